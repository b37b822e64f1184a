#!/bin/bash
# kernel-trace one short bench run -> gpurun_out/prof_$TAG
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG:-x} -o run --output-format csv -- python3 $R/bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu --pipeline ${PIPE:-wavefront} ${BENCH_ARGS} > $R/gpurun_out/prof_${TAG:-x}.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof_${TAG:-x}.log | cut -c1-300; exit $rc
