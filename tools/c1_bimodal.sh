#!/bin/bash
# the configs[0]-sized frame (65K paths) ran bimodally on eight slots.  Six runs of it with
# eight frames in flight, each under rocprofv3 --kernel-trace, then tools/c1_bimodal.py compares the
# slow and the fast runs' kernels (durations, overlap, gaps).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/c1b
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c1b/run$i -o run -- \
    python3 $R/bench.py --scene c1 --width 256 --height 256 --spp 1 --bounces 1 --steps 400 --warmup 20 \
    --frames-in-flight 8 --no-cpu --no-pmc --no-isolated > $R/gpurun_out/c1b/run$i.log 2>&1) || { echo "run $i failed"; tail -5 gpurun_out/c1b/run$i.log; exit 1; }
done
python3 tools/c1_bimodal.py gpurun_out/c1b
