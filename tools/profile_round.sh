#!/bin/bash
# The round's measurement artefacts (run from the repo root on the GPU box; copy the results into
# profiles/ under the round's tag):
#   1. the default bench line (with its live PMC passes and the CPU baseline)
#        -> gpurun_out/${TAG}_bench.json, PMC CSVs under gpurun_out/${TAG}_pmc/
#   2. rocprofv3 --kernel-trace --stats of the same workload with one frame in flight (the
#      kernels alone: what the roofline prices) -> gpurun_out/${TAG}_alone_kernel_stats.csv
#   3. the same with the default frames in flight -> gpurun_out/${TAG}_kernel_stats.csv
#   4. tools/roofline_check.py: the line's frac recomputed from 1 + 2
TAG=${TAG:-r04}
R=$PWD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --pmc-dir $R/gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
python3 tools/line_summary.py gpurun_out/${TAG}_bench.json bench
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_alone -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-pmc --frames-in-flight 1 > $R/gpurun_out/${TAG}_alone.log 2>&1 || { echo "kernel trace (alone) failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-pmc > $R/gpurun_out/${TAG}_prof.log 2>&1 || { echo "kernel trace failed"; exit 1; }
cd $R
cp gpurun_out/${TAG}_alone/run_kernel_stats.csv gpurun_out/${TAG}_alone_kernel_stats.csv
cp gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
python3 tools/roofline_check.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_alone_kernel_stats.csv
