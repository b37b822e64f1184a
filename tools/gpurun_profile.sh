#!/bin/bash
# Round artefacts (run from the repo root on the GPU box):
#   1. the default bench line (with the CPU baseline)           -> gpurun_out/${TAG}_bench.json
#   2. rocprofv3 --kernel-trace --stats of a bench run            -> gpurun_out/${TAG}_kernel_stats.csv
#   3. three --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT+TCC_MISS) -> gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_pmc_TCC_HIT_sum/run_counter_collection.csv
TAG=${TAG:-r02}
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || { echo "kernel trace failed"; exit 1; }
cp $R/gpurun_out/${TAG}_prof/run_kernel_stats.csv $R/gpurun_out/${TAG}_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=${c%% *}
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/${TAG}_pmc_$n -o run -- python3 $R/bench.py --no-cpu > $R/gpurun_out/${TAG}_pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
cd $R
python3 tools/traffic_json.py gpurun_out/${TAG}_pmc_FETCH_SIZE/run_counter_collection.csv,gpurun_out/${TAG}_pmc_WRITE_SIZE/run_counter_collection.csv gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_pmc_TCC_HIT_sum/run_counter_collection.csv
