#!/bin/bash
# Serial PMC analysis: one rocprofv3 --pmc pass per line of tools/pmc_sets.txt (each within the
# per-block counter limits of MI355X_MICROARCH.md 'rocprofv3 PMC slots'), over bench.py with the
# given arguments (default: the C3g frame, one frame in flight), then tools/pmc_report.py.
#   bash tools/pmc_passes.sh [bench args...]   -> gpurun_out/pmc/p<N>/run_counter_collection.csv
R=$PWD
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${*:---frames-in-flight 1 --steps 4 --warmup 1}
n=0
while IFS= read -r set; do
  [ -z "$set" ] && continue
  n=$((n + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$n -o run -- \
    python3 $R/bench.py --no-cpu --no-pmc --no-isolated $ARGS > $R/gpurun_out/pmc/p$n.log 2>&1) || { echo "pmc pass $n failed"; tail -5 gpurun_out/pmc/p$n.log; exit 1; }
done < tools/pmc_sets.txt
python3 tools/pmc_report.py wf_
