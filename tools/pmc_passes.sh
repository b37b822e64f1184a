#!/bin/bash
# Serial PMC analysis: one rocprofv3 --pmc pass per line of the counter-set file (each within the
# per-block counter limits of MI355X_MICROARCH.md 'rocprofv3 PMC slots'), over bench.py with the
# given arguments (default: the C3g frame, one frame in flight), then tools/pmc_report.py.
#   [PMC_SETS=file] [PMC_OUT=dir] bash tools/pmc_passes.sh [bench args...]
#   -> $PMC_OUT/p<N>/run_counter_collection.csv (default tools/pmc_sets.txt, gpurun_out/pmc)
R=$PWD
set -o pipefail
SETS=${PMC_SETS:-tools/pmc_sets.txt}
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${*:---frames-in-flight 1 --steps 4 --warmup 1}
n=0
while IFS= read -r set; do
  [ -z "$set" ] && continue
  n=$((n + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$n -o run -- \
    python3 $R/bench.py --no-cpu --no-pmc --no-isolated $ARGS > $R/$OUT/p$n.log 2>&1) || { echo "pmc pass $n failed"; tail -5 $OUT/p$n.log; exit 1; }
done < $SETS
python3 tools/pmc_report.py wf_ $OUT
