#!/bin/bash
# PMC passes over a short bench run; each line of $SETS is one rocprofv3 --pmc pass.
mkdir -p gpurun_out/pmc
R=$PWD
export TMPDIR=/tmp
cd /tmp
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --pipeline ${PIPE:-wavefront} ${BENCH_ARGS} > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done < $R/${SETS:-tools/pmc_sets.txt}
exit 0
