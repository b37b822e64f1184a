#!/bin/bash
# A/B/C... of environment settings on the default bench, alternating runs:
#   VARIANTS="base RT_NODE_PAD=1 RT_TRI_PAD=1" REPS=2 bash tools/gpurun_multiab.sh
# (a variant is "base" or a comma-separated list of VAR=value; EXTRA = more bench.py arguments)
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    o=gpurun_out/mab_${i}_$(echo "$v" | tr '=,' '__')
    env $envs timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 $EXTRA > $o.log 2>&1 || { tail -c 1500 $o.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
r=d['roofline']
print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], 'frac', r['frac'], 'stage', d['config']['stage_ms'], [(k['kernel'][:20], k['launch_ms']) for k in r['kernels']])" $o.log "$v" $i
  done
done
