#!/bin/bash
# A/B of one environment knob on the default bench: VAR=name A=value B=value (alternating runs)
mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for v in "$A" "$B"; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 $EXTRA > gpurun_out/envab_$v$i.log 2>&1 || { tail -c 1500 gpurun_out/envab_$v$i.log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/envab_$v$i.log') if x.startswith('{')][-1])
r=d['roofline']
print('$VAR=$v', $i, d['value'], d['ms_per_step'], d['config']['stage_ms'], 'npr', r['nodes_per_ray'], 'tpr', r['tris_per_ray'], 'frac', r['frac'], [(k['kernel'][:24], k['nodes_per_ray'], k['tris_per_ray']) for k in r['kernels']])"
  done
done
