#!/bin/bash
# device BVH builders on the default bench (--bvh lbvh): LBVH/PLOC x greedy/DP
mkdir -p gpurun_out
for i in $(seq ${REPS:-1}); do
  for cfg in "lbvh greedy" "lbvh dp" "ploc greedy" "ploc dp"; do
    set -- $cfg
    RT_DEVICE_BVH=$1 RT_DEVICE_COLLAPSE=$2 timeout -k 10 200 python -u bench.py --no-cpu --bvh lbvh --steps ${STEPS:-16} --warmup 2 $EXTRA > gpurun_out/devbvh_$1_$2_$i.log 2>&1 || { tail -c 2000 gpurun_out/devbvh_$1_$2_$i.log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/devbvh_$1_$2_$i.log') if x.startswith('{')][-1])
r=d['roofline']
print('$1 $2', $i, d['value'], d['ms_per_step'], 'setup', d['config']['setup_s'], 'npr', r['nodes_per_ray'], 'tpr', r['tris_per_ray'], [(k['kernel'][:22], k['nodes_per_ray'], k['tris_per_ray']) for k in r['kernels']])"
  done
done
