#!/bin/bash
# A/B of two builds of librt_hip.so (ab_old.so, ab_new.so at the repo root), alternating runs
mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for v in old new; do
    cp ab_$v.so metal4-raytracing_amd/librt_hip.so
    timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 $EXTRA > gpurun_out/ab_$v$i.log 2>&1 || { tail -c 1500 gpurun_out/ab_$v$i.log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/ab_$v$i.log') if x.startswith('{')][-1])
print('$v $i', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
cp ab_new.so metal4-raytracing_amd/librt_hip.so
