#!/bin/bash
# serial (one frame at a time) bench over several builds of librt_hip.so: LIBS="a b c" (ab_<name>.so)
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for v in $LIBS; do
    cp ab_$v.so metal4-raytracing_amd/librt_hip.so
    timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-16} --warmup 2 ${EXTRA:---frames-in-flight 1} > gpurun_out/multi_$v$i.log 2>&1 || { tail -c 1500 gpurun_out/multi_$v$i.log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/multi_$v$i.log') if x.startswith('{')][-1])
print('$v', $i, d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
