#!/bin/bash
# A/B/C... of library builds ab_<name>.so at the repo root, alternating runs:
#   LIBS="noslp iterative-ilp" REPS=3 bash tools/gpurun_libab.sh   (FINAL = the build left in place)
mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for v in ${LIBS}; do
    cp ab_$v.so metal4-raytracing_amd/librt_hip.so
    timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 $EXTRA > gpurun_out/lab_$v$i.log 2>&1 || { tail -c 1500 gpurun_out/lab_$v$i.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'], d['config']['stage_ms'])" gpurun_out/lab_$v$i.log "$v $i"
  done
done
cp ab_${FINAL:-${LIBS%% *}}.so metal4-raytracing_amd/librt_hip.so
