#!/bin/bash
# default bench at 2 / 3 / 4 frames in flight (alternating), value + dominant-kernel frac
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for f in 2 3 4; do
    timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 --frames-in-flight $f $EXTRA > gpurun_out/fif_$f$i.log 2>&1 || { tail -c 1500 gpurun_out/fif_$f$i.log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/fif_$f$i.log') if x.startswith('{')][-1])
r=d['roofline']
print('fif $f', $i, d['value'], d['ms_per_step'], 'frac', r['frac'], 'launch_ms', r['launch_ms'], [(k['kernel'][:22], k['ms_per_frame'], k['launch_ms']) for k in r['kernels']])"
  done
done
