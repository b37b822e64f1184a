#!/bin/bash
# Every BASELINE config through bench.py at the library defaults (one GPU)
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 6 "$@" > gpurun_out/cfg_$tag.log 2>&1 || { tail -c 1500 gpurun_out/cfg_$tag.log; exit 1; }
  python -c "
import json
d=json.loads([x for x in open('gpurun_out/cfg_$tag.log') if x.startswith('{')][-1])
r=d['roofline']; c=d['cpu_baseline']
print('$tag', d['value'], d['ms_per_step'], d['config']['frames_in_flight'], r['kernel'][:22], r['frac'], c and c['value'])"
}
run c1 --scene c1 --width 256 --height 256 --spp 1 --bounces 1 --steps 400 --warmup 20
run c2 --scene c2 --width 1280 --height 720 --spp 4 --bounces 4 --steps 128 --warmup 8
run c3d --scene c3d --steps 32 --warmup 4
run c5 --scene c5 --bounces 2 --animate --steps 64 --warmup 4
