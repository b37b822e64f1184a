#!/bin/bash
# usage: gpurun_cmp.sh  -> GPU tests + bench of both pipelines
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1
rc=$?; echo "TEST rc=$rc"; tail -4 gpurun_out/t.log
if [ $rc -gt 1 ]; then echo "tests crashed/timed out; stopping"; exit $rc; fi
for p in wavefront megakernel; do
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu --pipeline $p > gpurun_out/b_$p.json 2>gpurun_out/b_$p.err || { echo "bench $p failed"; tail gpurun_out/b_$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$p.json'));c=d['config'];print('$p',d['value'],d['ms_per_step'],c['stage_ms'],json.load(open('gpurun_out/b_$p.json'))['config'].get('stage6'),c['iterations'],d['roofline']['frac'])"
done
