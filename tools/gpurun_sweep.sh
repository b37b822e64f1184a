#!/bin/bash
# sweep env settings over short wavefront bench runs: SWEEP="VAR=a VAR=b,VAR2=c ..." (comma = same run)
mkdir -p gpurun_out
for kv in $SWEEP; do
  env ${kv//,/ } timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu --pipeline ${PIPE:-wavefront} ${BENCH_ARGS} > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo "fail $kv"; tail -3 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));c=d['config'];r=d['roofline'];print('$kv',d['value'],d['ms_per_step'],c['stage_ms'],c['iterations'],r['kernel'][:14],r['frac'],r.get('job_frac'))"
done
