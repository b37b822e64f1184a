#!/bin/bash
# HIP-event launch times (bench.py) against rocprofv3 kernel durations, per frames-in-flight count
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in ${FIFS:-2 4}; do
  timeout -k 10 200 python bench.py --no-cpu --frames-in-flight $f > gpurun_out/fp${f}_bench.json 2> gpurun_out/fp${f}_bench.err || { echo "bench failed"; exit 1; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fp${f}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --frames-in-flight $f > $R/gpurun_out/fp${f}_prof.log 2>&1 || { echo "kernel trace failed"; exit 1; }
  cd $R
  python3 -c "
import json,csv
d=json.loads(open('gpurun_out/fp${f}_bench.json').read().strip().splitlines()[-1])
print('fif $f value', d['value'], 'ms', d['ms_per_step'], [(k['kernel'][:24], round(k['launch_ms'],4), round(k['achieved'],1)) for k in d['roofline']['kernels']], 'job', d['roofline']['job_achieved'])
for r in csv.DictReader(open('gpurun_out/fp${f}_prof/run_kernel_stats.csv')):
    if 'wf_trace' in r['Name'] or 'finish' in r['Name']:
        print('   ', r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6)
"
done
