#!/bin/bash
# bench line + rocprof kernel-trace stats of the same command at FIF frames in flight and HWQ
# hardware queues: does the HIP-event launch time of the dominant kernel agree with rocprof's?
FIF=${FIF:-4}; HWQ=${HWQ:-8}
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=$HWQ
timeout -k 10 300 python bench.py --no-cpu --frames-in-flight $FIF > gpurun_out/fp_${FIF}_${HWQ}.json 2> gpurun_out/fp_${FIF}_${HWQ}.err || { tail -5 gpurun_out/fp_${FIF}_${HWQ}.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fp_prof_${FIF}_${HWQ} -o run --output-format csv -- python3 $R/bench.py --no-cpu --frames-in-flight $FIF > $R/gpurun_out/fp_prof_${FIF}_${HWQ}.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
python3 -c "
import json,csv,sys
d=json.load(open('gpurun_out/fp_${FIF}_${HWQ}.json')); r=d['roofline']
print('bench', d['value'], d['ms_per_step'], 'launch_ms', r['launch_ms'], 'frac', r['frac'])
for row in csv.DictReader(open('gpurun_out/fp_prof_${FIF}_${HWQ}/run_kernel_stats.csv')):
    if 'wf_trace<false, false>' in row['Name'] or 'wf_trace<true, false>' in row['Name'] or 'finish_step<false, false' in row['Name']:
        print(row['Name'][:40], row['Calls'], float(row['AverageNs'])/1e6)
"
