#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
RT_WF_LOG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/wflog.json 2> gpurun_out/wflog.err || { tail -5 gpurun_out/wflog.err; exit 1; }
grep "\[wf\]" gpurun_out/wflog.err | tail -14
SWEEP=${SWEEP:-"RT_DRAIN=0 RT_DRAIN=8 RT_DRAIN=16 RT_DRAIN=32 RT_DRAIN=16,RT_TAIL_RAYS=16777216 RT_DRAIN=32,RT_TAIL_RAYS=16777216"} bash tools/gpurun_sweep.sh
