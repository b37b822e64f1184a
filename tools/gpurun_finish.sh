#!/bin/bash
# GPU tests, per-iteration log, then the bench over finish-kernel settings
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
RT_WF_LOG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/wflog.json 2> gpurun_out/wflog.err || { tail -5 gpurun_out/wflog.err; exit 1; }
grep "\[wf\]" gpurun_out/wflog.err | tail -5
SWEEP=${SWEEP:-"RT_FINISH_STEP=0 RT_FINISH_STEP=1 RT_SHADE_MIN=8 RT_SHADE_MIN=32 RT_TAIL_RAYS=2097152 RT_TAIL_RAYS=4194304"} bash tools/gpurun_sweep.sh
