#!/bin/bash
# per-iteration log of one bench frame, then the bench over finish thresholds
mkdir -p gpurun_out
RT_WF_LOG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/wflog.json 2> gpurun_out/wflog.err || { tail -5 gpurun_out/wflog.err; exit 1; }
grep "\[wf\]" gpurun_out/wflog.err | tail -12
SWEEP=${SWEEP:-"RT_TAIL_RAYS=262144 RT_TAIL_RAYS=524288 RT_TAIL_RAYS=1048576 RT_TAIL_RAYS=2097152"} bash tools/gpurun_sweep.sh
