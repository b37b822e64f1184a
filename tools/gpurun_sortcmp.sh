#!/bin/bash
# GPU tests, then the default bench over hit-sort / XCD-mapping / steal settings.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
SWEEP=${SWEEP:-"RT_SORT_BINS=0,RT_STEAL=0 RT_SORT_BINS=0 RT_SORT_BINS=2048 RT_SORT_BINS=2048,RT_SORT_XCD=0 RT_SORT_BINS=2048,RT_STEAL=0"} bash tools/gpurun_sweep.sh
