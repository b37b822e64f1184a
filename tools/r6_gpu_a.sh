#!/bin/bash
# round 6 GPU call A: the full -m gpu suite, then (only if it ran to completion without a crash or a
# time limit) the triangle-record A/B sweep and the instance-motion table.
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=2 CASE_TIMEOUT=150 timeout -k 10 600 bash tools/sweep.sh tools/cases_r6_tri.txt > gpurun_out/sweep_tri.log 2>&1 || exit 3
REPS=1 CASE_TIMEOUT=150 timeout -k 10 400 bash tools/sweep.sh tools/cases_r6_move.txt > gpurun_out/sweep_move.log 2>&1 || exit 4
