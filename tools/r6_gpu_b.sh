#!/bin/bash
# round 6 GPU call B: the full -m gpu suite (all failures listed), then the lazy-id A/B, the
# frames-in-flight lines and the motion table's visit counts -- each only after the previous step
# ended without a crash or a time limit.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --maxfail=20 --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 CASE_TIMEOUT=150 timeout -k 10 700 bash tools/sweep.sh tools/cases_r6_lazy.txt > gpurun_out/sweep_lazy.log 2>&1 || exit 3
REPS=1 CASE_TIMEOUT=150 timeout -k 10 300 bash tools/sweep.sh tools/cases_r6_fif.txt > gpurun_out/sweep_fif.log 2>&1 || exit 4
REPS=1 CASE_TIMEOUT=150 timeout -k 10 400 bash tools/sweep.sh tools/cases_r6_move2.txt > gpurun_out/sweep_move2.log 2>&1 || exit 5
