#!/bin/bash
# round 6 closing measurement after the shading-latency changes: the full -m gpu suite, then the round's
# profiles (tools/profile_round.sh) -- each only after the previous step ended without a crash or a limit
mkdir -p gpurun_out
timeout -k 10 560 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests_final.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/gpu_tests_final.log
[ $rc -eq 0 ] || exit $rc
TAG=r06 timeout -k 10 600 bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || exit 3
