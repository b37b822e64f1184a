#!/bin/bash
# round 6 measurement call: the full -m gpu suite, then the round's profiles (tools/profile_round.sh:
# the default bench line with its PMC passes and CPU baseline, rocprofv3 kernel stats alone and in
# flight, roofline_check), then the serial PMC passes -- each only after the previous step ended
# without a crash or a time limit.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --maxfail=20 --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=r06 timeout -k 10 1000 bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || exit 3
PMC_OUT=gpurun_out/pmc timeout -k 10 600 bash tools/pmc_passes.sh > gpurun_out/pmc_serial.txt 2>&1 || exit 4
