#!/bin/bash
# round 6 GPU call C: parity of the fp16-plane node build (the traversal-heavy GPU tests), then the
# node-format A/B (80-B byte nodes vs 128-B fp16 nodes at 8 / 7 extend waves).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q --maxfail=10 --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_traversal_variants.py tests/test_gpu_fullsize.py tests/test_gpu_lbvh.py \
  tests/test_gpu_dynamic.py > gpurun_out/gpu_tests_c.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/gpu_tests_c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 CASE_TIMEOUT=150 timeout -k 10 900 bash tools/sweep.sh tools/cases_r6_n16.txt > gpurun_out/sweep_n16.log 2>&1 || exit 3
