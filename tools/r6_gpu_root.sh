#!/bin/bash
# the root-leaf-triangles-in-LDS variant: its traversal-heavy parity tests on ab_root.so, then the A/B
mkdir -p gpurun_out
cp metal4-raytracing_amd/librt_hip.so /tmp/librt_keep.so
cp ab_root.so metal4-raytracing_amd/librt_hip.so
timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_traversal_variants.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/root_tests.log 2>&1
rc=$?
cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so
echo "tests rc $rc" >> gpurun_out/root_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 CASE_TIMEOUT=150 timeout -k 10 800 bash tools/sweep.sh tools/cases_r6_root.txt > gpurun_out/sweep_root.log 2>&1 || exit 3
