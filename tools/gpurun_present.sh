set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_present.py -x -v --timeout 120 --timeout-method thread > gpurun_out/present_tests.log 2>&1
rc=$?; tail -8 gpurun_out/present_tests.log; exit $rc
