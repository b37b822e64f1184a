set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_qc.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_qc.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-base:base qc:qc qc2:qc2}" REPS=${REPS:-3} bash tools/gpurun_ab4.sh
