# Round-3 GPU check: the -m gpu suite (full-size parity included), the default bench line, then the
# scheduling sweep (tools/gpurun_sweep3.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -ne 0 ] && exit $rc
bash tools/gpurun_sweep3.sh
