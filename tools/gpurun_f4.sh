# Four frames in flight by default: the -m gpu suite, the tail threshold / finish share at four slots,
# and a rocprofv3 kernel trace of the default bench (HIP-event and device-clock launch times vs rocprof).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_f4.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_f4.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="d:f4 t1m:f4:RT_TAIL_RAYS=1048576 t13:f4:RT_TAIL_RAYS=1310720 t5:f4:RT_TAIL_RAYS=524288 fr20:f4:RT_FINISH_FRAC=20 fr33:f4:RT_FINISH_FRAC=33" REPS=2 bash tools/gpurun_ab4.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f4 -o run -- python3 bench.py --no-cpu > gpurun_out/prof_f4.log 2>&1
rc=$?; tail -2 gpurun_out/prof_f4.log; exit $rc
