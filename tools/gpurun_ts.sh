# Device-clock launch spans: the -m gpu suite, A/B of two vs three frames in flight, and a rocprofv3
# kernel trace of the three-frame bench to compare the spans with the dispatch durations.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ts.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_ts.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="fif2:ts fif3:ts:RT_FRAMES_IN_FLIGHT=3" REPS=2 bash tools/gpurun_ab4.sh || exit 1
RT_FRAMES_IN_FLIGHT=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fif3 -o run -- python3 bench.py --no-cpu --steps 32 --warmup 4 > gpurun_out/prof_fif3.log 2>&1
rc=$?; tail -2 gpurun_out/prof_fif3.log; exit $rc
