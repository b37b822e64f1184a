# Round-3 final: the -m gpu suite, the spans-off A/B (off = product library, fix = per-block spans
# on, qc = before the spans), the round's profile set (TAG=r03g) and the C3r bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="off:off fix:fix qc:qc:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20" REPS=2 EXTRA=--no-isolated bash tools/gpurun_ab4.sh || exit 1
TAG=r03g bash tools/gpurun_profile.sh || exit 1
timeout -k 10 300 python -u bench.py --scene c3r > gpurun_out/r03g_c3r_bench.json 2> gpurun_out/r03g_c3r_bench.err
rc=$?; cat gpurun_out/r03g_c3r_bench.json; exit $rc
