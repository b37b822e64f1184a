set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_textures.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tex_tests.log 2>&1
rc=$?; tail -8 gpurun_out/tex_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_tex.log 2>&1
  rc=$?; tail -c 400 gpurun_out/bench_tex.log; exit $rc
fi
