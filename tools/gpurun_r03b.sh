# Round-3 batch: library A/B (triangle copies, LDS top nodes), the full -m gpu suite on the current
# build, the suite's parity subset with frame graphs (RT_GRAPH=1), and a graph A/B.
set -o pipefail
mkdir -p gpurun_out
LIBS="noperm perm permnotop" REPS=3 bash tools/gpurun_ab3.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_b.log; [ $rc -ne 0 ] && exit $rc
RT_GRAPH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_inflight.py tests/test_gpu_inflight_edges.py tests/test_gpu_dynamic.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/graph_tests.log 2>&1
rc=$?; tail -3 gpurun_out/graph_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for g in 0 1; do
    RT_GRAPH=$g timeout -k 10 200 python -u bench.py --no-cpu --steps 48 > gpurun_out/g${g}_${i}.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/g${g}_${i}.json')); print('graph=$g', d['value'], d['ms_per_step'], d['config']['host_submit_ms'], d['roofline']['frac'], d['config']['stage_ms'])"
  done
done
