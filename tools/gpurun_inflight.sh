set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflight.py -x -v --timeout 120 --timeout-method thread > gpurun_out/inflight_tests.log 2>&1
rc=$?; tail -5 gpurun_out/inflight_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for f in ${FIFS:-1 2}; do
  timeout -k 10 300 python -u bench.py --no-cpu --frames-in-flight $f > gpurun_out/bench_fif$f.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -c 1500 gpurun_out/bench_fif$f.log; exit $rc; }
  python -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_fif$f.log') if x.startswith('{')][-1])
print('fif $f', d['value'], d['ms_per_step'], d['config']['stage_ms'], d['roofline']['frac'])"
done
