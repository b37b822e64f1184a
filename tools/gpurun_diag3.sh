# Round-3 diagnostics: kernel timeline of the default bench, the serial per-round log (RT_WF_LOG),
# and A/B runs (octant-grouped rays, three frames in flight).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
# the shadow-helper finish kernel (RT_SHADOW_HELP=1) against the oracle first
RT_SHADOW_HELP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c1_parity or glass or bunny or temporal or light or configs2 or golden" > gpurun_out/help_tests.log 2>&1
rc=$?; tail -3 gpurun_out/help_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03d_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 24 > $R/gpurun_out/r03d_prof.log 2>&1 || { echo "kernel trace failed"; tail $R/gpurun_out/r03d_prof.log; exit 1; }
cd $R
python3 tools/timeline_report.py gpurun_out/r03d_prof/run_kernel_trace.csv 16
RT_WF_LOG=1 timeout -k 10 200 python -u bench.py --no-cpu --frames-in-flight 1 --steps 3 --warmup 1 > gpurun_out/wflog.json 2> gpurun_out/wflog.err || { tail gpurun_out/wflog.err; exit 1; }
grep "\[wf\]" gpurun_out/wflog.err | tail -24
run() {  # name, env..., then bench args after --
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --steps 48 > gpurun_out/d3_$name.json 2> gpurun_out/d3_$name.err || { tail -5 gpurun_out/d3_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/d3_$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['frames_in_flight'], [round(x,3) for x in d['config']['stage_ms']])"
}
for i in 1 2; do
  run base_$i RT_RAY_SORT=0
  run sort_$i RT_RAY_SORT=1
  run fif3_$i RT_FRAMES_IN_FLIGHT=3
  run help_$i RT_SHADOW_HELP=1
done
