# Round-3 scheduling sweep (C3g, bench.py defaults): stagger on/off, then finish share, tail
# threshold and frames in flight with the stagger.  One JSON line per run in gpurun_out/sw_*.json.
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --steps 48 > gpurun_out/sw_$name.json 2> gpurun_out/sw_$name.err || { tail -5 gpurun_out/sw_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['frames_in_flight'], [round(x,3) for x in d['config']['stage_ms']])"
}
for i in 1 2; do
  run nostag_$i RT_STAGGER=0
  run stag_$i RT_STAGGER=1
done
run stag_ff20 RT_FINISH_FRAC=20
run stag_ff30 RT_FINISH_FRAC=30
run stag_ff55 RT_FINISH_FRAC=55
run stag_t786 RT_TAIL_RAYS=786432
run stag_t2m RT_TAIL_RAYS=2097152
run stag_sort RT_RAY_SORT=1
