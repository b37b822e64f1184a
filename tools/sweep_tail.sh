# Finish-threshold sweep (round 4 baseline): one frame at a time, four frames in flight, and one
# rank's share of the 8-way split, each at several RT_TAIL_RAYS values; plus an RT_WF_LOG frame.
set -o pipefail
mkdir -p gpurun_out
one() {   # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python -u bench.py --no-cpu "$@" > gpurun_out/sw_$name.log 2>&1 || { tail -c 2000 gpurun_out/sw_$name.log; return 1; }
  python3 tools/line_summary.py gpurun_out/sw_$name.log "$name"
}
RT_WF_LOG=1 timeout -k 10 200 python -u bench.py --no-cpu --no-isolated --frames-in-flight 1 --steps 2 --warmup 1 > gpurun_out/sw_wflog.log 2>&1 || exit 1
for t in ${TAILS1:-4194304 2097152 1048576 524288 262144}; do
  one f1_$t RT_TAIL_RAYS=$t -- --no-isolated --frames-in-flight 1 --steps 20 --warmup 3 || exit 1
done
for t in ${TAILS4:-786432 393216 196608}; do
  one f4_$t RT_TAIL_RAYS=$t -- --no-isolated --steps 60 --warmup 5 || exit 1
done
for t in ${TAILS8:-786432 262144 131072}; do
  one r8_$t RT_TAIL_RAYS=$t -- --no-isolated --emulate-ranks 8 --steps 200 --warmup 10 || exit 1
done
