# Bench sweep on the GPU box: each line of the case file ($1) is "name ENV=v ... -- bench args"; every case
# runs REPS times (alternating), one summary line per run (tools/line_summary.py).  Logs go to
# gpurun_out/sw_<name><rep>.log.
set -o pipefail
CASEFILE=$1
# a case's LIB=name runs it on ab_name.so (a variant build: make VARIANT=name DEFS=...); the
# product library is restored afterwards
cp metal4-raytracing_amd/librt_hip.so /tmp/librt_keep.so
trap 'cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so' EXIT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    set -- $line
    name=$1; shift
    envs=()
    lib=""
    while [ "$1" != "--" ]; do
      case "$1" in LIB=*) lib=${1#LIB=} ;; *) envs+=("$1") ;; esac
      shift
    done; shift
    if [ -n "$lib" ]; then cp ab_$lib.so metal4-raytracing_amd/librt_hip.so; else cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so; fi
    env "${envs[@]}" timeout -k 10 ${CASE_TIMEOUT:-200} python -u bench.py --no-cpu --no-pmc "$@" > gpurun_out/sw_$name$rep.log 2>&1 \
      || { tail -c 2000 gpurun_out/sw_$name$rep.log; exit 1; }
    python3 tools/line_summary.py gpurun_out/sw_$name$rep.log "$name$rep" || exit 1
  done < "$CASEFILE"
done
