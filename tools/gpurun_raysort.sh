# Extend / shadow ray grouping in wf_shade (RT_RAY_SORT = 0 off, 1 direction octant, 2 direction +
# origin octant): golden parity of each mode, alternating A/B on the default bench workload, and
# one TCC_HIT/TCC_MISS pass per mode (L2 hit rate of the extend launches that read the grouped
# rays) -> gpurun_out/${TAG}_l2_raysort.json; then the hit-sorted shade pass (gpurun_sorted_l2.sh).
set -o pipefail
R=$PWD
TAG=${TAG:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_env_variants.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/raysort_tests.log 2>&1
rc=$?; tail -3 gpurun_out/raysort_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # name, mode
  RT_RAY_SORT=$2 timeout -k 10 200 python -u bench.py --no-cpu --steps 48 > gpurun_out/rs_$1.json 2> gpurun_out/rs_$1.err || { tail -5 gpurun_out/rs_$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rs_$1.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], [(k['kernel'][:12], k['launch_ms']) for k in r['kernels']], [round(x,3) for x in d['config']['stage_ms']])"
}
for i in 1 2 3; do
  run off_$i 0 || exit 1
  run dir_$i 1 || exit 1
  run dirorg_$i 2 || exit 1
done
cd /tmp
for m in 0 1 2; do
  RT_RAY_SORT=$m timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/${TAG}_pmc_rs$m -o run -- python3 $R/bench.py --no-cpu --steps 8 > $R/gpurun_out/${TAG}_pmc_rs$m.log 2>&1 || { echo "pmc $m failed"; tail -5 $R/gpurun_out/${TAG}_pmc_rs$m.log; exit 1; }
done
cd $R
TAG=$TAG python3 - <<'PY'
import json, os, sys
T = os.environ["TAG"]
sys.path.insert(0, "tools")
from traffic_json import l2_hit_rates
out = {"config": "c3g 1920x1080x4spp 8 bounces, two frames in flight; RT_RAY_SORT = 0 / 1 / 2",
       "source": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum, all dispatches per kernel"}
for m in (0, 1, 2):
    out[f"ray_sort_{m}"] = l2_hit_rates(f"gpurun_out/{T}_pmc_rs{m}/run_counter_collection.csv")
json.dump(out, open(f"gpurun_out/{T}_l2_raysort.json", "w"), indent=1)
for m in (0, 1, 2):
    print(m, {k: v for k, v in out[f"ray_sort_{m}"].items() if "trace" in k or "shade" in k})
PY
TAG=$TAG bash tools/gpurun_sorted_l2.sh
