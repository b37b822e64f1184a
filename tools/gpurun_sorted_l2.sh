# L2 (TCC) hit rate of the sorted-hit shade kernel: one TCC_HIT/TCC_MISS pass of the bench with the
# per-bounce hit sort enabled (--sort-bins 2048), summarised per kernel into gpurun_out/<TAG>_l2_sorted.json
set -o pipefail
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/${TAG:-r02}_pmc_sorted -o run -- python3 $R/bench.py --no-cpu --sort-bins 2048 --steps 8 > $R/gpurun_out/${TAG:-r02}_pmc_sorted.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/${TAG:-r02}_pmc_sorted.log; exit 1; }
cd $R
TAG=${TAG:-r02} python3 - <<'PY'
import json, os, sys
T = os.environ["TAG"]
sys.path.insert(0, "tools")
from traffic_json import l2_hit_rates
r = l2_hit_rates(f"gpurun_out/{T}_pmc_sorted/run_counter_collection.csv")
json.dump({"config": "c3g 1920x1080x4spp 8 bounces, --sort-bins 2048", "l2_hit": r,
           "source": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum, all dispatches per kernel"},
          open(f"gpurun_out/{T}_l2_sorted.json", "w"), indent=1)
print(json.dumps(r))
PY

timeout -k 10 200 python3 bench.py --no-cpu --sort-bins 2048 > gpurun_out/${TAG:-r02}_bench_sorted.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG:-r02}_bench_sorted.json').read().strip().splitlines()[-1]); print('sorted', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
