#!/bin/bash
# Every BASELINE config through bench.py at the library defaults (one GPU), the emulated per-rank
# shares of the 2 / 4 / 8-way C3g split, and one rank of configs[3]'s 8-way 4K x 16 split
# (bench.py --emulate-ranks N: rank 0's tiles, no gather).  Every row runs bench.py's PMC passes, so
# its frac is an HBM fraction (rocprofv3 bytes over the launch time alone); the algorithmic rate is
# printed in GB/s beside it (it counts L2 / MALL hits too and is no fraction of HBM).  One summary
# line per run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/cfg_$tag.log 2>&1 || { tail -c 1500 gpurun_out/cfg_$tag.log; exit 1; }
  python3 - gpurun_out/cfg_$tag.log $tag <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r, c = d["roofline"], d["cpu_baseline"]
assert r["frac"] is not None and r["frac"] < 1, r.get("frac_source")
v = (r.get("valu_issue") or {}).get(r["kernel"]) or {}
print(sys.argv[2], d["value"], "ms/step", d["ms_per_step"], "ms/frame", d.get("ms_per_frame"), "fif", d["config"]["frames_in_flight"],
      r["kernel"][:24], "frac(pmc)", r["frac"], "l2_hit", r["l2_hit"] and r["l2_hit"].get(r["kernel"]),
      "alg_GBs", r.get("achieved_algorithmic"), "valu_issue", v.get("frac_valu_issue"), "lane_util", v.get("lane_util"),
      "visits", d["config"].get("visits_per_ray"), "cpu", c and c["value"], flush=True)
PY
}
run c1 --scene c1 --width 256 --height 256 --spp 1 --bounces 1 --steps 400 --warmup 20 --cpu-seconds 6
run c2 --scene c2 --width 1280 --height 720 --spp 4 --bounces 4 --steps 128 --warmup 8 --cpu-seconds 6
run c3g --steps 64 --warmup 6 --cpu-seconds 6
# the frames in flight a reference user would see: three (Renderer.swift:207) and the library's default
# without GPU_MAX_HW_QUEUES (four hardware queues -> four slots)
run c3g_fif3 --steps 64 --warmup 6 --frames-in-flight 3 --no-cpu
(export RT_HW_QUEUES=4; run c3g_q4 --steps 64 --warmup 6 --no-cpu) || exit 1
run c3d --scene c3d --steps 32 --warmup 4 --cpu-seconds 6
run c3r --scene c3r --steps 32 --warmup 4 --cpu-seconds 6
run c5 --scene c5 --bounces 2 --animate --steps 64 --warmup 4 --cpu-seconds 6
for n in 2 4 8; do
  run r$n --emulate-ranks $n --steps 300 --warmup 10 --no-cpu
done
run c4r8 --width 3840 --height 2160 --spp 16 --steps 6 --warmup 2 --emulate-ranks 8 --no-cpu
