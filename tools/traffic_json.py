"""Per-launch HBM traffic of the dominant kernel from the FETCH_SIZE / WRITE_SIZE passes, written
as the JSON bench.py reads for roofline.traffic (same kernel name and config as the bench line)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

csvs, bench_json, out = sys.argv[1], sys.argv[2], sys.argv[3]
line = json.loads(open(bench_json).read().strip().splitlines()[-1])
cfg = line["config"]
per_launch = bench.read_traffic(csvs.split(","), r"wf_trace<(true|false),false>")
res = {
    "kernel": line["roofline"]["kernel"],
    "config": [cfg["scene"], cfg["width"], cfg["height"], cfg["spp"], cfg["max_bounces"]],
    "bytes_per_launch": per_launch,
    "algorithmic_bytes_per_launch": line["roofline"]["bytes_per_launch"],
    "source": "rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, per wf_trace<*, false> dispatch, "
              + os.path.basename(out).split("_")[0],
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
