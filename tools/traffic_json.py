"""Per-launch HBM traffic of the dominant kernel from the FETCH_SIZE / WRITE_SIZE passes, plus the
L2 (TCC) hit rate per kernel from the TCC_HIT / TCC_MISS pass, written as the JSON bench.py reads
for roofline.traffic / roofline.l2_hit (same kernel name and config as the bench line).

usage: traffic_json.py FETCH.csv,WRITE.csv BENCH.json OUT.json [TCC.csv]
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def l2_hit_rates(path):
    """{kernel short name: TCC hit fraction} over all dispatches of each kernel."""
    hit, miss = collections.defaultdict(float), collections.defaultdict(float)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace(" ", "")
            if "rocclr" in k:
                continue
            v = float(row["Counter_Value"])
            if row["Counter_Name"].startswith("TCC_HIT"):
                hit[k] += v
            elif row["Counter_Name"].startswith("TCC_MISS"):
                miss[k] += v
    return {k: round(hit[k] / (hit[k] + miss[k]), 4) for k in hit if hit[k] + miss[k] > 0}


def main():
    csvs, bench_json, out = sys.argv[1], sys.argv[2], sys.argv[3]
    line = json.loads(open(bench_json).read().strip().splitlines()[-1])
    cfg = line["config"]
    per_launch = bench.read_traffic(csvs.split(","), bench.traffic_key(line["roofline"]["kernel"]))
    # every timed kernel of the line (the dominant one can change between runs)
    by_kernel = {k["kernel"]: bench.read_traffic(csvs.split(","), bench.traffic_key(k["kernel"]))
                 for k in line["roofline"].get("kernels", [])}
    res = {
        "kernel": line["roofline"]["kernel"],
        "config": [cfg["scene"], cfg["width"], cfg["height"], cfg["spp"], cfg["max_bounces"]],
        "bytes_per_launch": per_launch,
        "bytes_per_launch_by_kernel": by_kernel,
        "algorithmic_bytes_per_launch": line["roofline"]["bytes_per_launch"],
        "source": "rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, per dispatch of the dominant kernel, "
                  + os.path.basename(out).split("_")[0],
    }
    if len(sys.argv) > 4 and os.path.exists(sys.argv[4]):
        res["l2_hit"] = l2_hit_rates(sys.argv[4])
        res["l2_source"] = "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum, all dispatches per kernel"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
