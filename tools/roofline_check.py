#!/usr/bin/env python3
"""Recomputes a bench line's roofline from the rocprofv3 kernel-alone profile of the same workload:
the dominant kernel (most device time per frame with one frame in flight, by rocprof's kernel
trace) must be the line's, and frac = the line's PMC bytes per launch / rocprof's average duration
of that kernel / 8 TB/s must agree with the line's frac within 5 %.

  python3 tools/roofline_check.py BENCH.json ALONE_KERNEL_STATS.csv

Prints the comparison and exits non-zero when it does not hold."""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def rocprof_groups(stats_csv):
    """{kernel group: (calls, total ns)} of a rocprofv3 --stats kernel_stats.csv"""
    out = {}
    for row in csv.DictReader(open(stats_csv)):
        key = bench.kernel_key(row["Name"])
        if key is None:
            continue
        calls, total = out.get(key, (0, 0.0))
        out[key] = (calls + int(row["Calls"]), total + float(row["TotalDurationNs"]))
    return out


def check(line, stats_csv, tol=0.05):
    r = line["roofline"]
    groups = rocprof_groups(stats_csv)
    name_of = {k: n for k, n, _, _ in bench.KERNELS}
    top = max(groups, key=lambda k: groups[k][1])
    calls, total = groups[top]
    avg_ms = total / calls * 1e-6
    frac = r["traffic"] / (avg_ms * 1e-3) / 1e9 / r["peak"] if r.get("traffic") else None
    res = {"rocprof_top_kernel": name_of[top], "line_kernel": r["kernel"], "rocprof_avg_ms": round(avg_ms, 4),
           "line_launch_ms": r["launch_ms"], "frac_from_profiles": round(frac, 4) if frac else None,
           "line_frac": r["frac"],
           "rocprof_ms_per_kernel_group": {name_of[k]: round(v[1] * 1e-6, 3) for k, v in groups.items()}}
    ok = name_of[top] == r["kernel"] and frac is not None and abs(frac - r["frac"]) <= tol * r["frac"]
    return ok, res


def main():
    line = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
    ok, res = check(line, sys.argv[2])
    print(json.dumps(res, indent=1))
    print("roofline reproduces" if ok else "roofline does NOT reproduce")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
