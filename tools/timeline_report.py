#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (run_kernel_trace.csv): over the last K frames, the wall
span, how much of it some kernel was running (union of dispatch intervals), the mean number of
dispatches running at once, and per kernel the summed and mean duration.

  python3 tools/timeline_report.py gpurun_out/prof_x/run_kernel_trace.csv [frames]

A frame starts at a wf_generate (or megakernel) dispatch; with frames in flight the frames of
different streams interleave, so the window is "from the K-th last generate to the end"."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gen = [i for i, r in enumerate(rows) if "wf_generate" in r["Kernel_Name"] or "megakernel" in r["Kernel_Name"]]
    if len(gen) < frames + 1:
        frames = max(1, len(gen) - 1)
    w = rows[gen[-frames - 1]:]
    t0 = int(rows[gen[-frames - 1]]["Start_Timestamp"])
    ev = []
    per = collections.defaultdict(lambda: [0, 0.0])
    t1 = t0
    for r in w:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0:
            continue
        t1 = max(t1, e)
        ev.append((s, 1))
        ev.append((e, -1))
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace(" ", "")
        per[name][0] += 1
        per[name][1] += (e - s) / 1e3
    ev.sort()
    busy, area, cur, last = 0, 0, 0, t0
    for t, d in ev:
        if cur > 0:
            busy += t - last
        area += cur * (t - last)
        cur += d
        last = t
    span = t1 - t0
    print(f"window: {frames} frames, span {span / 1e3:.1f} us ({span / 1e3 / frames:.1f} us/frame)")
    print(f"busy (any dispatch running): {busy / span:.3f} of the span; mean dispatches running {area / max(span, 1):.2f}")
    for name, (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {name[:60]:60s} {n:5d} x {us / n:8.1f} us = {us / frames:8.1f} us/frame")


if __name__ == "__main__":
    main()
