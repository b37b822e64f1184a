#!/usr/bin/env python3
"""Per run of tools/c1_bimodal.sh: the bench value, and over the timed frames' kernels (the last 400
frames' worth of dispatches): each kernel group's mean duration, the mean number of kernels running at
once, and the share of the timed span with no kernel running (gaps)."""
import csv
import glob
import json
import os
import sys


def main(d):
    for log in sorted(glob.glob(os.path.join(d, "run*.log"))):
        run = os.path.basename(log)[:-4]
        line = [x for x in open(log) if x.startswith("{")]
        val = json.loads(line[-1])["value"] if line else None
        tr = glob.glob(os.path.join(d, run, "**", "*kernel_trace.csv"), recursive=True)
        if not tr:
            print(run, val, "no trace")
            continue
        rows = [r for r in csv.DictReader(open(tr[0])) if "rt::" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        rows = rows[len(rows) // 3:]   # past the counting frame and the warm-up
        spans = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")) for r in rows]
        t0, t1 = spans[0][0], max(e for _, e, _ in spans)
        busy = sum(e - s for s, e, _ in spans)
        # union of kernel intervals -> idle share
        cov, cur_s, cur_e = 0, None, None
        for s, e, _ in spans:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    cov += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        cov += cur_e - cur_s
        by = {}
        for s, e, n in spans:
            a = by.setdefault(n, [0, 0])
            a[0] += 1
            a[1] += e - s
        print(run, "value", val, "span_ms %.2f" % ((t1 - t0) / 1e6), "kernels_at_once %.2f" % (busy / (t1 - t0)),
              "idle_share %.3f" % (1 - cov / (t1 - t0)),
              {n: "%d x %.1f us" % (c, t / c / 1e3) for n, (c, t) in sorted(by.items())})


if __name__ == "__main__":
    main(sys.argv[1])
