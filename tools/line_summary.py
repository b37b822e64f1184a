#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (the last line starting with '{' in a log file):
value, ms per step, stage times and the per-kernel launch figures.  Used by the tools/ sweeps."""
import json
import sys


def main():
    path, name = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    d = json.loads([x for x in open(path) if x.startswith("{")][-1])
    r = d.get("roofline") or {}
    ks = [(k["kernel"][:16], k["launch_ms"], k.get("nodes_per_ray")) for k in r.get("kernels", [])]
    print(name, d["value"], d["ms_per_step"], "iters", d["config"].get("iterations"), "stage_ms",
          d["config"].get("stage_ms"), ks, flush=True)


if __name__ == "__main__":
    main()
