"""Diagnostics: node / triangle visits per ray of dumped wavefront queues (RT_WF_DUMP), traced on
the host through the library's own BVH + traversal (rt_debug_trace_host)."""
import glob
import importlib
import sys

import numpy as np

rt = importlib.import_module("metal4-raytracing_amd")
prefix, scene_name = sys.argv[1], sys.argv[2]
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
sc = rt.Scene.preset(scene_name)
for path in sorted(glob.glob(prefix + "_it*.bin")):
    a = np.fromfile(path, np.float32).reshape(-1, 8)
    n = len(a)
    if n == 0:
        continue
    idx = np.random.default_rng(0).choice(n, min(n, cap), replace=False)
    r = rt.debug_trace_host(sc, a[idx, 0:3], a[idx, 4:7])
    nodes, tris = r["nodes"], r["tris"]
    q = np.percentile(nodes, [50, 90, 99, 99.9])
    print(f"{path.split('_')[-1]:10s} n={n:8d} nodes mean {nodes.mean():7.2f} p50/90/99/99.9 {q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}/{q[3]:.0f} "
          f"max {nodes.max():5d}  tris mean {tris.mean():6.2f} max {tris.max():5d}  hit {np.mean(r['id'] != 0xFFFFFFFF):.3f}",
          flush=True)
