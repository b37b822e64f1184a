"""Times rt_bvh_build_device on a preset scene (default c3g: 881k triangles), each builder."""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rt = importlib.import_module("metal4-raytracing_amd")
scene = rt.Scene.preset(sys.argv[1] if len(sys.argv) > 1 else "c3g")
tu = rt.tuning_from_env()   # RT_DEVICE_BVH=lbvh selects the radix-tree builder (rt_tuning.device_bvh)
for k in ("graphs", "tail_paths", "frames_in_flight"):
    tu.pop(k, None)
R = rt.Renderer(scene, 64, 64, bvh="lbvh", tuning=tu)
for _ in range(2):
    R.rebuild(device=True)
R.wait()
n = 10
t0 = time.perf_counter()
for _ in range(n):
    R.rebuild(device=True)
R.wait()
print(os.environ.get("RT_DEVICE_BVH", "ploc"),
      "device build %.2f ms for %d triangles" % ((time.perf_counter() - t0) / n * 1e3, scene.triangle_count))
