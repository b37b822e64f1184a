"""How much throughput do two frames in flight add?  Two contexts (own streams and buffers) render
the C3g frame; frames are submitted without waiting in between, staggered by one frame, and the
rays / wall time compared with one context rendering frames back to back.

usage: python tools/overlap_probe.py [frames]
"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("metal4-raytracing_amd")

K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
scene = rt.Scene.preset("c3g")
Rs = [rt.Renderer(scene, 1920, 1080, pipeline="wavefront", seed=3) for _ in range(2)]
for R in Rs:
    R.samplesPerPixel = 4
    R.maxBounces = 8
    R.draw()
    R.wait()


def rays(R):
    st = R.stats()
    return st.closest_rays + st.shadow_rays


# one context, back to back
t0 = time.perf_counter()
n = 0
for _ in range(K):
    Rs[0].draw()
    Rs[0].wait()
    n += rays(Rs[0])
dt = time.perf_counter() - t0
print(f"serial : {n / dt / 1e9:.3f} Grays/s, {dt / K * 1e3:.3f} ms/frame", flush=True)

# two contexts, staggered: submit A(i+1) before waiting for B(i)
t0 = time.perf_counter()
n = 0
Rs[0].draw()
for i in range(K - 1):
    nxt, prev = Rs[(i + 1) % 2], Rs[i % 2]
    nxt.draw()
    prev.wait()
    n += rays(prev)
Rs[(K - 1) % 2].wait()
n += rays(Rs[(K - 1) % 2])
dt = time.perf_counter() - t0
print(f"2 in flight: {n / dt / 1e9:.3f} Grays/s, {dt / K * 1e3:.3f} ms/frame", flush=True)
