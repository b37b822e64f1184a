"""Regenerate the golden fixtures from the CPU oracle (oracle/rt_oracle.c).

The reference cannot run in this container (Swift/Metal absent), so these
fixtures are the oracle's own outputs for fixed seeds: they pin the oracle against silent
changes (tests/test_oracle_kat.py) and give the GPU path a second, independent anchor.
Run from the repo root:  python tests/golden/make_golden.py
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CASES = {
    # name: (preset, W, H, knobs, frames)
    "c1_pbr_b1": ("c1", 64, 64, dict(samplesPerPixel=1, maxBounces=1), 1),
    "c1_pbr_b4": ("c1", 64, 64, dict(samplesPerPixel=2, maxBounces=4), 1),
    "c1_legacy_b3": ("c1", 64, 48, dict(samplesPerPixel=1, maxBounces=3, shadingMode=1), 1),
    "c1_ema_f3": ("c1", 48, 48, dict(samplesPerPixel=1, maxBounces=2), 3),
    "c3g_small_b8": ("c3g", 64, 36, dict(samplesPerPixel=1, maxBounces=8), 1),
    "c2_small_b4": ("c2", 64, 36, dict(samplesPerPixel=1, maxBounces=4), 1),
    # c1 + the train with every texture map kind bound (tests/helpers.py textured_scene)
    "tex_b3": ("tex", 64, 48, dict(samplesPerPixel=1, maxBounces=3), 1),
    # c1 lit by the light types the AppScene does not use (Raytracing.metal:633-643) and by three
    # and four lights (the light pick of :588-589 with lightCount > 2), PBR and legacy shading
    "lights_point_b3": ("lights:point", 64, 48, dict(samplesPerPixel=2, maxBounces=3), 1),
    "lights_sun_b3": ("lights:sun", 64, 48, dict(samplesPerPixel=2, maxBounces=3), 1),
    "lights_mix4_b3": ("lights:area,spot,point,sun", 64, 48, dict(samplesPerPixel=2, maxBounces=3), 1),
    "lights_mix3_legacy_b3": ("lights:point,sun,area2", 64, 48, dict(samplesPerPixel=2, maxBounces=3, shadingMode=1), 1),
}
SEED = 11


def make_scene(rt, preset, assets):
    if preset == "tex":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from helpers import textured_scene
        return textured_scene(rt, assets)
    if preset.startswith("lights:"):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from helpers import lights_scene
        return lights_scene(rt, assets, preset.split(":", 1)[1].split(","))
    return rt.Scene.preset(preset, assets)


def render_case(rt, oracle, preset, W, H, knobs, frames, assets):
    scene = make_scene(rt, preset, assets)
    osc = oracle.OracleScene(scene.desc())
    rnd = rt.random_offsets(SEED, W, H)
    prev, motion = None, None
    for f in range(frames):
        u = rt.uniforms_default(W, H, scene.light_count)
        for k, v in knobs.items():
            setattr(u, k, v)
        u.frameIndex = f
        out = osc.render(u, rnd, accum_in=prev, motion_in=motion)
        prev, motion = out["radiance"], out["motion"]
    return out


def main(names=None):
    """Regenerates the named cases (default: all) and rewrites cases.json for every case."""
    rt = importlib.import_module("metal4-raytracing_amd")
    import oracle
    assets = os.path.join(ROOT, "assets")
    path = os.path.join(ROOT, "tests", "golden", "cases.json")
    meta = json.load(open(path)) if os.path.exists(path) else {}
    for name, (preset, W, H, knobs, frames) in CASES.items():
        if names and name not in names:
            continue
        out = render_case(rt, oracle, preset, W, H, knobs, frames, assets)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", name + ".npz"), radiance=out["radiance"][..., :3],
                            depth=out["depth"], motion=out["motion"],
                            counts=np.array([out["closest_rays"], out["shadow_rays"], out["paths"]], np.uint64))
        meta[name] = dict(preset=preset, width=W, height=H, knobs=knobs, frames=frames, seed=SEED,
                          closest_rays=int(out["closest_rays"]), shadow_rays=int(out["shadow_rays"]))
        print(name, meta[name])
    with open(os.path.join(ROOT, "tests", "golden", "cases.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
