"""GPU parity of the PBR texture path (SubMesh.swift:69-241,
Raytracing.metal:399-504): base color (sRGB), tangent-space normal, roughness, metallic,
emission (sRGB) and opacity maps, bilinear LOD-0 repeat sampling, the UV v-flip, the tangent
basis of computeTangentBasis, the texture debug views and the G-buffer, against the CPU oracle
on the same scene, seed and uniforms.  Textures are procedural (seeded) so the test needs no
files beyond the repo's assets.  Bar: bit-identical (the shared sampler specification,
tests/test_textures.py)."""
import os

import numpy as np
import pytest

from helpers import PIPELINES, make_renderer, parity_report, procedural_textures as _textures, textured_scene

pytestmark = pytest.mark.gpu


def _pair(rt, orc, assets, pipeline, W=96, H=64, frames=1, **knobs):
    sc = textured_scene(rt, assets)
    R = make_renderer(rt, sc, W, H, pipeline, seed=21)
    R.samplesPerPixel = 2
    R.maxBounces = 3
    for k, v in knobs.items():
        setattr(R, k, v)
    osc = orc.OracleScene(sc.desc())
    prev = motion = None
    for _ in range(frames):
        u = R.draw()
        R.wait()
        o = osc.render(u, R.random, accum_in=prev, motion_in=motion, gbuffer=bool(knobs.get("useTemporalDenoiser")))
        prev, motion = o["radiance"], o["motion"]
    g = R.radiance()
    gd, gm, gb = R.aux(gbuffer=bool(knobs.get("useTemporalDenoiser")))
    return R, sc, g, gd, gm, gb, R.stats(), o


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_textured_parity(rt, orc, assets, pipeline):
    R, sc, g, gd, gm, _, st, o = _pair(rt, orc, assets, pipeline, frames=2)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep
    assert rep["frac_bitwise"] == 1.0, rep
    assert np.array_equal(gd, o["depth"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront"])
@pytest.mark.parametrize("mode", [1, 2, 3, 4, 5, 6])
def test_texture_debug_views(rt, orc, assets, pipeline, mode):
    """DebugTextureMode BaseColor / Normal / Roughness / Metallic / AO / Emission (:459-490)."""
    R, sc, g, gd, gm, _, st, o = _pair(rt, orc, assets, pipeline, debugTextureMode=mode)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0 and rep["frac_bitwise"] == 1.0, rep
    if mode == 1:   # the textured floor shows its checker, untextured surfaces magenta
        rgb = g[..., :3].reshape(-1, 3)
        assert np.any(np.all(rgb == [1.0, 0.0, 1.0], axis=1))
        assert len(np.unique(rgb, axis=0)) > 50


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront"])
def test_textured_gbuffer(rt, orc, assets, pipeline):
    """G-buffer (:506-515) carries the sampled albedo / metallic / roughness and the mapped normal."""
    R, sc, g, gd, gm, gb, st, o = _pair(rt, orc, assets, pipeline, useTemporalDenoiser=True)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0 and rep["frac_bitwise"] == 1.0, rep
    assert np.array_equal(gb, o["gbuffer"])


def test_untextured_scene_unchanged(rt, orc, assets):
    """A scene without bound maps uploads no texture arrays (and keeps the untextured kernels);
    the textured one holds at least its texels."""
    sc = rt.Scene.preset("c1", assets)
    sc.add_model(os.path.join(assets, "train.obj"), (-0.3, 0.0, 0.4), scale=0.5)
    for v in _textures().values():
        sc.add_texture(v)   # added, never bound
    R = make_renderer(rt, sc, 64, 48, "wavefront", seed=3)
    R2 = make_renderer(rt, textured_scene(rt, assets), 64, 48, "wavefront", seed=3)
    texel_bytes = sum(v.size for v in _textures().values())
    assert R2.stats().device_bytes - R.stats().device_bytes >= texel_bytes


def test_flagged_slot_without_texture_rejected(rt, assets):
    sc = rt.Scene.preset("c1", assets)
    tid = sc.add_texture(np.zeros((2, 2, 4), np.uint8))
    sc.bind_texture(0, 0, "baseColor", tid)
    d = sc.desc()
    d.meshes[0].submeshes[0].textures[0] = 5   # out of range
    R = make_renderer(rt, rt.Scene.preset("c1", assets), 32, 32, "wavefront")
    from importlib import import_module
    with pytest.raises(import_module("metal4-raytracing_amd").RTError):
        R.upload(d)
