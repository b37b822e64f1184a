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

from helpers import PIPELINES, make_renderer, parity_report

pytestmark = pytest.mark.gpu


def _textures(seed=1):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:64, 0:64]
    base = np.zeros((64, 64, 4), np.uint8)
    chk = ((xx // 8 + yy // 8) % 2).astype(np.uint8)
    base[..., 0] = 40 + 200 * chk
    base[..., 1] = rng.integers(30, 220, size=(64, 64))
    base[..., 2] = 255 - 180 * chk
    base[..., 3] = 255
    # bumps: tangent-space normals from a height field
    hx = np.cos(xx / 64.0 * 2 * np.pi * 3) * 0.6
    hy = np.sin(yy / 64.0 * 2 * np.pi * 2) * 0.6
    n = np.stack([hx, hy, np.ones_like(hx)], axis=-1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    normal = np.concatenate([((n * 0.5 + 0.5) * 255).round().astype(np.uint8), np.full((64, 64, 1), 255, np.uint8)],
                            axis=-1)
    rough = np.repeat(((xx * 4) % 256).astype(np.uint8)[..., None], 4, axis=-1)
    metal = np.repeat((255 * ((yy // 4) % 2)).astype(np.uint8)[..., None], 4, axis=-1)
    emis = np.zeros((32, 32, 4), np.uint8)
    emis[::5, ::7, :3] = rng.integers(100, 256, size=emis[::5, ::7, :3].shape)
    emis[..., 3] = 255
    opac = np.full((16, 16, 4), 255, np.uint8)
    opac[4:12, 4:12, 0] = 40
    return dict(base=base, normal=normal, rough=rough, metal=metal, emis=emis, opac=opac)


def textured_scene(rt, assets):
    """c1 (floor with UVs, two spheres without, back wall) + the train (UVs, 6 submeshes)."""
    sc = rt.Scene.preset("c1", assets)
    sc.add_model(os.path.join(assets, "train.obj"), (-0.3, 0.0, 0.4), scale=0.5)
    T = {k: sc.add_texture(v) for k, v in _textures().items()}
    sc.bind_texture(0, 0, "baseColor", T["base"])        # floor
    sc.bind_texture(0, 0, "roughness", T["rough"])
    sc.bind_texture(0, 0, "normal", T["normal"])
    sc.bind_texture(1, 0, "baseColor", T["base"])        # sphere without UVs: samples (0, 1)
    sc.bind_texture(1, 0, "metallic", T["metal"])
    sc.bind_texture(4, 0, "normal", T["normal"])         # train submeshes
    sc.bind_texture(4, 0, "metallic", T["metal"])
    sc.bind_texture(4, 1, "emission", T["emis"])
    sc.bind_texture(4, 2, "opacity", T["opac"])
    sc.bind_texture(4, 3, "roughness", T["rough"])
    sc.bind_texture(4, 4, "baseColor", T["base"])
    sc.bind_texture(4, 5, "baseColor", T["base"])
    sc.bind_texture(4, 5, "normal", T["normal"])
    sc.bind_texture(4, 5, "ao", T["rough"])              # AO: bound, never sampled (ENABLE_AO 0)
    return sc


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
