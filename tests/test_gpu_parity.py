"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same scene, seed and
uniforms.  Bar: per-pixel relative L2 of radiance <= 1e-4 (BASELINE.json north star); in practice
the two are bit-identical because both evaluate the same operation order, so the
tests also report the bitwise fraction and require it for integer-like outputs (ray counts).
"""
import numpy as np
import pytest

from helpers import PIPELINES, REL_L2_TOL, make_renderer, parity_report

pytestmark = pytest.mark.gpu




def _render_pair(rt, orc, preset, W, H, assets, frames=1, seed=7, pipeline="megakernel", **knobs):
    scene = rt.Scene.preset(preset, assets)
    R = make_renderer(rt, scene, W, H, pipeline, seed=seed)
    for k, v in knobs.items():
        setattr(R, k, v)
    osc = orc.OracleScene(scene.desc())
    prev = None
    motion = None
    out = []
    for f in range(frames):
        u = R.draw()
        R.wait()
        g = R.radiance()
        gd, gm, _ = R.aux()
        st = R.stats()
        o = osc.render(u, R.random, accum_in=prev, motion_in=motion)
        prev = o["radiance"]
        motion = o["motion"]
        out.append((g, gd, gm, st, o))
    return out


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("preset,W,H,spp,bounces,mode", [
    ("c1", 64, 64, 1, 1, 0),          # config 1 (plumbing case), small
    ("c1", 256, 256, 1, 1, 0),        # config 1 at its full size
    ("c1", 96, 64, 2, 4, 0),          # more bounces, non-square
    ("c1", 64, 48, 2, 3, 1),          # legacy shading (ShadingModeLegacy)
])
def test_c1_parity(rt, orc, assets, preset, W, H, spp, bounces, mode, pipeline):
    (g, gd, gm, st, o), = _render_pair(rt, orc, preset, W, H, assets, samplesPerPixel=spp, maxBounces=bounces,
                                       shadingMode=mode, pipeline=pipeline)
    rep = parity_report(g, o["radiance"])
    print(rep, st.closest_rays, o["closest_rays"], st.shadow_rays, o["shadow_rays"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(gd, o["depth"])
    assert np.array_equal(gm, o["motion"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]
    assert st.paths == o["paths"]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_glass_dragon_parity(rt, orc, assets, pipeline):
    """C3g scene (glass dragon stand-in, 871k tris) at reduced resolution, 8 bounces."""
    (g, gd, gm, st, o), = _render_pair(rt, orc, "c3g", 96, 54, assets, samplesPerPixel=2, maxBounces=8,
                                       pipeline=pipeline)
    rep = parity_report(g, o["radiance"])
    print(rep)
    assert rep["n_bad"] == 0, rep
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_real_meshes_parity(rt, orc, assets, pipeline):
    """C3r: the reference's own coatball / teapot meshes (irregular, modelled geometry, 884k
    triangles, glass) in the dragon's place, 8 bounces (the irregular-geometry cross-check of the
    headline's procedural stand-in)."""
    (g, gd, gm, st, o), = _render_pair(rt, orc, "c3r", 128, 72, assets, samplesPerPixel=2, maxBounces=8,
                                       pipeline=pipeline)
    rep = parity_report(g, o["radiance"])
    print(rep, st.closest_rays, st.shadow_rays)
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(gd, o["depth"]) and np.array_equal(gm, o["motion"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_bunny_parity(rt, orc, assets, pipeline):
    (g, gd, gm, st, o), = _render_pair(rt, orc, "c2", 80, 45, assets, samplesPerPixel=2, maxBounces=4,
                                       pipeline=pipeline)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_temporal_accumulation(rt, orc, assets, pipeline):
    """frameIndex > 0: EMA with the history target (Raytracing.metal:796-817), 3 frames."""
    frames = _render_pair(rt, orc, "c1", 48, 48, assets, frames=3, samplesPerPixel=1, maxBounces=2,
                          pipeline=pipeline)
    for g, gd, gm, st, o in frames:
        rep = parity_report(g, o["radiance"])
        assert rep["n_bad"] == 0, rep


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("mode", range(1, 8))
def test_debug_modes(rt, orc, assets, mode, pipeline):
    (g, gd, gm, st, o), = _render_pair(rt, orc, "c1", 32, 32, assets, debugTextureMode=mode, pipeline=pipeline)
    assert parity_report(g, o["radiance"])["n_bad"] == 0


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_gbuffer(rt, orc, assets, pipeline):
    scene = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, scene, 40, 30, pipeline, seed=3)
    R.useTemporalDenoiser = True
    u = R.draw()
    _, _, gb = R.aux(gbuffer=True)
    o = orc.OracleScene(scene.desc()).render(u, R.random, gbuffer=True)
    assert np.array_equal(gb, o["gbuffer"])


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_tiles_bitwise(rt, assets, pipeline):
    """Tile-split rendering is bitwise identical to the full-image render."""
    import torch
    scene = rt.Scene.preset("c1", assets)
    W, H, T = 200, 136, 64
    full = make_renderer(rt, scene, W, H, pipeline, seed=5)
    full.maxBounces = 3
    full.draw()
    ref = full.radiance()
    n = 3
    canvas = np.zeros_like(ref)
    for rank in range(n):
        R = make_renderer(rt, scene, W, H, pipeline, seed=5)
        R.maxBounces = 3
        R.draw(tiles=(T, rank, n))
        cnt = R.tile_count(T, rank, n)
        buf = torch.empty((cnt, T, T, 4), dtype=torch.float32, device="cuda")
        R.pack_tiles(T, rank, n, buf.data_ptr())
        R.wait()
        torch.cuda.synchronize()
        packed = buf.cpu().numpy()
        tx = (W + T - 1) // T
        for k in range(cnt):
            tid = rank + k * n
            x0, y0 = (tid % tx) * T, (tid // tx) * T
            w, h = min(T, W - x0), min(T, H - y0)
            canvas[y0:y0 + h, x0:x0 + w] = packed[k, :h, :w]
    assert np.array_equal(canvas, ref)


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_tiles_depth_motion(rt, assets, pipeline):
    """A rank's depth and motion vectors (evaluated per own pixel by wf_motion after the pass)
    equal the full frame's on its tiles, after a camera move."""
    scene = rt.Scene.preset("c1", assets)
    W, H, T, n = 200, 136, 64, 3
    rs = [make_renderer(rt, scene, W, H, pipeline, seed=5) for _ in range(n + 1)]
    cam0 = rs[0].camera
    for i in range(2):
        for k, R in enumerate(rs):
            R.maxBounces = 3
            c = rt.Camera()
            c.position = type(cam0.position)(cam0.position.x + 0.04 * i, cam0.position.y, cam0.position.z, 0.0)
            c.right, c.up, c.forward = cam0.right, cam0.up, cam0.forward
            R.camera = c
            R.draw() if k == 0 else R.draw(tiles=(T, k - 1, n))
    ref_d, ref_m, _ = rs[0].aux()
    assert np.abs(ref_m).max() > 0
    tx = (W + T - 1) // T
    seen = np.zeros((H, W), bool)
    for rank in range(n):
        d, m, _ = rs[rank + 1].aux()
        for tid in range(rank, tx * ((H + T - 1) // T), n):
            x0, y0 = (tid % tx) * T, (tid // tx) * T
            sl = (slice(y0, min(y0 + T, H)), slice(x0, min(x0 + T, W)))
            assert np.array_equal(d[sl], ref_d[sl]) and np.array_equal(m[sl], ref_m[sl]), (rank, tid)
            seen[sl] = True
    assert seen.all()


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_counting_frame_matches(rt, assets, pipeline):
    """Counting frames produce the same image; node/triangle counters are populated."""
    scene = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, scene, 64, 64, pipeline, seed=9)
    R.draw()
    a = R.radiance()
    R2 = make_renderer(rt, scene, 64, 64, pipeline, seed=9)
    R2.set_counting(True)
    R2.draw()
    b = R2.radiance()
    st = R2.stats()
    assert np.array_equal(a, b)
    assert st.node_visits > st.closest_rays and st.tri_tests > 0
    if pipeline == "wavefront-bulk":   # every ray went through wf_trace
        assert st.trace_rays == st.closest_rays + st.shadow_rays
        assert st.trace_nodes == st.node_visits and st.trace_tris == st.tri_tests
        assert st.trace_launches == 2 * st.iterations


@pytest.mark.parametrize("W,H,spp,bounces", [(320, 180, 4, 8), (1920, 1080, 4, 8)])
def test_pipelines_agree_full_frame(rt, assets, W, H, spp, bounces):
    """All pipeline variants produce bit-identical frames and ray counts on the headline scene,
    up to the full BASELINE configuration (C3g 1920x1080x4spp, 8 bounces) — a size-independent
    property; the oracle checks the same scene at reduced size (test_glass_dragon_parity)."""
    scene = rt.Scene.preset("c3g", assets)
    imgs = []
    counts = []
    for pl in PIPELINES:
        R = make_renderer(rt, scene, W, H, pl, seed=3)
        R.samplesPerPixel = spp
        R.maxBounces = bounces
        R.draw()
        imgs.append(R.radiance())
        st = R.stats()
        counts.append((st.closest_rays, st.shadow_rays, st.paths))
        R.close()
    for k in range(1, len(PIPELINES)):
        assert counts[k] == counts[0], (PIPELINES[k], counts[k], counts[0])
        assert np.array_equal(imgs[k], imgs[0]), PIPELINES[k]
    assert np.isfinite(imgs[0]).all()


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("name", ["c1_pbr_b1", "c1_pbr_b4", "c1_legacy_b3", "c1_ema_f3", "c3g_small_b8", "c2_small_b4",
                                  "tex_b3", "lights_point_b3", "lights_sun_b3", "lights_mix4_b3",
                                  "lights_mix3_legacy_b3"])
def test_gpu_matches_golden_fixtures(rt, assets, name, pipeline):
    """The HIP path against the committed fixtures (tests/golden, oracle-generated, seed 11)."""
    import json
    import os
    from conftest import ROOT
    gdir = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gdir, "cases.json")))[name]
    g = np.load(os.path.join(gdir, name + ".npz"))
    import sys
    sys.path.insert(0, gdir)
    import make_golden
    scene = make_golden.make_scene(rt, meta["preset"], assets)
    R = make_renderer(rt, scene, meta["width"], meta["height"], pipeline, seed=meta["seed"])
    for k, v in meta["knobs"].items():
        setattr(R, k, v)
    for _ in range(meta["frames"]):
        R.draw()
    img = R.radiance()[..., :3]
    depth, motion, _ = R.aux()
    st = R.stats()
    rep = parity_report(img, g["radiance"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(depth, g["depth"])
    assert [st.closest_rays, st.shadow_rays] == g["counts"].tolist()[:2]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_triangle_soup_closest_hit(rt, orc, assets, tmp_path, pipeline):
    """Closest hit in a soup of overlapping triangles whose ids say nothing about their depth
    (helpers.write_triangle_soup): the nearest triangle must win every primary and secondary hit,
    as in the oracle's own traversal (t first, the id only on equal t)."""
    from helpers import write_triangle_soup
    write_triangle_soup(str(tmp_path / "soup.obj"))
    scene = rt.Scene.preset("c1", assets)
    scene.add_model(str(tmp_path / "soup.obj"), (0.0, 1.0, 0.0), scale=3.0)
    R = make_renderer(rt, scene, 64, 48, pipeline, seed=3)
    R.samplesPerPixel, R.maxBounces = 2, 3
    u = R.draw()
    R.wait()
    g = R.radiance()
    depth, _, _ = R.aux()
    st = R.stats()
    o = orc.OracleScene(scene.desc()).render(u, R.random)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(depth, o["depth"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_emissive_parity(rt, orc, assets, tmp_path, pipeline):
    """An emissive untextured material (MTL Ke): the common shading kernels add color * emission
    to the path radiance (:585), the only place shade changes it, over several frames (EMA)."""
    import os
    import shutil
    shutil.copy(os.path.join(assets, "sphere.obj"), tmp_path / "sphere.obj")
    (tmp_path / "sphere.mtl").write_text("newmtl None\nKd 0.6 0.7 0.5\nKe 1.5 0.75 0.25\nd 1\n")
    scene = rt.Scene.preset("c1", assets)
    scene.add_model(str(tmp_path / "sphere.obj"), (0.4, 0.6, 1.2), scale=0.5)
    R = make_renderer(rt, scene, 72, 56, pipeline, seed=9)
    R.samplesPerPixel, R.maxBounces = 2, 4
    osc = orc.OracleScene(scene.desc())
    prev = motion = None
    for _ in range(3):
        u = R.draw()
        R.wait()
        g = R.radiance()
        st = R.stats()
        o = osc.render(u, R.random, accum_in=prev, motion_in=motion)
        prev, motion = o["radiance"], o["motion"]
        rep = parity_report(g, o["radiance"])
        assert rep["n_bad"] == 0, rep
        assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]
    assert float(np.max(g[..., :3])) > 0.5   # the emitter shows


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kinds", [("point",), ("sun",), ("area", "spot", "point"), ("area", "spot", "point", "sun"),
                                   ("sun", "area2", "point", "spot")])
def test_light_types_parity(rt, orc, assets, kinds, mode, pipeline):
    """Point and sun lights (Raytracing.metal:633-643; a sun's shadow ray has tmax = inf - 1e-3 =
    inf, :716-743) and three or four lights (the light pick of :588-589 with lightCount > 2, the
    lightCount factor of :647), in PBR and legacy shading, over two EMA frames."""
    from helpers import lights_scene
    scene = lights_scene(rt, assets, list(kinds))
    R = make_renderer(rt, scene, 72, 48, pipeline, seed=13)
    R.samplesPerPixel, R.maxBounces, R.shadingMode = 2, 4, mode
    osc = orc.OracleScene(scene.desc())
    prev = motion = None
    for _ in range(2):
        u = R.draw()
        assert u.lightCount == len(kinds)
        R.wait()
        g = R.radiance()
        gd, gm, _ = R.aux()
        st = R.stats()
        o = osc.render(u, R.random, accum_in=prev, motion_in=motion)
        prev, motion = o["radiance"], o["motion"]
        rep = parity_report(g, o["radiance"])
        assert rep["n_bad"] == 0, rep
        assert np.array_equal(gd, o["depth"]) and np.array_equal(gm, o["motion"])
        assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]
    assert float(np.max(g[..., :3])) > 0.0


def test_tuning_api_roundtrip_and_validation(rt, assets):
    """rt_set_tuning / rt_get_tuning (the library reads no environment for its scheduling): defaults
    resolved, a set value read back, out-of-range values refused, the frame unchanged by them."""
    scene = rt.Scene.preset("c1", assets)
    R = rt.Renderer(scene, 64, 48, seed=2)
    d = R.tuning()
    assert d["trace_chunk"] == 64 and d["finish_chunk"] == 64 and d["shade_blocks"] == 2048 and d["team"] == 0
    R.samplesPerPixel, R.maxBounces = 1, 3
    R.draw()
    R.wait()
    a = R.radiance()
    R.set_tuning(finish_chunk=5, team=4, shade_min_drained=-100, refill_min=3)
    t = R.tuning()
    assert t["finish_chunk"] == 5 and t["team"] == 4 and t["shade_min_drained"] == -100 and t["refill_min"] == 3
    R.frameIndex = 0
    R.draw()
    R.wait()
    assert np.array_equal(R.radiance(), a)
    assert d["finish_grid_pct"] == 0 and d["trace_grid_pct"] == 0   # chosen per frame (rt_api.h)
    for bad in ({"team": 3}, {"refill_min": 65}, {"log": 3}, {"shade_min_drained": -101}, {"trace_chunk": 4097},
                {"finish_chunk": 1 << 30}, {"shade_blocks": 65537}, {"finish_grid_pct": 101}):
        with pytest.raises(rt.RTError):
            R.set_tuning(**bad)
    R.set_tuning()
    assert R.tuning() == d
    R.close()


def test_radiance_half_is_fp32_rounded_to_nearest(rt, assets):
    """rt_read_radiance_half (RGBA16F, Renderer.swift:685): the fp32 target rounded to nearest even,
    bit for bit what numpy's float32 -> float16 conversion gives; on a PBR frame and an EMA frame."""
    scene = rt.Scene.preset("c1", assets)
    R = rt.Renderer(scene, 96, 64, seed=4)
    R.samplesPerPixel, R.maxBounces = 2, 3
    for _ in range(2):
        R.draw()
        R.wait()
        a = R.radiance()
        h = R.radiance_half()
        assert h.dtype == np.float16 and h.shape == a.shape
        want = a.astype(np.float16)
        assert np.array_equal(h.view(np.uint16), want.view(np.uint16))
        assert float(np.max(a[..., :3])) > 0.0
    R.close()
