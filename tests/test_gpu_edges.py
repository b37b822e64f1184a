"""Edge cases of the hot path against the oracle (sizes, bounces, samples at their
limits): no bounces at all, one-pixel and ragged frames (not multiples of the 16x16 dispatch
block or the 64-pixel tile), many samples with the motion-adaptive extra samples at their
maximum, and a tile split with more ranks than tiles (a rank that owns nothing)."""
import numpy as np
import pytest

from helpers import PIPELINES, make_renderer, parity_report

pytestmark = pytest.mark.gpu


def _pair(rt, orc, assets, W, H, pipeline, frames=1, camera_step=0.0, **knobs):
    sc = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, sc, W, H, pipeline, seed=13)
    for k, v in knobs.items():
        setattr(R, k, v)
    osc = orc.OracleScene(sc.desc())
    cam0 = R.camera
    prev = motion = None
    for f in range(frames):
        if camera_step:
            c = rt.Camera()
            c.position = type(cam0.position)(cam0.position.x + camera_step * f, cam0.position.y, cam0.position.z, 0.0)
            c.right, c.up, c.forward = cam0.right, cam0.up, cam0.forward
            R.camera = c
        u = R.draw()
        R.wait()
        o = osc.render(u, R.random, accum_in=prev, motion_in=motion)
        prev, motion = o["radiance"], o["motion"]
    g = R.radiance()
    gd, gm, _ = R.aux()
    st = R.stats()
    R.close()
    return g, gd, gm, st, o


def _check(g, gd, gm, st, o):
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(gd, o["depth"]) and np.array_equal(gm, o["motion"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_zero_bounces(rt, orc, assets, pipeline):
    """maxBounces = 0: the bounce loop never runs (Raytracing.metal:311), no ray is traced and
    the accumulation is the EMA of zero radiance."""
    g, gd, gm, st, o = _pair(rt, orc, assets, 40, 24, pipeline, frames=2, maxBounces=0)
    _check(g, gd, gm, st, o)
    assert st.closest_rays == 0 and st.shadow_rays == 0
    assert not np.any(g[..., :3])


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("W,H", [(1, 1), (17, 9), (130, 67)])
def test_ragged_frames(rt, orc, assets, pipeline, W, H):
    g, gd, gm, st, o = _pair(rt, orc, assets, W, H, pipeline, samplesPerPixel=2, maxBounces=3)
    _check(g, gd, gm, st, o)


@pytest.mark.parametrize("pipeline", ["wavefront", "wavefront-mixed", "megakernel"])
def test_many_samples_and_max_extra(rt, orc, assets, pipeline):
    """16 spp plus up to 8 motion-adaptive extra samples per pixel under camera motion."""
    g, gd, gm, st, o = _pair(rt, orc, assets, 48, 32, pipeline, frames=3, camera_step=0.4, samplesPerPixel=16,
                             maxBounces=2, motionSamplingMaxExtraSamples=8)
    _check(g, gd, gm, st, o)
    assert st.paths > 48 * 32 * 16   # extra samples ran


def test_rank_without_tiles(rt, assets):
    """More ranks than 64x64 tiles: a rank that owns none renders nothing and packs nothing;
    the others' tiles still reassemble the full frame."""
    import torch
    sc = rt.Scene.preset("c1", assets)
    W, H, T, n = 100, 60, 64, 5          # 2 x 1 tiles over 5 ranks
    full = make_renderer(rt, sc, W, H, "wavefront", seed=5)
    full.maxBounces = 2
    full.draw()
    ref = full.radiance()
    canvas = np.zeros_like(ref)
    tx = (W + T - 1) // T
    for rank in range(n):
        R = make_renderer(rt, sc, W, H, "wavefront", seed=5)
        R.maxBounces = 2
        R.draw(tiles=(T, rank, n))
        R.wait()
        cnt = R.tile_count(T, rank, n)
        st = R.stats()
        if rank >= 2:
            assert cnt == 0 and st.paths == 0 and st.closest_rays == 0
            continue
        buf = torch.empty((cnt, T, T, 4), dtype=torch.float32, device="cuda")
        R.pack_tiles(T, rank, n, buf.data_ptr())
        R.wait()
        torch.cuda.synchronize()
        packed = buf.cpu().numpy()
        for k in range(cnt):
            tid = rank + k * n
            x0, y0 = (tid % tx) * T, (tid // tx) * T
            w, h = min(T, W - x0), min(T, H - y0)
            canvas[y0:y0 + h, x0:x0 + w] = packed[k, :h, :w]
    assert np.array_equal(canvas, ref)
