"""Frames in flight (Renderer.swift:1406-1409 keeps up to three command buffers in flight): a
context renders consecutive wavefront frames on two streams, each frame overlapping the previous
one until its extra-sample pass and resolve, which read that frame's accumulation and motion
outputs.  The images, auxiliary targets and ray counts must be bit-identical to rendering one
frame at a time, through camera motion (EMA history, motion vectors, motion-adaptive extra
samples) and through scene updates between frames (which drain the frames in flight)."""
import os

import numpy as np
import pytest

from helpers import PIPELINES, make_renderer

pytestmark = pytest.mark.gpu


def _moved(rt, cam, dx, dy):
    c = rt.Camera()
    c.position = type(cam.position)(cam.position.x + dx, cam.position.y + dy, cam.position.z, 0.0)
    c.right, c.up, c.forward = cam.right, cam.up, cam.forward
    return c


def _run(rt, sc, desc, pipeline, fif, frames, move_at=None, gbuffer=False):
    W, H = 96, 64
    R = make_renderer(rt, sc, W, H, pipeline, seed=11, frames_in_flight=fif)
    R.samplesPerPixel = 2
    R.maxBounces = 3
    if gbuffer:
        R.useTemporalDenoiser = True
    cam0 = R.camera
    for i in range(frames):
        if move_at is not None and i == move_at:
            mats = np.stack([np.frombuffer(bytes(desc.meshes[k].transform), np.float32).reshape(4, 3).copy()
                             for k in range(desc.mesh_count)])
            mats[0, 3, 0] += 0.2
            R.set_instance_transforms(mats)
            R.refit()
        # orbit-ish camera drift: every frame moves, frames 3.. move by more than the extra-sample
        # threshold in places
        R.camera = _moved(rt, cam0, 0.05 * i * i, 0.02 * i)
        R.draw()
    img = R.radiance()
    depth, motion, gb = R.aux(gbuffer=gbuffer)
    st = R.stats()
    return R, img, depth, motion, gb, st


@pytest.mark.parametrize("pipeline,fif", [(p, 2) for p in PIPELINES] + [("wavefront", 3), ("wavefront-mixed", 3), ("wavefront", 4), ("wavefront-mixed", 4), ("wavefront", 8)])
def test_in_flight_matches_serial(rt, assets, pipeline, fif):
    sc = rt.Scene.preset("c2", assets)
    desc = sc.desc()
    _, a_img, a_d, a_m, _, a_st = _run(rt, sc, desc, pipeline, 1, 7)
    _, b_img, b_d, b_m, _, b_st = _run(rt, sc, desc, pipeline, fif, 7)
    assert np.array_equal(a_img, b_img)
    assert np.array_equal(a_d, b_d)
    assert np.array_equal(a_m, b_m)
    assert np.abs(a_m).max() > 0   # motion vectors exercised
    assert a_st.frames_in_flight == 1
    assert b_st.frames_in_flight == (fif if pipeline != "megakernel" else 1)
    assert a_st.frames_total == b_st.frames_total == 7
    for f in ("total_closest_rays", "total_shadow_rays", "total_paths", "closest_rays", "shadow_rays", "paths"):
        assert getattr(a_st, f) == getattr(b_st, f), f
    assert b_st.total_paths > 7 * 96 * 64 * 2   # the extra-sample pass ran in some frames


@pytest.mark.parametrize("pipeline", ["wavefront", "wavefront-mixed"])
def test_in_flight_scene_update_and_gbuffer(rt, assets, pipeline):
    """An instance transform + refit after frame 3 drains the frames in flight; the G-buffer and
    depth read back are the newest frame's."""
    sc = rt.Scene.preset("c2", assets)
    desc = sc.desc()
    _, a_img, a_d, a_m, a_g, a_st = _run(rt, sc, desc, pipeline, 1, 6, move_at=3, gbuffer=True)
    _, b_img, b_d, b_m, b_g, b_st = _run(rt, sc, desc, pipeline, 2, 6, move_at=3, gbuffer=True)
    assert np.array_equal(a_img, b_img)
    assert np.array_equal(a_d, b_d)
    assert np.array_equal(a_m, b_m)
    assert np.array_equal(a_g, b_g)
    assert a_st.total_closest_rays == b_st.total_closest_rays


def test_in_flight_then_megakernel_frame(rt, assets):
    """Wavefront frames in flight followed by a frame the megakernel renders (the motion debug
    view): the megakernel frame follows the newest wavefront frame's motion target."""
    sc = rt.Scene.preset("c2", assets)
    desc = sc.desc()
    out = []
    for fif in (1, 2, 3):
        R, *_ = _run(rt, sc, desc, "wavefront", fif, 4)
        R.debugTextureMode = 7   # DebugTextureModeMotion: megakernel only
        R.camera = _moved(rt, R.camera, 0.05, 0.0)
        R.draw()
        out.append((R.radiance(), R.aux()[1]))
    for img, mot in out[1:]:
        assert np.array_equal(out[0][0], img)
        assert np.array_equal(out[0][1], mot)


# 0: the library default for a rank's small frame: at most four slots below 512K paths
# (rt_api.cpp kSmallFramePaths), whatever the hardware queue count
@pytest.mark.parametrize("fif,expect", [(2, 2), (0, 4)])
def test_in_flight_tile_gather(rt, assets, fif, expect):
    """Two ranks' renderers (tile split, frames in flight) with the per-frame gather enqueued on
    a separate stream without host waits (rank 1 packs, rank 0 unpacks, the pattern of
    TileGather.gather over RCCL): rank 0's image after the last frame equals the one-GPU image,
    through camera motion (each pixel's history stays its own rank's)."""
    import torch
    sc = rt.Scene.preset("c1", assets)
    W, H, T, K = 200, 136, 64, 5
    full = make_renderer(rt, sc, W, H, "wavefront", seed=5, frames_in_flight=1)
    ranks = [make_renderer(rt, sc, W, H, "wavefront", seed=5, frames_in_flight=fif) for _ in range(2)]
    for R in [full] + ranks:
        R.maxBounces = 3
    cam0 = full.camera
    cnt = ranks[1].tile_count(T, 1, 2)
    s = torch.cuda.Stream()
    keep = []
    for i in range(K):
        for R in [full] + ranks:
            R.camera = _moved(rt, cam0, 0.05 * i * i, 0.02 * i)
        full.draw()
        for r, R in enumerate(ranks):
            R.draw(tiles=(T, r, 2))
        with torch.cuda.stream(s):
            buf = torch.empty((cnt, T, T, 4), dtype=torch.float32, device="cuda")
            ranks[1].pack_tiles(T, 1, 2, buf.data_ptr(), stream=s.cuda_stream)
            ranks[0].unpack_tiles(T, 1, 2, buf.data_ptr(), stream=s.cuda_stream)
        keep.append(buf)
    ref = full.radiance()
    img = ranks[0].radiance()
    assert ranks[0].stats().frames_in_flight == expect
    assert np.array_equal(img, ref)
