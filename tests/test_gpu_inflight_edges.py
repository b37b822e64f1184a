"""Edge cases of frames in flight (rt_api.cpp FrameSlot rotation): a resize between frames in
flight, switching to a caller's stream mid-sequence (one slot from then on), a rank that owns no
tiles, re-uploading the scene, and the on-device BVH rebuild between in-flight frames.  Each
sequence must give the same bytes as one-frame-at-a-time rendering."""
import numpy as np
import pytest

from helpers import make_renderer

pytestmark = pytest.mark.gpu


def _seq(rt, assets, fif, steps):
    sc = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, sc, 72, 48, "wavefront", seed=6, frames_in_flight=fif)
    R.samplesPerPixel, R.maxBounces = 2, 3
    out = []
    for st in steps:
        st(rt, R, sc)
        R.draw()
    out.append(R.radiance())
    out.append(R.aux()[0])
    return out, R


def _draws(n):
    return [lambda rt, R, sc: None] * n


def _check_same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_resize_between_frames(rt, assets):
    def resize(rt, R, sc):
        R.resize(88, 56, seed=9)
    steps = _draws(3) + [resize] + _draws(3)
    a, _ = _seq(rt, assets, 1, steps)
    b, Rb = _seq(rt, assets, 2, steps)
    assert a[0].shape == (56, 88, 4)
    _check_same(a, b)
    assert Rb.stats().frames_in_flight == 2


def test_switch_to_caller_stream(rt, assets):
    import torch
    s = torch.cuda.Stream()

    def to_stream(rt, R, sc):
        R.set_stream(s.cuda_stream)

    def back(rt, R, sc):
        R.set_stream(None)
    steps = _draws(3) + [to_stream] + _draws(2) + [back] + _draws(2)
    a, _ = _seq(rt, assets, 1, steps)
    b, Rb = _seq(rt, assets, 2, steps)
    _check_same(a, b)


def test_caller_stream_uses_one_slot(rt, assets):
    import torch
    s = torch.cuda.Stream()
    sc = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, sc, 64, 48, "wavefront", seed=6, frames_in_flight=2, stream=s.cuda_stream)
    R.draw()
    R.draw()
    assert R.stats().frames_in_flight == 1


def test_rank_without_tiles(rt, assets):
    sc = rt.Scene.preset("c1", assets)
    R = make_renderer(rt, sc, 64, 64, "wavefront", seed=6, frames_in_flight=2)
    assert R.tile_count(64, 3, 4) == 0   # one 64x64 tile, four ranks
    for _ in range(3):
        R.draw(tiles=(64, 3, 4))
    st = R.stats()
    assert st.frames_total == 3 and st.total_closest_rays == 0 and st.paths == 0


def test_reupload_and_device_rebuild_between_frames(rt, assets):
    def reupload(rt, R, sc):
        R.upload(sc.desc())

    def rebuild(rt, R, sc):
        R.rebuild(device=True)
    steps = _draws(2) + [reupload] + _draws(2) + [rebuild] + _draws(2)
    a, _ = _seq(rt, assets, 1, steps)
    b, _ = _seq(rt, assets, 2, steps)
    _check_same(a, b)


def _animated(rt, assets, fif, frames=6, rebuild_at=None, move=False, rebuild_every=None):
    sc = rt.Scene.preset("c5", assets)
    d = sc.desc()
    skinned = [m for m in range(d.mesh_count) if d.meshes[m].joint_count > 0]
    mats = np.stack([np.frombuffer(bytes(d.meshes[k].transform), np.float32).reshape(4, 3).copy()
                     for k in range(d.mesh_count)])
    R = make_renderer(rt, sc, 80, 56, "wavefront", seed=12, frames_in_flight=fif)
    R.samplesPerPixel, R.maxBounces = 2, 3
    for i in range(frames):
        for m in skinned:
            R.skin(m, sc.joint_matrices(m, i / 60.0))
        if move:
            mats[skinned[0], 3, 0] += 0.01
            R.set_instance_transforms(mats)
        if rebuild_every is not None:
            R.rebuild(device=rebuild_every == "device")
        elif rebuild_at is not None and i == rebuild_at:
            R.rebuild(device=True)
        else:
            R.refit()
        R.draw()
    img = R.radiance()
    depth, motion, _ = R.aux()
    return img, depth, motion, R.stats()


@pytest.mark.parametrize("kw", [dict(), dict(move=True), dict(rebuild_at=3), dict(rebuild_every="device"),
                                dict(rebuild_every="host", move=True)])
@pytest.mark.parametrize("fif", [2, 4])
def test_animated_frames_in_flight(rt, assets, kw, fif):
    """Per-frame skinning + refit (configs[4] shape) with frames in flight: the updates go to the
    other geometry generation while the previous frame still renders; bytes equal the serial run."""
    a = _animated(rt, assets, 1, **kw)
    b = _animated(rt, assets, fif, **kw)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert np.abs(a[2]).max() > 0   # the robot moved: motion vectors exercised
    assert a[3].total_closest_rays == b[3].total_closest_rays
    assert b[3].frames_in_flight == fif
