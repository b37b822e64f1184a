"""GPU parity at the BASELINE.json configurations themselves (not reduced sizes): the HIP path,
through the C-ABI with the defaults the bench uses, against the CPU oracle's restatement of
Raytracing.metal:220-831 on the same scene, seed and uniforms.

  configs[1]  C2  bunny stand-in, 1280x720x4 spp, 4 bounces
  configs[2]  C3g glass dragon stand-in, 1920x1080x4 spp, 8 bounces (+ C3d, the opaque red dragon);
              two frames submitted back to back (frames in flight, frame 1 = temporal EMA)
  configs[3]  C3g at 3840x2160x16 spp, 8 bounces, split 8 ways in 64x64 tiles: rank r's share
  configs[4]  C5  skinned robot stand-in, 1920x1080x4 spp: frame 0 at rest, one skinning tick
              (t = 1/60 s) + refit, frame 1 with motion vectors, motion-adaptive extra samples and
              the EMA

Bar (BASELINE.json north star): per-pixel relative L2 of the radiance <= 1e-4 (tests/helpers.py);
depth, motion vectors and the ray / path counts must be equal.  In practice every pixel is
bit-identical, which the report prints.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import make_renderer, parity_report

pytestmark = pytest.mark.gpu

_ORACLE = {}   # (preset, ...) -> oracle results, shared by the pipelines of one configuration


def _oracle_frames(orc, scene, key, uniforms, random, tiles=None):
    """Oracle renders of the given uniforms in order (each frame's history = the previous one)."""
    if key not in _ORACLE:
        osc = orc.OracleScene(scene.desc())
        out, prev, motion = [], None, None
        for u in uniforms:
            o = osc.render(u, random, accum_in=prev, motion_in=motion, tiles=tiles)
            prev, motion = o["radiance"], o["motion"]
            out.append(o)
        _ORACLE[key] = out
        osc.close()
    return _ORACLE[key]


def _check(R, o, mask=None, counts=True):
    g = R.radiance()
    gd, gm, _ = R.aux()
    st = R.stats()
    if mask is not None:
        g, ref, gd, od, gm, om = g[mask], o["radiance"][mask], gd[mask], o["depth"][mask], gm[mask], o["motion"][mask]
    else:
        ref, od, om = o["radiance"], o["depth"], o["motion"]
    rep = parity_report(g, ref)
    print(rep, "closest", st.closest_rays, o["closest_rays"], "shadow", st.shadow_rays, o["shadow_rays"],
          "paths", st.paths, o["paths"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(gd, od)
    assert np.array_equal(gm, om)
    if counts:
        assert (st.closest_rays, st.shadow_rays, st.paths) == (o["closest_rays"], o["shadow_rays"], o["paths"])
    assert np.isfinite(g).all()
    return rep


@pytest.mark.parametrize("pipeline", ["wavefront", "megakernel"])
@pytest.mark.parametrize("preset", ["c3g", "c3d"])
def test_configs2_dragon_full_frame(rt, orc, assets, preset, pipeline):
    """configs[2]: 1920x1080x4 spp, 8 bounces, whole frame.  The wavefront renderer submits frames 0
    and 1 back to back (two frames in flight, as in bench.py) and frame 1 blends with frame 0's
    history; the megakernel renders frame 0."""
    scene = rt.Scene.preset(preset, assets)
    R = make_renderer(rt, scene, 1920, 1080, pipeline, seed=3)
    R.samplesPerPixel, R.maxBounces = 4, 8
    frames = 2 if pipeline == "wavefront" else 1
    us = [R.draw() for _ in range(frames)]   # no wait in between: the frames overlap
    if frames == 1:
        us.append(R.uniforms())   # frame 1's uniforms for the shared oracle sequence
    outs = _oracle_frames(orc, scene, (preset, 1920, 1080, 4, 8), us, R.random)
    if frames == 2:
        # frame 1 blends with frame 0's radiance (EMA), so frame 0 is checked through it
        assert R.stats().frames_total == 2
    _check(R, outs[frames - 1])


@pytest.mark.parametrize("pipeline", ["wavefront", "megakernel"])
def test_configs1_bunny_full_frame(rt, orc, assets, pipeline):
    """configs[1]: bunny stand-in, 1280x720x4 spp, 4 bounces, whole frame."""
    scene = rt.Scene.preset("c2", assets)
    R = make_renderer(rt, scene, 1280, 720, pipeline, seed=2)
    R.samplesPerPixel, R.maxBounces = 4, 4
    u = R.draw()
    o, = _oracle_frames(orc, scene, ("c2", 1280, 720, 4, 4), [u], R.random)
    _check(R, o)


@pytest.mark.parametrize("rank", [0, 5])
def test_configs3_rank_share(rt, orc, assets, rank):
    """configs[3]: 3840x2160x16 spp, 8 bounces, 8-way split in 64x64 tiles.  Rank r renders its own
    tiles (global pixel coordinates, the global random offsets) exactly as bench.py's rank does;
    the oracle renders the same tiles.  Every pixel of the share and the share's ray counts."""
    W, H, T, N = 3840, 2160, 64, 8
    scene = rt.Scene.preset("c3g", assets)
    R = make_renderer(rt, scene, W, H, "wavefront", seed=4)
    R.samplesPerPixel, R.maxBounces = 16, 8
    u = R.draw(tiles=(T, rank, N))
    o, = _oracle_frames(orc, scene, ("c3g", W, H, 16, 8, T, rank, N), [u], R.random, tiles=(T, rank, N))
    _ORACLE.pop(("c3g", W, H, 16, 8, T, rank, N))
    tx = (W + T - 1) // T
    yy, xx = np.mgrid[0:H, 0:W]
    own = ((yy // T) * tx + xx // T) % N == rank
    assert 0 < own.sum() <= R.tile_count(T, rank, N) * T * T   # 2160 = 33.75 tiles: the last row is partial
    _check(R, o, mask=own)
    # the packed share (what the RCCL gather moves) holds exactly these pixels
    import torch
    buf = torch.empty((R.tile_count(T, rank, N), T, T, 4), dtype=torch.float32, device="cuda")
    R.pack_tiles(T, rank, N, buf.data_ptr())
    R.wait()
    torch.cuda.synchronize()
    canvas = np.zeros((H, W, 4), np.float32)
    packed = buf.cpu().numpy()
    for k in range(packed.shape[0]):
        tid = rank + k * N
        x0, y0 = (tid % tx) * T, (tid // tx) * T
        h = min(T, H - y0)
        canvas[y0:y0 + h, x0:x0 + T] = packed[k, :h]
    assert np.array_equal(canvas[own][:, :3], o["radiance"][own][:, :3])


@pytest.mark.parametrize("rank", [0, 5])
def test_configs2_rank_share_team_drain(rt, orc, assets, rank):
    """configs[2] split 8 ways (the per-GPU frame of bench.py --gpus 8): rank r's 1.04M paths take
    the finish kernel's team drain by default (frames of 256K .. 2.5M paths).  Two
    frames back to back (frame 1 = EMA over frame 0), every pixel of the share and its ray counts."""
    W, H, T, N = 1920, 1080, 64, 8
    scene = rt.Scene.preset("c3g", assets)
    R = make_renderer(rt, scene, W, H, "wavefront", seed=6)
    R.samplesPerPixel, R.maxBounces = 4, 8
    us = [R.draw(tiles=(T, rank, N)) for _ in range(2)]
    key = ("c3g", W, H, 4, 8, T, rank, N)
    o = _oracle_frames(orc, scene, key, us, R.random, tiles=(T, rank, N))[1]
    _ORACLE.pop(key)
    tx = (W + T - 1) // T
    yy, xx = np.mgrid[0:H, 0:W]
    own = ((yy // T) * tx + xx // T) % N == rank
    assert 256 * 1024 <= R.tile_count(T, rank, N) * T * T * 4 <= 2500000   # the team drain's range
    assert R.stats().frames_total == 2
    _check(R, o, mask=own)


def _f4(ptr, n):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_float)), shape=(n, 4))


def test_configs4_skinned_full_frame(rt, orc, assets):
    """configs[4]: the skinned robot stand-in at 1920x1080x4 spp, 8 bounces (bench.py --animate).
    Frame 0 at rest; then one SkinningPass tick (t = 1/60 s) and a refit; frame 1 carries motion
    vectors, motion-adaptive extra samples (:779-789) and the motion-adaptive EMA (:796-817)."""
    from test_gpu_dynamic import _desc_with, _skinned_mesh
    W, H = 1920, 1080
    sc = rt.Scene.preset("c5", assets)
    desc = sc.desc()
    m = _skinned_mesh(desc)
    md = desc.meshes[m]
    n = md.vertex_count
    rest_p, rest_n = _f4(md.positions, n).copy(), _f4(md.normals, n).copy()
    ji = np.ctypeslib.as_array(md.joint_indices, shape=(n, 4)).copy()
    jw = np.ctypeslib.as_array(md.joint_weights, shape=(n, 4)).copy()
    R = make_renderer(rt, sc, W, H, "wavefront", seed=5)
    R.samplesPerPixel, R.maxBounces = 4, 8
    # frame 0: the skeleton's pose at t = 0 (the bench skins before every frame)
    J0 = sc.joint_matrices(m, 0.0)
    R.skin(m, J0)
    R.refit()
    u0 = R.draw()
    J1 = sc.joint_matrices(m, 1.0 / 60.0)
    R.skin(m, J1)
    R.refit()
    u1 = R.draw()
    R.wait()
    p0, n0 = orc.skin(rest_p, rest_n, ji, jw, J0)
    p1, n1 = orc.skin(rest_p, rest_n, ji, jw, J1)
    osc0 = orc.OracleScene(_desc_with(rt, desc, m, positions=p0, normals=n0))
    osc0.set_previous(m, prev_positions=rest_p)   # before frame 0's tick: the rest pose
    o0 = osc0.render(u0, R.random)
    osc1 = orc.OracleScene(_desc_with(rt, desc, m, positions=p1, normals=n1))
    osc1.set_previous(m, prev_positions=p0)
    o1 = osc1.render(u1, R.random, accum_in=o0["radiance"], motion_in=o0["motion"])
    assert np.abs(o1["motion"]).max() > 0
    _check(R, o1)
    print("extra samples in frame 1:", o1["paths"] - W * H * 4)
