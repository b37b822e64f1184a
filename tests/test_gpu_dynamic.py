"""GPU parity for the dynamic rows of SURVEY.md §8: skinning (a25, Skinning.metal:7-49), BVH refit
(a26, Renderer.swift:1084-1202), instance-transform motion (a5/a16, Renderer.swift:939-944,
Raytracing.metal:342-389) and the motion-adaptive extra samples they trigger (a23, :779-789).

The oracle scene is rebuilt from a descriptor holding the skinned / moved geometry, and its
motion history is set to what the device holds (positions before the skinning tick, the previous
instance transform), so radiance, depth and motion must agree bit for bit."""
import ctypes as C

import numpy as np
import pytest

from helpers import PIPELINES, make_renderer, parity_report

pytestmark = pytest.mark.gpu



def _f4(ptr, n):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_float)), shape=(n, 4))


def _skinned_mesh(desc):
    for m in range(desc.mesh_count):
        if desc.meshes[m].joint_count > 0:
            return m
    raise AssertionError("no skinned mesh in the scene")


def _desc_with(rt, desc, mesh, positions=None, normals=None, transform=None):
    """A copy of desc whose mesh `mesh` points at other positions / normals / transform."""
    from importlib import import_module
    A = import_module("metal4-raytracing_amd._abi")
    arr = (A.MeshDesc * desc.mesh_count)()
    for m in range(desc.mesh_count):
        C.pointer(arr[m])[0] = desc.meshes[m]
    md = arr[mesh]
    if positions is not None:
        md.positions = C.cast(positions.ctypes.data, C.POINTER(A.Float3))
    if normals is not None:
        md.normals = C.cast(normals.ctypes.data, C.POINTER(A.Float3))
    if transform is not None:
        C.memmove(C.byref(md.transform), np.ascontiguousarray(transform, np.float32).ctypes.data, 48)
    d = A.SceneDesc()
    d.mesh_count, d.light_count, d.meshes, d.lights = desc.mesh_count, desc.light_count, arr, desc.lights
    d.texture_count, d.textures = desc.texture_count, desc.textures
    d._keep = (arr, positions, normals)
    return d


def _check_frame(R, o):
    g = R.radiance()
    gd, gm, _ = R.aux()
    st = R.stats()
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep
    assert np.array_equal(gd, o["depth"])
    assert np.array_equal(gm, o["motion"])
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]
    assert st.paths == o["paths"]
    return rep


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("rebuild", ["refit", "host", "device"])
def test_skinning_refit_parity(rt, orc, assets, pipeline, rebuild):
    """C5: skin the robot stand-in at t = 0.35 s, refit the BVH or rebuild it (host SAH build, or
    the on-device LBVH build), render; oracle on the host-skinned mesh with prevPositions = rest
    pose."""
    W, H = 96, 64
    sc = rt.Scene.preset("c5", assets)
    desc = sc.desc()
    m = _skinned_mesh(desc)
    md = desc.meshes[m]
    n = md.vertex_count
    rest_p, rest_n = _f4(md.positions, n).copy(), _f4(md.normals, n).copy()
    ji = np.ctypeslib.as_array(md.joint_indices, shape=(n, 4)).copy()
    jw = np.ctypeslib.as_array(md.joint_weights, shape=(n, 4)).copy()
    J = sc.joint_matrices(m, 0.35)
    R = make_renderer(rt, sc, W, H, pipeline, seed=5)
    R.samplesPerPixel = 2
    R.maxBounces = 2
    R.skin(m, J)
    R.refit() if rebuild == "refit" else R.rebuild(device=rebuild == "device")
    u = R.draw()
    R.wait()
    sp, sn = orc.skin(rest_p, rest_n, ji, jw, J)
    d2 = _desc_with(rt, desc, m, positions=sp, normals=sn)
    osc = orc.OracleScene(d2)
    osc.set_previous(m, prev_positions=rest_p)
    o = osc.render(u, R.random)
    _check_frame(R, o)
    # the robot moved: some pixels carry motion, so the motion vectors are exercised
    assert np.abs(o["motion"]).max() > 0


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("shift", [0.15, -3.5])
def test_instance_motion_and_extra_samples(rt, orc, assets, pipeline, shift):
    """Move the hero mesh between frames (set_instance_transforms + refit): frame 1's motion
    vectors come from prev_inst, and motion-adaptive sampling adds extra samples where the
    motion exceeds the threshold (defaults: up to 2 extra, 1-6 px)."""
    W, H = 96, 64
    sc = rt.Scene.preset("c2", assets)
    desc = sc.desc()
    R = make_renderer(rt, sc, W, H, pipeline, seed=9)
    R.samplesPerPixel = 1
    R.maxBounces = 2
    assert R.useMotionAdaptiveSampling
    osc0 = orc.OracleScene(desc)
    u0 = R.draw()
    R.wait()
    o0 = osc0.render(u0, R.random)
    _check_frame(R, o0)
    # frame 1: hero (mesh 0) translated along x (a large shift re-pads the refitted boxes)
    mats = np.stack([np.frombuffer(bytes(desc.meshes[k].transform), np.float32).reshape(4, 3).copy()
                     for k in range(desc.mesh_count)])
    old0 = mats[0].copy()
    mats[0, 3, 0] += shift
    R.set_instance_transforms(mats)
    R.refit()
    u1 = R.draw()
    R.wait()
    d1 = _desc_with(rt, desc, 0, transform=mats[0])
    osc1 = orc.OracleScene(d1)
    osc1.set_previous(0, prev_transform=old0)
    o1 = osc1.render(u1, R.random, accum_in=o0["radiance"], motion_in=o0["motion"])
    _check_frame(R, o1)
    if abs(shift) < 1.0:   # the hero stays in view: motion-adaptive extra samples were taken
        assert o1["paths"] > W * H


class _DescScene:
    """A scene descriptor built in the test, for Renderer (which only calls desc())."""

    def __init__(self, d):
        self._d = d
        self.synthetic = False

    def desc(self):
        return self._d


def _desc_dup_hero(rt, desc, transforms):
    """desc plus a second instance of mesh 0; every mesh at transforms[m] (the copy's last)."""
    from importlib import import_module
    A = import_module("metal4-raytracing_amd._abi")
    n = desc.mesh_count + 1
    arr = (A.MeshDesc * n)()
    for m in range(n):
        C.pointer(arr[m])[0] = desc.meshes[m if m < desc.mesh_count else 0]
        C.memmove(C.byref(arr[m].transform), np.ascontiguousarray(transforms[m], np.float32).ctypes.data, 48)
    d = A.SceneDesc()
    d.mesh_count, d.light_count, d.meshes, d.lights = n, desc.light_count, arr, desc.lights
    d.texture_count, d.textures = desc.texture_count, desc.textures
    d._keep = (arr,)
    return d


def test_refit_degradation_triggers_device_rebuild(rt, orc, assets):
    """rt_tuning.refit_rebuild_pct (Renderer.swift:1252-1277 rebuilds where a refit is not enough):
    two coincident copies of the hero interleave in the tree's nodes; moving one 5 units away makes
    every shared node span both, the refit's node-area sum grows past 150 % of the build's, and the
    next frame rebuilds the tree on the device (rt_stats.total_auto_rebuilds).  The frame on the
    rebuilt tree equals a freshly built renderer's and the oracle's bit for bit; a small move keeps
    the refit (no rebuild)."""
    W, H = 96, 64
    sc = rt.Scene.preset("c2", assets)
    base = sc.desc()
    mats0 = [np.frombuffer(bytes(base.meshes[k].transform), np.float32).reshape(4, 3).copy()
             for k in range(base.mesh_count)]
    mats0.append(mats0[0].copy())
    d0 = _desc_dup_hero(rt, base, mats0)

    def renderer(d):
        R = make_renderer(rt, _DescScene(d), W, H, "wavefront", seed=9)
        R.samplesPerPixel, R.maxBounces = 1, 2
        R.useMotionAdaptiveSampling = False
        return R

    R = renderer(d0)
    s0 = R.stats()
    built = s0.bvh_cost_built
    assert built > 0.0 and s0.total_auto_rebuilds == 0
    # a small move: the refit keeps the tree
    small = [m.copy() for m in mats0]
    small[-1][3, 0] += 0.02
    R.set_instance_transforms(np.stack(small))
    R.refit()
    for _ in range(2):
        R.draw()
        R.wait()
    s1 = R.stats()
    assert s1.total_auto_rebuilds == 0 and s1.bvh_cost_refit <= 1.5 * built, (s1.bvh_cost_refit, built)
    # a large move: the refit degrades, the next frame rebuilds on the device
    big = [m.copy() for m in mats0]
    big[-1][3, 0] += 5.0
    R.set_instance_transforms(np.stack(big))
    R.set_instance_transforms(np.stack(big))   # previous = current: no motion history
    R.refit()
    for _ in range(2):
        R.frameIndex = 0
        u = R.draw()
        R.wait()
    s2 = R.stats()
    assert s2.total_auto_rebuilds == 1, (s2.total_auto_rebuilds, s2.bvh_cost_refit, built)
    assert s2.bvh_cost_refit > 1.5 * built                         # the refit that triggered it
    assert built < s2.bvh_cost_built < 1.5 * built                 # the rebuilt tree
    g = R.radiance()
    d1 = _desc_dup_hero(rt, base, big)
    R2 = renderer(d1)
    u2 = R2.draw()
    R2.wait()
    assert np.array_equal(R2.radiance(), g)
    assert R2.stats().closest_rays == s2.closest_rays and R2.stats().shadow_rays == s2.shadow_rays
    o = orc.OracleScene(d1).render(u2, R2.random)
    _check_frame(R2, o)
    R.close()
    R2.close()
