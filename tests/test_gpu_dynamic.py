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
