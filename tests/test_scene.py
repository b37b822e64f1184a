"""Host scene ingest (Scene/Model/Mesh/Submesh mirror) on CPU: OBJ/MTL conventions, transforms,
camera, uniforms, random offsets, procedural stand-ins."""
import ctypes as C
import math
import os

import numpy as np
import pytest


def _meshes(scene):
    d = scene.desc()
    out = []
    for i in range(d.mesh_count):
        m = d.meshes[i]
        n = m.vertex_count
        P = np.ctypeslib.as_array(C.cast(m.positions, C.POINTER(C.c_float)), shape=(n * 4,)).reshape(n, 4)[:, :3]
        N = np.ctypeslib.as_array(C.cast(m.normals, C.POINTER(C.c_float)), shape=(n * 4,)).reshape(n, 4)[:, :3]
        subs = []
        for k in range(m.submesh_count):
            sm = m.submeshes[k]
            idx = np.ctypeslib.as_array(sm.indices, shape=(sm.index_count,)).reshape(-1, 3).copy()
            subs.append((idx, sm.material))
        T = np.array([[m.transform.columns[c][r] for r in range(3)] for c in range(4)], np.float32)
        out.append(dict(P=P.copy(), N=N.copy(), subs=subs, T=T))
    return out


@pytest.mark.parametrize("name,tris,nsub", [("plane", 2, 1), ("plane-back", 2, 1), ("sphere", 4900, 1),
                                            ("train", 3624, 6), ("treefir", 352, 2)])
def test_obj_triangle_counts(rt, assets, name, tris, nsub):
    s = rt.Scene()
    s.add_model(os.path.join(assets, name + ".obj"), (0, 0, 0))
    assert s.triangle_count == tris
    (m,) = _meshes(s)
    assert len(m["subs"]) == nsub


def test_obj_materials_and_vertex_streams(rt, assets):
    s = rt.Scene()
    s.add_model(os.path.join(assets, "plane.obj"), (0, 0, 0))
    (m,) = _meshes(s)
    idx, mat = m["subs"][0]
    assert [mat.baseColor.x, mat.baseColor.y, mat.baseColor.z] == [0.5, 0.5, 0.5]   # Kd
    assert mat.refractionIndex == 1.0 and mat.opacity == 1.0 and mat.textureFlags == 0
    assert mat.specularExponent == 0.0   # Material(material:) reads it only for float3 (SubMesh.swift:309)
    assert len(m["P"]) == 4                  # one vertex per unique (v, vt, vn)
    assert np.allclose(m["N"], [0, 1, 0])
    assert idx.tolist() == [[0, 1, 2], [0, 2, 3]]   # fan triangulation of the quad
    s2 = rt.Scene()
    s2.add_model(os.path.join(assets, "sphere.obj"), (0, 0, 0))
    (m2,) = _meshes(s2)
    _, mat2 = m2["subs"][0]
    assert [mat2.baseColor.x, mat2.baseColor.y, mat2.baseColor.z] == [1.0, 1.0, 0.5]


def test_obj_without_normals_leaves_zero(rt, tmp_path):
    p = tmp_path / "tri.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    s = rt.Scene()
    s.add_model(str(p), (0, 0, 0))
    (m,) = _meshes(s)
    assert np.all(m["N"] == 0)   # kernel then uses -ray.direction (Raytracing.metal:395-397)
    _, mat = m["subs"][0]
    assert mat.refractionIndex == 1.0 and mat.opacity == 1.0


def test_missing_asset_raises(rt, tmp_path):
    s = rt.Scene()
    with pytest.raises(rt.RTError) as e:
        s.add_model(str(tmp_path / "nope.obj"), (0, 0, 0))
    assert e.value.code == rt._abi.RT_ERR_IO


def test_model_transform_trs(rt, assets):
    """worldTransform = T * Rx*Ry*Rz * S (Model.swift:55-58, Utilities.swift:339-347)."""
    s = rt.Scene()
    rot = (0.3, math.pi / 2 * 1.2, -0.2)
    s.add_model(os.path.join(assets, "plane.obj"), (0.3, 0.38, 2.5), rot, 1.2)
    (m,) = _meshes(s)

    def R(axis, a):
        c, sn = math.cos(a), math.sin(a)
        x, y, z = axis
        return np.array([[c + x * x * (1 - c), x * y * (1 - c) - z * sn, x * z * (1 - c) + y * sn],
                         [y * x * (1 - c) + z * sn, c + y * y * (1 - c), y * z * (1 - c) - x * sn],
                         [z * x * (1 - c) - y * sn, z * y * (1 - c) + x * sn, c + z * z * (1 - c)]])
    M = R((1, 0, 0), rot[0]) @ R((0, 1, 0), rot[1]) @ R((0, 0, 1), rot[2]) * 1.2
    T = m["T"]
    assert np.allclose(T[:3, :].T, M, atol=1e-6)
    assert np.allclose(T[3], [0.3, 0.38, 2.5])


def test_glass_override(rt):
    o = rt.glass_override()
    assert list(o.base_color) == pytest.approx([0.95, 0.98, 1.0]) and o.refraction_index == pytest.approx(1.52)
    assert o.opacity == pytest.approx(0.08)


def test_default_camera_appendix_c(rt):
    c = rt.camera_default(256, 256)
    assert c.position.tolist() == pytest.approx([0, 1, 5.38])
    assert c.forward.tolist() == pytest.approx([0, -0.1827436, -0.9831606], abs=1e-6)
    assert c.up.tolist() == pytest.approx([0, 0.40723846, -0.07569488], abs=1e-6)
    assert c.right.tolist() == pytest.approx([0.41421356, 0, 0], abs=1e-6)
    c2 = rt.camera_default(1920, 1080)
    assert c2.right.x == pytest.approx(0.73637967, abs=1e-6)


def test_uniform_defaults(rt):
    u = rt.uniforms_default(320, 200, 2)
    assert (u.samplesPerPixel, u.maxBounces, u.lightCount, u.frameIndex) == (2, 2, 2, 0)
    assert u.accumulationWeight == pytest.approx(0.9) and u.enableMotionAdaptiveAccumulation == 1
    assert u.motionSamplingMaxExtraSamples == 2 and u.blocksWide == 20 and u.shadingMode == 0


def test_random_offsets_splitmix(rt):
    r = rt.random_offsets(42, 16, 8)
    M = (1 << 64) - 1
    st = 42
    ref = []
    for _ in range(16 * 8):
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        ref.append(z % (1 << 20))
    assert r.tolist() == ref
    assert r.max() < (1 << 20)


def test_default_lights(rt):
    s = rt.Scene()
    d = s.desc()
    assert d.light_count == 2
    area, spot = d.lights[0], d.lights[1]
    assert area.type == rt._abi.LightTypeAreaLight and area.position.tolist() == pytest.approx([0, 1.98, 0])
    assert spot.type == rt._abi.LightTypeSpotlight and spot.coneAngle == pytest.approx(25 / 180 * math.pi)
    s.set_light_intensity(15)
    assert s.desc().lights[1].color.tolist() == [15, 15, 15]


@pytest.mark.parametrize("kind,tris", [("dragon", 871414), ("bunny", 69450), ("knot", 871414)])
def test_procedural_standins_closed_outward(rt, kind, tris):
    s = rt.Scene()
    s.add_procedural(kind, (0, 0, 0))
    assert s.triangle_count == tris
    (m,) = _meshes(s)
    P = m["P"].astype(np.float64)
    I = np.concatenate([x[0] for x in m["subs"]])
    vol = np.einsum("ij,ij->i", P[I[:, 0]], np.cross(P[I[:, 1]], P[I[:, 2]])).sum() / 6
    assert vol > 0, "outward winding / normals"
    n = np.linalg.norm(m["N"], axis=1)
    assert np.allclose(n, 1, atol=1e-5)


def test_presets(rt, assets):
    c1 = rt.Scene.preset("c1", assets)
    assert c1.triangle_count == 2 + 4900 + 4900 + 2 and not c1.synthetic
    c3 = rt.Scene.preset("c3g", assets)
    assert c3.triangle_count == 871414 + 9804 and c3.synthetic
    d = c3.desc()
    mat = d.meshes[0].submeshes[0].material
    assert mat.refractionIndex == pytest.approx(1.52) and mat.opacity == pytest.approx(0.08)
    c3d = rt.Scene.preset("c3d", assets)
    m2 = c3d.desc().meshes[0].submeshes[0].material
    assert [m2.baseColor.x, m2.baseColor.y, m2.baseColor.z] == [1, 0, 0]   # dragon.mtl Kd
    with pytest.raises(rt.RTError):
        rt.Scene.preset("nope", assets)


def test_robot_joint_matrices(rt):
    s = rt.Scene.preset("c5")
    J0 = s.joint_matrices(0, 0.0)
    assert J0.shape[0] == 5
    J1 = s.joint_matrices(0, 0.5)
    assert not np.allclose(J0, J1)
