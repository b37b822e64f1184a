"""GPU parity for a USD-loaded skinned model (SURVEY.md §8f rank 3 feeding rows a25 / a26): the
test asset of tests/test_usd.py, written as a .usdz crate package, placed in the C1 scene, skinned
on the device with the joint matrices of Model.update + SkinningPass (rt_scene_joint_matrices),
refit or rebuilt, rendered through every pipeline and compared bit for bit with the oracle on the
host-skinned mesh (as tests/test_gpu_dynamic.py does for the procedural robot)."""
import numpy as np
import pytest

import usd_writers as W
from helpers import PIPELINES, make_renderer
from test_gpu_dynamic import _check_frame, _desc_with, _f4, _skinned_mesh
from test_usd import TEX, robot_prims

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def usdz(tmp_path_factory):
    prims, _ = robot_prims()
    p = tmp_path_factory.mktemp("gpu_usd") / "robot.usdz"
    p.write_bytes(W.write_usdz("robot.usdc", W.write_usdc(prims), [("textures/tex.png", TEX)]))
    return str(p)


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("rebuild", ["refit", "device"])
@pytest.mark.parametrize("t", [0.6, 1.5])
def test_usd_skinned_model_parity(rt, orc, assets, usdz, pipeline, rebuild, t):
    W_, H = 96, 64
    sc = rt.Scene.preset("c1", assets)
    sc.add_usd(usdz, (-0.4, 0.0, 1.2), (0.0, 0.5, 0.0), 0.45)
    desc = sc.desc()
    m = _skinned_mesh(desc)
    md = desc.meshes[m]
    n = md.vertex_count
    rest_p, rest_n = _f4(md.positions, n).copy(), _f4(md.normals, n).copy()
    ji = np.ctypeslib.as_array(md.joint_indices, shape=(n, 4)).copy()
    jw = np.ctypeslib.as_array(md.joint_weights, shape=(n, 4)).copy()
    J = sc.joint_matrices(m, t)
    R = make_renderer(rt, sc, W_, H, pipeline, seed=7)
    R.samplesPerPixel = 2
    R.maxBounces = 3
    R.skin(m, J)
    R.refit() if rebuild == "refit" else R.rebuild(device=True)
    u = R.draw()
    R.wait()
    sp, sn = orc.skin(rest_p, rest_n, ji, jw, J)
    assert np.abs(sp - rest_p).max() > 1e-3   # the arm moved
    d2 = _desc_with(rt, desc, m, positions=sp, normals=sn)
    osc = orc.OracleScene(d2)
    osc.set_previous(m, prev_positions=rest_p)
    o = osc.render(u, R.random)
    _check_frame(R, o)
    R.close()
