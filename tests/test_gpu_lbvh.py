"""The on-device BVH build (rt_bvh_build_device, SURVEY.md §8f rank 1: LBVH + 8-wide collapse).

The tree differs from the host SAH tree, but traversal is exact (conservative boxes, watertight
triangles, ties to the smaller triangle id), so frames must be bit-identical to the
host-built ones and match the oracle."""
import time

import numpy as np
import pytest

from helpers import parity_report

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,W,H,spp,bounces", [
    ("c1", 64, 64, 1, 2),
    ("c2", 80, 45, 2, 4),
    ("c3g", 96, 54, 2, 8),
])
def test_lbvh_oracle_parity(rt, orc, assets, preset, W, H, spp, bounces):
    scene = rt.Scene.preset(preset, assets)
    R = rt.Renderer(scene, W, H, pipeline="wavefront", seed=7, bvh="lbvh")
    R.samplesPerPixel = spp
    R.maxBounces = bounces
    u = R.draw()
    g = R.radiance()
    st = R.stats()
    o = orc.OracleScene(scene.desc()).render(u, R.random)
    rep = parity_report(g, o["radiance"])
    assert rep["n_bad"] == 0, rep
    assert st.closest_rays == o["closest_rays"] and st.shadow_rays == o["shadow_rays"]
    R.close()


@pytest.mark.parametrize("W,H", [(320, 180), (1920, 1080)])
def test_lbvh_matches_host_build(rt, assets, W, H):
    """Full headline scene (up to the BASELINE size): LBVH and SAH trees give the same frame."""
    scene = rt.Scene.preset("c3g", assets)
    imgs, counts = [], []
    for bvh in ("sah", "lbvh"):
        R = rt.Renderer(scene, W, H, pipeline="wavefront", seed=3, bvh=bvh)
        R.samplesPerPixel = 4
        R.maxBounces = 8
        R.draw()
        imgs.append(R.radiance())
        st = R.stats()
        counts.append((st.closest_rays, st.shadow_rays))
        R.close()
    assert counts[0] == counts[1]
    assert np.array_equal(imgs[0], imgs[1])


def test_lbvh_rebuild_time_and_shape(rt, assets):
    """The device build of the 881k-triangle dragon scene takes milliseconds; the tree fits the
    traversal stack and covers every triangle once."""
    scene = rt.Scene.preset("c3g", assets)
    R = rt.Renderer(scene, 64, 64, pipeline="wavefront", seed=3, bvh="lbvh")
    t0 = time.perf_counter()
    for _ in range(3):
        R.rebuild(device=True)
    dt = (time.perf_counter() - t0) / 3
    st = R.stats()
    print(f"device BVH build: {dt * 1e3:.2f} ms, {st.bvh_nodes} nodes for {st.triangles} triangles")
    assert 0 < st.bvh_nodes < st.triangles
    assert dt < 0.5
    R.close()
