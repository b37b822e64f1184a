"""Product BVH (binned-SAH BVH2 collapsed to the compressed 8-wide layout) + the product traversal
loop, run on the host through rt_debug_trace_host, against the oracle's independent median BVH.

The reference delegates this to Metal's intersector (Raytracing.metal:275-291: closest hit,
triangle geometry, instancing; :622-636 shadow any-hit) — parity unpinned against Apple's
intersector, pinned here against the oracle's brute-force-checked traversal.  Closest hits must
agree bit-exactly (t, triangle id, barycentrics); any-hit must agree on occlusion."""
import numpy as np
import pytest


def _rays(rng, desc_scene, n, orc):
    # rays from points around the scene toward random points inside its bounds
    lo, hi = np.array([-3.0, -0.5, -2.0]), np.array([4.0, 3.0, 4.0])
    o = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    tgt = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


@pytest.mark.parametrize("preset,n", [("c1", 3000), ("c2", 1500), ("c3g_synthetic", 600)])
def test_closest_hit_matches_oracle(rt, orc, assets, preset, n):
    sc = rt.Scene.preset(preset, assets)
    o_s = orc.OracleScene(sc.desc())
    rng = np.random.default_rng(5)
    o, d = _rays(rng, sc, n, orc)
    res = rt.debug_trace_host(sc, o, d)
    mism = 0
    for k in range(n):
        ref = o_s.intersect(o[k], d[k])
        if ref is None:
            mism += int(res["id"][k] != 0xFFFFFFFF)
            continue
        t, i, u, v = ref
        same = (res["id"][k] == i and np.float32(res["t"][k]) == np.float32(t)
                and np.float32(res["u"][k]) == np.float32(u) and np.float32(res["v"][k]) == np.float32(v))
        mism += int(not same)
    assert mism == 0, f"{mism}/{n} rays differ"
    # traversal visits a bounded number of wide nodes (sanity of the collapsed tree)
    assert res["nodes"].mean() < 200


@pytest.mark.parametrize("preset", ["c1", "c3g_synthetic"])
def test_any_hit_matches_oracle(rt, orc, assets, preset):
    sc = rt.Scene.preset(preset, assets)
    o_s = orc.OracleScene(sc.desc())
    rng = np.random.default_rng(9)
    n = 800
    o, d = _rays(rng, sc, n, orc)
    tmax = rng.uniform(0.1, 6.0, size=n).astype(np.float32)
    res = rt.debug_trace_host(sc, o, d, tmax=tmax, any_hit=True)
    for k in range(n):
        ref = o_s.intersect(o[k], d[k], tmax=float(tmax[k]), any_hit=True)
        assert (ref is not None) == (res["id"][k] != 0xFFFFFFFF), k


def test_empty_and_parallel_rays(rt, orc, assets):
    sc = rt.Scene.preset("c1", assets)
    # axis-parallel rays (zero direction components) and rays pointing away from everything
    o = np.array([[0, 5, 0], [0, 0.5, 10], [0, 0.5, 10], [100, 100, 100]], np.float32)
    d = np.array([[0, -1, 0], [0, 0, -1], [0, 0, 1], [1, 0, 0]], np.float32)
    res = rt.debug_trace_host(sc, o, d)
    o_s = orc.OracleScene(sc.desc())
    for k in range(len(o)):
        ref = o_s.intersect(o[k], d[k])
        if ref is None:
            assert res["id"][k] == 0xFFFFFFFF
        else:
            assert res["id"][k] == ref[1] and np.float32(res["t"][k]) == np.float32(ref[0])
