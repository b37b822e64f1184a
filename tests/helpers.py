"""Shared helpers for the parity tests (tolerances and comparison)."""
import numpy as np

# North-star parity bar (BASELINE.json): per-pixel relative L2 of RGB radiance <= 1e-4.
REL_L2_TOL = 1e-4


def rel_l2_per_pixel(a, b):
    """Per-pixel ||a-b|| / max(||b||, 1e-6) over RGB."""
    a = np.asarray(a, np.float64)[..., :3]
    b = np.asarray(b, np.float64)[..., :3]
    num = np.linalg.norm(a - b, axis=-1)
    den = np.maximum(np.linalg.norm(b, axis=-1), 1e-6)
    return num / den


def parity_report(gpu, ref):
    e = rel_l2_per_pixel(gpu, ref)
    exact = np.mean(np.all(np.asarray(gpu)[..., :3] == np.asarray(ref)[..., :3], axis=-1))
    return dict(max_rel=float(e.max()), n_bad=int((e > REL_L2_TOL).sum()), frac_bitwise=float(exact))


# Pipeline variants of the GPU tests: the per-pixel megakernel, and the wavefront pipeline with
# the default finish threshold (small frames run almost entirely in the persistent finish
# kernel), with no finish kernel at all (every bounce through extend / shade / connect) and
# with a small threshold (bulk rounds, then finish).  "wavefront-bulk-sort" and the mixed variant
# also sort hits by BVH leaf bin between extend and shade (off by default).
PIPELINES = ["megakernel", "wavefront", "wavefront-bulk", "wavefront-mixed", "wavefront-bulk-sort"]
_VARIANTS = {"megakernel": ("megakernel", 0, 0), "wavefront": ("wavefront", 0, 0),
             "wavefront-bulk": ("wavefront", 1, 0), "wavefront-mixed": ("wavefront", 2048, 4096),
             "wavefront-bulk-sort": ("wavefront", 1, 2048)}


def make_renderer(rt, scene, W, H, pipeline="wavefront", **kw):
    pl, tail, sort_bins = _VARIANTS[pipeline]
    return rt.Renderer(scene, W, H, pipeline=pl, tail_paths=tail, sort_bins=sort_bins, **kw)
