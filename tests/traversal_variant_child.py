"""Child process of test_gpu_traversal_variants.py: the adversarial closest-hit scenes (the
triangle soup and the exact-tie scene, tests/helpers.py) through the given pipelines, against the
CPU oracle, in a process whose environment selects a traversal instance (RT_TEAM lanes per query
in the finish kernel's drain, RT_FCHUNK ...: tests/helpers.make_renderer maps these onto the
library's rt_set_tuning).  Prints one line per case; exits non-zero on the first mismatch."""
import importlib
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]

from helpers import make_renderer, parity_report, traversal_scene   # noqa: E402


def main(specs, pipelines):
    rt = importlib.import_module("metal4-raytracing_amd")
    import oracle
    assets = os.path.join(ROOT, "assets")
    tmp = tempfile.mkdtemp(prefix="rt_trav_")
    for spec in specs:   # kind:W:H:spp:bounces
        kind, W, H, spp, nb = spec.split(":")
        scene = traversal_scene(rt, assets, kind, tmp)
        osc = oracle.OracleScene(scene.desc())
        ref = None
        for pipeline in pipelines:
            R = make_renderer(rt, scene, int(W), int(H), pipeline, seed=3)
            R.samplesPerPixel, R.maxBounces = int(spp), int(nb)
            u = R.draw()
            R.wait()
            g = R.radiance()
            depth, _, _ = R.aux()
            st = R.stats()
            if ref is None:
                ref = osc.render(u, R.random)
            rep = parity_report(g, ref["radiance"])
            ok = (rep["n_bad"] == 0 and np.array_equal(depth, ref["depth"])
                  and (st.closest_rays, st.shadow_rays) == (ref["closest_rays"], ref["shadow_rays"]))
            print(spec, pipeline, "ok" if ok else "MISMATCH", rep, st.closest_rays, ref["closest_rays"], flush=True)
            R.close()
            if not ok:
                return 1
        osc.close()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1].split(","), sys.argv[2].split(",")))
