"""Child process of test_gpu_env_variants.py: the golden-fixture parity of test_gpu_parity.py for a
few cases and pipelines, in a process whose environment selects a runtime variant (the library
reads RT_* switches once per process).  Exits non-zero on the first mismatch."""
import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]

from helpers import make_renderer, parity_report   # noqa: E402
import make_golden   # noqa: E402


def main(cases, pipelines):
    rt = importlib.import_module("metal4-raytracing_amd")
    assets = os.path.join(ROOT, "assets")
    meta_all = json.load(open(os.path.join(HERE, "golden", "cases.json")))
    for name in cases:
        meta = meta_all[name]
        g = np.load(os.path.join(HERE, "golden", name + ".npz"))
        for pipeline in pipelines:
            scene = make_golden.make_scene(rt, meta["preset"], assets)
            R = make_renderer(rt, scene, meta["width"], meta["height"], pipeline, seed=meta["seed"])
            for k, v in meta["knobs"].items():
                setattr(R, k, v)
            for _ in range(meta["frames"]):
                R.draw()
            img = R.radiance()[..., :3]
            depth, _, _ = R.aux()
            st = R.stats()
            rep = parity_report(img, g["radiance"])
            ok = (rep["n_bad"] == 0 and np.array_equal(depth, g["depth"])
                  and [st.closest_rays, st.shadow_rays] == g["counts"].tolist()[:2])
            print(name, pipeline, "ok" if ok else "MISMATCH", rep, flush=True)
            if not ok:
                return 1
            R.close()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1].split(","), sys.argv[2].split(",")))
