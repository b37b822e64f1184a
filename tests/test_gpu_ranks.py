"""The multi-rank frame flow on one GPU (Renderer.swift:1405-1503 renders on one
device): `bench.py --gpus 2 --gather-backend gloo` starts two rank processes through its own
launcher, both render their tiles on the box's GPU with the HIP path, pack them with the device
kernel, gather the packed tiles over gloo (host-staged: RCCL refuses two ranks on one device) and
rank 0 unpacks them with the device kernel.  Everything but RCCL's transport runs; the gathered
frame must equal the one-rank frame bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--scene", "c1", "--width", "200", "--height", "136", "--spp", "2", "--bounces", "3", "--steps", "3",
        "--warmup", "1", "--no-cpu", "--no-pmc", "--no-isolated"]


def _bench(*extra):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, *extra], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_ranks_share_one_gpu_gloo_gather_bitwise(tmp_path, n):
    one = _bench("--dump-radiance", str(tmp_path / "one.npy"))
    many = _bench("--gpus", str(n), "--gather-backend", "gloo", "--dump-radiance", str(tmp_path / "many.npy"))
    assert one["n_gpus"] == 1 and many["n_gpus"] == n and many["world_size"] == n
    assert many["config"]["parallelism"] == f"tiles{n}" and "gloo" in many["config"]["workload"]
    # all ranks' rays: the split frame traces the same rays as the whole one
    assert many["config"]["rays_per_frame"] == one["config"]["rays_per_frame"]
    pr = many["config"]["per_rank"]   # each rank's own figures (load balance of the split)
    assert [x["rank"] for x in pr] == list(range(n)) and all(x["ms_per_step"] > 0 for x in pr)
    assert abs(sum(x["rays_per_frame"] for x in pr) - many["config"]["rays_per_frame"]) <= n   # per-rank truncation
    a, b = np.load(tmp_path / "one.npy"), np.load(tmp_path / "many.npy")
    assert a.shape == b.shape == (136, 200, 4)
    diff = np.any(a != b, axis=-1)
    if diff.any():   # which tiles differ: rank 0's own (rendering) or the gathered ones (transport)
        tiles_x = (200 + 63) // 64
        tid = (np.arange(136)[:, None] // 64) * tiles_x + (np.arange(200)[None, :] // 64)
        owner = tid % n
        by_rank = {r: int(diff[owner == r].sum()) for r in range(n)}
        ys, xs = np.nonzero(diff)
        pytest.fail(f"{int(diff.sum())} of {diff.size} pixels differ; by owning rank {by_rank}; "
                    f"max |diff| {float(np.abs(a - b).max())}; first differing pixels (y, x) "
                    f"{list(zip(ys[:8].tolist(), xs[:8].tolist()))} (both frames kept in {tmp_path})")
