"""The Python RCCL gather path (tiles.TileGather over dist.init_process_group("nccl"), device
buffers) executed end to end at world size 1, in a fresh child process (tests/rccl_child.py):
render, device pack on torch's stream, dist.gather over RCCL, device unpack, all bitwise against
the frame itself and an untiled frame.  Multi-rank RCCL needs more than the pool's one GPU; the
2- and 3-rank flow runs over gloo in test_gpu_ranks.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_tilegather_rccl_world1_device_buffers_bitwise():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_child.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    out = json.loads(lines[-1])
    assert out["backend"] == "nccl" and out["world_size"] == 1, out
    assert out["pack_equal"] and out["unpack_equal"] and out["untiled_equal"], out
    assert out["frame_changed"] and out["nonzero"], out
    assert r.returncode == 0, r.stderr[-3000:]
