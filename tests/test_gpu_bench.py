"""bench.py's contract on a small workload (the driver parses its one JSON line): required keys,
the roofline and cpu_baseline objects, and the per-rank emulation mode."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_line_contract():
    d = _run("--scene", "c1", "--width", "128", "--height", "96", "--spp", "2", "--bounces", "3", "--steps", "3",
             "--warmup", "1", "--cpu-seconds", "0.5")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["unit"] == "Grays/s"
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1
    # a small frame (< 8M allocated paths) keeps four frames in flight: bench.py fixes HIP's
    # hardware queues at four (rt_api.cpp small_frame_slots)
    assert d["config"]["frames_in_flight"] == 4
    # with frames in flight the line carries the traversal launches measured alone (one frame in
    # flight, after the timed region) and says whether the shared-GPU launch time is a kernel time
    iso = r["isolated"]
    assert iso["frames_in_flight"] == 1 and iso["launch_ms"] > 0 and 0 < iso["frac"] < 1
    assert isinstance(r["not_a_kernel_measurement"], bool)


def test_bench_emulated_rank_and_animation():
    d = _run("--scene", "c5", "--width", "128", "--height", "96", "--spp", "1", "--bounces", "2", "--steps", "3",
             "--warmup", "1", "--no-cpu", "--animate", "--emulate-ranks", "2")
    assert d["value"] > 0 and d["config"]["animate"] is True and d["cpu_baseline"] is None
