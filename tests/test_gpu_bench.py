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
    # 12 steps over the frame slots: each slot's first frame may capture, the later ones replay
    d = _run("--scene", "c1", "--width", "128", "--height", "96", "--spp", "2", "--bounces", "3", "--steps", "12",
             "--warmup", "4", "--cpu-seconds", "0.5")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 12 and d["value"] > 0 and d["unit"] == "Grays/s"
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["frac"] > 0
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1
    # a frame below 512K paths keeps four frames in flight although bench.py gives the process
    # eight hardware queues (rt_api.cpp kSmallFramePaths)
    assert d["config"]["frames_in_flight"] == 4
    _roofline_consistent(d)
    # the timed frames replay captured HIP graphs
    g = d["config"]["graphs"]
    assert g["fallbacks"] == 0 and g["eager"] == 0 and g["replays"] >= 4 and g["replays"] + g["captures"] == 12


def _roofline_consistent(d):
    """The roofline is internally consistent: the dominant kernel has the most device time per frame
    with the kernels alone, that time fits in the single-frame latency, and frac recomputes from the
    line's own fields (PMC bytes per launch / launch time alone / 8 TB/s)."""
    r = d["roofline"]
    ks = r["kernels"]
    dom = max(ks, key=lambda k: k["ms_per_frame"])
    assert r["kernel"] == dom["kernel"] and r["launch_ms"] == dom["launch_ms"]
    assert d["ms_per_frame"] > 0 and r["ms_per_frame_alone"] <= d["ms_per_frame"] * 1.02
    assert sum(k["ms_per_frame"] for k in ks) <= d["ms_per_frame"] * 1.05
    assert r["frac_source"].startswith("pmc"), r["frac_source"]
    assert r["traffic"] > 0
    frac = r["traffic"] / (r["launch_ms"] * 1e-3) / 1e9 / r["peak"]
    assert abs(frac - r["frac"]) <= 1e-3 + 0.01 * frac
    assert r["l2_hit"] and all(0 < v < 1 for v in r["l2_hit"].values())
    if any(k["kernel"].startswith("rt::wf_shade") for k in ks):   # a small frame may run entirely in the finish
        assert r["shade_l2_hit"] is not None and 0 < r["shade_l2_hit"] < 1
    # the timed frames are graph replays, which carry no per-stage events under torch's HIP runtime
    assert "in_flight" in r and r["in_flight"]["ms_per_step"] > 0


def test_bench_emulated_rank_and_animation():
    d = _run("--scene", "c5", "--width", "128", "--height", "96", "--spp", "1", "--bounces", "2", "--steps", "3",
             "--warmup", "1", "--no-cpu", "--no-pmc", "--animate", "--emulate-ranks", "2")
    assert d["value"] > 0 and d["config"]["animate"] is True and d["cpu_baseline"] is None
    # --no-pmc: no HBM byte count, so no HBM fraction; the algorithmic rate is reported beside it
    r = d["roofline"]
    assert r["frac"] is None and r["achieved"] is None and r["traffic"] is None
    assert r["frac_source"].startswith("none") and r["frac_algorithmic"] > 0
