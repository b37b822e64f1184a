"""Frames submitted as HIP graph replays (the replacement of the reference's per-frame
command buffers, Renderer.swift:1405-1490): rt_stats counts how every wavefront frame was submitted
(replayed, captured, refused capture -> eager, eager by choice).  The default C3g frame, through the
Python mirror and through the C host driver, is captured once per frame slot and replayed after
that, never refused; and the graph shape the library uses (the cross-frame wait between two
graphs) runs under the system ROCm runtime the C host links (tests/graph_repro)."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPRO = os.path.join(ROOT, "tests", "graph_repro", "graph_wait_repro")


def test_c3g_frames_replay_graphs(rt, assets):
    R = rt.Renderer(rt.Scene.preset("c3g", assets), 1920, 1080, seed=3)
    R.samplesPerPixel, R.maxBounces = 4, 8
    frames = 10
    for _ in range(frames):
        R.draw()
    R.wait()
    s = R.stats()
    nfl = s.frames_in_flight
    assert nfl >= 2
    assert s.total_graph_fallbacks == 0 and s.total_graph_eager == 0
    assert s.total_graph_captures == nfl               # each slot's first frame
    assert s.total_graph_replays == frames - nfl       # every later frame
    # a changed launch argument (here the sample count: queue sizes, grid) captures again once per slot
    R.samplesPerPixel = 2
    for _ in range(nfl + 1):
        R.draw()
    R.wait()
    t = R.stats()
    assert t.total_graph_captures - s.total_graph_captures == nfl
    assert t.total_graph_replays - s.total_graph_replays == 1 and t.total_graph_fallbacks == 0
    R.close()


def test_rtbench_c3g_replays_graphs(rt, assets):
    exe = os.path.join(ROOT, "host", "rtbench")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "host")], check=True)
    r = subprocess.run([exe, "--scene", "c3g", "--assets", assets, "--width", "1920", "--height", "1080", "--spp", "4",
                        "--bounces", "8", "--frames", "8", "--warmup", "2"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    nfl = line["frames_in_flight"]
    assert line["graph_fallbacks"] == 0 and line["graph_eager"] == 0
    assert line["graph_captures"] == nfl and line["graph_replays"] == 10 - nfl


def test_graph_repro_split_wait_runs():
    """The library's shape: two graphs per frame, the previous frame's `done` waited on between
    them as a plain stream wait; eight frames over two slots, captured once, replayed."""
    if not os.path.exists(REPRO):
        subprocess.run(["make", "-s", "-C", os.path.dirname(REPRO)], check=True)
    r = subprocess.run([REPRO, "split"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ok: 8 frames" in r.stderr
