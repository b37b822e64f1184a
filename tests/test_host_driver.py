"""The C host driver (host/rtbench.c) over the C-ABI: it builds with plain gcc against the
headers and the library, and (GPU) renders frames in flight, reports Grays/s from the library's
running totals and writes the presented frame as a PNG."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "host", "rtbench")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "host")], check=True)
    return EXE


def test_rtbench_builds_and_parses_args():
    exe = _build()
    r = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "usage: rtbench" in r.stderr
    r = subprocess.run([exe, "--bogus", "1"], capture_output=True, text=True)
    assert r.returncode == 2


@pytest.mark.gpu
def test_rtbench_renders(rt, assets, tmp_path):
    exe = EXE if os.path.exists(EXE) else _build()
    png = tmp_path / "c1.png"
    r = subprocess.run([exe, "--scene", "c1", "--assets", assets, "--width", "128", "--height", "96", "--spp", "2",
                        "--bounces", "3", "--frames", "4", "--warmup", "1", "--png", str(png)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["grays_per_s"] > 0 and line["frames_in_flight"] == 4   # default for a small frame
    img = rt.decode_png(png.read_bytes())
    assert img.shape == (96, 128, 4)
    # same frames through the Python mirror: identical display bytes
    R = rt.Renderer(rt.Scene.preset("c1", assets), 128, 96, seed=3)
    R.samplesPerPixel, R.maxBounces = 2, 3
    for _ in range(5):
        R.draw()
    assert np.array_equal(R.present(), img)


def test_rtbench_rank_launcher_args():
    """--rank / --nranks without an id file, or a rank outside the split, is a usage error."""
    exe = _build()
    r = subprocess.run([exe, "--rank", "0", "--nranks", "2"], capture_output=True, text=True)
    assert r.returncode == 2
    r = subprocess.run([exe, "--rank", "3", "--nranks", "2", "--id-file", "/tmp/x"], capture_output=True, text=True)
    assert r.returncode == 2


@pytest.mark.gpu
def test_rtbench_rccl_split(rt, assets, tmp_path):
    """--ranks 1: the launcher starts one rank process, which builds an RCCL communicator (id
    through the file), renders its tiles, packs them, ncclGathers them to rank 0 and unpacks them;
    the presented frame equals the single-process one.  (More ranks need more GPUs than the
    test box has: RCCL refuses two ranks on one device.)"""
    exe = EXE if os.path.exists(EXE) else _build()
    png = tmp_path / "split.png"
    r = subprocess.run([exe, "--ranks", "1", "--scene", "c1", "--assets", assets, "--width", "200", "--height", "136",
                        "--spp", "2", "--bounces", "3", "--frames", "3", "--warmup", "1", "--png", str(png)],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["ranks"] == 1 and line["grays_per_s"] > 0
    img = rt.decode_png(png.read_bytes())
    R = rt.Renderer(rt.Scene.preset("c1", assets), 200, 136, seed=3)
    R.samplesPerPixel, R.maxBounces = 2, 3
    for _ in range(4):
        R.draw(tiles=(64, 0, 1))
    assert np.array_equal(R.present(), img)
