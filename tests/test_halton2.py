"""The base-2 Halton dimension in closed form (rt_math.h halton_base2, used by the primary-ray
jitter) is bit-identical to the reference radical-inverse loop (Raytracing.metal:42-57, rt_math.h
halton_fast).  tools/halton2_check.c compares them; the full check over all 2^31 positive indices
was run when it was written (~2 min on 4 cores); here: the first 2^22 indices, the last 2^20, and
the carry / tie cases around every power of two."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("h2") / "h2")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-I", ROOT, "-x", "c++",
                    os.path.join(ROOT, "tools", "halton2_check.c"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("lo,hi", [(1, 1 << 22), ((1 << 31) - (1 << 20), (1 << 31) - 1)] +
                         [((1 << k) - 64, (1 << k) + 64) for k in range(7, 31)])
def test_base2_closed_form_matches_loop(checker, lo, hi):
    r = subprocess.run([checker, str(lo), str(hi)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
