"""The square-root-free length comparisons of the shading code (rt_math.h length_lt_* /
length_gt_*) give the same result as comparing sqrtf(dot(v, v)) for every input:
tools/sqrt_thresholds.c recomputes each dot-product bound and checks the floats around it (the
full check over every non-negative float, ~40 s, ran when the bounds were written)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sqrt_thresholds_band(tmp_path):
    exe = str(tmp_path / "st")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tools", "sqrt_thresholds.c"), "-o", exe,
                    "-lm"], check=True)
    r = subprocess.run([exe, "band", str(1 << 22)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    # the bounds compiled into rt_math.h are the ones the tool checks
    src = open(os.path.join(ROOT, "metal4-raytracing_amd", "csrc", "rt_math.h")).read()
    for lit in ("0x1.79ca1p-67f", "0x1.0c6f7ap-20f", "0x1.5798eep-27f"):
        assert lit in src
