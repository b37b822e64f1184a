"""The host readers of untrusted asset bytes (USD text / crate / zip, PNG, OBJ) under
AddressSanitizer + UBSan on mutated inputs (tools/fuzz_host.sh; DESIGN.md §8e 'Hostile input').
A short campaign per reader: any sanitizer report aborts the run and fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_asset_readers_survive_mutated_inputs():
    env = dict(os.environ, ITERS="200", SEED="3")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "fuzz_host.sh")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    for mode in ("usda", "usdc", "usdz", "png", "obj"):
        assert f"{mode}: 200 inputs" in r.stdout, r.stdout
