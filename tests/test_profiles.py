"""The committed measurement of the newest round reproduces (VERDICT r03 'next' 1): the bench line's
dominant kernel is rocprofv3's top kernel in the kernel-alone profile of the same workload, and the
line's roofline fraction (PMC bytes per launch over the launch time alone) recomputes from that
profile's average duration within 5 % (tools/roofline_check.py)."""
import importlib
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _newest(pattern):
    names = sorted(f for f in os.listdir(PROF) if re.fullmatch(pattern, f)) if os.path.isdir(PROF) else []
    return os.path.join(PROF, names[-1]) if names else None


def test_committed_roofline_reproduces():
    bench_json = _newest(r"r(0[4-9]|[1-9]\d)_bench\.json")
    if bench_json is None:
        pytest.skip("no round-4+ bench line under profiles/")
    tag = os.path.basename(bench_json).split("_")[0]
    stats = os.path.join(PROF, f"{tag}_alone_kernel_stats.csv")
    assert os.path.exists(stats), f"{stats} missing beside {bench_json}"
    check = importlib.import_module("roofline_check").check
    line = json.loads([x for x in open(bench_json) if x.startswith("{")][-1])
    ok, res = check(line, stats)
    assert ok, res
    assert line["roofline"]["frac_source"].startswith("pmc")
