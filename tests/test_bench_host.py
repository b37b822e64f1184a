"""bench.py's host-side pieces on the CPU: the rocprofv3 PMC CSV reader (per kernel group: HBM bytes
per dispatch = FETCH_SIZE x 2 + WRITE_SIZE in KB, L2 hit rate) and the kernel-name grouping."""
import csv
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = importlib.import_module("bench")


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"], r)))


def test_kernel_key_groups():
    k = bench.kernel_key
    assert k("void rt::wf_trace<false, false>(rt::DevScene, ...)") == "trace"
    assert k("rt::wf_trace<true, false>(rt::DevScene)") == "trace"
    assert k("rt::wf_trace<true, true>(rt::DevScene)") is None   # counting frame
    assert k("rt::wf_shade<false, false>(rt::DevScene)") == "shade"
    assert k("rt::wf_finish_step<false, false>(rt::DevScene)") == "finish"
    assert k("rt::wf_finish_step<true, false>(rt::DevScene)") is None
    assert k("rt::wf_generate(rt::DevScene)") == "generate"
    assert k("rt::wf_resolve(rt::DevScene)") == "resolve" and k("rt::wf_motion(rt::DevScene)") == "resolve"
    assert k("__amd_rocclr_fillBufferAligned") is None


def test_read_pmc(tmp_path):
    fa, fw, fh = tmp_path / "f.csv", tmp_path / "w.csv", tmp_path / "h.csv"
    _write(fa, [(1, "rt::wf_finish_step<false, false>(x)", "FETCH_SIZE", 1000.0),
                (2, "rt::wf_finish_step<false, false>(x)", "FETCH_SIZE", 3000.0),
                (3, "rt::wf_trace<false, false>(x)", "FETCH_SIZE", 10.0)])
    _write(fw, [(1, "rt::wf_finish_step<false, false>(x)", "WRITE_SIZE", 100.0),
                (2, "rt::wf_finish_step<false, false>(x)", "WRITE_SIZE", 300.0),
                (3, "rt::wf_trace<false, false>(x)", "WRITE_SIZE", 2.0)])
    _write(fh, [(1, "rt::wf_finish_step<false, false>(x)", "TCC_HIT_sum", 60.0),
                (1, "rt::wf_finish_step<false, false>(x)", "TCC_MISS_sum", 40.0),
                (5, "rt::wf_shade<false, false>(x)", "TCC_HIT_sum", 3.0),
                (5, "rt::wf_shade<false, false>(x)", "TCC_MISS_sum", 1.0)])
    p = bench.read_pmc([str(fa), str(fw), str(fh)])
    assert p["finish"]["bytes_per_launch"] == int((2 * 2000.0 + 200.0) * 1024) and p["finish"]["dispatches"] == 2
    assert p["finish"]["l2_hit"] == 0.6 and p["shade"]["l2_hit"] == 0.75
    assert p["trace"]["bytes_per_launch"] == int((20.0 + 2.0) * 1024)
    assert "bytes_per_launch" not in p["shade"]


def test_pmc_child_args_keep_the_workload():
    a = bench.parse(["--scene", "c2", "--width", "1280", "--height", "720", "--bounces", "4", "--emulate-ranks", "8"])
    args = bench.pmc_child_args(a)
    assert args[0] == "--pmc-child"
    for k, v in (("--scene", "c2"), ("--width", "1280"), ("--height", "720"), ("--bounces", "4"),
                 ("--emulate-ranks", "8")):
        assert args[args.index(k) + 1] == v
