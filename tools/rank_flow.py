"""configs[3]'s rank flow end to end on one GPU (tool, GPU box): the 3840x2160x16spp dragon frame,
8 bounces, rendered once by one rank and once by 8 gloo ranks sharing the box's GPU
(`bench.py --gpus 8 --gather-backend gloo`: tile split, device pack, host-staged gather, device
unpack on rank 0).  Rank 0's gathered frame must equal the one-rank frame bit for bit; the
per-rank figures of the 8-rank run show the split's load balance.  Prints one summary (JSON) and
writes it to gpurun_out/rank_flow.json; the frames stay in /tmp (too big for gpurun_out).

    python tools/rank_flow.py [--width 3840 --height 2160 --spp 16 --ranks 8]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench(args, extra, timeout):
    t0 = time.time()
    log = f"/tmp/rank_flow_{len(extra)}.log"
    with open(log, "w") as f:
        proc = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args, *extra], stdout=subprocess.PIPE,
                                stderr=f, text=True, cwd=ROOT, start_new_session=True)
        while proc.poll() is None:   # a heartbeat line every 30 s (a silent GPU command reads as hung)
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                print(f"  ... {time.time() - t0:.0f} s", flush=True)
                if time.time() - t0 > timeout:   # the launcher and its rank processes (own group)
                    os.killpg(proc.pid, 9)
                    proc.wait()
        stdout = proc.stdout.read()
    if proc.returncode != 0:
        sys.stderr.write(open(log).read()[-4000:])
        raise SystemExit(f"bench.py {' '.join(extra)} failed: {proc.returncode}")
    lines = [x for x in stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0]), time.time() - t0


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--spp", type=int, default=16)
    p.add_argument("--bounces", type=int, default=8)
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--timeout", type=int, default=420)
    a = p.parse_args()
    common = ["--width", str(a.width), "--height", str(a.height), "--spp", str(a.spp), "--bounces", str(a.bounces),
              "--steps", str(a.steps), "--warmup", "1", "--no-cpu", "--no-pmc", "--no-isolated"]
    one_f, many_f = "/tmp/rank_flow_one.npy", "/tmp/rank_flow_many.npy"
    one, t_one = bench(common, ["--dump-radiance", one_f], a.timeout)
    print(f"one rank: {one['value']} Grays/s, {one['ms_per_step']} ms/step ({t_one:.0f} s)", flush=True)
    many, t_many = bench(common, ["--gpus", str(a.ranks), "--gather-backend", "gloo", "--dump-radiance", many_f],
                         a.timeout)
    print(f"{a.ranks} ranks: {many['value']} Grays/s, {many['ms_per_step']} ms/step ({t_many:.0f} s)", flush=True)
    x, y = np.load(one_f), np.load(many_f)
    diff = np.any(x != y, axis=-1) if x.shape == y.shape else None
    T = 64
    tiles_x, tiles_y = (a.width + T - 1) // T, (a.height + T - 1) // T
    pr = many["config"]["per_rank"]
    ms = [r["ms_per_step"] for r in pr]
    rays = [r["rays_per_frame"] for r in pr]
    out = {
        "workload": many["config"]["workload"],
        "frame": [a.width, a.height, a.spp, a.bounces], "ranks": a.ranks, "steps": a.steps,
        "tiles": {"size": T, "grid": [tiles_x, tiles_y], "last_row_pixels": a.height - (tiles_y - 1) * T},
        "bitwise_equal": bool(diff is not None and not diff.any()),
        "differing_pixels": None if diff is None else int(diff.sum()),
        "one_rank": {"grays_s": one["value"], "ms_per_step": one["ms_per_step"],
                     "rays_per_frame": one["config"]["rays_per_frame"],
                     "frames_in_flight": one["config"]["frames_in_flight"]},
        "many_ranks": {"grays_s": many["value"], "ms_per_step": many["ms_per_step"],
                       "rays_per_frame": many["config"]["rays_per_frame"],
                       "gather_ms_per_step": many["config"]["gather_ms_per_step"],
                       "frames_in_flight": many["config"]["frames_in_flight"]},
        "per_rank": pr,
        "balance": {"rays_max_over_mean": round(max(rays) / (sum(rays) / len(rays)), 4),
                    "ms_max_over_min": round(max(ms) / min(ms), 4)},
        "note": "all ranks share ONE MI355X (gloo, host-staged gather): per-rank wall times include waiting for "
                "the CUs the other ranks' kernels hold; no RCCL transport ran",
    }
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "rank_flow.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1), flush=True)
    return 0 if out["bitwise_equal"] else 1


if __name__ == "__main__":
    sys.exit(main())
