#!/usr/bin/env python3
"""Headline benchmark: Grays/s + ms/frame, dragon scene, 1920x1080x4spp, 8 bounces (BASELINE.json
metric; workload = configs[2], the dragon config that fits one MI355X).

One step = one frame of the hot path (raytracingKernel equivalent) over the whole image.
N GPUs (one process per GPU, torch.distributed over RCCL): the frame is tile-partitioned
(64x64 tiles, tile_id % N == rank), every rank renders its tiles, packs them, and rank 0
gathers the packed radiance over RCCL/xGMI and unpacks it into the full frame ("strong"
scaling: the frame is fixed, N GPUs share it).

`python bench.py --gpus N` with no WORLD_SIZE in the environment starts the N ranks itself: the
parent never touches the GPU (it does not import torch); it starts N child processes of this
script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, passes rank 0's JSON
line through (the children share its stdout) and exits non-zero if any child fails.  Under
torch.distributed.run (WORLD_SIZE set) the process is one rank.

Grays/s = (closest-hit + shadow rays traced, all ranks) / wall time of the K timed frames
(barrier + device sync on both sides, max over ranks).  Inputs (scene, BVH, random offsets)
are resident in HBM before the timed region.
"""
import argparse
import importlib
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np

# Hardware queues per process, fixed before anything initialises HIP so every run sees the same
# count: RT_HW_QUEUES if set, else eight (the library keeps one frame in flight per queue, up to
# eight: rt_api.cpp small_frame_slots).  Since the slot streams stopped waiting on the context
# stream (round 5), eight queues / eight frames in flight measured, against HIP's default four
# (which the GPU boxes export): C3g 9.47-9.51 vs 9.26-9.31 Grays/s at 20 steps, 9.55-9.56 vs
# 9.35-9.38 at 32; configs[1] 10.03 vs 9.78; the 8-way rank share 6.76 vs 6.18; configs[3] +-0;
# but the animated configs[4] (skin + refit every frame) 10.21-10.33 vs 10.77-10.86, so --animate
# keeps four (profiles/r05_finish_experiments.txt).
# (Only when run as a program: tests import this module for its helpers.)
if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES") or ("4" if "--animate" in sys.argv else "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
# MI355X_MICROARCH.md 'Indexed rows': rows gathered from a table every workgroup shares, served by
# the XCD's L2, 16.8-18.8 TB/s chip-wide (the lower figure).  The traversal's node / triangle
# working set (48 MB for C3g) lives in L2 and the Infinity Cache (L2 hit 0.63), so its algorithmic
# rate is also priced against this cache-gather ceiling.
L2_GATHER_PEAK_GBS = 16800.0
# Random 128-B line requests per second (tools/ubench/lane_loads, profiles/r04_gather_ceiling.txt):
# ~255 G/s for lines that hit the XCD's L2, ~60 G/s for L2 misses (Infinity Cache or HBM); a lane's
# loads inside one line cost one request.  `frac_of_line_ceiling` prices a kernel's L2 requests
# (TCC_HIT + TCC_MISS per launch, PMC) against them: hits / 255 G + misses / 60 G per second.
L2_HIT_LINES_PER_S = 255e9
L2_MISS_LINES_PER_S = 60e9
SCENES = {"c3g": "glass dragon scene (configs[2])", "c3": "glass dragon scene (configs[2])",
          "c3d": "opaque dragon scene", "c1": "AppScene base (configs[0])", "c2": "bunny scene (configs[1])",
          "c5": "skinned robot scene (configs[4])",
          "c3r": "irregular-geometry check: the reference's coatball / teapot meshes, glass, in the dragon's place"}   # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic bytes (DESIGN.md §6 'Roofline'): per traced ray its 48-B queue entry (extend: 32 B ray
# in + 16 B hit out; connect: 48 B shadow entry in); per 8-wide node fetched from memory 80 B; per
# triangle tested 48 B; per closest hit shaded inside the finish kernel 16 B triangle record +
# 3 x 16 B normals + 48 B instance transform.
B_RAY = 48
B_NODE = 80  # compressed 8-wide node (Bvh8Node)
B_TRI = 48
B_HIT = 16 + 48 + 48
B_QRAY = 48
# wf_shade, per shaded hit: ray + hit + colour of the queue entry (64 B), the triangle's normal
# record (48 B of its 64) and instance transform (48 B) in; the next ray + colour (48 B) and the
# shadow entry (48 B) out
B_SHADE_HIT = 64 + 48 + 48 + 48 + 48
# wf_generate: per path its ray (32 B) and accumulator (16 B); per pixel depth, motion, hit record (28 B)
B_GEN_PATH, B_GEN_PIXEL = 48, 28
# wf_motion + wf_resolve, per pixel: the samples' accumulators (16 B each), motion in / out and
# history in / out (48 B)
B_RESOLVE_PIXEL = 48
# The frame's kernels, grouped as the roofline prices them: key, name, stage_ms slots (rt_stats
# kernel_ms: [generate, extend, shade, connect, resolve, finish, hit sort]), and the rocprofv3
# kernel-name pattern of their timed (non-counting) instantiations
KERNELS = [
    ("trace", "rt::wf_trace<{false,true}, false> (extend + connect)", (1, 3), r"wf_trace<(true|false),false>"),
    ("shade", "rt::wf_shade<false, false>", (2,), r"wf_shade<"),
    ("finish", "rt::wf_finish_step<false, false>", (5,), r"wf_finish_step<false,"),
    ("generate", "rt::wf_generate", (0,), r"wf_generate"),
    ("resolve", "rt::wf_motion + rt::wf_resolve", (4,), r"wf_(motion|resolve|extra)\b"),
]
PMC_PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"], ["TCC_HIT_sum", "TCC_MISS_sum"],
              ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]]
# VALU issue (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles on its SIMD;
# 256 CUs x 4 SIMDs; SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE is summed
# over the 8 XCDs, so GRBM_GUI_ACTIVE / 8 is the launch's length in cycles)
VALU_ISSUE_CYCLES = 2
SIMDS = 1024
NOMINAL_CLOCK_HZ = 2.4e9


def kernel_key(name):
    """the KERNELS key of a rocprofv3 kernel name (None: not one of the frame's timed kernels)"""
    k = name.split("(")[0].replace("void ", "").replace(" ", "")
    for key, _, _, pat in KERNELS:
        if re.search(pat, k):
            return key
    return None


def read_pmc(paths):
    """Per kernel group from rocprofv3 --pmc counter_collection CSVs (one pass per file): HBM bytes
    per dispatch (FETCH_SIZE x 2 + WRITE_SIZE, KB units; gfx950's FETCH_SIZE counts half of wide
    reads, MI355X_MICROARCH.md 'HBM'), the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS) and the
    dispatches seen."""
    import csv
    acc = {}
    for path in paths:
        if not path or not os.path.exists(path):
            continue
        with open(path) as f:
            for row in csv.DictReader(f):
                key = kernel_key(row.get("Kernel_Name", ""))
                if key is None:
                    continue
                name = row.get("Counter_Name", "")
                g = acc.setdefault(key, {})
                c = g.setdefault(name, [0.0, set()])
                c[0] += float(row.get("Counter_Value", 0) or 0)
                c[1].add(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(c[1]))
    out = {}
    for key, g in acc.items():
        r = {}
        if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
            f, w = g["FETCH_SIZE"], g["WRITE_SIZE"]
            r["bytes_per_launch"] = int((2 * f[0] / max(len(f[1]), 1) + w[0] / max(len(w[1]), 1)) * 1024)
            r["dispatches"] = len(f[1])
        hit, miss = g.get("TCC_HIT_sum", [0.0, ()])[0], g.get("TCC_MISS_sum", [0.0, ()])[0]
        if hit + miss > 0:
            r["l2_hit"] = round(hit / (hit + miss), 4)
            nd = max(len(g.get("TCC_HIT_sum", [0.0, ()])[1]), 1)
            r["l2_hits_per_launch"], r["l2_misses_per_launch"] = int(hit / nd), int(miss / nd)
        per = lambda c: g[c][0] / max(len(g[c][1]), 1) if c in g else None
        valu, act, thr, wcyc, gui = (per(c) for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU",
                                                      "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"))
        if valu:
            r["valu_insts_per_launch"] = int(valu)
        if act and thr:
            # active lanes per VALU instruction / 64 (both counters in the same quad-cycle units)
            r["lane_util"] = round(thr / (64.0 * act), 4)
        if gui:
            r["cycles_per_launch"] = int(gui / 8)
            if wcyc:
                # average waves resident per SIMD over the launch (SQ_WAVE_CYCLES in quad-cycles)
                r["waves_per_simd"] = round(4.0 * wcyc / (gui / 8.0) / SIMDS, 3)
        out[key] = r
    return out


def pmc_child_args(a):
    """bench.py arguments of a PMC pass: the same workload, one frame in flight, a few frames"""
    args = ["--pmc-child", "--scene", a.scene, "--width", str(a.width), "--height", str(a.height), "--spp", str(a.spp),
            "--bounces", str(a.bounces), "--tile", str(a.tile), "--pipeline", a.pipeline, "--sort-bins",
            str(a.sort_bins), "--bvh", a.bvh]
    if a.emulate_ranks > 1:
        args += ["--emulate-ranks", str(a.emulate_ranks), "--emulate-rank", str(a.emulate_rank)]
    if a.animate:
        args += ["--animate"] + (["--rebuild"] if a.rebuild else [])
    if a.move:
        args += ["--move", str(a.move), "--move-mode", a.move_mode]
    return args


def apply_move(R, scene, a):
    """--move: mesh 0 translated along x (both the current and the previous transform, so no
    motion history), then the tree refit (automatic rebuild off) or rebuilt on the device / host."""
    if not a.move:
        return
    import numpy as np
    d = scene.desc()
    mats = np.stack([np.frombuffer(bytes(d.meshes[k].transform), np.float32).reshape(4, 3).copy()
                     for k in range(d.mesh_count)])
    mats[0, 3, 0] += a.move
    R.set_instance_transforms(mats)
    R.set_instance_transforms(mats)
    if a.move_mode == "refit":
        R.set_tuning(**dict(R.tuning(), refit_rebuild_pct=-1))
        R.refit()
    else:
        R.rebuild(device=a.move_mode == "device")
    R.wait()


def run_pmc(a):
    """The rocprofv3 --pmc passes of PMC_PASSES, each its own process (rocprofv3 -- python3 bench.py
    --pmc-child ...: the same workload, kernels alone), started before this process touches the GPU.
    Returns (read_pmc result, {counter: csv path}, error or None)."""
    import glob
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, {}, "rocprofv3 not found"
    base = a.pmc_dir or tempfile.mkdtemp(prefix="rt_pmc_", dir="/tmp")
    csvs = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for counters in PMC_PASSES:
        d = os.path.join(base, counters[0])
        os.makedirs(d, exist_ok=True)
        cmd = [prof, "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), *pmc_child_args(a)]
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=a.pmc_timeout,
                               start_new_session=True)
        except subprocess.TimeoutExpired:
            return None, csvs, f"pmc pass {counters[0]} timed out"
        found = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
        if r.returncode != 0 or not found:
            return None, csvs, f"pmc pass {counters[0]} failed (rc {r.returncode}): {r.stderr[-300:]}"
        csvs[counters[0]] = found[-1]
    return read_pmc(list(csvs.values())), csvs, None


def _env_tuning(rt):
    """The sweep tools' RT_* variables (tools/sweep.sh case files) as explicit rt_tuning fields and
    Renderer options: the library reads no environment (rt_set_tuning), the harness does."""
    tu = rt.tuning_from_env()
    tu.pop("frames_in_flight", None)   # --frames-in-flight sets that
    return tu


def pmc_child(a):
    """--pmc-child: the workload with one frame in flight (kernels alone), warm-up frame + 3 frames;
    prints nothing.  Runs under rocprofv3 --pmc (run_pmc)."""
    rt = importlib.import_module("metal4-raytracing_amd")
    scene = rt.Scene.preset(a.scene)
    tu = _env_tuning(rt)
    tu.pop("graphs", None)
    R = rt.Renderer(scene, a.width, a.height, device=0, pipeline=a.pipeline, seed=3, sort_bins=a.sort_bins, bvh=a.bvh,
                    frames_in_flight=1, tail_paths=tu.pop("tail_paths", 0), tuning=tu)
    R.samplesPerPixel = a.spp
    R.maxBounces = a.bounces
    apply_move(R, scene, a)
    tiles = (a.tile, a.emulate_rank, a.emulate_ranks) if a.emulate_ranks > 1 else None
    for _ in range(4):
        R.draw(tiles=tiles)
    R.wait()
    R.close()


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--scene", default="c3g")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=4)
    p.add_argument("--bounces", type=int, default=8)
    p.add_argument("--tile", type=int, default=64)
    p.add_argument("--pipeline", default="wavefront", choices=["wavefront", "megakernel"])
    p.add_argument("--sort-bins", type=int, default=0, help="hit-sort bins (0 = library default, -1 = no sort)")
    p.add_argument("--bvh", default="sah", choices=["sah", "lbvh"], help="host binned-SAH or on-device LBVH build")
    p.add_argument("--frames-in-flight", type=int, default=0,
                   help="frames the renderer overlaps (0 = library default: one per hardware queue: 8 with the queues set here (4 with --animate or RT_HW_QUEUES=4), within a 96 GB budget; 1 = one at a time)")
    p.add_argument("--animate", action="store_true",
                   help="configs[4] shape: skin every skinned mesh at t = frame/60 s and refit the BVH before each frame")
    p.add_argument("--rebuild", action="store_true", help="with --animate: rebuild the BVH on the device instead of refitting")
    p.add_argument("--move", type=float, default=0.0,
                   help="instance motion (Renderer.swift:937-973): translate mesh 0 (the hero) by this many units along x "
                        "before the run, then update the tree by --move-mode")
    p.add_argument("--move-mode", default="refit", choices=["refit", "device", "host"],
                   help="with --move: refit the flattened tree (the automatic rebuild off), rebuild on the device, or on the host")
    p.add_argument("--emulate-ranks", type=int, default=0,
                   help="tuning aid: one process renders rank 0's tiles of an N-way split (no gather)")
    p.add_argument("--emulate-rank", type=int, default=0, help="with --emulate-ranks: which rank's tiles")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-isolated", action="store_true", help="skip the one-frame-in-flight traversal measurement")
    p.add_argument("--isolated-frames", type=int, default=6)
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the rocprofv3 --pmc passes (HBM bytes and L2 hit rates per kernel); roofline.frac then falls back to algorithmic bytes")
    p.add_argument("--pmc-dir", default=None, help="keep the PMC pass outputs here (default: a /tmp directory)")
    p.add_argument("--pmc-timeout", type=float, default=150.0)
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--gather-backend", default="nccl", choices=["nccl", "gloo"],
                   help="multi-GPU tile gather: nccl (RCCL over xGMI, device buffers) or gloo (the packed tiles staged "
                        "through host memory; ranks may share a GPU, which RCCL refuses)")
    p.add_argument("--dump-radiance", default=None,
                   help="rank 0 writes the newest frame's radiance (H, W, 4) float32 here (.npy) after the timed region")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher / collective test on the CPU: gloo instead of RCCL, a stub frame instead of the renderer")
    return p.parse_args(argv)


# ---- launcher -----------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n, argv):
    """Starts n ranks of this script (one process per GPU) and waits for them; returns the exit
    status (the first failing rank's, after stopping the others).  Touches no GPU itself."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    status = 0
    try:
        while procs:
            for p in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 1
                    for q in procs:   # a failed rank leaves the collectives hanging: stop the others
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
            p.wait()
    return status


# ---- one rank -----------------------------------------------------------------------------------
class StubFrames:
    """--dry-run: a constant 'frame' per rank with fixed ray counts, so the launcher, barriers,
    max-over-ranks timing and the tile gather run without a GPU."""

    RAYS = 1000

    def __init__(self, a, rank, n):
        from importlib import import_module
        tiles = import_module("metal4-raytracing_amd.tiles")
        self.gather = tiles.TileGather(a.width, a.height, a.tile, rank, n, "cpu") if n > 1 else None
        self.img = np.full((a.height, a.width, 4), float(rank + 1), np.float32)
        self.frames = 0

    def submit(self):
        self.frames += 1
        if self.gather is not None:
            out = self.gather.gather(self.img)
            if out is not None:   # rank 0: every rank's tiles arrived
                assert np.all(out[..., 0] >= 1.0)

    def totals(self):
        return dict(frames=self.frames, closest=self.frames * self.RAYS, shadow=self.frames * self.RAYS // 2)


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    world_env = int(os.environ.get("WORLD_SIZE") or 0)
    if a.pmc_child:
        return pmc_child(a)
    if a.gpus > 1 and world_env == 0:
        sys.exit(launch(a.gpus, argv))
    # PMC passes (one GPU, before this process touches the GPU): HBM bytes and L2 hit rates per
    # kernel, measured on the same workload with the kernels alone
    pmc, pmc_csvs, pmc_err = None, {}, None
    if not a.no_pmc and not a.dry_run and max(world_env, 1) == 1 and a.pipeline == "wavefront":
        pmc, pmc_csvs, pmc_err = run_pmc(a)
    import torch
    import torch.distributed as dist

    world = max(world_env, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = world
    gloo = a.dry_run or a.gather_backend == "gloo"
    if not a.dry_run:
        # gloo ranks may outnumber the GPUs (a one-GPU box): rank r renders on GPU r mod count
        ndev = torch.cuda.device_count()
        local = local % max(ndev, 1) if gloo else local
    if world > 1:
        if gloo:
            if not a.dry_run:
                torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world

    def barrier():
        if n > 1:
            dist.barrier()
        if not a.dry_run:
            torch.cuda.synchronize()

    if a.dry_run:
        stub = StubFrames(a, rank, n)
        for _ in range(a.warmup):
            stub.submit()
        barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            stub.submit()
        barrier()
        dt = time.perf_counter() - t0
        tot = torch.tensor([dt, float(a.steps * (StubFrames.RAYS + StubFrames.RAYS // 2))], dtype=torch.float64)
        per_rank = None
        if n > 1:
            allt = [torch.zeros_like(tot) for _ in range(n)]
            dist.all_gather(allt, tot)
            per_rank = [{"rank": r, "ms_per_step": round(float(x[0]) / max(a.steps, 1) * 1e3, 3),
                         "rays_per_frame": int(float(x[1]) / max(a.steps, 1))} for r, x in enumerate(allt)]
            mx, sm = tot.clone(), tot.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(sm, op=dist.ReduceOp.SUM)
            dt, rays = float(mx[0]), float(sm[1])
        else:
            dt, rays = float(tot[0]), float(tot[1])
        if rank == 0:
            print(json.dumps({"metric": "dry-run (stub frames, gloo)", "value": rays / dt / 1e9, "unit": "Grays/s",
                              "n_gpus": n, "world_size": n, "steps": a.steps, "warmup": a.warmup,
                              "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
                              "vs_baseline": None, "dtype": "f32", "data": "stub",
                              "config": {"workload": "dry-run", "per_rank": per_rank}}),
                  flush=True)
        if n > 1:
            dist.destroy_process_group()
        return

    rt = importlib.import_module("metal4-raytracing_amd")
    scene = rt.Scene.preset(a.scene)
    t0 = time.time()
    tu = _env_tuning(rt)
    graphs_env = tu.pop("graphs", None)
    R = rt.Renderer(scene, a.width, a.height, device=local, pipeline=a.pipeline, seed=3, sort_bins=a.sort_bins,
                    bvh=a.bvh, frames_in_flight=a.frames_in_flight, tail_paths=tu.pop("tail_paths", 0), tuning=tu)
    setup_s = time.time() - t0
    if graphs_env is not None:
        R.set_graphs(bool(graphs_env))
    if a.frames_in_flight == 1:
        # one frame at a time is the kernel-alone measurement: enqueue launch by launch, so every
        # stage's HIP events are recorded (graph replays carry none under torch's HIP runtime)
        R.set_graphs(False)
    R.samplesPerPixel = a.spp
    R.maxBounces = a.bounces
    apply_move(R, scene, a)
    tiles = (a.tile, rank, n) if n > 1 else None
    if a.emulate_ranks > 1 and n == 1:
        tiles = (a.tile, a.emulate_rank, a.emulate_ranks)
    T = a.tile
    dev = torch.device("cuda", local)
    gather = None
    if n > 1:
        tiles_mod = importlib.import_module("metal4-raytracing_amd.tiles")
        gather = tiles_mod.TileGather(a.width, a.height, T, rank, n, "cpu" if gloo else dev, renderer=R)

    skinned = []
    if a.animate:
        d = scene.desc()
        skinned = [m for m in range(d.mesh_count) if d.meshes[m].joint_count > 0]
    tick = [0]

    def animate():
        # SkinningPass tick (Renderer.swift:1280-1326): joint matrices at t, skin, refit
        if not skinned:
            return
        t = tick[0] / 60.0
        tick[0] += 1
        for m in skinned:
            R.skin(m, scene.joint_matrices(m, t))
        R.rebuild(device=True) if a.rebuild else R.refit()

    gather_events = []

    def submit(timed=False):
        # one step: the frame is submitted and, multi-GPU, its tiles packed, gathered to rank 0
        # over RCCL and unpacked there, all enqueued without a host wait (the renderer keeps
        # frames in flight and waits for a slot's previous frame itself).  Timed steps bracket
        # the collective (after the pack, through the unpack) with events on torch's stream.
        animate()
        R.draw(tiles=tiles)
        if gather is not None:
            ev = None
            if timed:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            gather.gather(events=ev)
            if ev is not None:
                gather_events.append(ev)

    # counting frame (untimed): node visits / triangle tests per ray for the roofline numerator
    R.set_counting(True)
    R.frameIndex = 0
    R.draw(tiles=tiles)
    R.wait()
    cst = R.stats()
    R.set_counting(False)
    R.samplesPerPixel = a.spp  # resets frameIndex (didSet)

    for _ in range(a.warmup):
        submit()
    R.wait()
    s0 = R.stats()
    barrier()
    t0 = time.perf_counter()
    t_host = 0.0
    for _ in range(a.steps):
        th = time.perf_counter()
        submit(timed=True)
        t_host += time.perf_counter() - th
    R.wait()
    barrier()
    dt = time.perf_counter() - t0
    # the running totals of every frame of the timed region (HIP events per stage on the
    # renderer's streams, ray counters read back per frame)
    s1 = R.stats()
    assert s1.frames_total - s0.frames_total == a.steps
    gather_ms = sum(e0.elapsed_time(e1) for e0, e1 in gather_events) / a.steps if gather_events else 0.0
    d = lambda f: getattr(s1, f) - getattr(s0, f)
    closest = d("total_closest_rays")
    rays = closest + d("total_shadow_rays")
    kms_local = d("total_frame_ms") / a.steps

    tot = torch.tensor([dt, float(rays), float(closest), kms_local, gather_ms], dtype=torch.float64,
                       device="cpu" if gloo else dev)
    per_rank = None
    if n > 1:
        # every rank's own figures (load balance of the tile split)
        allt = [torch.zeros_like(tot) for _ in range(n)]
        dist.all_gather(allt, tot)
        per_rank = [{"rank": r, "ms_per_step": round(float(x[0]) / a.steps * 1e3, 3),
                     "rays_per_frame": int(float(x[1]) / a.steps), "kernel_ms_per_frame": round(float(x[3]), 3),
                     "gather_ms_per_step": round(float(x[4]), 4)} for r, x in enumerate(t.cpu() for t in allt)]
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        dt, rays_all, kms, gather_ms = float(mx[0]), float(sm[1]), float(mx[3]), float(mx[4])
    else:
        rays_all, kms = float(rays), kms_local
    if rank != 0:
        dist.destroy_process_group()
        return
    if a.dump_radiance:
        np.save(a.dump_radiance, R.radiance())

    value = rays_all / dt / 1e9
    ms_per_step = dt / a.steps * 1e3
    try:
        cus = torch.cuda.get_device_properties(local).multi_processor_count
    except Exception:
        cus = 256
    ranks = n if n > 1 else max(a.emulate_ranks, 1)
    pixels = a.width * a.height / ranks
    table = kernel_table(a, cst, s0, s1, a.steps, pixels, cus)
    if s1.frames_in_flight > 1 and not a.no_isolated:
        # after the timed region: the same frame with one frame in flight, so every kernel has the
        # GPU to itself; the roofline prices these launches, and their wall time per frame is the
        # single-frame latency
        i0, i1, ms_frame, cst_alone = isolated(R, tiles, torch, dev, a.isolated_frames)
        alone, shared = kernel_table(a, cst_alone, i0, i1, a.isolated_frames, pixels, cus), table
        stage_alone = (np.array(list(i1.total_kernel_ms)) - np.array(list(i0.total_kernel_ms))) / a.isolated_frames
    elif s1.frames_in_flight == 1:
        alone, shared, ms_frame, stage_alone = table, None, ms_per_step, None
    else:   # --no-isolated: the shared-GPU launches, flagged
        alone, shared, ms_frame, stage_alone = table, None, None, None
    roof = roofline(alone, shared, pmc, pmc_err, ms_frame, ms_per_step, pmc_csvs)
    if roof.get("shade_l2_hit") is not None:
        roof["shade_l2_hit_kernel"] = ("wf_shade on hit-sorted input (--sort-bins)" if a.sort_bins > 0 else
                                       "wf_shade of the default pipeline: hits shaded in queue order (rays grouped by "
                                       "octant inside each block's appends only; no queue-wide ray or hit sort, DESIGN.md §3.5)")
    if alone is table and s1.frames_in_flight > 1:
        roof["not_a_kernel_measurement"] = True
    stage_ms = (np.array(list(s1.total_kernel_ms)) - np.array(list(s0.total_kernel_ms))) / a.steps
    graphs = {k: int(d("total_graph_" + k)) for k in ("replays", "captures", "fallbacks", "eager")}

    cpu = None
    if not a.no_cpu and n == 1:
        cpu = cpu_baseline(rt, scene, R, a)

    line = {
        "metric": "Grays/sec (closest-hit + shadow rays traced) at 1920x1080x4spp, dragon; ms/frame",
        "value": round(value, 4),
        "unit": "Grays/s",
        "n_gpus": n,
        # the communicator's own count (a multi-rank line proves the collective saw every rank)
        "world_size": dist.get_world_size() if n > 1 else 1,
        "dist_backend": dist.get_backend() if n > 1 else None,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        # single-frame latency: one frame in flight, wall time per frame (the metric's ms/frame);
        # ms_per_step is the throughput interval with frames in flight
        "ms_per_frame": round(ms_frame, 3) if ms_frame else None,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: procedural 871,414-triangle dragon stand-in (dragon.obj absent from the reference "
                "snapshot), real plane/sphere OBJ assets, seeded random offsets" if scene.synthetic else
                "reference OBJ assets, seeded random offsets",
        "config": {
            "workload": f"{a.scene}: {SCENES.get(a.scene, a.scene + ' scene')} {a.width}x{a.height}x{a.spp}spp, {a.bounces} bounces, "
                        f"one frame per step, {'tile-split ' + str(T) + 'px + ' + ('gloo (host-staged)' if gloo else 'RCCL') + ' gather' if n > 1 else 'single GPU'}"
                        f", frames submitted back to back (overlapping frames in flight)",
            "scene": a.scene, "triangles": scene.triangle_count, "width": a.width, "height": a.height,
            "spp": a.spp, "max_bounces": a.bounces, "pipeline": a.pipeline, "parallelism": f"tiles{n}",
            "rays_per_frame": int(rays_all / a.steps), "kernel_ms_per_frame": round(kms, 3),
            "setup_s": round(setup_s, 2),
            # [generate, extend, shade, connect, resolve, finish, hit sort]
            "stage_ms": [round(x, 3) for x in stage_ms], "sort_bins": a.sort_bins, "bvh": a.bvh,
            "stage_ms_alone": [round(x, 3) for x in stage_alone] if stage_alone is not None else None,
            "pipeline_used": ["megakernel", "wavefront"][s1.pipeline], "iterations": s1.iterations,
            "frames_in_flight": s1.frames_in_flight, "animate": bool(skinned),
            # host time inside the submit calls per step (includes waiting for a free frame slot)
            "host_submit_ms": round(t_host / a.steps * 1e3, 3),
            # how the timed frames were submitted (rt_stats total_graph_*): replays of the slots'
            # captured HIP graphs, fresh captures, refused captures (eager), eager by choice
            # the counting frame's BVH work per traced ray (closest-hit + shadow)
            "visits_per_ray": {"nodes": round(cst.node_visits / max(cst.closest_rays + cst.shadow_rays, 1), 3),
                               "tris": round(cst.tri_tests / max(cst.closest_rays + cst.shadow_rays, 1), 3)},
            "graphs": graphs,
            "move": {"dx": a.move, "mode": a.move_mode, "auto_rebuilds": int(s1.total_auto_rebuilds),
                     "bvh_cost_built": round(float(s1.bvh_cost_built), 2),
                     "bvh_cost_refit": round(float(s1.bvh_cost_refit), 2)} if a.move else None,
            # multi-GPU: device time per step from the end of the pack through the unpack on rank 0's
            # side of the RCCL gather (max over ranks), and its share of the step
            "gather_ms_per_step": round(gather_ms, 4) if n > 1 else None,
            "gather_share": round(gather_ms / ms_per_step, 4) if n > 1 else None,
            # multi-rank: each rank's wall ms per step (to its own end of the timed region), rays
            # and summed kernel ms per frame (ranks sharing one GPU share its CUs)
            "per_rank": per_rank,
        },
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if n > 1:
        dist.destroy_process_group()


def kernel_table(a, cst, s0, s1, frames, pixels, cus):
    """Per kernel group (KERNELS) over the frames between stats s0 and s1: launches per frame, the
    average launch time (HIP events around each launch on its render stream), device time per
    frame, and algorithmic bytes per launch.  Node / triangle counts per ray come
    from the untimed counting frame `cst`: wf_trace counts its own visits, the finish kernel's are
    the rest."""
    d = lambda f: getattr(s1, f) - getattr(s0, f)
    stage_ms = np.array(list(s1.total_kernel_ms)) - np.array(list(s0.total_kernel_ms))
    if s1.pipeline != 1:   # megakernel: the whole frame is one launch; every node comes from memory
        rays_c = cst.closest_rays + cst.shadow_rays
        rays = (d("total_closest_rays") + d("total_shadow_rays")) / frames
        npr, tpr = cst.node_visits / max(rays_c, 1), cst.tri_tests / max(rays_c, 1)
        b = rays * (B_RAY + npr * B_NODE + tpr * B_TRI) + d("total_closest_rays") / frames * B_HIT + pixels * 56
        ms = d("total_frame_ms") / frames
        return [dict(key="megakernel", kernel="rt::megakernel<false, false>", launches=1.0, launch_ms=ms,
                     ms_per_frame=ms, bytes_per_launch=b, nodes_per_ray=npr, tris_per_ray=tpr)]
    rays_c = cst.closest_rays + cst.shadow_rays
    q_nodes = cst.trace_nodes / max(cst.trace_rays, 1)
    q_tris = cst.trace_tris / max(cst.trace_rays, 1)
    f_rays_c = rays_c - cst.trace_rays
    f_nodes = (cst.node_visits - cst.trace_nodes) / max(f_rays_c, 1)
    f_tris = (cst.tri_tests - cst.trace_tris) / max(f_rays_c, 1)
    trace_rays, trace_launches = d("total_trace_rays"), d("total_trace_launches")
    trace_closest, finish_launches = d("total_trace_closest_rays"), d("total_finish_launches")
    closest, rays = d("total_closest_rays"), d("total_closest_rays") + d("total_shadow_rays")
    paths = d("total_paths") / frames
    out = []
    for key, name, stages, _ in KERNELS:
        ms = float(sum(stage_ms[i] for i in stages))
        if key == "trace":
            n = trace_launches
            rpl = trace_rays / max(n, 1)
            b = rpl * (B_QRAY + q_nodes * B_NODE + q_tris * B_TRI)
            extra = dict(rays_per_launch=rpl, nodes_per_ray=q_nodes, tris_per_ray=q_tris)
        elif key == "finish":
            n = finish_launches
            f_rays = (rays - trace_rays) / max(n, 1)
            f_closest = (closest - trace_closest) / max(n, 1)
            b = f_rays * (B_RAY + f_nodes * B_NODE + f_tris * B_TRI) + f_closest * B_HIT
            extra = dict(rays_per_launch=f_rays, nodes_per_ray=f_nodes, tris_per_ray=f_tris)
        elif key == "shade":
            n = trace_launches / 2   # one per bulk round (extend + connect are the round's wf_trace pair)
            b = trace_closest / max(n, 1) * B_SHADE_HIT
            extra = dict(hits_per_launch=trace_closest / max(n, 1))
        elif key == "generate":
            n = frames
            b = paths * B_GEN_PATH + pixels * B_GEN_PIXEL
            extra = {}
        else:   # resolve (+ motion vectors): two launches a frame
            n = 2 * frames
            b = pixels * (16 * a.spp + B_RESOLVE_PIXEL) / 2
            extra = {}
        if n <= 0:
            continue
        out.append(dict(key=key, kernel=name, launches=n / frames, launch_ms=ms / n, ms_per_frame=ms / frames,
                        bytes_per_launch=b, **extra))
    return out


def valu_fields(p, launch_ms):
    """The VALU-issue bound of a kernel (the bound the traversal kernels sit at):
    VALU wave-instructions per launch, lane utilisation, average waves per SIMD and
    frac_valu_issue = VALU instructions x 2 cycles / (1,024 SIMDs x the launch's cycles), the share of
    the chip's VALU issue slots the launch used.  The launch's cycles come from GRBM_GUI_ACTIVE of
    the PMC pass (the clock it ran at); without it, from the bench's launch time at 2.4 GHz."""
    v = p.get("valu_insts_per_launch")
    if not v:
        return {}
    cyc = p.get("cycles_per_launch") or launch_ms * 1e-3 * NOMINAL_CLOCK_HZ
    out = {"valu_insts": v, "lane_util": p.get("lane_util"), "waves_per_simd": p.get("waves_per_simd"),
           "frac_valu_issue": round(v * VALU_ISSUE_CYCLES / (SIMDS * cyc), 4)}
    if p.get("cycles_per_launch"):
        out["clock_GHz"] = round(p["cycles_per_launch"] / (launch_ms * 1e-3) / 1e9, 3)
    return out


def roofline(alone, shared, pmc, pmc_err, ms_frame_alone, ms_per_step, pmc_csvs):
    """The bench line's roofline: the dominant kernel is the one with the most device
    time per frame with the kernels alone (one frame in flight); `frac` = its HBM bytes per launch
    (rocprofv3 PMC, FETCH_SIZE x 2 + WRITE_SIZE, same workload, kernels alone) over its average
    launch time alone, against 8 TB/s.  The algorithmic-byte fraction and the L2-gather figure are
    secondary fields; the shared-GPU figures of the timed region (frames in flight) are under
    `in_flight`."""
    if not any(k["ms_per_frame"] > 0 for k in alone):
        # --no-isolated over graph replays: no launch of the run was timed on its own
        return {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": None, "achieved": None, "frac": None,
                "traffic": None, "ms_per_step": round(ms_per_step, 4),
                "note": "no per-kernel times: the timed frames were graph replays (DESIGN.md §3.4) and --no-isolated "
                        "skipped the kernels-alone frames"}
    dom = max(alone, key=lambda k: k["ms_per_frame"])
    pmc = pmc or {}
    kernels = []
    for k in alone:
        p = pmc.get(k["key"], {})
        t = p.get("bytes_per_launch")
        alg = k["bytes_per_launch"] / (k["launch_ms"] * 1e-3) / 1e9
        hbm = t / (k["launch_ms"] * 1e-3) / 1e9 if t else None
        kernels.append({
            "kernel": k["kernel"], "ms_per_frame": round(k["ms_per_frame"], 4), "launches": round(k["launches"], 2),
            "launch_ms": round(k["launch_ms"], 4), "traffic": t, "hbm_GBs": round(hbm, 1) if hbm else None,
            "frac": round(hbm / HBM_PEAK_GBS, 4) if hbm else None, "l2_hit": p.get("l2_hit"),
            "algorithmic_bytes_per_launch": int(k["bytes_per_launch"]), "achieved_algorithmic_GBs": round(alg, 1),
            "frac_algorithmic": round(alg / HBM_PEAK_GBS, 4),
            "frac_of_line_ceiling": round((p["l2_hits_per_launch"] / L2_HIT_LINES_PER_S +
                                           p["l2_misses_per_launch"] / L2_MISS_LINES_PER_S) / (k["launch_ms"] * 1e-3), 4)
            if "l2_hits_per_launch" in p else None,
            **{x: round(k[x], 3) for x in ("nodes_per_ray", "tris_per_ray") if x in k},
            **valu_fields(p, k["launch_ms"])})
    d = next(k for k in kernels if k["kernel"] == dom["kernel"])
    r = {
        "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": dom["kernel"],
        # HBM bytes from the PMC pass only: without one, achieved / frac stay null and the
        # algorithmic-byte figures below are the only rate (they count L2 / MALL hits as well, so
        # they are not an HBM fraction and can exceed 1)
        "achieved": d["hbm_GBs"],
        "frac": d["frac"],
        "frac_source": "pmc: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch, kernels alone, over the launch time alone"
        if d["frac"] is not None else "none: no PMC pass (" + (pmc_err or "--no-pmc") + "); see frac_algorithmic",
        "traffic": d["traffic"], "launch_ms": d["launch_ms"], "ms_per_frame_alone": d["ms_per_frame"],
        "frame_ms_alone": round(ms_frame_alone, 4) if ms_frame_alone else None,
        "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"],
        "achieved_algorithmic": d["achieved_algorithmic_GBs"], "frac_algorithmic": d["frac_algorithmic"],
        "frac_of_l2_gather_peak": round(d["achieved_algorithmic_GBs"] / L2_GATHER_PEAK_GBS, 4),
        "frac_of_line_ceiling": d["frac_of_line_ceiling"],
        "l2_hit": {k["kernel"]: k["l2_hit"] for k in kernels if k["l2_hit"] is not None} or None,
        # the bound the traversal kernels actually sit at: VALU issue (fraction of the chip's VALU
        # issue slots per kernel, with its lane utilisation), beside the HBM fraction above
        "valu_issue": {k["kernel"]: {x: k.get(x) for x in ("frac_valu_issue", "lane_util", "valu_insts", "waves_per_simd")}
                       for k in kernels if k.get("valu_insts")} or None,
        # north star: the L2 hit rate of the shade kernel (it shades the hits of the rays as the
        # extend launch traced them), measured in this run
        "shade_l2_hit": next((k["l2_hit"] for k in kernels if k["kernel"].startswith("rt::wf_shade")), None),
        # which shade kernel that is: the default pipeline shades hits in queue order (no ray or hit
        # sort; the sorts were measured slower)
        "shade_l2_hit_kernel": None,   # set by main(): which shade kernel that is
        "pmc_files": {c: os.path.relpath(p, ROOT) if p.startswith(ROOT) else p for c, p in pmc_csvs.items()} or None,
        "kernels": kernels,
    }
    if shared is not None and sum(k["ms_per_frame"] for k in shared) == 0:
        r["in_flight"] = {"ms_per_step": round(ms_per_step, 4),
                          "note": "the timed frames were graph replays, which record no per-stage times under this HIP "
                                  "runtime (DESIGN.md §3.4)"}
    elif shared is not None:
        r["in_flight"] = {
            "note": "frames in flight share the GPU: a launch's time includes the time its workgroups wait for CUs "
                    "other frames' kernels hold, so these are not kernel measurements",
            "ms_per_step": round(ms_per_step, 4),
            "kernels": [{"kernel": k["kernel"], "ms_per_frame": round(k["ms_per_frame"], 4),
                         "launch_ms": round(k["launch_ms"], 4)} for k in shared]}
    return r


def isolated(R, tiles, torch, dev, frames):
    """The bench frame with one frame in flight, after the timed region: the renderer on a caller's
    stream keeps one slot (rt_set_stream), so every launch has the GPU to itself.  Returns the stats
    before / after, the wall time per frame (single-frame latency) and the stats of a counting frame
    of the same configuration (one slot: the single-frame finish threshold, so its launches trace
    other rays than the timed region's)."""
    s = torch.cuda.Stream(device=dev)
    R.set_stream(s.cuda_stream)
    R.set_graphs(False)   # enqueued launch by launch: every stage's HIP events are recorded
    try:
        R.set_counting(True)   # warms the single slot and counts its node / triangle visits
        R.draw(tiles=tiles)
        R.wait()
        cst = R.stats()
        R.set_counting(False)
        R.draw(tiles=tiles)
        R.wait()
        i0 = R.stats()
        t0 = time.perf_counter()
        for _ in range(frames):
            R.draw(tiles=tiles)
            R.wait()
        wall = (time.perf_counter() - t0) / frames
        i1 = R.stats()
    finally:
        R.set_graphs(True)
        R.set_stream(None)
    return i0, i1, wall * 1e3, cst


def host_cpu():
    """nproc, the CPUs this process may use, the cgroup's CPU quota and the CPU model."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpus"] = None
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["model"] = model
    return info


def cpu_baseline(rt, scene, R, a):
    """The C oracle (oracle/, a port: binned-SAH BVH2, nearer child first) built -O3 -march=native
    on this host, on a bounded row subset of the same frame, on the host CPUs this process may use
    (at most 16: the CPU share of one GPU on the GPU boxes, whose nproc is the whole machine)."""
    import oracle
    native = oracle.build_native()
    if native:
        oracle.use_library(native)
    threads = oracle.default_threads()
    osc = oracle.OracleScene(scene.desc())
    u = R.uniforms()
    u.frameIndex = 0
    probe_step = 64
    t0 = time.perf_counter()
    o = osc.render(u, R.random, row_start=0, row_step=probe_step, threads=threads)
    t_probe = time.perf_counter() - t0
    step = max(1, int(probe_step * t_probe / max(a.cpu_seconds, 0.1)))
    step = min(step, probe_step)
    # a whole frame shorter than the target: repeat it so the sample still spans ~cpu_seconds
    reps = 1 if step > 1 else max(1, int(round(a.cpu_seconds / max(t_probe * probe_step, 1e-3))))
    rays, t = 0, 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        o = osc.render(u, R.random, row_start=0, row_step=step, threads=threads)
        t += time.perf_counter() - t0
        rays += o["closest_rays"] + o["shadow_rays"]
    hc = host_cpu()
    return {"value": round(rays / t / 1e9, 6), "unit": "Grays/s", "cores": threads, "kind": "port",
            "build": "gcc -O3 -march=native -ffp-contract=off" if native else "gcc -O3 -ffp-contract=off (portable)",
            "host": hc,
            "sample": f"every {step}th row of frame 0 ({(a.height + step - 1) // step} rows x {a.width} px x "
                      f"{a.spp} spp) x {reps}, {rays} rays in {t:.1f} s on {threads} threads"}


if __name__ == "__main__":
    main()
