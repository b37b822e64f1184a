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
# count: RT_HW_QUEUES if set, else the caller's GPU_MAX_HW_QUEUES, else four (HIP's default, also
# what the GPU boxes export).  Small frames (a multi-GPU rank's share) keep as many frames in
# flight as there are queues, up to eight (rt_api.cpp small_frame_slots); with the final round-2
# kernels four queues / four slots measured 4.21 / 4.24 Grays/s per rank against eight / eight
# 4.11 / 4.10.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES") or os.environ.get("GPU_MAX_HW_QUEUES") or "4"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
# MI355X_MICROARCH.md 'Indexed rows': rows gathered from a table every workgroup shares, served by
# the XCD's L2, 16.8-18.8 TB/s chip-wide (the lower figure).  The traversal's node / triangle
# working set (48 MB for C3g) lives in L2 and the Infinity Cache (L2 hit 0.63), so its algorithmic
# rate is also priced against this cache-gather ceiling.
L2_GATHER_PEAK_GBS = 16800.0
SCENES = {"c3g": "glass dragon scene (configs[2])", "c3": "glass dragon scene (configs[2])",
          "c3d": "opaque dragon scene", "c1": "AppScene base (configs[0])", "c2": "bunny scene (configs[1])",
          "c5": "skinned robot scene (configs[4])",
          "c3r": "irregular-geometry check: the reference's coatball / teapot meshes, glass, in the dragon's place"}   # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic bytes (DESIGN.md §6 'Roofline'): per traced ray its 48-B queue entry (extend: 32 B ray
# in + 16 B hit out; connect: 48 B shadow entry in); per 8-wide node fetched from memory 80 B; per
# triangle tested 48 B; per closest hit shaded inside the finish kernel 16 B triangle record +
# 3 x 16 B normals + 48 B instance transform.  Node tests served from an LDS copy of the BVH's top
# levels (a build with RT_TOP_NODES > 0; the rt_stats *_lds counters) move no memory per visit:
# they are charged once per block (the staging read, B_NODE x kTopNodes per block).
B_RAY = 48
B_NODE = 80  # compressed 8-wide node (Bvh8Node)
B_TRI = 48
B_HIT = 16 + 48 + 48
B_PIXEL = 4 + 16 + 16 + 4 + 16
B_QRAY = 48
TOP_NODES = 32          # rt_device.h kTopNodes
TRACE_BLOCKS_PER_CU = 8   # wf_trace: 256-thread blocks at 8 waves / SIMD
FINISH_BLOCKS_PER_CU = 4  # wf_finish_step: 4 waves / SIMD
# PMC traffic of the newest round (profiles/rNN_traffic.json, tools/gpurun_profile.sh)
_TRAFFIC = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if re.fullmatch(r"r\d+_traffic\.json", f)) \
    if os.path.isdir(os.path.join(ROOT, "profiles")) else []
TRAFFIC_JSON_REL = "profiles/" + (_TRAFFIC[-1] if _TRAFFIC else "r01_traffic.json")
TRAFFIC_JSON = os.path.join(ROOT, TRAFFIC_JSON_REL)


def _newest_profile(pattern):
    d = os.path.join(ROOT, "profiles")
    names = sorted(f for f in os.listdir(d) if re.fullmatch(pattern, f)) if os.path.isdir(d) else []
    return os.path.join(d, names[-1]) if names else None


def sorted_l2_hit():
    """L2 hit rates of the opt-in sorted runs (north star: the sorted-ray shade kernel's L2 hit rate):
    the hit-sorted shade (--sort-bins 2048, tools/gpurun_sorted_l2.sh) and the wf_shade ray grouping
    modes (RT_RAY_SORT, tools/gpurun_raysort.sh), from the newest profiles/rNN_l2_*.json."""
    out = {}
    p = _newest_profile(r"r\d+_l2_sorted\.json")
    if p:
        hits = json.load(open(p)).get("l2_hit") or {}
        out["hit_sorted"] = {k: v for k, v in hits.items() if re.search(r"wf_(trace|shade|finish)", k)}
        out["hit_sorted_source"] = "profiles/" + os.path.basename(p)
    p = _newest_profile(r"r\d+_l2_raysort\.json")
    if p:
        rs = json.load(open(p))
        for m in ("ray_sort_0", "ray_sort_1", "ray_sort_2"):
            if m in rs:
                out[m] = {k: v for k, v in rs[m].items() if re.search(r"wf_(trace|shade)", k)}
        out["ray_sort_source"] = "profiles/" + os.path.basename(p)
    return out or None


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
                   help="frames the renderer overlaps (0 = library default: one per hardware queue, 4 with the queues set here, 8 with RT_HW_QUEUES=8, within a 96 GB budget; 1 = one at a time)")
    p.add_argument("--animate", action="store_true",
                   help="configs[4] shape: skin every skinned mesh at t = frame/60 s and refit the BVH before each frame")
    p.add_argument("--rebuild", action="store_true", help="with --animate: rebuild the BVH on the device instead of refitting")
    p.add_argument("--emulate-ranks", type=int, default=0,
                   help="tuning aid: one process renders rank 0's tiles of an N-way split (no gather)")
    p.add_argument("--emulate-rank", type=int, default=0, help="with --emulate-ranks: which rank's tiles")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-isolated", action="store_true", help="skip the one-frame-in-flight traversal measurement")
    p.add_argument("--isolated-frames", type=int, default=6)
    p.add_argument("--traffic-csv", default=None, help="rocprofv3 --pmc counter_collection.csv for traffic")
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
    if a.gpus > 1 and world_env == 0:
        sys.exit(launch(a.gpus, argv))
    import torch
    import torch.distributed as dist

    world = max(world_env, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = world
    if world > 1:
        if a.dry_run:
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
        if n > 1:
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
                              "vs_baseline": None, "dtype": "f32", "data": "stub", "config": {"workload": "dry-run"}}),
                  flush=True)
        if n > 1:
            dist.destroy_process_group()
        return

    rt = importlib.import_module("metal4-raytracing_amd")
    scene = rt.Scene.preset(a.scene)
    t0 = time.time()
    R = rt.Renderer(scene, a.width, a.height, device=local, pipeline=a.pipeline, seed=3, sort_bins=a.sort_bins,
                    bvh=a.bvh, frames_in_flight=a.frames_in_flight)
    setup_s = time.time() - t0
    R.samplesPerPixel = a.spp
    R.maxBounces = a.bounces
    tiles = (a.tile, rank, n) if n > 1 else None
    if a.emulate_ranks > 1 and n == 1:
        tiles = (a.tile, a.emulate_rank, a.emulate_ranks)
    T = a.tile
    dev = torch.device("cuda", local)
    gather = None
    if n > 1:
        tiles_mod = importlib.import_module("metal4-raytracing_amd.tiles")
        gather = tiles_mod.TileGather(a.width, a.height, T, rank, n, dev, renderer=R)

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

    tot = torch.tensor([dt, float(rays), float(closest), kms_local, gather_ms], dtype=torch.float64, device=dev)
    if n > 1:
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

    value = rays_all / dt / 1e9
    ms_per_step = dt / a.steps * 1e3
    try:
        cus = torch.cuda.get_device_properties(local).multi_processor_count
    except Exception:
        cus = 256
    roof = roofline(a, cst, s0, s1, rays, closest, kms_local, ms_per_step, cus)
    if s1.pipeline == 1 and s1.frames_in_flight > 1 and not a.no_isolated:
        # after the timed region: the same frame with one frame in flight, so the dominant kernel's
        # launches have the GPU to themselves (its own roofline, beside the shared-GPU figure above)
        roof["isolated"] = isolated(R, tiles, torch, dev, a, cst, cus, roof["kernel"], a.isolated_frames)

    cpu = None
    if not a.no_cpu and n == 1:
        cpu = cpu_baseline(rt, scene, R, a)

    line = {
        "metric": "Grays/sec (closest-hit + shadow rays traced) at 1920x1080x4spp, dragon; ms/frame",
        "value": round(value, 4),
        "unit": "Grays/s",
        "n_gpus": n,
        "world_size": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: procedural 871,414-triangle dragon stand-in (dragon.obj absent from the reference "
                "snapshot), real plane/sphere OBJ assets, seeded random offsets" if scene.synthetic else
                "reference OBJ assets, seeded random offsets",
        "config": {
            "workload": f"{a.scene}: {SCENES.get(a.scene, a.scene + ' scene')} {a.width}x{a.height}x{a.spp}spp, {a.bounces} bounces, "
                        f"one frame per step, {'tile-split ' + str(T) + 'px + RCCL gather' if n > 1 else 'single GPU'}"
                        f", frames submitted back to back (overlapping frames in flight)",
            "scene": a.scene, "triangles": scene.triangle_count, "width": a.width, "height": a.height,
            "spp": a.spp, "max_bounces": a.bounces, "pipeline": a.pipeline, "parallelism": f"tiles{n}",
            "rays_per_frame": int(rays_all / a.steps), "kernel_ms_per_frame": round(kms, 3),
            "setup_s": round(setup_s, 2),
            # [generate, extend, shade, connect, resolve, finish, hit sort]
            "stage_ms": [round(x, 3) for x in roof.pop("_stage_ms")], "sort_bins": a.sort_bins, "bvh": a.bvh,
            "pipeline_used": ["megakernel", "wavefront"][s1.pipeline], "iterations": s1.iterations,
            "frames_in_flight": s1.frames_in_flight, "animate": bool(skinned),
            # host time inside the submit calls per step (includes waiting for a free frame slot)
            "host_submit_ms": round(t_host / a.steps * 1e3, 3),
            # multi-GPU: device time per step from the end of the pack through the unpack on rank 0's
            # side of the RCCL gather (max over ranks), and its share of the step
            "gather_ms_per_step": round(gather_ms, 4) if n > 1 else None,
            "gather_share": round(gather_ms / ms_per_step, 4) if n > 1 else None,
        },
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if n > 1:
        dist.destroy_process_group()


def roofline(a, cst, s0, s1, rays_local, closest_local, kms_local, ms_per_step, cus):
    """The dominant kernel's algorithmic bytes per launch over its average launch time (HIP events
    around each launch on its render stream, over the timed region), with node bytes counted for
    the nodes fetched from memory only.  The device-clock span of the same launches
    (first workgroup start to last wave end, s_memrealtime) is reported beside it
    (launch_ms_device).  With frames in flight, launches of different frames share the GPU: a
    launch's span, as rocprofv3's kernel trace records it too, is then longer than it would be
    alone, and the per-frame kernel times add up to more than the step."""
    d = lambda f: getattr(s1, f) - getattr(s0, f)
    steps = a.steps
    trace_rays, trace_launches, trace_ms = d("total_trace_rays"), d("total_trace_launches"), d("total_trace_ms")
    trace_closest, finish_launches = d("total_trace_closest_rays"), d("total_finish_launches")
    trace_dev_ms, trace_dev_launches = d("total_trace_dev_ms"), d("total_trace_dev_launches")
    finish_dev_ms, finish_dev_launches = d("total_finish_dev_ms"), d("total_finish_dev_launches")
    stage_ms = np.array(list(s1.total_kernel_ms)) - np.array(list(s0.total_kernel_ms))
    # per-ray visits of the counting frame: wf_trace's own, and the finish kernel's (the rest)
    rays_c = cst.closest_rays + cst.shadow_rays
    q_nodes = cst.trace_nodes / max(cst.trace_rays, 1)
    q_nodes_lds = cst.trace_nodes_lds / max(cst.trace_rays, 1)
    q_tris = cst.trace_tris / max(cst.trace_rays, 1)
    f_rays_c = rays_c - cst.trace_rays
    f_nodes = (cst.node_visits - cst.trace_nodes) / max(f_rays_c, 1)
    f_nodes_lds = (cst.node_visits_lds - cst.trace_nodes_lds) / max(f_rays_c, 1)
    f_tris = (cst.tri_tests - cst.trace_tris) / max(f_rays_c, 1)
    kernels = []
    if s1.pipeline == 1 and trace_launches > 0:
        rpl = trace_rays / trace_launches
        blocks = cus * TRACE_BLOCKS_PER_CU
        kernels.append(dict(
            kernel="rt::wf_trace<{false,true}, false> (extend + connect)", launches=trace_launches / steps,
            launch_ms=trace_ms / trace_launches,
            launch_ms_device=trace_dev_ms / trace_dev_launches if trace_dev_launches else None,
            rays_per_launch=rpl, nodes_per_ray=q_nodes,
            lds_nodes_per_ray=q_nodes_lds, tris_per_ray=q_tris,
            bytes_per_launch=rpl * (B_QRAY + (q_nodes - q_nodes_lds) * B_NODE + q_tris * B_TRI)
            + (blocks * TOP_NODES * B_NODE if q_nodes_lds > 0 else 0),
            bytes_all_nodes=rpl * (B_QRAY + q_nodes * B_NODE + q_tris * B_TRI)))
    if s1.pipeline == 1 and finish_launches > 0:
        # wf_finish_step: its rays (48 B ray + hit) + nodes + triangles as above, + the shading
        # gathers per closest hit (B_HIT); the path state in and out once per path is left out
        f_rays = (rays_local - trace_rays) / finish_launches
        f_closest = (closest_local - trace_closest) / finish_launches
        blocks = cus * FINISH_BLOCKS_PER_CU
        kernels.append(dict(
            kernel="rt::wf_finish_step<false, false>", launches=finish_launches / steps,
            launch_ms=float(stage_ms[5]) / finish_launches,
            launch_ms_device=finish_dev_ms / finish_dev_launches if finish_dev_launches else None,
            rays_per_launch=f_rays, nodes_per_ray=f_nodes,
            lds_nodes_per_ray=f_nodes_lds, tris_per_ray=f_tris,
            bytes_per_launch=f_rays * (B_RAY + (f_nodes - f_nodes_lds) * B_NODE + f_tris * B_TRI) + f_closest * B_HIT
            + (blocks * TOP_NODES * B_NODE if f_nodes_lds > 0 else 0),
            bytes_all_nodes=f_rays * (B_RAY + f_nodes * B_NODE + f_tris * B_TRI) + f_closest * B_HIT))
    if not kernels:
        # megakernel: the whole frame is one launch; every node comes from memory
        rpl = rays_local / steps
        npr = cst.node_visits / max(rays_c, 1)
        tpr = cst.tri_tests / max(rays_c, 1)
        b = (rpl * (B_RAY + npr * B_NODE + tpr * B_TRI) + closest_local / steps * B_HIT
             + a.width * a.height / max(1, int(os.environ.get("WORLD_SIZE", "1"))) * B_PIXEL)
        kernels.append(dict(kernel="rt::megakernel<false, false>", launches=1, launch_ms=kms_local,
                            launch_ms_device=None, rays_per_launch=rpl,
                            nodes_per_ray=npr, lds_nodes_per_ray=0.0, tris_per_ray=tpr, bytes_per_launch=b,
                            bytes_all_nodes=b))
    for k in kernels:
        k["achieved"] = k["bytes_per_launch"] / (k["launch_ms"] * 1e-3) / 1e9
        k["achieved_all_nodes"] = k["bytes_all_nodes"] / (k["launch_ms"] * 1e-3) / 1e9
        k["ms_per_frame"] = k["launch_ms"] * k["launches"]
    dom = max(kernels, key=lambda k: k["ms_per_frame"])
    # the whole frame: every timed kernel's algorithmic bytes over the wall time per frame
    job_bytes = sum(k["bytes_per_launch"] * k["launches"] for k in kernels)
    job_achieved = job_bytes / (ms_per_step * 1e-3) / 1e9
    traffic, traffic_src, l2_hit = None, None, None
    if a.traffic_csv:
        traffic = read_traffic(a.traffic_csv.split(","), traffic_key(dom["kernel"]))
        traffic_src = "live: " + a.traffic_csv
    elif os.path.exists(TRAFFIC_JSON):
        with open(TRAFFIC_JSON) as f:
            tj = json.load(f)
        if tj.get("config") == [a.scene, a.width, a.height, a.spp, a.bounces]:
            by_kernel = tj.get("bytes_per_launch_by_kernel") or {}
            if by_kernel.get(dom["kernel"]) is not None:
                traffic, traffic_src = by_kernel[dom["kernel"]], TRAFFIC_JSON_REL + " (" + tj.get("source", "") + ")"
            # TCC hit rates (rocprofv3 TCC_HIT/TCC_MISS pass) of the traversal, shade and finish kernels
            hits = tj.get("l2_hit") or {}
            l2_hit = {k: v for k, v in hits.items() if re.search(r"wf_(trace|shade|finish)", k)} or None
    # frames in flight: launches of different frames share the GPU, so a launch's time is not the
    # kernel's alone; when the dominant kernel's time per frame exceeds the step, say so
    shared = dom["ms_per_frame"] > ms_per_step
    r = {
        "bound": "hbm", "achieved": round(dom["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(dom["achieved"] / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
        "frac_of_l2_gather_peak": round(dom["achieved"] / L2_GATHER_PEAK_GBS, 4),
        # the same launch with every node visit charged 80 B (round-2 accounting: LDS-served top
        # nodes counted as memory bytes)
        "frac_all_nodes": round(dom["achieved_all_nodes"] / HBM_PEAK_GBS, 4),
        # measured HBM bytes of one launch (PMC) over the launch time: what actually crossed HBM
        "hbm_GBs": round(traffic / (dom["launch_ms"] * 1e-3) / 1e9, 1) if traffic else None,
        "l2_hit": l2_hit,
        "l2_hit_sorted": sorted_l2_hit(),
        "job_achieved": round(job_achieved, 1), "job_frac": round(job_achieved / HBM_PEAK_GBS, 4),
        "job_bytes_per_frame": int(job_bytes),
        "not_a_kernel_measurement": shared,
        "note": ("frames in flight share the GPU: the launch time includes time its workgroups wait for CUs "
                 "other frames' kernels hold (see 'isolated' for the kernel alone)") if shared else None,
        "kernel": dom["kernel"], "launch_ms": round(dom["launch_ms"], 4),
        "launch_ms_device": round(dom["launch_ms_device"], 4) if dom["launch_ms_device"] else None,
        "bytes_per_launch": int(dom["bytes_per_launch"]),
        "rays_per_launch": int(dom["rays_per_launch"]), "nodes_per_ray": round(dom["nodes_per_ray"], 3),
        "lds_nodes_per_ray": round(dom["lds_nodes_per_ray"], 3), "tris_per_ray": round(dom["tris_per_ray"], 3),
        # every timed kernel of the frame with its own roofline, for comparison
        "kernels": [{"kernel": k["kernel"], "ms_per_frame": round(k["ms_per_frame"], 3),
                     "launch_ms": round(k["launch_ms"], 4),
                     "launch_ms_device": round(k["launch_ms_device"], 4) if k["launch_ms_device"] else None,
                     "achieved_GBs": round(k["achieved"], 1), "bytes_per_launch": int(k["bytes_per_launch"]),
                     "frac": round(k["achieved"] / HBM_PEAK_GBS, 4), "nodes_per_ray": round(k["nodes_per_ray"], 3),
                     "lds_nodes_per_ray": round(k["lds_nodes_per_ray"], 3),
                     "tris_per_ray": round(k["tris_per_ray"], 3)} for k in kernels],
        "_stage_ms": list(stage_ms[:7] / steps),
    }
    return r


def isolated(R, tiles, torch, dev, a, cst, cus, kernel, frames):
    """The bench frame with one frame in flight: the renderer on a caller's stream keeps one slot
    (rt_set_stream), so every launch has the GPU to itself.  After the timed region, not part of
    the bench value: the dominant kernel's algorithmic bytes per launch (same accounting as the
    timed region) over these launches' own HIP-event and device-clock times."""
    s = torch.cuda.Stream(device=dev)
    R.set_stream(s.cuda_stream)
    R.set_device_spans(True)   # the stamps cost ~1 % of a frame: on for these frames only
    try:
        R.draw(tiles=tiles)   # capture / warm the single slot
        R.wait()
        i0 = R.stats()
        t0 = time.perf_counter()
        for _ in range(frames):
            R.draw(tiles=tiles)
            R.wait()
        wall = (time.perf_counter() - t0) / frames
        i1 = R.stats()
    finally:
        R.set_device_spans(False)
        R.set_stream(None)
    d = lambda f: getattr(i1, f) - getattr(i0, f)
    b = argparse.Namespace(**vars(a))
    b.steps = frames
    closest = d("total_closest_rays")
    r = roofline(b, cst, i0, i1, closest + d("total_shadow_rays"), closest, d("total_frame_ms") / frames,
                 wall * 1e3, cus)
    k = next((k for k in r["kernels"] if k["kernel"] == kernel), None)
    if k is None:
        return None
    return {"frames_in_flight": i1.frames_in_flight, "frames": frames, "kernel": kernel,
            "launch_ms": k["launch_ms"], "launch_ms_device": k["launch_ms_device"],
            "achieved": k["achieved_GBs"], "frac": k["frac"],
            "frac_of_l2_gather_peak": round(k["achieved_GBs"] / L2_GATHER_PEAK_GBS, 4),
            "frac_device": round(k["bytes_per_launch"] / (k["launch_ms_device"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if k["launch_ms_device"] else None,
            "ms_per_frame": round(wall * 1e3, 3), "kernel_ms_per_frame": round(d("total_frame_ms") / frames, 3),
            # [generate, extend, shade, connect, resolve, finish, hit sort] per frame, one frame at a time
            "stage_ms": [round(x, 3) for x in r["_stage_ms"]]}


TRAFFIC_KEYS = {"rt::wf_trace": r"wf_trace<(true|false),false>", "rt::wf_finis": r"wf_finish_step<false,false"}


def traffic_key(kernel):
    """rocprof kernel-name pattern of the bench line's dominant kernel"""
    return TRAFFIC_KEYS.get(kernel[:12], r"megakernel<false,")


def read_traffic(paths, kernel_key):
    """Per-launch HBM bytes of the dominant kernel from rocprofv3 --pmc counter_collection CSVs
    (FETCH_SIZE and WRITE_SIZE come from separate passes; KB units; gfx950 FETCH_SIZE reports half
    of wide reads -> x2, MI355X_MICROARCH.md 'HBM').  COUNT=true instantiations are excluded."""
    import csv
    fetch, write, nf, nw = 0.0, 0.0, 0, 0
    for path in paths:
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "").split("(")[0].replace(" ", "")
                if not re.search(kernel_key, k):
                    continue
                name = row.get("Counter_Name", "")
                v = float(row.get("Counter_Value", 0))
                if name == "FETCH_SIZE":
                    fetch += v
                    nf += 1
                elif name == "WRITE_SIZE":
                    write += v
                    nw += 1
    if nf == 0 or nw == 0:
        return None
    return int((2 * fetch / nf + write / nw) * 1024)


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
