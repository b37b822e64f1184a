#!/usr/bin/env python3
"""Headline benchmark: Grays/s + ms/frame, dragon scene, 1920x1080x4spp, 8 bounces (BASELINE.json
metric; workload = configs[2], the dragon config that fits one MI355X).

One step = one frame of the hot path (raytracingKernel equivalent) over the whole image.
N GPUs (one process per GPU, torch.distributed over RCCL): the frame is tile-partitioned
(64x64 tiles, tile_id % N == rank), every rank renders its tiles, packs them, and rank 0
gathers the packed radiance over RCCL/xGMI and unpacks it into the full frame ("strong"
scaling: the frame is fixed, N GPUs share it).

Grays/s = (closest-hit + shadow rays traced, all ranks) / wall time of the K timed frames
(barrier + device sync on both sides, max over ranks).  Inputs (scene, BVH, random offsets)
are resident in HBM before the timed region.
"""
import argparse
import importlib
import json
import os
import re
import sys
import time

import numpy as np

# Hardware queues per process, fixed before anything initialises HIP so every run sees the same
# count: four (HIP's default, also what the GPU boxes export).  Small frames (a multi-GPU rank's
# share) keep as many frames in flight as there are queues, up to eight (rt_api.cpp
# small_frame_slots).  Final round-2 kernels, 8-way rank share: four queues / four slots 4.21 /
# 4.24 Grays/s against eight / eight 4.11 / 4.10 (round 1's slower kernels preferred eight).
# RT_HW_QUEUES overrides (tuning runs).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES", "4")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic bytes: per traced ray 32 B in (o, tmin, d, tmax) + 16 B hit out;
# per BVH node fetched 64 B; per triangle tested 48 B; per closest hit shading 16 B tri record
# + 3x16 B normals + 48 B instance transform; per pixel 4 B offset + 16 B history read +
# 16 B accumulation write + 4 B depth + 8+8 B motion read/write.
B_RAY = 48
B_NODE = 80  # compressed 8-wide node (Bvh8Node)
B_TRI = 48
B_HIT = 16 + 48 + 48
B_PIXEL = 4 + 16 + 16 + 4 + 16
B_QRAY = 48  # wf_trace queue entry: extend 32 B ray in + 16 B hit out; connect 48 B shadow entry in
_ROOT = os.path.dirname(os.path.abspath(__file__))
# PMC traffic of the newest round (profiles/rNN_traffic.json, tools/gpurun_profile.sh)
_TRAFFIC = sorted(f for f in os.listdir(os.path.join(_ROOT, "profiles")) if re.fullmatch(r"r\d+_traffic\.json", f)) \
    if os.path.isdir(os.path.join(_ROOT, "profiles")) else []
TRAFFIC_JSON_REL = "profiles/" + (_TRAFFIC[-1] if _TRAFFIC else "r01_traffic.json")
TRAFFIC_JSON = os.path.join(_ROOT, TRAFFIC_JSON_REL)


def parse():
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
                   help="frames the renderer overlaps (0 = library default: 2; below 8M allocated paths per frame 4 with the 4 hardware queues set here, 8 with RT_HW_QUEUES=8; 1 = one at a time)")
    p.add_argument("--animate", action="store_true",
                   help="configs[4] shape: skin every skinned mesh at t = frame/60 s and refit the BVH before each frame")
    p.add_argument("--rebuild", action="store_true", help="with --animate: rebuild the BVH on the device instead of refitting")
    p.add_argument("--emulate-ranks", type=int, default=0,
                   help="tuning aid: one process renders rank 0's tiles of an N-way split (no gather)")
    p.add_argument("--emulate-rank", type=int, default=0, help="with --emulate-ranks: which rank's tiles")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--traffic-csv", default=None, help="rocprofv3 --pmc counter_collection.csv for traffic")
    return p.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    rt = importlib.import_module("metal4-raytracing_amd")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    n = max(world, 1)

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

    def frame():
        R.draw(tiles=tiles)
        R.wait()
        st = R.stats()
        if gather is not None:
            gather.gather()   # packed tiles -> rank 0 over RCCL, unpacked into its radiance target
        return st

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

    def submit():
        # one step: the frame is submitted and, multi-GPU, its tiles packed, gathered to rank 0
        # over RCCL and unpacked there, all enqueued without a host wait (the renderer keeps two
        # frames in flight and waits for a slot's previous frame itself)
        animate()
        R.draw(tiles=tiles)
        if gather is not None:
            gather.gather()

    def barrier():
        if n > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # counting frame (untimed): node visits / triangle tests per ray for the roofline numerator
    R.set_counting(True)
    R.frameIndex = 0
    cst = frame()
    R.set_counting(False)
    rays_c = cst.closest_rays + cst.shadow_rays
    nodes_per_ray = cst.node_visits / max(rays_c, 1)
    tris_per_ray = cst.tri_tests / max(rays_c, 1)
    # the queue traversal kernel alone (wavefront): its own node / triangle visits per traced ray
    q_nodes_per_ray = cst.trace_nodes / max(cst.trace_rays, 1)
    q_tris_per_ray = cst.trace_tris / max(cst.trace_rays, 1)
    # the persistent finish kernel: the rest of the visits, over the rays it traced
    f_rays_c = rays_c - cst.trace_rays
    f_nodes_per_ray = (cst.node_visits - cst.trace_nodes) / max(f_rays_c, 1)
    f_tris_per_ray = (cst.tri_tests - cst.trace_tris) / max(f_rays_c, 1)
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
        submit()
        t_host += time.perf_counter() - th
    R.wait()
    barrier()
    dt = time.perf_counter() - t0
    # the running totals of every frame of the timed region (HIP events per stage on the
    # renderer's streams, ray counters read back per frame)
    last_st = s1 = R.stats()
    assert s1.frames_total - s0.frames_total == a.steps
    d = lambda f: getattr(s1, f) - getattr(s0, f)
    closest = d("total_closest_rays")
    rays = closest + d("total_shadow_rays")
    trace_rays, trace_launches, trace_ms = d("total_trace_rays"), d("total_trace_launches"), d("total_trace_ms")
    trace_closest, finish_launches = d("total_trace_closest_rays"), d("total_finish_launches")
    stage_ms = np.array(list(s1.total_kernel_ms)) - np.array(list(s0.total_kernel_ms))
    kernel_ms = [d("total_frame_ms") / a.steps]

    rays_local, closest_local = rays, closest   # this rank's, for the per-kernel roofline
    tot = torch.tensor([dt, float(rays), float(closest), float(np.mean(kernel_ms))], dtype=torch.float64, device=dev)
    if n > 1:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        dt, rays, closest, kms = float(mx[0]), float(sm[1]), float(sm[2]), float(mx[3])
    else:
        kms = float(tot[3])
    if rank != 0:
        dist.destroy_process_group()
        return

    value = rays / dt / 1e9
    ms_per_step = dt / a.steps * 1e3
    kernels = []
    if last_st.pipeline == 1 and trace_launches > 0:
        # wf_trace (extend + connect launches), per launch.  Algorithmic bytes per traced ray: 48 B
        # queue entry in (+ hit record out) + 80 B per 8-wide node fetched + 48 B per triangle
        # tested (DESIGN.md 'Roofline').
        rpl = trace_rays / trace_launches
        kernels.append(dict(
            kernel="rt::wf_trace<{false,true}, false> (extend + connect)", launches=trace_launches / a.steps,
            launch_ms=trace_ms / trace_launches, rays_per_launch=rpl, nodes_per_ray=q_nodes_per_ray,
            tris_per_ray=q_tris_per_ray,
            bytes_per_launch=rpl * (B_QRAY + q_nodes_per_ray * B_NODE + q_tris_per_ray * B_TRI)))
    if last_st.pipeline == 1 and finish_launches > 0:
        # wf_finish_step: the tail paths to completion.  Per ray 48 B (ray + hit) + nodes + triangles
        # as above; per closest hit the shading gathers (B_HIT); the path state in and out (48 B x 2)
        # once per path is left out (not counted per ray).
        f_rays = (rays_local - trace_rays) / finish_launches
        f_closest = (closest_local - trace_closest) / finish_launches
        kernels.append(dict(
            kernel="rt::wf_finish_step<false, false, 4>", launches=finish_launches / a.steps,
            launch_ms=float(stage_ms[5]) / finish_launches, rays_per_launch=f_rays, nodes_per_ray=f_nodes_per_ray,
            tris_per_ray=f_tris_per_ray,
            bytes_per_launch=f_rays * (B_RAY + f_nodes_per_ray * B_NODE + f_tris_per_ray * B_TRI) + f_closest * B_HIT))
    if not kernels:
        # megakernel: the whole frame is one launch
        rpl = rays_local / a.steps
        kernels.append(dict(
            kernel="rt::megakernel<false, false>", launches=1, launch_ms=kms, rays_per_launch=rpl,
            nodes_per_ray=nodes_per_ray, tris_per_ray=tris_per_ray,
            bytes_per_launch=(rpl * (B_RAY + nodes_per_ray * B_NODE + tris_per_ray * B_TRI)
                              + closest_local / a.steps * B_HIT + a.width * a.height / n * B_PIXEL)))
    for k in kernels:
        k["achieved"] = k["bytes_per_launch"] / (k["launch_ms"] * 1e-3) / 1e9
        k["ms_per_frame"] = k["launch_ms"] * k["launches"]
    # the dominant kernel: the most device time per frame
    dom = max(kernels, key=lambda k: k["ms_per_frame"])
    # the whole frame: every timed kernel's algorithmic bytes over the wall time per frame (with
    # frames in flight the kernels of two frames share the GPU, so per-launch durations stretch
    # while the aggregate rate rises)
    job_bytes = sum(k["bytes_per_launch"] * k["launches"] for k in kernels)
    job_achieved = job_bytes / (dt / a.steps) / 1e9   # per GPU (rank 0's kernels)
    kernel, launch_ms, bytes_per_launch = dom["kernel"], dom["launch_ms"], dom["bytes_per_launch"]
    rays_per_launch, npr, tpr, achieved = dom["rays_per_launch"], dom["nodes_per_ray"], dom["tris_per_ray"], dom["achieved"]
    traffic, traffic_src, l2_hit = None, None, None
    if a.traffic_csv:
        traffic = read_traffic(a.traffic_csv.split(","), traffic_key(kernel))
        traffic_src = "live: " + a.traffic_csv
    elif os.path.exists(TRAFFIC_JSON):
        with open(TRAFFIC_JSON) as f:
            tj = json.load(f)
        if tj.get("config") == [a.scene, a.width, a.height, a.spp, a.bounces]:
            by_kernel = tj.get("bytes_per_launch_by_kernel") or {}
            if tj.get("kernel") == kernel:
                by_kernel.setdefault(kernel, tj["bytes_per_launch"])
            if by_kernel.get(kernel) is not None:
                traffic, traffic_src = by_kernel[kernel], TRAFFIC_JSON_REL + " (" + tj.get("source", "") + ")"
            # TCC hit rates (rocprofv3 TCC_HIT/TCC_MISS pass) of the traversal, shade and finish kernels
            hits = tj.get("l2_hit") or {}
            l2_hit = {k: v for k, v in hits.items() if re.search(r"wf_(trace|shade|finish)", k)} or None

    cpu = None
    if not a.no_cpu and n == 1:
        cpu = cpu_baseline(rt, scene, R, a)

    line = {
        "metric": "Grays/sec (closest-hit + shadow rays traced) at 1920x1080x4spp, dragon; ms/frame",
        "value": round(value, 4),
        "unit": "Grays/s",
        "n_gpus": n,
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
            "workload": f"{a.scene}: glass dragon scene (configs[2]) {a.width}x{a.height}x{a.spp}spp, {a.bounces} bounces, "
                        f"one frame per step, {'tile-split ' + str(T) + 'px + RCCL gather' if n > 1 else 'single GPU'}"
                        f"{', frames submitted back to back (overlapping frames in flight)' if n == 1 else ''}",
            "scene": a.scene, "triangles": scene.triangle_count, "width": a.width, "height": a.height,
            "spp": a.spp, "max_bounces": a.bounces, "pipeline": a.pipeline, "parallelism": f"tiles{n}",
            "rays_per_frame": int(rays / a.steps), "kernel_ms_per_frame": round(kms, 3),
            "setup_s": round(setup_s, 2),
            # [generate, extend, shade, connect, resolve, finish, hit sort]
            "stage_ms": [round(x / a.steps, 3) for x in stage_ms[:7]], "sort_bins": a.sort_bins, "bvh": a.bvh,
            "pipeline_used": ["megakernel", "wavefront"][last_st.pipeline], "iterations": last_st.iterations,
            "frames_in_flight": last_st.frames_in_flight, "animate": bool(skinned),
            # host time inside the submit calls per step (includes waiting for a free frame slot)
            "host_submit_ms": round(t_host / a.steps * 1e3, 3),
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
            # measured HBM bytes of one launch (PMC) over the launch time: what actually crossed HBM
            "hbm_GBs": round(traffic / (launch_ms * 1e-3) / 1e9, 1) if traffic else None,
            "l2_hit": l2_hit,
            "job_achieved": round(job_achieved, 1), "job_frac": round(job_achieved / HBM_PEAK_GBS, 4),
            "job_bytes_per_frame": int(job_bytes),
            "kernel": kernel, "launch_ms": round(launch_ms, 4), "bytes_per_launch": int(bytes_per_launch),
            "rays_per_launch": int(rays_per_launch), "nodes_per_ray": round(npr, 3), "tris_per_ray": round(tpr, 3),
            # every timed kernel of the frame with its own roofline, for comparison
            "kernels": [{"kernel": k["kernel"], "ms_per_frame": round(k["ms_per_frame"], 3),
                         "launch_ms": round(k["launch_ms"], 4), "achieved_GBs": round(k["achieved"], 1),
                         "frac": round(k["achieved"] / HBM_PEAK_GBS, 4), "nodes_per_ray": round(k["nodes_per_ray"], 3),
                         "tris_per_ray": round(k["tris_per_ray"], 3)} for k in kernels],
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if n > 1:
        dist.destroy_process_group()


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


def cpu_baseline(rt, scene, R, a):
    """The C oracle (oracle/, a port) on a bounded row subset of the same frame, host cores."""
    import oracle
    threads = min(16, os.cpu_count() or 1)
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
    return {"value": round(rays / t / 1e9, 6), "unit": "Grays/s", "cores": threads, "kind": "port",
            "sample": f"every {step}th row of frame 0 ({(a.height + step - 1) // step} rows x {a.width} px x "
                      f"{a.spp} spp) x {reps}, {rays} rays in {t:.1f} s"}


if __name__ == "__main__":
    main()
