"""Multi-rank tile split + gather on CPU (gloo, world_size 2 and 3): the protocol bench.py runs
over RCCL, with the library's own tile layout (rt_pack_tiles_host /
rt_unpack_tiles_host share tile_pixel() with the device kernels).

Each rank's "render" is the oracle's frame restricted to that rank's tiles, so the gathered
image must equal the one-process frame bit for bit."""
import importlib
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tile_mask(w, h, tile, rank, n):
    m = np.zeros((h, w), bool)
    tx = (w + tile - 1) // tile
    ty = (h + tile - 1) // tile
    for t in range(rank, tx * ty, n):
        x0, y0 = (t % tx) * tile, (t // tx) * tile
        m[y0:y0 + tile, x0:x0 + tile] = True
    return m


def _worker(rank, n, port, w, h, tile, full, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=n)
    try:
        rt = importlib.import_module("metal4-raytracing_amd")
        from importlib import import_module
        tiles = import_module("metal4-raytracing_amd.tiles")
        # this rank's render: only its own tiles are valid, the rest is garbage
        mine = np.where(_tile_mask(w, h, tile, rank, n)[..., None], full, np.float32(-7.0)).astype(np.float32)
        g = tiles.TileGather(w, h, tile, rank, n, device="cpu")
        out = g.gather(mine)
        if rank == 0:
            q.put(("ok", out))
        dist.barrier()
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,w,h,tile", [(2, 200, 136, 64), (3, 256, 256, 64), (2, 64, 48, 16)])
def test_gloo_tile_gather_bitwise(n, w, h, tile):
    import torch.multiprocessing as mp
    rng = np.random.default_rng(n * 1000 + w)
    full = rng.standard_normal((h, w, 4)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, w, h, tile, full, q)) for r in range(n)]
    for p in procs:
        p.start()
    status, out = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", out
    assert np.array_equal(out, full)


def test_tile_partition_covers_frame(rt):
    tiles = importlib.import_module("metal4-raytracing_amd.tiles")
    w, h, tile = 1920, 1080, 64
    for n in (1, 2, 4, 8):
        counts = [tiles.tile_count(w, h, tile, r, n) for r in range(n)]
        assert sum(counts) == ((w + 63) // 64) * ((h + 63) // 64)
        assert max(counts) - min(counts) <= 1
        cover = np.zeros((h, w), np.int32)
        for r in range(n):
            cover += _tile_mask(w, h, tile, r, n)
        assert (cover == 1).all()


def test_pack_unpack_roundtrip_with_oracle_frame(rt, orc, assets):
    """A real (oracle) C1 frame through pack -> unpack for every rank of a 3-way split."""
    tiles = importlib.import_module("metal4-raytracing_amd.tiles")
    sc = rt.Scene.preset("c1", assets)
    W, H = 96, 80
    U = rt.uniforms_default(W, H, sc.light_count)
    U.samplesPerPixel = 1
    U.maxBounces = 1
    osc = orc.OracleScene(sc.desc())
    img = osc.render(U, rt.random_offsets(1, W, H))["radiance"].reshape(H, W, 4).astype(np.float32)
    out = np.full_like(img, np.nan)
    for r in range(3):
        p = tiles.pack_host(img, 32, r, 3)
        tiles.unpack_host(p, out, 32, r, 3)
    assert np.array_equal(out, img)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n", [2, 3])
def test_bench_launcher_starts_ranks(n):
    """`python bench.py --gpus N` with no WORLD_SIZE starts N rank processes itself (the parent
    never touches a GPU), they meet over torch.distributed (gloo in --dry-run, RCCL on GPUs), run
    the barrier / max-over-ranks timing and the tile gather, and rank 0's single JSON line comes
    through with n_gpus = world_size = N."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run", "--steps", "3",
                        "--warmup", "1", "--width", "200", "--height", "136"], capture_output=True, text=True,
                       timeout=200, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_size"] == n and d["steps"] == 3 and d["value"] > 0
    pr = d["config"]["per_rank"]   # every rank's own figures, gathered to rank 0
    assert [x["rank"] for x in pr] == list(range(n)) and all(x["ms_per_step"] > 0 for x in pr)
    assert sum(x["rays_per_frame"] for x in pr) * 3 / (d["ms_per_step"] * 3e-3) / 1e9 == pytest.approx(d["value"], rel=1e-6)


@pytest.mark.timeout(120)
def test_bench_launcher_fails_when_a_rank_fails():
    """Ranks that fail (an invalid frame size reaches every child) make the launcher exit non-zero
    instead of hanging."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "0",
                        "--warmup", "0", "--scene", "c1", "--width", "-5"], capture_output=True, text=True, timeout=100,
                       cwd=ROOT, env=env)
    assert r.returncode != 0
