"""Child process of tests/test_gpu_rccl.py: the Python RCCL gather path of tiles.TileGather with
device buffers, at world size 1 under dist.init_process_group("nccl") (the pool's boxes hold one
GPU and RCCL refuses two ranks on one device).  Started fresh, before any GPU call in it.

Steps: render a tile-split frame (rank 0 of 1), pack it on torch's stream with the device kernel,
dist.gather the packed device buffer over RCCL, check the gathered buffer against the host packing
of the frame, render a different frame, unpack the gathered tiles into the target with the device
kernel on torch's stream, and require the target to equal the first frame again; the first frame
must also equal an untiled frame of a second renderer (Renderer.swift:1405-1503 renders one
device's frame).  Prints one JSON line; exits non-zero on a mismatch."""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29533")
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    rt = importlib.import_module("metal4-raytracing_amd")
    tiles = importlib.import_module("metal4-raytracing_amd.tiles")
    W, H, T = 200, 136, 64
    scene = rt.Scene.preset("c1")

    def renderer():
        R = rt.Renderer(scene, W, H, device=0, seed=3)
        R.samplesPerPixel, R.maxBounces = 2, 3
        return R

    R = renderer()
    R.draw(tiles=(T, 0, 1))
    g = tiles.TileGather(W, H, T, 0, 1, torch.device("cuda", 0), renderer=R)
    assert g.packed.is_cuda and not g.staging
    g.gather()                          # device pack on torch's stream + dist.gather over RCCL
    torch.cuda.current_stream().synchronize()
    R.wait()
    a = R.radiance()
    got = g.recv[0].cpu().numpy()
    want = tiles.pack_host(a, T, 0, 1, g.max_own)
    pack_equal = bool(np.array_equal(got, want))
    R.draw()                            # frame 1 (EMA over frame 0): a different target
    R.wait()
    b = R.radiance()
    changed = bool(np.any(b != a))
    R.unpack_tiles(T, 0, 1, g.recv[0].data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    R.wait()
    c = R.radiance()
    unpack_equal = bool(np.array_equal(c, a))
    R.close()
    R1 = renderer()                     # the same frame untiled, another context
    R1.draw()
    R1.wait()
    untiled_equal = bool(np.array_equal(R1.radiance(), a))
    R1.close()
    out = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "pack_equal": pack_equal,
           "frame_changed": changed, "unpack_equal": unpack_equal, "untiled_equal": untiled_equal,
           "nonzero": bool(np.any(a[..., :3] > 0))}
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0 if all(out[k] for k in ("pack_equal", "frame_changed", "unpack_equal", "untiled_equal", "nonzero")) else 1


if __name__ == "__main__":
    sys.exit(main())
