"""Tile-split frames across ranks and the radiance gather.

Each rank renders the 64x64 tiles with tile_id % nranks == rank (global pixel coordinates and the
global random-offset image, so the pixels are bitwise those of a one-GPU frame), packs them into
a buffer of max_tiles x T x T x RGBA fp32 (ranks padded to equal size), and ONE
torch.distributed.gather moves the packed buffers to the destination rank, which unpacks the
other ranks' tiles into its radiance target.  On GPUs the backend is "nccl" (RCCL over xGMI) and
pack/unpack are the library's device kernels; the host forms (rt_pack_tiles_host /
rt_unpack_tiles_host, same layout) serve gathers into host memory and the gloo tests.

The reference renders on one device only (Renderer.draw, Renderer.swift:1405-1503); this is
the multi-GPU frame split of BASELINE configs[3].
"""
import ctypes as C

import numpy as np

from ._abi import TileSet


def _lib():
    from . import lib
    return lib()


def _check(st):
    from . import _check as chk
    chk(st)


def tile_count(width, height, tile, rank, nranks):
    return int(_lib().rt_tile_count(width, height, C.byref(TileSet(tile, rank, nranks, 0))))


def pack_host(img, tile, rank, nranks, count=None):
    """img: (H, W, 4) float32 -> (count, T, T, 4) packed tiles of `rank` (zero padded)."""
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape[:2]
    own = tile_count(w, h, tile, rank, nranks)
    out = np.zeros((max(own, count or 0), tile, tile, 4), np.float32)
    fp = C.POINTER(C.c_float)
    _check(_lib().rt_pack_tiles_host(w, h, C.byref(TileSet(tile, rank, nranks, 0)), img.ctypes.data_as(fp),
                                     out.ctypes.data_as(fp)))
    return out


def unpack_host(packed, img, tile, rank, nranks):
    """Writes the tiles of `rank` from packed (>= own, T, T, 4) into img (H, W, 4) in place."""
    packed = np.ascontiguousarray(packed, np.float32)
    assert img.dtype == np.float32 and img.flags.c_contiguous
    h, w = img.shape[:2]
    fp = C.POINTER(C.c_float)
    _check(_lib().rt_unpack_tiles_host(w, h, C.byref(TileSet(tile, rank, nranks, 0)), packed.ctypes.data_as(fp),
                                       img.ctypes.data_as(fp)))
    return img


class TileGather:
    """One rank's side of the per-frame gather.

    renderer: a Renderer whose latest radiance target holds this rank's tiles (device path), or
    None for the host path (gather(image) with a host image).  device: torch device of the
    packed buffers (cuda for RCCL, cpu for gloo).  A renderer with a cpu `device` stages through
    host memory: the device pack kernel writes a device buffer, the packed tiles cross to the host,
    gloo gathers them, and the destination unpacks them with the device kernel (the rank flow of
    the RCCL path with another transport: bench.py --gather-backend gloo, e.g. several ranks on
    one GPU, which RCCL refuses)."""

    def __init__(self, width, height, tile, rank, nranks, device, renderer=None, dst=0):
        import torch
        self.w, self.h, self.T, self.rank, self.n, self.dst = width, height, tile, rank, nranks, dst
        self.R = renderer
        self.own = tile_count(width, height, tile, rank, nranks)
        self.max_own = max(tile_count(width, height, tile, r, nranks) for r in range(nranks))
        self.packed = torch.zeros((self.max_own, tile, tile, 4), dtype=torch.float32, device=device)
        self.recv = ([torch.empty_like(self.packed) for _ in range(nranks)] if rank == dst else None)
        self.staging = renderer is not None and torch.device(device).type == "cpu"
        if self.staging:   # device-side buffers of the host-staged path
            self.d_packed = torch.zeros(self.packed.shape, dtype=torch.float32, device="cuda")
            self.d_recv = [torch.empty_like(self.d_packed) for _ in range(nranks)] if rank == dst else None

    def gather(self, image=None, events=None):
        """Gathers this frame's tiles on the dst rank. Device path: enqueued without a host wait;
        after the dst renderer's wait() its target holds the full frame (returns None). Host path:
        returns the full (H, W, 4) image on dst, None elsewhere.  events (device path, optional): a
        pair of torch.cuda.Event recorded on the current stream after the pack and after the
        unpack (dst) / the gather (other ranks), i.e. around the collective."""
        import torch
        import torch.distributed as dist
        if self.R is not None:
            # after the newest frame, on the stream the collective is ordered on; the renderer's
            # next frame overlaps the pack and the gather
            self.R.pack_tiles(self.T, self.rank, self.n, (self.d_packed if self.staging else self.packed).data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
            if events is not None:
                events[0].record()
            if self.staging:
                self.packed.copy_(self.d_packed)   # waits for the pack on the current stream
        else:
            self.packed.copy_(torch.from_numpy(pack_host(image, self.T, self.rank, self.n, self.max_own)))
        dist.gather(self.packed, self.recv, dst=self.dst)
        if self.rank != self.dst:
            if events is not None and self.R is not None:
                events[1].record()
            return None
        if self.R is not None:
            s = torch.cuda.current_stream().cuda_stream
            for r in range(self.n):
                if r != self.rank:
                    src = self.recv[r]
                    if self.staging:
                        self.d_recv[r].copy_(src)
                        src = self.d_recv[r]
                    self.R.unpack_tiles(self.T, r, self.n, src.data_ptr(), stream=s)
            if events is not None:
                events[1].record()
            return None
        out = np.zeros((self.h, self.w, 4), np.float32)
        for r in range(self.n):
            unpack_host(self.recv[r].numpy(), out, self.T, r, self.n)
        return out
