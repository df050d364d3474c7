"""Multi-GPU framebuffer sharding and the RCCL gather of the final image.

SURVEY §8(e): every pixel-sample is independent, so each rank renders the
32x32 tiles t with t % world == rank (interleaved for load balance) with the
scene replicated, and the only collective is one gather of the framebuffer to
rank 0 (torch.distributed "nccl" = RCCL over xGMI; "gloo" in CPU tests).
The reference has no multi-GPU path (cu:1874-1897 only enumerates devices).

Everything a frame's gather needs besides the sums themselves (the owned-pixel
lists of all ranks, the receive buffers, the device-side scatter index) is
built once per frame shape and cached: at 8 ranks a 1024x1024 frame is ~5 ms
of rendering per GPU, so per-frame host work would dominate it.
"""
from __future__ import annotations

import functools

import numpy as np


@functools.lru_cache(maxsize=16)
def _tile_order(width, height, tile, nranks):
    """Every pixel in the slot order of pt_owned_pixels (tile by tile, row-major
    inside the clipped tile) and, per rank, the [start, end) of its pixels in
    the rank-major concatenation (ranks own tiles t with t % nranks == rank)."""
    ntx = -(-width // tile)
    y, x = np.divmod(np.arange(width * height, dtype=np.int64), width)
    t = (y // tile) * ntx + x // tile
    r = t % nranks
    key = ((r * (ntx * -(-height // tile)) + t) * tile + y % tile) * tile + x % tile
    order = np.argsort(key, kind="stable")
    counts = np.bincount(r, minlength=nranks)
    starts = np.concatenate([[0], np.cumsum(counts)])
    order.setflags(write=False)
    return order, starts


def owned_pixels(width, height, tile, rank, nranks):
    """Global pixel indices owned by `rank`, in the slot order of pt_owned_pixels."""
    order, starts = _tile_order(width, height, tile, nranks)
    return order[starts[rank]:starts[rank + 1]]


def local_sums_tensor(ctx, device, out=None):
    """This rank's per-pixel radiance sums (float4 per owned pixel, slot order
    of pt_owned_pixels) as a torch tensor on `device` (a GPU: device-to-device
    copy by pt_copy_owned_sums on the context's stream, which it synchronises;
    "cpu": to host).  `out`: a tensor with at least that many rows to reuse
    (the result is then a view of it)."""
    import torch
    n = ctx.owned_count()
    if out is not None and out.shape[0] >= n and out.device == torch.device(device):
        buf = out[:n]
    else:
        buf = torch.empty((n, 4), dtype=torch.float32, device=device)
    if buf.device.type != "cpu":
        # the copy runs on the context's stream: torch's stream must be done
        # with the buffer (its allocation, or the last frame's gather copy)
        torch.cuda.synchronize(buf.device)
    if n:
        ctx.copy_owned_sums(buf.data_ptr(), n * 16, on_device=buf.device.type != "cpu")
    return buf


class _Layout:
    """Cached per (frame shape, world, device): counts, padded send / receive
    buffers and the scatter index of the received rows into the frame (padding
    rows go to a spare row past the last pixel)."""

    def __init__(self, width, height, tile, world, device):
        import torch
        order, starts = _tile_order(width, height, tile, world)
        self.counts = [int(starts[r + 1] - starts[r]) for r in range(world)]
        self.maxn = max(self.counts)
        npix = width * height
        dst = np.full((world, self.maxn), npix, dtype=np.int64)
        for r in range(world):
            dst[r, :self.counts[r]] = order[starts[r]:starts[r + 1]]
        self.dst = torch.as_tensor(dst.reshape(-1), device=device)
        self.send = torch.zeros((self.maxn, 4), dtype=torch.float32, device=device)
        self.recv = torch.empty((world, self.maxn, 4), dtype=torch.float32, device=device)
        self.npix = npix


@functools.lru_cache(maxsize=8)
def _layout(width, height, tile, world, device):
    return _Layout(width, height, tile, world, device)


def gather_frame(local_sums, width, height, tile, spp, group=None):
    """Gather every rank's owned-pixel sums to rank 0 and assemble the image.

    local_sums: torch tensor (n_local, 4) on this rank's device (cuda for RCCL,
    cpu for gloo).  Returns the (height, width, 4) float32 image on rank 0
    (radiance / spp, alpha 1), None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    L = _layout(width, height, tile, world, local_sums.device)
    assert local_sums.shape[0] == L.counts[rank]
    L.send[: L.counts[rank]].copy_(local_sums)
    recv = list(L.recv.unbind(0)) if rank == 0 else None
    # dst is a global rank: the group's rank 0
    dist.gather(L.send, recv, dst=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    if rank != 0:
        return None
    frame = torch.empty((L.npix + 1, 4), dtype=torch.float32, device=local_sums.device)
    frame.index_copy_(0, L.dst, L.recv.view(-1, 4))
    frame = frame[: L.npix]
    frame[:, :3] /= float(spp)
    frame[:, 3] = 1.0
    return frame.view(height, width, 4)
