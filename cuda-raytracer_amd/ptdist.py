"""Multi-GPU framebuffer sharding and the RCCL gather of the final image.

SURVEY §8(e): every pixel-sample is independent, so each rank renders the
32x32 tiles t with t % world == rank (interleaved for load balance) with the
scene replicated, and the only collective is one gather of the framebuffer to
rank 0 (torch.distributed "nccl" = RCCL over xGMI; "gloo" in CPU tests).
The reference has no multi-GPU path (cu:1874-1897 only enumerates devices).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def owned_pixels(width, height, tile, rank, nranks):
    """Global pixel indices owned by `rank`, in the slot order of pt_owned_pixels."""
    ntx, nty = -(-width // tile), -(-height // tile)
    out = []
    for t in range(rank, ntx * nty, nranks):
        ty, tx = divmod(t, ntx)
        rows = np.arange(ty * tile, min(height, (ty + 1) * tile))
        cols = np.arange(tx * tile, min(width, (tx + 1) * tile))
        out.append((rows[:, None] * width + cols[None, :]).reshape(-1))
    return np.concatenate(out).astype(np.int64) if out else np.zeros(0, np.int64)


_hip = None


def _hip_memcpy_d2d(dst, src, nbytes):
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.restype = C.c_int
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    rc = _hip.hipMemcpy(C.c_void_p(dst), C.c_void_p(src), C.c_size_t(nbytes), 3)  # DeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed ({rc})")


def local_sums_tensor(ctx, device):
    """This rank's per-pixel radiance sums (float4 per owned pixel) as a torch tensor on `device`."""
    import torch
    idx, dptr = ctx.owned_pixels()
    buf = torch.empty((len(idx), 4), dtype=torch.float32, device=device)
    if len(idx):
        torch.cuda.synchronize(device)
        _hip_memcpy_d2d(buf.data_ptr(), dptr, len(idx) * 16)
    return buf


def gather_frame(local_sums, width, height, tile, spp, group=None):
    """Gather every rank's owned-pixel sums to rank 0 and assemble the image.

    local_sums: torch tensor (n_local, 4) on this rank's device (cuda for RCCL,
    cpu for gloo).  Returns the (height, width, 4) float32 image on rank 0
    (radiance / spp, alpha 1), None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [len(owned_pixels(width, height, tile, r, world)) for r in range(world)]
    assert local_sums.shape[0] == counts[rank]
    maxn = max(counts)
    send = torch.zeros((maxn, 4), dtype=torch.float32, device=local_sums.device)
    send[: counts[rank]] = local_sums
    recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, recv, dst=0, group=group)
    if rank != 0:
        return None
    frame = torch.zeros((height * width, 4), dtype=torch.float32, device=local_sums.device)
    for r in range(world):
        idx = torch.as_tensor(owned_pixels(width, height, tile, r, world), device=local_sums.device)
        frame[idx] = recv[r][: counts[r]]
    frame[:, :3] /= float(spp)
    frame[:, 3] = 1.0
    return frame.reshape(height, width, 4)
