"""Multi-GPU framebuffer sharding and the RCCL gather of the final image.

SURVEY §8(e): every pixel-sample is independent, so each rank renders the
32x32 tiles t with t % world == rank (interleaved for load balance) with the
scene replicated, and the only collective is one gather of the framebuffer to
rank 0 (torch.distributed "nccl" = RCCL over xGMI; "gloo" in CPU tests).
The reference has no multi-GPU path (cu:1874-1897 only enumerates devices).
"""
from __future__ import annotations

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


def local_sums_tensor(ctx, device):
    """This rank's per-pixel radiance sums (float4 per owned pixel, slot order
    of pt_owned_pixels) as a torch tensor on `device` (a GPU: device-to-device
    copy by pt_copy_owned_sums on the context's stream; "cpu": to host)."""
    import torch
    idx, _ = ctx.owned_pixels()
    buf = torch.empty((len(idx), 4), dtype=torch.float32, device=device)
    if len(idx):
        on_dev = buf.device.type != "cpu"
        if on_dev:
            torch.cuda.synchronize(buf.device)  # (the allocation is ordered on torch's stream)
        ctx.copy_owned_sums(buf.data_ptr(), len(idx) * 16, on_device=on_dev)
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
    # dst is a global rank: the group's rank 0
    dist.gather(send, recv, dst=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    if rank != 0:
        return None
    frame = torch.zeros((height * width, 4), dtype=torch.float32, device=local_sums.device)
    for r in range(world):
        idx = torch.as_tensor(owned_pixels(width, height, tile, r, world), device=local_sums.device)
        frame[idx] = recv[r][: counts[r]]
    frame[:, :3] /= float(spp)
    frame[:, 3] = 1.0
    return frame.reshape(height, width, 4)
