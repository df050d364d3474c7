"""Multi-rank path on the HIP renderer (BASELINE config 5).

* world 2 over gloo, both ranks on cuda:0: each rank renders its interleaved
  tiles through libptcore (small path pool), hands ptdist.local_sums_tensor
  (pt_copy_owned_sums, device-to-device) to ptdist.gather_frame, and rank 0's
  assembled frame equals the single-rank HIP frame, which equals the oracle;
* config 5's sharding on the dragon proxy: 8 ranks' tile shares (rendered one
  after another on this GPU) add up to the full HIP frame, bit for bit, and
  the full frame equals the oracle.
RCCL itself cannot run two ranks on one GPU; the driver's 8-GPU bench runs the
same gather over "nccl"."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import ptdist
import ptrace
import pyoracle
from conftest import ROOT, load_fixture

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, tile, spp, out_path):
    import sys
    sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "tests")]
    import torch
    import torch.distributed as dist
    import ptrace as pt
    from conftest import load_fixture as lf
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ctx = pt.Context(0)
    ctx.load_scene(lf("CBbunny"))
    ctx.render(W, H, spp, max_bounces=6, batch_paths=4096, tile_size=tile, rank=rank, nranks=world)
    local = ptdist.local_sums_tensor(ctx, torch.device("cuda", 0))
    assert local.device.type == "cuda"
    frame = ptdist.gather_frame(local.cpu(), W, H, tile, spp)  # gloo gathers host tensors
    if rank == 0:
        np.save(out_path, frame.numpy())
    ctx.close()
    dist.destroy_process_group()


def test_two_ranks_gather_equals_single_rank_hip_frame(gpu_ctx, tmp_path):
    W, H, tile, spp = 72, 56, 16, 2
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(2, _free_port(), W, H, tile, spp, out), nprocs=2, join=True)
    frame = np.load(out)
    sc = load_fixture("CBbunny")
    gpu_ctx.load_scene(sc)
    gpu_ctx.clear()
    gpu_ctx.render(W, H, spp, max_bounces=6, tile_size=tile)
    full = gpu_ctx.get_image()
    assert np.array_equal(frame, full)
    o, _ = pyoracle.image(sc.desc(), W, H, spp, max_bounces=6, tile=tile)
    assert np.array_equal(full, o)


def test_local_sums_tensor_matches_owned_pixels(gpu_ctx):
    import torch
    gpu_ctx.load_scene(load_fixture("CBgems"))
    gpu_ctx.clear()
    gpu_ctx.render(40, 30, 3, max_bounces=4, tile_size=8, rank=1, nranks=3)
    sums = ptdist.local_sums_tensor(gpu_ctx, torch.device("cuda", 0)).cpu().numpy()
    host = ptdist.local_sums_tensor(gpu_ctx, "cpu").numpy()
    idx, _ = gpu_ctx.owned_pixels()
    assert np.array_equal(idx, ptdist.owned_pixels(40, 30, 8, 1, 3))
    img = gpu_ctx.get_image().reshape(-1, 4)
    assert np.array_equal(sums, host)
    assert np.array_equal(sums[:, :3] / np.float32(3), img[idx, :3])


def test_config5_dragon_proxy_tile_shards(gpu_ctx):
    """BASELINE config 5's decomposition on its scene (the dragon proxy),
    scaled down: 8 ranks' interleaved 8x8 tiles of a 64x64 frame."""
    import scenes
    sc = scenes.dragon_proxy()
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    W = H = 64
    spp, tile, world = 2, 8, 8
    acc = np.zeros((H, W, 4), np.float32)
    for r in range(world):
        gpu_ctx.clear()
        gpu_ctx.render(W, H, spp, max_bounces=8, tile_size=tile, rank=r, nranks=world)
        part = gpu_ctx.get_image()
        own = np.zeros(H * W, bool)
        own[ptdist.owned_pixels(W, H, tile, r, world)] = True
        assert (part.reshape(-1, 4)[~own] == 0).all()
        acc += part
    gpu_ctx.clear()
    gpu_ctx.render(W, H, spp, max_bounces=8, tile_size=tile)
    full = gpu_ctx.get_image()
    assert np.array_equal(acc, full)
    o, _ = pyoracle.image(d, W, H, spp, max_bounces=8, tile=tile)
    assert np.array_equal(full, o)
