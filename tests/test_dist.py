"""Multi-rank path on the CPU: world_size 2 over gloo.  Each rank
renders its interleaved tiles (here with the CPU oracle standing in for the GPU
renderer, which has the same tile ownership: tests/test_gpu_parity.py
test_tile_sharding_union), ptdist.gather_frame collects the framebuffer on rank
0, and the assembled image equals a single-rank render."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import ptdist
from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, tile, spp, out_path):
    import sys
    sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
    import torch
    import torch.distributed as dist
    import ptrace  # noqa: F401
    import pyoracle
    from conftest import load_fixture
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    d = load_fixture("CBgems").desc()
    sums, _ = pyoracle.render(d, W, H, spp, max_bounces=4, tile=tile, rank=rank, nranks=world, threads=2)
    idx = ptdist.owned_pixels(W, H, tile, rank, world)
    local = torch.from_numpy(sums.reshape(-1, 4)[idx].copy())
    frame = ptdist.gather_frame(local, W, H, tile, spp)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_shard_gather_equals_single_rank(tmp_path, world):
    W, H, tile, spp = 45, 38, 8, 2
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, tile, spp, out), nprocs=world, join=True)
    frame = np.load(out)
    import pyoracle
    from conftest import load_fixture
    ref, _ = pyoracle.image(load_fixture("CBgems").desc(), W, H, spp, max_bounces=4, tile=tile)
    assert np.array_equal(frame[..., :3], ref[..., :3])


def test_owned_pixels_partition():
    W, H, tile = 100, 37, 16
    seen = np.concatenate([ptdist.owned_pixels(W, H, tile, r, 5) for r in range(5)])
    assert sorted(seen.tolist()) == list(range(W * H))


def _worker_frames(rank, world, port, out_path):
    """Two frames through the cached gather layout: the second frame's result
    must not keep anything of the first (reused send / receive buffers)."""
    import sys
    sys.path[:0] = [str(ROOT / "cuda-raytracer_amd")]
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    W, H, tile = 37, 29, 8
    frames = []
    for f in range(2):
        idx = ptdist.owned_pixels(W, H, tile, rank, world)
        vals = (idx.astype(np.float32) + 1000.0 * f)[:, None] * np.array([1, 2, 3, 4], np.float32)
        frame = ptdist.gather_frame(torch.from_numpy(vals), W, H, tile, spp=2)
        if rank == 0:
            frames.append(frame.numpy().copy())
    if rank == 0:
        np.save(out_path, np.stack(frames))
    dist.destroy_process_group()


def test_gather_layout_reused_across_frames(tmp_path):
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker_frames, args=(3, _free_port(), out), nprocs=3, join=True)
    frames = np.load(out)
    pix = np.arange(37 * 29, dtype=np.float32).reshape(29, 37)
    for f in range(2):
        v = pix + 1000.0 * f
        assert np.array_equal(frames[f][..., 0], v / 2)
        assert np.array_equal(frames[f][..., 2], 3 * v / 2)
        assert np.all(frames[f][..., 3] == 1.0)


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N launches N ranks itself, but not onto GPUs that are
    not there (no GPU in this container)."""
    import subprocess
    import sys
    from conftest import ROOT, have_gpu
    if have_gpu():
        pytest.skip("GPU box: covered by test_gpu_regress.py")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr
