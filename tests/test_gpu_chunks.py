"""Multi-chunk frames.  pt_render splits a frame of
npix x spp paths into chunks of floor(chunk_paths / npix) samples; each
chunk's per-path radiance is summed into the owned pixels' accumulators in
sample order, so the image cannot depend on the chunking -- the property the
reference's renderAccumulate gives across frames (cudaRenderer.cu:2419-2457:
accumulate one frame's samples after the previous frame's).  PT_CHUNK_PATHS
(read at pt_create) shrinks the chunk so the oracle-sized renders here cross
chunks, on the single-leaf path (CBempty) and the wavefront path (CBbunny,
the dragon proxy), including a ragged last chunk; and config 5's own size
(2048x2048, 1024 spp: 16 chunks of 2^28 paths) is checked against the oracle
on every 512th tile, with its eight 1/8 tile shares (the per-GPU work at 8
GPUs) against the whole frame."""
import os

import numpy as np
import pytest

import ptrace
import pyoracle

pytestmark = pytest.mark.gpu
SEED = 15618


def _scene(name):
    import scenes
    return scenes.load(name)


def _ctx_with_env(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return ptrace.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _ctx_with_chunk(chunk):
    return _ctx_with_env(PT_CHUNK_PATHS=chunk)


@pytest.fixture(scope="module")
def chunk_ctxs(gpu_ctx):
    # W x H = 96 x 80 = 7680 pixels: chunks of 4 samples (4 chunks at 16 spp),
    # of 5 samples (5, 5, 5, 1: a ragged last chunk) and of one sample with a
    # chunk smaller than the frame (16 chunks)
    npix = 96 * 80
    ctxs = {k: _ctx_with_chunk(c) for k, c in (("4", 4 * npix), ("5", 5 * npix + 17), ("1", npix // 3))}
    yield ctxs
    for c in ctxs.values():
        c.close()


@pytest.mark.parametrize("name", ["CBempty", "CBbunny", "dragon_proxy"])
def test_multi_chunk_frame_bit_exact(gpu_ctx, chunk_ctxs, name):
    W, H, SPP, B = 96, 80, 16, 8
    sc = _scene(name)
    d = sc.desc()
    o, orays = pyoracle.image(d, W, H, SPP, max_bounces=B, seed=SEED, threads=16)
    gpu_ctx.load_scene(sc)
    gpu_ctx.clear()
    gpu_ctx.render(W, H, SPP, max_bounces=B, seed=SEED)
    one = gpu_ctx.get_image()
    assert np.array_equal(one[..., :3], o[..., :3])
    for key, ctx in chunk_ctxs.items():
        ctx.load_scene(sc)
        ctx.reset_stats()
        ctx.clear()
        ctx.render(W, H, SPP, max_bounces=B, seed=SEED)
        g = ctx.get_image()
        bad = np.argwhere(g[..., :3] != o[..., :3])
        assert len(bad) == 0, f"{name} chunk {key}: {len(bad)} values differ, max {np.abs(g - o).max()}"
        assert ctx.stats().rays == orays
        assert np.isfinite(g).all() and o[..., :3].mean() > 1e-3


@pytest.mark.parametrize("name", ["CBempty", "CBbunny"])
def test_async_frames_across_chunks(gpu_ctx, chunk_ctxs, name):
    """PT_FLAG_ASYNC (the bench's timed frames): a single-leaf launch's per-path
    results are summed by the next launch's leading workgroups (two result
    buffers alternate; pt_clear switches accumulation buffers while sums or
    images are pending; an image waits for its sums) -- progressive renders
    (two calls, 6 + 10 samples) and a cleared second frame, queued back to
    back with their image copies, equal the synchronous renders bit for bit,
    on every chunking, with 8 leading workgroups and with none (a k_accum per
    launch); the wavefront renderer (CBbunny) ignores the flag.  The counters
    read after the queued frames cover all of them."""
    import torch
    W, H, B = 96, 80, 8
    sc = _scene(name)
    gpu_ctx.load_scene(sc)
    want, rays = [], []
    for seed in (SEED, 7):
        gpu_ctx.reset_stats()
        gpu_ctx.clear()
        gpu_ctx.render(W, H, 6, max_bounces=B, seed=seed)
        gpu_ctx.render(W, H, 10, max_bounces=B, seed=seed, sample_offset=6)
        want.append(gpu_ctx.get_image())
        rays.append(gpu_ctx.stats().rays)
    A = ptrace.PT_FLAG_ASYNC
    extra = [("acc8", _ctx_with_env(PT_ACC_BLOCKS=8)), ("acc0", _ctx_with_env(PT_ACC_BLOCKS=0))]
    for key, ctx in [("1chunk", gpu_ctx)] + list(chunk_ctxs.items()) + extra:
        ctx.load_scene(sc)
        ctx.clear()
        ctx.render(W, H, 16, max_bounces=B, seed=SEED)  # (camera culling, framebuffer: set up synchronously)
        ctx.reset_stats()
        bufs = [torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True) for _ in range(3)]
        for k, seed in enumerate((SEED, 7, SEED)):
            ctx.clear()
            ctx.render(W, H, 6, max_bounces=B, seed=seed, flags=A)
            ctx.render(W, H, 10, max_bounces=B, seed=seed, sample_offset=6, flags=A)
            ctx.get_image_async(bufs[k])
        ctx.wait_image()
        for k, w in enumerate((0, 1, 0)):
            bad = np.argwhere(bufs[k].numpy() != want[w])
            assert len(bad) == 0, f"{name} {key} frame {k}: {len(bad)} values differ"
        assert ctx.stats().rays == 2 * rays[0] + rays[1]  # (pt_get_stats waits for the queued frames)
        ctx.sync()
        assert ctx.samples() == 16
    for _, ctx in extra:
        ctx.close()
    assert not np.array_equal(want[0], want[1])


def test_async_images_between_progressive_renders(gpu_ctx):
    """An image requested while its frame's sums are pending (PT_FLAG_ASYNC)
    shows the samples rendered when it was requested, not those of a later
    progressive render into the same accumulation buffer; three requests in
    a row (two wait at most, the third flushes the sums) give the same
    frame."""
    import torch
    W, H, B = 96, 80, 8
    gpu_ctx.load_scene(_scene("CBempty"))
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 6, max_bounces=B, seed=SEED)
    img6 = gpu_ctx.get_image()
    gpu_ctx.render(W, H, 10, max_bounces=B, seed=SEED, sample_offset=6)
    img16 = gpu_ctx.get_image()
    A = ptrace.PT_FLAG_ASYNC
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True) for _ in range(5)]
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 6, max_bounces=B, seed=SEED, flags=A)
    gpu_ctx.get_image_async(bufs[0])
    gpu_ctx.render(W, H, 10, max_bounces=B, seed=SEED, sample_offset=6, flags=A)
    for b in bufs[1:4]:
        gpu_ctx.get_image_async(b)
    gpu_ctx.clear()  # (the next frame's buffer: the pending images keep theirs)
    gpu_ctx.render(W, H, 6, max_bounces=B, seed=SEED, flags=A)
    gpu_ctx.get_image_async(bufs[4])
    gpu_ctx.wait_image()
    assert np.array_equal(bufs[0].numpy(), img6)
    for b in bufs[1:4]:
        assert np.array_equal(b.numpy(), img16)
    assert np.array_equal(bufs[4].numpy(), img6)
    assert not np.array_equal(img6, img16)


def test_multi_chunk_wavefront_with_batches(chunk_ctxs):
    """A small path pool (several shade workgroups' regeneration plus the tail
    compaction in every chunk) across chunks: same pixels as the oracle."""
    W, H, SPP, B = 96, 80, 12, 8
    sc = _scene("CBbunny")
    o, _ = pyoracle.image(sc.desc(), W, H, SPP, max_bounces=B, seed=SEED, threads=16)
    ctx = chunk_ctxs["5"]
    ctx.load_scene(sc)
    ctx.clear()
    ctx.render(W, H, SPP, max_bounces=B, seed=SEED, batch_paths=8192)
    assert np.array_equal(ctx.get_image()[..., :3], o[..., :3])


def _owned_mask(W, H, tile, k):
    ntx = (W + tile - 1) // tile
    r = np.arange(H)[:, None] // tile
    c = np.arange(W)[None, :] // tile
    return ((r * ntx + c) % k) == 0


def test_config5_fullsize_frame(gpu_ctx):
    """BASELINE config 5 at its own size on one GPU: the dragon proxy at
    2048x2048, 1024 spp, 8 bounces (2^32 paths = 16 chunks of 2^28).  The
    oracle renders every 512th 32x32 tile (8 tiles, 8 M paths); those pixels
    agree bit for bit, and the same tiles alone on the GPU cast the oracle's
    rays.  Each of the eight 1/8 tile shares (what one rank renders at 8 GPUs)
    gives the whole frame's pixels on its tiles, and their ray counts add up
    to the whole frame's."""
    W = H = 2048
    SPP, B, TILE, K = 1024, 8, 32, 512
    sc = _scene("dragon_proxy")
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    gpu_ctx.reset_stats()
    gpu_ctx.clear()
    gpu_ctx.render(W, H, SPP, max_bounces=B, seed=SEED)
    whole_rays = gpu_ctx.stats().rays
    g = gpu_ctx.get_image()
    assert np.isfinite(g).all() and g[..., :3].mean() > 1e-3
    o, orays = pyoracle.image(d, W, H, SPP, max_bounces=B, seed=SEED, tile=TILE, rank=0, nranks=K, threads=16)
    m = _owned_mask(W, H, TILE, K)
    assert m.sum() == 8 * TILE * TILE
    bad = np.argwhere(g[m][:, :3] != o[m][:, :3])
    assert len(bad) == 0, f"{len(bad)} values differ, max {np.abs(g[m] - o[m]).max()}"
    gpu_ctx.reset_stats()
    gpu_ctx.clear()
    gpu_ctx.render(W, H, SPP, max_bounces=B, seed=SEED, tile_size=TILE, rank=0, nranks=K)
    assert gpu_ctx.stats().rays == orays
    share_rays = 0
    for r in range(8):
        gpu_ctx.reset_stats()
        gpu_ctx.clear()
        gpu_ctx.render(W, H, SPP, max_bounces=B, seed=SEED, tile_size=TILE, rank=r, nranks=8)
        share_rays += gpu_ctx.stats().rays
        ntx = W // TILE
        t = (np.arange(H)[:, None] // TILE) * ntx + np.arange(W)[None, :] // TILE
        ms = (t % 8) == r
        assert np.array_equal(gpu_ctx.get_image()[ms], g[ms]), f"share {r}"
    assert share_rays == whole_rays


@pytest.mark.parametrize("name", ["bunny", "CBbunny"])
def test_camera_ray_culling(gpu_ctx, name):
    """pt_render leaves out of the path space the pixels whose camera rays
    provably miss the root box (pt_device.hip cull_rect: the box's projection
    widened by 4 pixels) and counts their rays as cast: the frame and the ray
    count equal an unculled render (PT_CULL=0) and the oracle's bit for bit.
    bunny.dae (an open scene) culls most of its frame, the Cornell box the
    margins around its open front."""
    W, H, SPP, B = 160, 120, 4, 8
    sc = _scene(name)
    o, orays = pyoracle.image(sc.desc(), W, H, SPP, max_bounces=B, seed=SEED, threads=16)
    old = os.environ.get("PT_CULL")
    os.environ["PT_CULL"] = "0"
    try:
        nc = ptrace.Context(0)
    finally:
        if old is None:
            del os.environ["PT_CULL"]
        else:
            os.environ["PT_CULL"] = old
    try:
        out = []
        for ctx in (gpu_ctx, nc):
            ctx.load_scene(sc)
            ctx.reset_stats()
            ctx.clear()
            ctx.render(W, H, SPP, max_bounces=B, seed=SEED)
            out.append((ctx.get_image(), ctx.stats()))
    finally:
        nc.close()
    (g, st), (g0, st0) = out
    assert np.array_equal(g[..., :3], o[..., :3]) and np.array_equal(g0[..., :3], o[..., :3])
    assert st.rays == orays and st0.rays == orays and st0.culled_rays == 0
    assert 0 < st.culled_rays < W * H * SPP
    if name == "bunny":
        assert st.culled_rays > W * H * SPP // 4, st.culled_rays
