"""Deterministic regression tests for two memory-safety fixes of round 2, each
on a fresh context of its own (not dependent on the session context's scene
order), and the bench's own rank launcher.

* 6881d6f (host heap corruption): the root table's detached leaves of a
  scene were applied to the next scene loaded after a single-leaf scene.
  CBbunny -> CBempty -> CBbunny on one context must trace and render exactly
  as the oracle does.
* 6f3f032 (device buffer overrun): ensure_paths allocated fewer path slots
  than pt_render then launched, after a queue overflow doubled the queue
  factor on a context holding a 3-slot reference-schedule pool.  A
  reference-schedule render, then an overflowing 16.8 M-path render on the
  same context must give the fresh context's image bit for bit."""
import json
import subprocess
import sys

import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import ROOT, load_fixture
from rays import camera_rays, interior_rays

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    from conftest import have_gpu
    if not have_gpu():
        pytest.skip("no GPU")


def test_scene_reload_after_single_leaf_scene():
    ctx = ptrace.Context(0)
    try:
        for name in ("CBbunny", "CBempty", "CBbunny", "CBempty"):
            sc = load_fixture(name)
            d = sc.desc()
            ctx.load_scene(sc)
            rays = np.concatenate([camera_rays(d, 3000, seed=1), interior_rays(d, 3000, seed=2)])
            assert np.array_equal(ctx.intersect(rays), pyoracle.intersect(d, rays, use_bvh=True)), name
            ctx.clear()
            ctx.render(40, 32, 2, max_bounces=5)
            o, _ = pyoracle.image(d, 40, 32, 2, max_bounces=5)
            assert np.array_equal(ctx.get_image(), o), name
    finally:
        ctx.close()


def _soup():
    rng = np.random.default_rng(11)
    c = rng.random((3000, 1, 3), dtype=np.float32)
    return ptrace.Scene.from_triangles((c + 0.6 * (rng.random((3000, 3, 3), dtype=np.float32) - 0.5)).reshape(-1, 9))


def test_overflow_rerun_after_reference_schedule_pool():
    sc = _soup()
    W = H = 1024
    spp = 16  # 16.8 M paths: more than a 3-slot pool holds once the queue factor doubles
    ref_ctx = ptrace.Context(0)
    try:
        ref_ctx.load_scene(sc)
        ref_ctx.render(W, H, spp, max_bounces=2, seed=15618)
        ref = ref_ctx.get_image()
        assert ref_ctx.stats().queue_factor > 4  # the soup overflows the default factor
    finally:
        ref_ctx.close()
    ctx = ptrace.Context(0)
    try:
        ctx.load_scene(sc)
        ctx.render(64, 64, 2, max_bounces=2, seed=15618, flags=ptrace.PT_FLAG_REF_SCHEDULE)  # 3 ray slots per path
        ctx.clear()
        ctx.reset_stats()
        ctx.render(W, H, spp, max_bounces=2, seed=15618)
        assert ctx.stats().queue_factor > 4
        assert np.array_equal(ctx.get_image(), ref)
    finally:
        ctx.close()


def _bench(tmp_path, gpus, tag):
    out = tmp_path / f"frame{tag}.npy"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--backend", "gloo", "--steps", "1",
           "--warmup", "0", "--configs", "none", "--config5", "off", "--ref-arith", "none", "--no-cpu",
           "--no-1spp", "--width", "96", "--height", "64", "--spp", "4", "--bounces", "4", "--batch", "8192",
           "--save-frame", str(out), "--detail-out", str(tmp_path / f"detail{tag}.json")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    return line, np.load(out)


def test_rccl_gather_on_one_gpu(tmp_path):
    """The nccl (RCCL) gather path on one GPU:
    torch.distributed.run with one rank and --force-gather runs
    ptdist.local_sums_tensor into a device tensor, dist.gather over RCCL and
    the device index_copy_ into the frame; the gathered frame equals
    pt_get_image's bit for bit."""
    import socket
    one, f1 = _bench(tmp_path, 1, "1")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "frame_rccl.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "1", "--force-gather",
           "--backend", "nccl", "--steps", "1", "--warmup", "0", "--configs", "none", "--config5", "off",
           "--ref-arith", "none", "--no-cpu", "--no-1spp", "--width", "96", "--height", "64", "--spp", "4",
           "--bounces", "4", "--batch", "8192", "--save-frame", str(out), "--detail-out", str(tmp_path / "d.json")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["rays_per_frame"] == one["rays_per_frame"]
    f2 = np.load(out)
    assert np.array_equal(f1, f2) and f1[..., :3].mean() > 0


def test_bench_launches_ranks_itself(tmp_path):
    """bench.py --gpus 2 (no launcher around it) starts two ranks; both render
    their tiles and the gathered frame equals the one-rank frame bit for bit
    (gloo: both ranks share this box's GPU)."""
    one, f1 = _bench(tmp_path, 1, "1")
    two, f2 = _bench(tmp_path, 2, "2")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["rays_per_frame"] == two["rays_per_frame"]
    assert np.array_equal(f1, f2)
    assert f1[..., :3].mean() > 0


def test_origin_bound(gpu_ctx):
    """Camera and query-ray origins beyond 64x the scene's largest coordinate
    magnitude are refused (the boxes' guard band G = 2^-14 M keeps the fp32
    box test conservative to ~180x); origins inside still work."""
    sc = load_fixture("CBbunny")
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    cam = ptrace.pt_camera.from_buffer_copy(bytes(d.camera))
    cam.origin[2] = 1e4
    with pytest.raises(ptrace.PTError) as e:
        gpu_ctx.set_camera(cam)
    assert e.value.code == ptrace.PT_E_UNSUPPORTED
    rays = camera_rays(d, 100, seed=3)
    rays[7, 0] = -1e5
    with pytest.raises(ptrace.PTError) as e:
        gpu_ctx.intersect(rays)
    assert e.value.code == ptrace.PT_E_UNSUPPORTED
    rays[7, 0] = 60.0  # CBbunny's largest coordinate magnitude is ~1.5: 64 x is ~96
    assert np.array_equal(gpu_ctx.intersect(rays), pyoracle.intersect(d, rays, use_bvh=True))


@pytest.mark.parametrize("name", ["CBbunny", "CBgems"])
def test_scotty_farthest_camera(gpu_ctx, name):
    """Scotty3D's framing zooms out to max_view_distance = 20 canonical view
    distances = 15 |bbox extent| from the bbox centroid (application.cpp:
    395-408); a camera placed there is accepted by pt_set_camera
    and its frame is bit-exact against the oracle."""
    sc = load_fixture(name)
    d = sc.desc()
    q = sc.a["prims"]
    tri = (q[:, 3].view(np.uint32) >> 28) == 0
    v = q[tri][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].reshape(-1, 3).astype(np.float64)
    lo, hi = v.min(0), v.max(0)
    canonical = np.linalg.norm(hi - lo) / 2 * 1.5
    cam, _, _ = ptrace.scotty_camera_place(50.0, 35.0, 64, 48, (lo + hi) / 2, 0.9, 0.4, 20 * canonical,
                                           0.0, 20 * canonical, [[0.5, 0.5]])
    gpu_ctx.load_scene(sc)
    gpu_ctx.set_camera(cam)
    gpu_ctx.render(64, 48, 2, max_bounces=4, seed=15618)
    g = gpu_ctx.get_image()
    d.camera = cam
    o, _ = pyoracle.image(d, 64, 48, 2, max_bounces=4, seed=15618)
    assert np.array_equal(g[..., :3], o[..., :3])


def _in_plane_scene():
    """Axis-aligned right triangles in the planes z = 0, y = 0.5 and x = 0.25,
    and rays lying in or parallel to those planes (W.d = 0: t = NaN or +-inf;
    with t = +inf and the ray's tmax = inf, the ordered inside test of round 3's
    first Baldwin-Weber build took u = inf, v = NaN for a hit at t = inf)."""
    P = np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0],
                  [1, 1, 0, 0, 1, 0, 1, 0, 0],
                  [0, 0.5, 0, 1, 0.5, 0, 0, 0.5, 1],
                  [0.25, 0, 0, 0.25, 1, 0, 0.25, 0, 1]], np.float32)
    bsdf = ptrace.pt_bsdf()
    bsdf.type = ptrace.PT_BSDF_DIFFUSE
    sc = ptrace.Scene.from_mesh(P, [bsdf], tri_bsdf=np.zeros(len(P), np.int32))
    rays = []
    for o, d in [((-1, 0.25, 0), (1, 0, 0)), ((0.3, -1, 0), (0, 1, 0)), ((-1, -1, 0), (0.6, 0.8, 0)),
                 ((-1, 0.5, 0.3), (1, 0, 0)), ((0.2, 0.5, -1), (0, 0, 1)), ((0.25, -1, 0.5), (0, 1, 0)),
                 ((0.25, 0.3, -1), (0, 0, 1)), ((0.25, 0.0, 0.0), (0, 0.6, 0.8)),
                 # parallel to a plane just off it: t = +inf on one side
                 ((-1, 0.25, -0.3), (1, 0, 0)), ((-1, 0.25, 0.3), (1, 0, 0)), ((0.3, -1, -0.2), (0, 1, 0)),
                 ((0.2, 0.3, -1), (0, 0, 1)), ((0.2, 0.7, -1), (0, 0, 1)), ((0.05, -1, 0.5), (0, 1, 0)),
                 ((0.45, -1, 0.5), (0, 1, 0))]:
        rays.append([*o, np.inf, *d, 0.0])
    return sc, np.array(rays, np.float32)


def test_rays_in_a_triangle_plane_miss_it(gpu_ctx):
    """A ray lying in a triangle's plane has no plane hit (the reference
    rejects |N.d| < 1e-6, cu:230): the Baldwin-Weber test's t = +-inf / NaN
    must not become a hit at t = inf (unordered inside test, trace.hip
    bw_test), on the GPU and in the oracle alike."""
    sc, rays = _in_plane_scene()
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    o = pyoracle.intersect(d, rays, use_bvh=False)
    assert np.array_equal(gpu_ctx.intersect(rays), o)
    t = ptrace.hit_t(o)
    assert not np.isinf(t[o != ptrace.PT_HIT_NONE]).any()


@pytest.mark.parametrize("batch", [None, 700])
def test_tail_compaction_matches_oracle(batch, monkeypatch):
    """Tail compaction (k_shade_push with ShadeArgs::compact, then passes over
    the compacted slots): a context with it (the default) and one without
    (PT_COMPACT=0, read at pt_create) give the oracle's image and ray count,
    with the default schedule and the reference schedule (two shadow-ray slots
    per path), in one chunk and in many small ones (batch_paths=700)."""
    sc = load_fixture("CBbunny")
    d = sc.desc()
    W, H, SPP = 48, 40, 3
    kw = {} if batch is None else {"batch_paths": batch}
    for flags in (0, ptrace.PT_FLAG_REF_SCHEDULE):
        o, orays = pyoracle.image(d, W, H, SPP, max_bounces=8, seed=15618, flags=flags)
        for comp in ("2", "0"):
            monkeypatch.setenv("PT_COMPACT", comp)
            ctx = ptrace.Context(0)
            try:
                ctx.load_scene(sc)
                ctx.reset_stats()
                ctx.render(W, H, SPP, max_bounces=8, seed=15618, flags=flags, **kw)
                assert np.array_equal(ctx.get_image(), o), (flags, comp)
                assert ctx.stats().rays == orays, (flags, comp)
            finally:
                ctx.close()


def test_fast_sqrt_rcp_are_ieee(gpu_ctx):
    """sqrt_rn and rcp_rn (ptmath.h: the hardware approximations plus one
    correction, without the IEEE sequences' range scaling) give the IEEE
    results bit for bit on every fp32 input of the ranges their call sites
    are restricted to: sqrt_rn for 0 and every x >= 2^-96 up to +inf, rcp_rn
    for |b| in [2^-100, 2^100] (exhaustive, ~1.9 G patterns each, on the
    device against the compiler's correctly rounded sqrtf and 1/b).  Below
    2^-96 sqrt_rn does differ (which is why the IEEE sequence pre-scales)."""
    ok = [(0, 0x00000000, 0x00000001), (0, 0x0F800000, 0x7F800001),
          (1, 0x0D800000, 0x71800001), (1, 0x8D800000, 0xF1800001)]
    for which, lo, hi in ok:
        n, first = gpu_ctx.check_fast_math(which, lo, hi)
        assert n == 0, (which, hex(lo), hex(hi), n, hex(first))
    n, _ = gpu_ctx.check_fast_math(0, 0x00800000, 0x0F800000)  # (normal inputs below 2^-96)
    assert n > 0


def test_triangle_test_division_is_ieee(gpu_ctx):
    """The Baldwin-Weber test divides without the IEEE sequence's range
    scaling and fixup (trace.hip div_rn): over 20 M operand pairs spanning the
    magnitudes a scene produces (|num| in [2^-60, 2^40], |den| in [2^-60, 2^4],
    both signs) every quotient equals IEEE division bit for bit; a zero
    numerator gives a zero of either sign (bw_test returns t + 0, so the sign
    of a zero t never leaves it); for den = 0 (a ray parallel to the plane) it
    gives NaN or an infinity, which the test treats as a miss like IEEE's
    infinity."""
    rng = np.random.default_rng(5)
    n = 20_000_000
    num = (rng.uniform(1, 2, n) * np.exp2(rng.integers(-60, 41, n)) * rng.choice([-1, 1], n)).astype(np.float32)
    den = (rng.uniform(1, 2, n) * np.exp2(rng.integers(-60, 5, n)) * rng.choice([-1, 1], n)).astype(np.float32)
    num[:1000] = 0.0
    num[1000:2000] = -0.0
    q = gpu_ctx.check_division(num, den)
    with np.errstate(all="ignore"):
        ref = num / den
    nz = num != 0
    assert np.array_equal(q[nz].view(np.uint32), ref[nz].view(np.uint32))
    assert np.all(q[~nz] == 0.0)
    z = gpu_ctx.check_division(np.array([1.0, -1.0, 0.0], np.float32), np.zeros(3, np.float32))
    assert np.all(np.isnan(z) | np.isinf(z))
    # small numerators: down to |num| = 2^-100 the residuals stay
    # normal and every quotient is IEEE's; below that (|num| in [2^-126,
    # 2^-101]: the fma residuals are subnormal) a quotient may differ from
    # IEEE's -- by at most one ulp.  That band is a t below ~2^-96 at a unit
    # ray (an origin on the plane to 29 decimal places): not pinned.
    m = 4_000_000
    num = (rng.uniform(1, 2, m) * np.exp2(rng.integers(-100, -59, m)) * rng.choice([-1, 1], m)).astype(np.float32)
    den = (rng.uniform(1, 2, m) * np.exp2(rng.integers(-60, 5, m)) * rng.choice([-1, 1], m)).astype(np.float32)
    q = gpu_ctx.check_division(num, den)
    assert np.array_equal(q.view(np.uint32), (num / den).view(np.uint32))
    num = (rng.uniform(1, 2, m) * np.exp2(rng.integers(-126, -100, m)) * rng.choice([-1, 1], m)).astype(np.float32)
    den = (rng.uniform(1, 2, m) * np.exp2(rng.integers(-4, 5, m)) * rng.choice([-1, 1], m)).astype(np.float32)
    q = gpu_ctx.check_division(num, den)
    with np.errstate(all="ignore"):
        ref = num / den
    ulps = np.abs(q.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1, ulps.max()
    # the camera's pixel coordinate over the image size (shade.hip camera_dir):
    # num in {0} U [2^-24, 2^15], den an image size in [1, 2^15]
    num = (rng.uniform(1, 2, m) * np.exp2(rng.integers(-24, 15, m))).astype(np.float32)
    num[:1000] = 0.0
    den = rng.integers(1, 1 << 15, m).astype(np.float32)
    q = gpu_ctx.check_division(num, den)
    assert np.array_equal(q.view(np.uint32), (num / den).view(np.uint32))


def _bench_c5(tmp_path, gpus, tag):
    """bench.py with BASELINE config 5's branch at a small size (--config5-size)."""
    out, out5 = tmp_path / f"h{tag}.npy", tmp_path / f"c5_{tag}.npy"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--backend", "gloo", "--steps", "1",
           "--warmup", "0", "--configs", "none", "--config5", "on", "--config5-size", "96x64x3", "--tile", "8",
           "--ref-arith", "none", "--no-cpu", "--no-1spp", "--width", "64", "--height", "48", "--spp", "2",
           "--bounces", "4", "--batch", "8192", "--save-frame", str(out), "--save-config5", str(out5),
           "--detail-out", str(tmp_path / f"detail{tag}.json")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    return line, np.load(out), np.load(out5)


def test_bench_eight_ranks_config5_branch(tmp_path):
    """bench.py --gpus 8 runs BASELINE config 5's 8-rank branch (tiles over
    all ranks + the gather), here over gloo with the eight
    ranks sharing this box's GPU and config 5 shrunk to 96x64x3 on the
    dragon proxy: the gathered config-5 frame equals one GPU's whole frame of
    the same workload (the world-1 branch), and the headline frame the
    world-1 headline, bit for bit."""
    one, h1, c1 = _bench_c5(tmp_path, 1, "1")
    eight, h8, c8 = _bench_c5(tmp_path, 8, "8")
    assert one["n_gpus"] == 1 and eight["n_gpus"] == 8
    cfg8 = [c for c in eight["configs"] if c["scene"] == "dragon_proxy"]
    assert len(cfg8) == 1 and "tiles over all ranks + gloo gather" in cfg8[0]["config"]
    whole1 = [c for c in one["configs"] if c["scene"] == "dragon_proxy" and "whole" in c["config"]]
    assert len(whole1) == 1
    assert cfg8[0]["value"] > 0 and one["rays_per_frame"] == eight["rays_per_frame"]
    assert c1.shape == (64, 96, 4) and c1[..., :3].mean() > 0
    assert np.array_equal(h1, h8)
    assert np.array_equal(c1, c8)


def test_async_image_overlaps_next_frame(gpu_ctx):
    """pt_get_image_async (the bench's frame readback): the copy of frame A
    is queued, frame B is cleared and rendered while it may still run, and
    after pt_wait_image both host buffers hold exactly what the synchronous
    pt_get_image returns for each frame (the copy reads a staged frame of its
    own, two alternate, so the next clear / render cannot change it)."""
    import torch
    gpu_ctx.load_scene(load_fixture("CBgems"))
    W, H = 160, 96
    want = []
    for spp, seed in ((3, 15618), (2, 7)):
        gpu_ctx.clear()
        gpu_ctx.render(W, H, spp, max_bounces=6, seed=seed)
        want.append(gpu_ctx.get_image())
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True) for _ in range(3)]
    for k, (spp, seed) in enumerate(((3, 15618), (2, 7), (3, 15618))):
        gpu_ctx.clear()
        gpu_ctx.render(W, H, spp, max_bounces=6, seed=seed)
        gpu_ctx.get_image_async(bufs[k])
    gpu_ctx.wait_image()
    assert np.array_equal(bufs[0].numpy(), want[0])
    assert np.array_equal(bufs[1].numpy(), want[1])
    assert np.array_equal(bufs[2].numpy(), want[0])
    assert not np.array_equal(want[0], want[1])
