"""GPU parity: the HIP path (libptcore.so through the C ABI) against the CPU
oracle (oracle/ptoracle.c) on the same inputs.

Bar:
  * closest hit: bit-equal {t, prim} keys on every ray;
  * images: bit-equal fp32 per pixel (the kernels and the oracle share the
    operation order, -ffp-contract=off, IEEE div/sqrt, Philox streams).  The
    documented fallback tolerance, relative L2 <= 1e-3 and |G-C| <= 1e-3*max(1,|C|)
    on >= 99.9 % of pixels, is asserted as well so a failure says which bar broke.
"""
import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import load_fixture
from rays import camera_rays, edge_rays, interior_rays

pytestmark = pytest.mark.gpu

SCENES = ["CBempty", "CBspheres", "CBgems", "CBcoil", "CBbunny"]


@pytest.mark.parametrize("name", SCENES)
def test_closest_hit_bit_exact(gpu_ctx, name):
    sc = load_fixture(name)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    rays = np.concatenate([camera_rays(d, 20000, seed=7), interior_rays(d, 20000, seed=8),
                           interior_rays(d, 5000, seed=9, tmax=0.5)])
    g = gpu_ctx.intersect(rays)
    o = pyoracle.intersect(d, rays, use_bvh=True)
    assert (o != ptrace.PT_HIT_NONE).sum() > 1000
    bad = np.nonzero(g != o)[0]
    assert len(bad) == 0, f"{len(bad)} mismatching hits, first {bad[:5]}: gpu {g[bad[:5]]} oracle {o[bad[:5]]}"
    # the oracle's BVH walk equals its brute force on a subset
    sub = rays[::97]
    assert np.array_equal(pyoracle.intersect(d, sub, use_bvh=True), pyoracle.intersect(d, sub, use_bvh=False))


@pytest.mark.parametrize("name", ["CBbunny", "CBcoil"])
def test_level_skip_off_matches(gpu_ctx, name, monkeypatch):
    """PT_NO_SKIP_L1=1 restores the root -> level-1 pass; both schedules must
    report the same closest hits (the traversal order never changes results)."""
    sc = load_fixture(name)
    d = sc.desc()
    rays = np.concatenate([camera_rays(d, 20000, seed=17), interior_rays(d, 20000, seed=18)])
    gpu_ctx.load_scene(sc)
    g_skip = gpu_ctx.intersect(rays)
    monkeypatch.setenv("PT_NO_SKIP_L1", "1")
    gpu_ctx.load_scene(sc)
    g_full = gpu_ctx.intersect(rays)
    monkeypatch.delenv("PT_NO_SKIP_L1")
    gpu_ctx.load_scene(sc)
    assert np.array_equal(g_skip, g_full)
    assert np.array_equal(g_skip, pyoracle.intersect(d, rays, use_bvh=True))


@pytest.mark.parametrize("env", [("PT_ENTRY_LEVEL", "1"), ("PT_ENTRY_LEVEL", "2"), ("PT_INLINE_MAX", "0"),
                                 ("PT_NO_ROOT_CLUSTER", "1"), ("PT_NO_ROOT_CLUSTER_SHADOW", "1")])
def test_schedule_options_match(gpu_ctx, env, monkeypatch):
    """Ray-entry queues below the root targets (PT_ENTRY_LEVEL), the root
    pass without inline leaves (PT_INLINE_MAX=0) and the inline leaves tested
    whole instead of by candidate clusters (PT_NO_ROOT_CLUSTER, for shadow
    rays only PT_NO_ROOT_CLUSTER_SHADOW) give the same closest hits and the
    same image as the default schedule."""
    sc = load_fixture("CBbunny")
    d = sc.desc()
    rays = np.concatenate([camera_rays(d, 20000, seed=27), interior_rays(d, 20000, seed=28)])
    monkeypatch.setenv(*env)
    gpu_ctx.load_scene(sc)
    g = gpu_ctx.intersect(rays)
    gpu_ctx.clear()
    gpu_ctx.render(32, 32, 2, max_bounces=6, seed=15618)
    img = gpu_ctx.get_image()
    monkeypatch.delenv(env[0])
    gpu_ctx.load_scene(sc)
    assert np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=True))
    o, _ = pyoracle.image(d, 32, 32, 2, max_bounces=6, seed=15618)
    assert np.array_equal(img, o)


def test_queue_overflow_rerun(monkeypatch):
    """A context started with the smallest queue factor (PT_QFACTOR=1) on a
    soup of large overlapping triangles overflows a level queue, abandons the
    pass and re-runs it with twice the capacity (pt_intersect and pt_render):
    hits and image still equal the oracle's."""
    rng = np.random.default_rng(11)
    c = rng.random((3000, 1, 3), dtype=np.float32)
    tris = (c + 0.6 * (rng.random((3000, 3, 3), dtype=np.float32) - 0.5)).reshape(-1, 9)
    sc = ptrace.Scene.from_triangles(tris)
    d = sc.desc()
    monkeypatch.setenv("PT_QFACTOR", "1")
    ctx = ptrace.Context(0)
    monkeypatch.delenv("PT_QFACTOR")
    try:
        ctx.load_scene(sc)
        rays = interior_rays(d, 50000, seed=41)
        g = ctx.intersect(rays)
        assert np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=True))
        assert (g != ptrace.PT_HIT_NONE).sum() > 10000
        assert ctx.stats().queue_factor > 1  # the overflow path did run
        ctx.render(32, 32, 2, max_bounces=4, seed=15618)
        o, _ = pyoracle.image(d, 32, 32, 2, max_bounces=4, seed=15618)
        assert np.array_equal(ctx.get_image(), o)
    finally:
        ctx.close()


def test_render_overflow_rerun_counts_and_queues(monkeypatch):
    """A render (not an intersect) that overflows a level queue at its first
    chunk: the passes queued behind the abandoned one have pushed rays into
    the root targets' queues, so the re-run must start from zeroed (node,
    lane) counters -- stale counts read that many stale ids from the
    reallocated queues, a memory fault when the recycled memory held floats --
    and must count only its own rays (the abandoned passes' are taken back):
    image and ray count equal the oracle's."""
    rng = np.random.default_rng(11)
    c = rng.random((3000, 1, 3), dtype=np.float32)
    tris = (c + 0.6 * (rng.random((3000, 3, 3), dtype=np.float32) - 0.5)).reshape(-1, 9)
    sc = ptrace.Scene.from_triangles(tris)
    d = sc.desc()
    monkeypatch.setenv("PT_QFACTOR", "1")
    ctx = ptrace.Context(0)
    monkeypatch.delenv("PT_QFACTOR")
    try:
        ctx.load_scene(sc)
        for k in range(2):  # (the second render runs at the doubled factor, after the first one's buffers)
            ctx.reset_stats()
            ctx.clear()
            ctx.render(64, 64, 4, max_bounces=4, seed=15618 + k)
            o, orays = pyoracle.image(d, 64, 64, 4, max_bounces=4, seed=15618 + k)
            assert np.array_equal(ctx.get_image(), o)
            assert ctx.stats().rays == orays
        assert ctx.stats().queue_factor > 1  # the overflow path did run
    finally:
        ctx.close()


def test_overflow_rerun_shrinks_large_batch(gpu_ctx):
    """A large path pool whose level queues overflow: the chunk re-runs with
    twice the queue factor, which the pool no longer fits under u32 queue
    offsets, so the batch shrinks (it used to fail with PT_E_UNSUPPORTED).
    The soup of overlapping triangles overflows the default queue factor
    twice; the image equals the default context's bit for bit."""
    rng = np.random.default_rng(11)
    c = rng.random((3000, 1, 3), dtype=np.float32)
    tris = (c + 0.6 * (rng.random((3000, 3, 3), dtype=np.float32) - 0.5)).reshape(-1, 9)
    sc = ptrace.Scene.from_triangles(tris)
    W = H = 1024
    spp, batch = 144, 150_000_000  # 151 M paths; the pool asks for 150 M slots
    gpu_ctx.load_scene(sc)
    gpu_ctx.clear()
    gpu_ctx.render(W, H, spp, max_bounces=2, seed=15618)
    ref = gpu_ctx.get_image()
    ctx = ptrace.Context(0)
    try:
        ctx.load_scene(sc)
        ctx.reset_stats()
        ctx.render(W, H, spp, max_bounces=2, seed=15618, batch_paths=batch)
        assert np.array_equal(ctx.get_image(), ref)
        st = ctx.stats()
        # the re-runs did run (queue factor 4 -> 16: a pool of 42 M slots no
        # longer fits u32 offsets at 8), with a smaller pool
        assert st.queue_factor >= 8 and st.batch_paths < 40_000_000, (st.queue_factor, st.batch_paths)
    finally:
        ctx.close()


def test_tie_break_lowest_prim(gpu_ctx):
    # two identical triangles: every hit must report the lower sorted index
    tri = np.array([[-1, -1, 0, 1, -1, 0, 0, 1, 0]] * 2, np.float32)
    rng = np.random.default_rng(0)
    extra = rng.random((100, 9), dtype=np.float32) + 5
    sc = ptrace.Scene.from_triangles(np.concatenate([tri, extra]))
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    r = np.zeros((1000, 8), np.float32)
    r[:, 0:2] = rng.random((1000, 2), dtype=np.float32) * 0.5 - 0.25
    r[:, 2] = -3
    r[:, 3] = np.inf
    r[:, 6] = 1
    g = gpu_ctx.intersect(r)
    o = pyoracle.intersect(d, r, use_bvh=False)
    assert np.array_equal(g, o)
    perm = sc.sorted_to_input()
    hit_inputs = set(perm[ptrace.hit_prim(g)[ptrace.hit_prim(g) >= 0]].tolist())
    assert len(hit_inputs) == 1


def _images_equal(gimg, oimg):
    # NaN pixels (PT_FLAG_REF_GUIDE reproduces the reference's NaN frame)
    # must be NaN on both sides; they count as equal
    gn, on = np.isnan(gimg[..., :3]), np.isnan(oimg[..., :3])
    assert np.array_equal(gn, on), "NaN pixels differ"
    gimg = np.where(gn, 0.0, gimg[..., :3])
    oimg = np.where(on, 0.0, oimg[..., :3])
    diff = np.abs(gimg[..., :3] - oimg[..., :3])
    ref = np.abs(oimg[..., :3])
    l2 = np.linalg.norm(diff) / max(np.linalg.norm(ref), 1e-30)
    frac_ok = np.mean(np.all(diff <= 1e-3 * np.maximum(1.0, ref), axis=-1))
    return float(diff.max()), float(l2), float(frac_ok)


REF = ptrace.PT_FLAG_REF_SCHEDULE | ptrace.PT_FLAG_REF_DROP_ON_MISS
# every reference-arithmetic switch (SURVEY §8(a) parity decisions; pt_api.h
# PT_FLAG_REF_ARITH): the kernels' expressions of cu:217-270, 347-354,
# 416-446, 570-653, 1205-1234 with the reference schedule and REAL_TIME
REF_FULL = REF | ptrace.PT_FLAG_REF_ARITH | ptrace.PT_FLAG_NO_EMISSION


@pytest.mark.parametrize("name,flags", [("CBbunny", 0), ("CBspheres", 0), ("CBgems", 0), ("CBempty", 0),
                                        ("CBcoil", ptrace.PT_FLAG_COSINE_DIFFUSE),
                                        # reference-quirk modes (SURVEY §8(a) parity decisions)
                                        ("CBbunny", REF), ("CBempty", REF | ptrace.PT_FLAG_NO_EMISSION),
                                        ("CBspheres", REF), ("CBcoil", ptrace.PT_FLAG_REF_GUIDE),
                                        ("CBempty", ptrace.PT_FLAG_REF_GUIDE),
                                        # reference arithmetic (PT_FLAG_REF_ARITH), alone and with
                                        # every other reference switch
                                        ("CBbunny", ptrace.PT_FLAG_REF_ARITH), ("CBcoil", ptrace.PT_FLAG_REF_ARITH),
                                        ("CBempty", ptrace.PT_FLAG_REF_ARITH), ("CBbunny", REF_FULL),
                                        ("CBcoil", REF_FULL | ptrace.PT_FLAG_REF_GUIDE), ("CBempty", REF_FULL),
                                        # glass read as the reference reads it: a MirrorBSDF cast (cu:1713-1719)
                                        ("CBgems", ptrace.PT_FLAG_REF_ARITH), ("CBgems", REF_FULL)])
def test_render_bit_exact(gpu_ctx, name, flags):
    sc = load_fixture(name)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    W = H = 48
    spp, B = 3, 8
    gpu_ctx.clear()
    gpu_ctx.render(W, H, spp, max_bounces=B, seed=15618, flags=flags)
    g = gpu_ctx.get_image()
    o, rays = pyoracle.image(d, W, H, spp, max_bounces=B, seed=15618, flags=flags)
    mx, l2, ok = _images_equal(g, o)
    assert l2 <= 1e-3 and ok >= 0.999, (mx, l2, ok)
    assert mx == 0.0, f"not bit-exact: max |diff| {mx}, rel L2 {l2}"
    assert o[..., :3].mean() > 0.01


def _sparse_soup():
    """300 small diffuse triangles scattered in a 4-unit cube under a point
    light, seen from 8 units away: most paths leave the scene early."""
    rng = np.random.default_rng(5)
    c = rng.random((300, 1, 3), dtype=np.float32) * 4.0 - 2.0
    tris = (c + 0.4 * (rng.random((300, 3, 3), dtype=np.float32) - 0.5)).reshape(-1, 9)
    b = ptrace.pt_bsdf()
    b.type = ptrace.PT_BSDF_DIFFUSE
    L = ptrace.pt_light()
    L.type = ptrace.PT_LIGHT_POINT
    cam = ptrace.pt_camera()
    for k in range(3):
        b.albedo[k] = 0.8
        L.radiance[k] = 20.0
        L.position[k] = (0.5, 3.0, 2.5)[k]
        cam.origin[k], cam.look_at[k], cam.left[k], cam.up[k] = (0, 0, 8)[k], (0, 0, -1)[k], (1, 0, 0)[k], (0, 1, 0)[k]
    return ptrace.Scene.from_mesh(tris, [b], tri_bsdf=np.zeros(len(tris), np.int32), light=L, camera=cam)


@pytest.mark.parametrize("W,H,spp", [(37, 23, 3), (61, 5, 7), (13, 11, 1)])
def test_shade_tail_workgroups_sparse_paths(gpu_ctx, W, H, spp):
    """The shade kernel's root pass reads cluster records that its loader
    waves copied into LDS (global_load_lds, counted by vmcnt): each loader
    wave waits for its copies before the barrier, also when it holds no live
    slot.  A sparse soup (most camera rays and nearly every bounce escape)
    rendered at sizes that are not multiples of the workgroup leaves each
    pass's last workgroups with loader waves and no live paths; image and ray
    count equal the oracle's."""
    sc = _sparse_soup()
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    gpu_ctx.reset_stats()
    gpu_ctx.clear()
    gpu_ctx.render(W, H, spp, max_bounces=8, seed=15618)
    o, orays = pyoracle.image(d, W, H, spp, max_bounces=8, seed=15618)
    assert np.array_equal(gpu_ctx.get_image(), o)
    assert gpu_ctx.stats().rays == orays
    assert orays > W * H * spp  # some paths do bounce


@pytest.mark.parametrize("name", ["CBempty", "CBgems", "CBcoil", "CBbunny"])
def test_closest_hit_ref_arith_bit_exact(gpu_ctx, name):
    """PT_FLAG_REF_ARITH: the literal cu:217-270 triangle test (edge tests
    dot(N, cross(e_k, P - v_k)), N and N.v0 per the reference) through the
    breadth-first traversal equals the oracle's per-call restatement, on the
    fixture rays and on rays aimed at triangle edges (where the literal and
    the default Baldwin-Weber forms disagree: see DESIGN.md §2)."""
    sc = load_fixture(name)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    rays = np.concatenate([camera_rays(d, 20000, seed=7), interior_rays(d, 20000, seed=8), edge_rays(d, 10000, seed=3)])
    g = gpu_ctx.intersect(rays, flags=ptrace.PT_FLAG_REF_ARITH)
    o = pyoracle.intersect(d, rays, use_bvh=True, flags=ptrace.PT_FLAG_REF_ARITH)
    assert (o != ptrace.PT_HIT_NONE).sum() > 1000
    bad = np.nonzero(g != o)[0]
    assert len(bad) == 0, f"{len(bad)} mismatching hits, first {bad[:5]}: gpu {g[bad[:5]]} oracle {o[bad[:5]]}"
    # the default (Baldwin-Weber) test differs from it on edge-aimed rays only
    dflt = gpu_ctx.intersect(rays)
    assert np.array_equal(dflt, pyoracle.intersect(d, rays, use_bvh=True))


def test_ref_arith_refuses_spheres(gpu_ctx):
    """The reference renders triangles only (cu:1765 casts every primitive to
    a Triangle): spheres are refused under PT_FLAG_REF_ARITH."""
    gpu_ctx.load_scene(load_fixture("CBspheres"))
    with pytest.raises(ptrace.PTError) as e:
        gpu_ctx.render(16, 16, 1, flags=ptrace.PT_FLAG_REF_ARITH)
    assert e.value.code == ptrace.PT_E_UNSUPPORTED


def test_ref_arith_glass_is_the_reference_mirror(gpu_ctx):
    """Under PT_FLAG_REF_ARITH a glass BSDF is the reference's MirrorBSDF
    reinterpret_cast (cu:1713-1719): the CBgems frame equals, bit for bit, the
    frame of the same scene with each glass BSDF replaced by a mirror of
    reflectance (roughness, reflectance.r, reflectance.g) (bsdf.h:138-139 over
    bsdf.h:206-210) -- and differs from the default glass frame."""
    from test_oracle import gems_glass_as_mirror
    sc, mir = gems_glass_as_mirror()
    W = H = 40
    imgs = []
    for s, fl in ((sc, ptrace.PT_FLAG_REF_ARITH), (mir, ptrace.PT_FLAG_REF_ARITH), (sc, 0)):
        gpu_ctx.load_scene(s)
        gpu_ctx.clear()
        gpu_ctx.render(W, H, 2, max_bounces=8, seed=15618, flags=fl)
        imgs.append(gpu_ctx.get_image())
    assert np.array_equal(imgs[0], imgs[1])
    assert not np.array_equal(imgs[0], imgs[2])


def test_dragon_proxy_parity(gpu_ctx):
    """~100k triangles, 9 levels: closest hits and a small render bit-exact."""
    import scenes
    sc = scenes.dragon_proxy()
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    rays = np.concatenate([camera_rays(d, 20000, seed=27), interior_rays(d, 20000, seed=28)])
    g = gpu_ctx.intersect(rays)
    o = pyoracle.intersect(d, rays, use_bvh=True)
    assert (o != ptrace.PT_HIT_NONE).sum() > 1000
    assert np.array_equal(g, o)
    W = H = 32
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 2, max_bounces=8, seed=15618)
    gi = gpu_ctx.get_image()
    oi, _ = pyoracle.image(d, W, H, 2, max_bounces=8, seed=15618)
    mx, l2, ok = _images_equal(gi, oi)
    assert mx == 0.0, f"not bit-exact: max |diff| {mx}, rel L2 {l2}"


def test_bunny_dae_parity(gpu_ctx):
    """bunny.dae (BASELINE config 4, 33,696 triangles): its BVH level 6 holds
    1,167 nodes -- the level that overflows the reference's per-level
    buffers.  Closest hits (default and reference arithmetic) and
    a small render (lit by CBbunny's area light, scenes.bunny_lit) bit-exact."""
    import scenes
    sc = scenes.bunny_lit()
    d = sc.desc()
    assert sc.level_counts() == [1, 4, 16, 64, 239, 780, 1167, 45]
    gpu_ctx.load_scene(sc)
    rays = np.concatenate([camera_rays(d, 20000, seed=47), interior_rays(d, 20000, seed=48), edge_rays(d, 5000)])
    o = pyoracle.intersect(d, rays, use_bvh=True)
    assert (o != ptrace.PT_HIT_NONE).sum() > 5000
    assert np.array_equal(gpu_ctx.intersect(rays), o)
    assert np.array_equal(gpu_ctx.intersect(rays, flags=ptrace.PT_FLAG_REF_ARITH),
                          pyoracle.intersect(d, rays, use_bvh=True, flags=ptrace.PT_FLAG_REF_ARITH))
    gpu_ctx.reset_stats()
    for flags in (0, REF_FULL):
        gpu_ctx.clear()
        gpu_ctx.render(40, 40, 2, max_bounces=8, seed=15618, flags=flags | ptrace.PT_FLAG_STATS)
        gi = gpu_ctx.get_image()
        oi, _ = pyoracle.image(d, 40, 40, 2, max_bounces=8, seed=15618, flags=flags)
        mx, l2, ok = _images_equal(gi, oi)
        # (the reference mode drops every path that escapes the open scene)
        assert mx == 0.0 and oi[..., :3].mean() > (0.005 if flags == 0 else 5e-4), (flags, mx, l2)
    st = gpu_ctx.stats()
    assert st.level_visits[6] > 0  # the 1,167-node level was traversed


def test_batching_and_progressive_invariance(gpu_ctx):
    sc = load_fixture("CBbunny")
    gpu_ctx.load_scene(sc)
    W = H = 40
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 6, max_bounces=5, batch_paths=W * H)  # 6 batches of 1 spp
    a = gpu_ctx.get_image()
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 6, max_bounces=5, batch_paths=W * H * 6)  # 1 batch
    b = gpu_ctx.get_image()
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 2, max_bounces=5, sample_offset=0)
    gpu_ctx.render(W, H, 4, max_bounces=5, sample_offset=2)
    c = gpu_ctx.get_image()
    assert np.array_equal(a, b)
    assert np.array_equal(a, c)


def test_tile_sharding_union(gpu_ctx):
    sc = load_fixture("CBgems")
    gpu_ctx.load_scene(sc)
    W, H = 70, 45  # ragged tiles
    full = None
    parts = []
    for rank in range(3):
        gpu_ctx.clear()
        gpu_ctx.render(W, H, 2, max_bounces=4, tile_size=16, rank=rank, nranks=3)
        parts.append(gpu_ctx.get_image())
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 2, max_bounces=4, tile_size=16)
    full = gpu_ctx.get_image()
    assert np.array_equal(sum(p[..., :3] for p in parts), full[..., :3])


@pytest.mark.parametrize("name,flags", [("CBbunny", 0), ("CBempty", 0), ("CBbunny", REF), ("CBempty", REF)])
def test_ray_count_matches_oracle(gpu_ctx, name, flags):
    sc = load_fixture(name)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    gpu_ctx.reset_stats()
    gpu_ctx.clear()
    gpu_ctx.render(32, 32, 2, max_bounces=8, flags=flags)
    st = gpu_ctx.stats()
    _, rays = pyoracle.render(d, 32, 32, 2, max_bounces=8, flags=flags)
    assert st.rays == rays
    assert st.visits >= st.rays


def test_scotty_camera_render(gpu_ctx):
    """camera=scotty framing (pt_scene_camera_scotty, fixture made from
    CBbunny.dae at 64x48): the kernels render it bit-exactly like the oracle."""
    from conftest import ROOT
    sc = load_fixture("CBbunny")
    cam = ptrace.pt_camera.from_buffer_copy(np.load(ROOT / "tests/golden/camera_scotty_CBbunny_64x48.npy").tobytes())
    gpu_ctx.load_scene(sc)
    gpu_ctx.set_camera(cam)
    gpu_ctx.clear()
    gpu_ctx.render(64, 48, 2, max_bounces=6)
    g = gpu_ctx.get_image()
    d = sc.desc()
    d.camera = cam
    o, _ = pyoracle.image(d, 64, 48, 2, max_bounces=6)
    assert np.array_equal(g, o) and o[..., :3].mean() > 0.01



@pytest.mark.parametrize("name", ["CBempty", "CBspheres"])
@pytest.mark.parametrize("chunk,regions", [(64, 1), (128, 3), (4096, 32)])
def test_path_grab_schedules_match(monkeypatch, name, chunk, regions):
    """Other path-grab schedules of the single-leaf kernel (grab size,
    path regions: PT_PATH_CHUNK / PT_PATH_REGIONS) give the oracle's image
    too: scheduling never changes a path's result, and every path is taken
    exactly once (the ray count equals the default schedule's)."""
    sc = load_fixture(name)
    d = sc.desc()
    counts = []
    for env in ({}, {"PT_PATH_CHUNK": str(chunk), "PT_PATH_REGIONS": str(regions)}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ctx = ptrace.Context(0)
        for k in env:
            monkeypatch.delenv(k)
        try:
            ctx.load_scene(sc)
            ctx.clear()
            ctx.reset_stats()
            ctx.render(48, 48, 3, max_bounces=8, seed=15618)
            o, _ = pyoracle.image(d, 48, 48, 3, max_bounces=8, seed=15618)
            assert np.array_equal(ctx.get_image(), o)
            counts.append(ctx.stats().rays)
        finally:
            ctx.close()
    assert counts[0] == counts[1]
