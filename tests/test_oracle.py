"""The CPU oracle pinned: Philox known-answer vectors, sampling math, BVH walk ==
brute force, tmax/tie semantics, thread-count independence and a committed
golden render (regression pin of the oracle itself)."""
import math

import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import ROOT, load_fixture
from rays import camera_rays, interior_rays

GOLDEN = ROOT / "tests" / "golden"


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert pyoracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert pyoracle.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert pyoracle.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_sincos2pi_accuracy():
    for u in np.linspace(0, 1, 4097, endpoint=False, dtype=np.float32):
        s, c = pyoracle.sincos2pi(float(u))
        assert abs(s - math.sin(2 * math.pi * float(u))) < 2e-7
        assert abs(c - math.cos(2 * math.pi * float(u))) < 2e-7


@pytest.mark.parametrize("name", ["CBempty", "CBspheres", "CBgems", "CBcoil", "CBbunny"])
def test_bvh_walk_equals_brute_force(name):
    d = load_fixture(name).desc()
    rays = np.concatenate([camera_rays(d, 1500, seed=3), interior_rays(d, 1500, seed=4),
                           interior_rays(d, 500, seed=5, tmax=0.3)])
    b = pyoracle.intersect(d, rays, use_bvh=False)
    v = pyoracle.intersect(d, rays, use_bvh=True)
    assert np.array_equal(b, v)
    assert (b != ptrace.PT_HIT_NONE).mean() > 0.3


def test_tmax_is_inclusive():
    d = load_fixture("CBcoil").desc()
    r = np.array([[0, 0.75, 3, np.inf, 0, 0, -1, 0]], np.float32)
    t = ptrace.hit_t(pyoracle.intersect(d, r))[0]
    r[0, 3] = t
    assert ptrace.hit_t(pyoracle.intersect(d, r))[0] == t
    r[0, 3] = np.nextafter(t, np.float32(0))
    assert pyoracle.intersect(d, r)[0] == ptrace.PT_HIT_NONE


def test_render_thread_independent_and_progressive():
    d = load_fixture("CBgems").desc()
    a, ra = pyoracle.render(d, 24, 20, 3, max_bounces=6, threads=1)
    b, rb = pyoracle.render(d, 24, 20, 3, max_bounces=6, threads=8)
    assert np.array_equal(a, b) and ra == rb
    # per-pixel sums are sums over samples: s[0:3] == s[0:1] + s[1:3] is NOT
    # bitwise (fp association), but the samples themselves are independent:
    c1, _ = pyoracle.render(d, 24, 20, 1, max_bounces=6, sample_offset=2)
    c2, _ = pyoracle.render(d, 24, 20, 1, max_bounces=6, sample_offset=2, threads=3)
    assert np.array_equal(c1, c2)


def test_golden_render_regression():
    g = np.load(GOLDEN / "render_CBgems_16x16x2.npz", allow_pickle=False)
    d = load_fixture("CBgems").desc()
    sums, rays = pyoracle.render(d, 16, 16, 2, max_bounces=8, seed=15618)
    assert int(g["rays"]) == rays
    assert np.array_equal(g["sums"], sums)


def gems_glass_as_mirror():
    """(CBgems, CBgems with every glass BSDF replaced by the MirrorBSDF the
    reference's reinterpret_cast reads: reflectance (roughness, refl.r,
    refl.g), bsdf.h:138-139 against bsdf.h:206-210)."""
    sc = load_fixture("CBgems")
    mir = ptrace.ArrayScene(dict(sc.a))
    sz = ptrace.C.sizeof(ptrace.pt_bsdf)
    raw = bytearray(sc.a["bsdfs"].tobytes())
    nglass = 0
    for i in range(len(raw) // sz):
        b = ptrace.pt_bsdf.from_buffer(raw, i * sz)
        if b.type == ptrace.PT_BSDF_GLASS:
            r, g = b.albedo[0], b.albedo[1]
            b.albedo[0], b.albedo[1], b.albedo[2] = b.roughness, r, g
            b.type = ptrace.PT_BSDF_MIRROR
            nglass += 1
    assert nglass == 3
    mir.a["bsdfs"] = np.frombuffer(bytes(raw), dtype=np.uint8).copy()
    return sc, mir


def test_oracle_ref_arith_glass_reads_as_mirror():
    """PT_FLAG_REF_ARITH (cu:1713-1719): the oracle renders CBgems' glass as
    the reference's mirror cast -- the same frame as a scene whose glass
    BSDFs are those mirrors; with roughness 0 (every media file) the red
    channel of a glass bounce is 0."""
    sc, mir = gems_glass_as_mirror()
    a, ra = pyoracle.render(sc.desc(), 24, 20, 2, max_bounces=8, flags=ptrace.PT_FLAG_REF_ARITH, threads=4)
    b, rb = pyoracle.render(mir.desc(), 24, 20, 2, max_bounces=8, flags=ptrace.PT_FLAG_REF_ARITH, threads=4)
    assert np.array_equal(a, b) and ra == rb
    c, _ = pyoracle.render(sc.desc(), 24, 20, 2, max_bounces=8, threads=4)
    assert not np.array_equal(a, c)


def test_fixture_bsdf_roughness():
    """Fixtures carry the COLLADA <roughness> of glass (pt_bsdf.roughness):
    0 in every reference media file; pre-roughness (32-byte) records load
    with roughness 0."""
    sc = load_fixture("CBgems")
    d = sc.desc()
    kinds = [d.bsdfs[i].type for i in range(d.n_bsdfs)]
    assert kinds.count(ptrace.PT_BSDF_GLASS) == 3
    assert all(d.bsdfs[i].roughness == 0.0 for i in range(d.n_bsdfs))
    old = dict(sc.a)
    n = d.n_bsdfs
    old["bsdfs"] = sc.a["bsdfs"].reshape(n, -1)[:, :32].reshape(-1).copy()
    del old["bsdf_size"]
    up = ptrace._upgrade_bsdfs(old)
    assert np.array_equal(up["bsdfs"], sc.a["bsdfs"])


def test_oracle_quirk_modes():
    """Reference-quirk modes of the oracle (SURVEY §8(a) parity decisions)."""
    d = load_fixture("CBempty").desc()
    W = H = 12
    base, r0 = pyoracle.render(d, W, H, 1, max_bounces=8, threads=4)
    drop, r1 = pyoracle.render(d, W, H, 1, max_bounces=8, threads=4, flags=ptrace.PT_FLAG_REF_DROP_ON_MISS)
    # (i): a sample either keeps its radiance or (its path escaped) is dropped
    same = np.all(drop[..., :3] == base[..., :3], axis=-1)
    zero = np.all(drop[..., :3] == 0.0, axis=-1)
    assert np.all(same | zero) and r1 == r0 and zero.sum() > 0
    # (vi): 2 bounces with NEE samples 2, 2, 1; max_bounces is ignored
    a, ra = pyoracle.render(d, W, H, 1, max_bounces=8, threads=4, flags=ptrace.PT_FLAG_REF_SCHEDULE)
    b, rb = pyoracle.render(d, W, H, 1, max_bounces=1, threads=4, flags=ptrace.PT_FLAG_REF_SCHEDULE)
    assert np.array_equal(a, b) and ra == rb
    assert ra <= W * H * (3 + 5)  # 3 extension rays + 2 + 2 + 1 shadow rays per path at most
    assert not np.array_equal(a, base)


def test_ref_arith_oracle_consistent():
    """PT_FLAG_REF_ARITH in the oracle: the literal triangle test's BVH walk
    equals its brute force, it finds the same primitives as the default
    Baldwin-Weber form on generic rays, and a full reference-mode render is finite."""
    import ptrace
    from conftest import load_fixture
    from rays import camera_rays, edge_rays, interior_rays
    RA = ptrace.PT_FLAG_REF_ARITH
    for name in ["CBempty", "CBbunny"]:
        d = load_fixture(name).desc()
        rays = np.concatenate([camera_rays(d, 3000, seed=5), interior_rays(d, 3000, seed=6)])
        a = pyoracle.intersect(d, rays, use_bvh=True, flags=RA)
        assert np.array_equal(a, pyoracle.intersect(d, rays, use_bvh=False, flags=RA))
        b = pyoracle.intersect(d, rays, use_bvh=True)
        assert np.array_equal(ptrace.hit_prim(a), ptrace.hit_prim(b))
        e = edge_rays(d, 2000, seed=4)
        assert np.array_equal(pyoracle.intersect(d, e, use_bvh=True, flags=RA),
                              pyoracle.intersect(d, e, use_bvh=False, flags=RA))
        flags = RA | ptrace.PT_FLAG_REF_SCHEDULE | ptrace.PT_FLAG_REF_DROP_ON_MISS | ptrace.PT_FLAG_NO_EMISSION
        img, rays_cast = pyoracle.image(d, 24, 24, 2, flags=flags)
        assert np.isfinite(img).all() and img[..., :3].mean() > 0.01 and rays_cast > 24 * 24 * 2


@pytest.mark.parametrize("name", ["CBempty", "CBspheres", "CBbunny"])
def test_oracle_bvh_walk_equals_brute_force_on_grazing_rays(name):
    """The oracle's double-precision BVH walk over the guard-banded host boxes
    finds exactly the brute-force closest hit on grazing rays (walls' edges and
    vertices, sphere silhouettes)."""
    from rays import axis_aligned_tris, edge_rays, sphere_tangent_rays
    d = load_fixture(name).desc()
    rays = [edge_rays(d, 2000, seed=1, vertex_frac=0.4, prims=axis_aligned_tris(d)), edge_rays(d, 2000, seed=2)]
    if name == "CBspheres":
        rays.append(sphere_tangent_rays(d, 2000, seed=3))
    rays = np.concatenate(rays)
    assert np.array_equal(pyoracle.intersect(d, rays, use_bvh=True), pyoracle.intersect(d, rays, use_bvh=False))


def test_oracle_in_plane_rays_do_not_hit_at_infinity():
    """The oracle's Baldwin-Weber test (ptoracle.c pto_tri): rays lying in a
    triangle's plane never report a hit at t = inf (tests/test_gpu_regress.py
    checks the GPU against the same rays)."""
    import ptrace
    from test_gpu_regress import _in_plane_scene
    sc, rays = _in_plane_scene()
    o = pyoracle.intersect(sc.desc(), rays, use_bvh=False)
    t = ptrace.hit_t(o)
    hit = o != ptrace.PT_HIT_NONE
    assert np.isfinite(t[hit]).all()
