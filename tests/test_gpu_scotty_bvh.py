"""StaticScene::BVHAccel on the GPU (scotty/scotty_pt.h, bvh.h:111-149) and
pt_intersect's t_min (the 8th float of a ray).

BVHAccel(primitives, max_leaf_size) takes Scotty3D primitives (a Mesh's
Triangles and SphereObjects' Spheres); intersect(ray, isect) must return the
closest hit with min_t <= t <= max_t (Triangle::intersect's segment test,
triangle.cpp:187-193), the Intersection's primitive, and Triangle::intersect's
normal: the vertex normals blended with the hit's barycentric weights, flipped
toward the ray origin's side, unit length (triangle.cpp:195-202); a sphere's is
the outward normal (sphere.h).

Oracle: the brute-force closest hit of oracle/ptoracle.c over the same
flattened scene (pt_scene_from_mesh of the same fp32 arrays), the fp32 ray
with min_t rounded up and max_t rounded down (bit-exact t and primitive); the
normal from numpy fp64 (within 1e-12)."""
import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import load_fixture

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    from conftest import have_gpu
    if not have_gpu():
        pytest.skip("no GPU")


def _round_up(x):
    f = np.float32(x)
    return np.nextafter(f, np.float32(np.inf)) if np.float64(f) < x else f


def _round_down(x):
    f = np.float32(x)
    return np.nextafter(f, np.float32(-np.inf)) if np.float64(f) > x else f


def _scene(tri_name, sphere_name=None, n_tris=None):
    """A Scotty3D mesh (one vertex per triangle corner) from a fixture's
    primitives, plus the spheres of another fixture."""
    q = load_fixture(tri_name).a
    prims, shading = q["prims"], q["shading"]
    tri = (prims[:, 3].view(np.uint32) >> 28) == 0
    P = prims[tri][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].astype(np.float32)
    N = shading[tri][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].astype(np.float32)
    if n_tris:
        P, N = P[:n_tris], N[:n_tris]
    sph = np.zeros((0, 4), np.float32)
    if sphere_name:
        s = load_fixture(sphere_name).a["prims"]
        m = (s[:, 3].view(np.uint32) >> 28) == 1
        sph = np.concatenate([s[m][:, 0:3], s[m][:, 4:5]], axis=1).astype(np.float32)
    return P, N, sph


def _reference(P, N, sph, rays64):
    """Oracle answers for rays (n, 8) float64 = o, d, min_t, max_t."""
    bsdf = ptrace.pt_bsdf()
    bsdf.type = ptrace.PT_BSDF_DIFFUSE
    sc = ptrace.Scene.from_mesh(P, [bsdf, bsdf], normals=N, tri_bsdf=np.zeros(len(P), np.int32),
                                spheres=sph if len(sph) else None,
                                sphere_bsdf=np.ones(len(sph), np.int32) if len(sph) else None)
    d = sc.desc()
    r32 = np.zeros((len(rays64), 8), np.float32)
    r32[:, 0:3] = rays64[:, 0:3]
    r32[:, 4:7] = rays64[:, 3:6]
    r32[:, 3] = [_round_down(x) for x in rays64[:, 7]]
    r32[:, 7] = [_round_up(x) for x in rays64[:, 6]]
    keys = pyoracle.intersect(d, r32, use_bvh=False)
    s2i = sc.sorted_to_input()
    prim = ptrace.hit_prim(keys)
    prim = np.where(prim >= 0, s2i[np.maximum(prim, 0)], -1)
    return prim, ptrace.hit_t(keys)


def _normals(P, N, sph, rays64, prim, t):
    """Intersection::n per triangle.cpp:170-202 (fp64) / sphere.h."""
    out = np.zeros((len(rays64), 3))
    nt = len(P)
    for i in np.nonzero(prim >= 0)[0]:
        o, dv = rays64[i, 0:3], rays64[i, 3:6]
        k = prim[i]
        if k < nt:
            p1, p2, p3 = (P[k, 3 * j:3 * j + 3].astype(np.float64) for j in range(3))
            n1, n2, n3 = (N[k, 3 * j:3 * j + 3].astype(np.float64) for j in range(3))
            s, e1, e2 = o - p1, p2 - p1, p3 - p1
            t1, t2 = np.cross(e1, dv), np.cross(s, e2)
            den = 1.0 / np.dot(t1, e2)
            u, v = np.dot(-t2, dv) * den, np.dot(t1, s) * den
            n = u * n2 + v * n3 + (1 - u - v) * n1
            n = n * (1 if np.dot(s, n) > 0 else -1)
        else:
            c = sph[k - nt, 0:3].astype(np.float64)
            n = o + t[i] * dv - c
        out[i] = n / np.linalg.norm(n)
    return out


def _rays(P, sph, n, seed):
    """Camera-like rays, interior rays and rays leaving surface points (with
    their self-hit at t ~ 0), as (n, 8) float64 with min_t = 0, max_t = inf."""
    rng = np.random.default_rng(seed)
    lo = np.minimum(P[:, 0:3].min(0), P[:, 6:9].min(0))
    hi = np.maximum(P[:, 0:3].max(0), P[:, 6:9].max(0))
    r = np.zeros((n, 8))
    k = n // 3
    # interior rays
    r[:k, 0:3] = lo + (hi - lo) * rng.random((k, 3))
    # from outside toward the scene
    r[k:2 * k, 0:3] = (lo + hi) / 2 + (hi - lo) * np.array([0.1, 0.2, 1.5]) + rng.normal(size=(k, 3)) * 0.05
    # from points on triangles (fp32 barycentric points)
    idx = rng.integers(0, len(P), n - 2 * k)
    w = rng.dirichlet([1, 1, 1], n - 2 * k).astype(np.float32)
    pts = (w[:, 0:1] * P[idx, 0:3] + w[:, 1:2] * P[idx, 3:6] + w[:, 2:3] * P[idx, 6:9]).astype(np.float32)
    r[2 * k:, 0:3] = pts
    dirs = rng.normal(size=(n, 3))
    dirs[k:2 * k] = (lo + hi) / 2 - r[k:2 * k, 0:3] + rng.normal(size=(k, 3)) * 0.3
    r[:, 3:6] = dirs / np.linalg.norm(dirs, axis=1, keepdims=True)
    r[:, 0:6] = r[:, 0:6].astype(np.float32)  # the fp32 rays the GPU traces, exactly
    r[:, 6] = 0.0
    r[:, 7] = np.inf
    return r


def _check(bvh, P, N, sph, rays, single=False):
    hit, t, prim, nrm = bvh.intersect(rays, single=single)
    rp, rt = _reference(P, N, sph, rays)
    assert np.array_equal(prim, np.where(hit, prim, -1))
    assert np.array_equal(np.where(hit, prim, -1), rp), np.nonzero(np.where(hit, prim, -1) != rp)[0][:10]
    assert np.array_equal(t[hit], rt[hit].astype(np.float64))
    en = _normals(P, N, sph, rays, rp, t)
    assert np.abs(nrm[hit] - en[hit]).max(initial=0) < 1e-12
    # bool intersect(const Ray&): one GPU call per ray, so on a subset
    assert np.array_equal(bvh.occluded(rays[::97]), hit[::97])
    return hit, t, prim


@pytest.mark.parametrize("tri,sph", [("CBbunny", None), ("CBgems", "CBspheres"), ("CBcoil", None)])
def test_bvhaccel_min_t(tri, sph):
    P, N, S = _scene(tri, sph)
    bvh = ptrace.ScottyBVH(P.reshape(-1, 3), N.reshape(-1, 3), np.arange(3 * len(P)).reshape(-1, 3), S)
    rays = _rays(P, S, 6000, seed=11)
    hit0, t0, _ = _check(bvh, P, N, S, rays)
    assert hit0.mean() > 0.5
    # min_t = 1e-4: the surface rays' self-hits (t ~ 0) are skipped
    r = rays.copy()
    r[:, 6] = 1e-4
    hit1, t1, _ = _check(bvh, P, N, S, r)
    assert (t1[hit1] >= 1e-4).all()
    # min_t = the first hit's t: inclusive, the same hit is found again
    r = rays.copy()
    r[hit0, 6] = t0[hit0]
    hit2, t2, _ = _check(bvh, P, N, S, r)
    assert np.array_equal(hit2[hit0], np.ones(hit0.sum(), bool)) and np.array_equal(t2[hit0], t0[hit0])
    # min_t just above it: that hit is excluded
    r[hit0, 6] = np.nextafter(t0[hit0].astype(np.float32), np.float32(np.inf)).astype(np.float64)
    hit3, t3, _ = _check(bvh, P, N, S, r)
    assert (t3[hit3 & hit0] > t0[hit3 & hit0]).all()
    # max_t below min_t: nothing
    r[:, 7] = r[:, 6] * 0.5
    h4, _, _, _ = bvh.intersect(r)
    assert not h4[hit0].any()
    # the one-ray form (one GPU call per ray) agrees with the batch
    _check(bvh, P, N, S, rays[::150], single=True)
    bvh.close()


def test_bvhaccel_max_leaf_and_segments():
    """max_leaf_size (bvh.h:111) changes the tree, not the answers; finite
    segments [min_t, max_t] both inclusive."""
    P, N, S = _scene("CBbunny", n_tris=4000)
    rays = _rays(P, S, 2000, seed=5)
    rays[:, 6] = 0.05
    rays[:, 7] = 0.8
    res = []
    for leaf in (4, 32, 100):
        bvh = ptrace.ScottyBVH(P.reshape(-1, 3), N.reshape(-1, 3), np.arange(3 * len(P)).reshape(-1, 3), S,
                               max_leaf=leaf)
        res.append(_check(bvh, P, N, S, rays))
        bvh.close()
    for h, t, p in res[1:]:
        assert np.array_equal(h, res[0][0]) and np.array_equal(t, res[0][1]) and np.array_equal(p, res[0][2])


@pytest.mark.parametrize("name", ["CBbunny", "CBspheres"])
def test_pt_intersect_tmin_matches_oracle(gpu_ctx, name):
    """pt_intersect's t_min through the C ABI: random t_min per ray against the
    oracle's brute force and BVH walk (bit-exact keys)."""
    scene = load_fixture(name)
    d = scene.desc()
    gpu_ctx.load_scene(scene)
    from rays import camera_rays, interior_rays
    rays = np.concatenate([camera_rays(d, 5000, seed=3), interior_rays(d, 5000, seed=4)])
    base = ptrace.hit_t(pyoracle.intersect(d, rays, use_bvh=False))
    rng = np.random.default_rng(9)
    fin = np.isfinite(base)
    rays[fin, 7] = (base[fin] * rng.random(fin.sum()) * 2.0).astype(np.float32)
    rays[::7, 7] = -1.0  # negative t_min means 0
    g = gpu_ctx.intersect(rays)
    assert np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=False))
    assert np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=True))
    t = ptrace.hit_t(g)
    assert (t[np.isfinite(t)] >= np.maximum(rays[np.isfinite(t), 7], 0)).all()


def test_bvhaccel_non_unit_directions(gpu_ctx):
    """Scotty3D callers may pass non-unit directions (a shadow ray o + t (light
    - o) over [eps, 1]).  With spheres in the scene BVHAccel traces (o, d/|d|)
    over [min_t |d|, max_t |d|] and scales t back (the sphere test assumes a
    unit d): the same primitives as the unit rays over the same
    segments, t within fp32 rounding.  The C ABI refuses non-unit directions
    on sphere scenes, and takes them as given on triangle-only scenes (the
    triangle test's t is parametric: bit-exact against the oracle's brute
    force on the same non-unit rays)."""
    P, N, S = _scene("CBgems", "CBspheres")
    bvh = ptrace.ScottyBVH(P.reshape(-1, 3), N.reshape(-1, 3), np.arange(3 * len(P)).reshape(-1, 3), S)
    rays = _rays(P, S, 6000, seed=21)
    rays[:, 6] = 1e-3
    h0, t0, p0, _ = bvh.intersect(rays)
    s = np.exp(np.random.default_rng(4).uniform(np.log(0.05), np.log(20.0), len(rays)))
    r2 = rays.copy()
    r2[:, 3:6] *= s[:, None]
    r2[:, 6] /= s
    h1, t1, p1, _ = bvh.intersect(r2)
    assert h0.mean() > 0.5 and (p0[h0] >= len(P)).sum() > 50  # sphere hits among them
    same = (p0 == p1)
    assert same.mean() > 0.999, same.mean()
    both = h0 & h1 & same
    assert np.all(np.abs(t1[both] * s[both] - t0[both]) <= 1e-5 * np.maximum(1.0, t0[both]))
    bvh.close()
    # the C ABI on a sphere scene: unit directions only
    sph = load_fixture("CBspheres")
    gpu_ctx.load_scene(sph)
    from rays import camera_rays
    cr = camera_rays(sph.desc(), 64, seed=1)
    gpu_ctx.intersect(cr)
    bad = cr.copy()
    bad[:, 4:7] *= 2.0
    with pytest.raises(ptrace.PTError) as e:
        gpu_ctx.intersect(bad)
    assert e.value.code == ptrace.PT_E_INVALID
    # triangle-only: non-unit directions as given, bit-exact
    sc = load_fixture("CBbunny")
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    cr = camera_rays(d, 4000, seed=2)
    cr[:, 4:7] *= np.float32(3.0)
    g = gpu_ctx.intersect(cr)
    assert (g != ptrace.PT_HIT_NONE).sum() > 1000
    assert np.array_equal(g, pyoracle.intersect(d, cr, use_bvh=False))
