"""Deterministic ray batches for closest-hit parity tests (inputs only)."""
import numpy as np


def camera_rays(desc, n, seed=0, width=256, height=256):
    """Pinhole rays of the reference camera model (cu:338-354) at random pixels."""
    rng = np.random.default_rng(seed)
    o = np.array(desc.camera.origin, np.float32)
    L, U, K = (np.array(v, np.float32) for v in (desc.camera.left, desc.camera.up, desc.camera.look_at))
    ss = rng.random((n, 2), dtype=np.float32) * np.array([height, width], np.float32)
    kx = ss[:, 1] / np.float32(width) - np.float32(0.5)
    ky = -(ss[:, 0] / np.float32(height) - np.float32(0.5))
    d = kx[:, None] * L + ky[:, None] * U + K
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = o
    r[:, 3] = np.inf
    r[:, 4:7] = d
    return r


def interior_rays(desc, n, seed=1, tmax=np.inf):
    """Rays from random points inside the scene bounds in random directions."""
    rng = np.random.default_rng(seed)
    nodes = np.frombuffer(bytes(desc.nodes[0]), dtype=np.float32, count=24).reshape(6, 4)
    if desc.nodes[0].prim_count > 0:
        lo, hi = np.array([-1, 0, -1], np.float32), np.array([1, 1.5, 1], np.float32)
    else:
        valid = np.array(desc.nodes[0].child) >= 0
        lo = np.array([nodes[0][valid].min(), nodes[2][valid].min(), nodes[4][valid].min()], np.float32)
        hi = np.array([nodes[1][valid].max(), nodes[3][valid].max(), nodes[5][valid].max()], np.float32)
    o = lo + (hi - lo) * rng.random((n, 3), dtype=np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = o
    r[:, 3] = tmax
    r[:, 4:7] = d
    return r


def _prims(desc):
    import ctypes as C
    return np.ctypeslib.as_array(C.cast(desc.prims, C.POINTER(C.c_float)), shape=(desc.n_prims, 24))


def axis_aligned_tris(desc):
    """Indices of triangles whose normal lies along a coordinate axis (the
    Cornell walls): their boxes are flat in one axis."""
    q = _prims(desc)
    tri = (q[:, 3].view(np.uint32) >> 28) == 0
    N = q[:, 12:15]
    flat = (np.count_nonzero(np.abs(N) > 1e-6 * np.abs(N).max(axis=1, keepdims=True), axis=1) == 1)
    return np.nonzero(tri & flat)[0]


def edge_rays(desc, n, seed=2, vertex_frac=0.25, prims=None):
    """Rays from near the camera aimed at points on triangle edges (and, for a
    `vertex_frac` share, exactly at vertices) of `prims` (default: every
    triangle): the grazing cases where edge-test rounding and box
    conservativeness matter."""
    rng = np.random.default_rng(seed)
    q = _prims(desc)
    tri = np.nonzero((q[:, 3].view(np.uint32) >> 28) == 0)[0] if prims is None else np.asarray(prims)
    idx = rng.choice(tri, n)
    v = np.stack([q[idx, 0:3], q[idx, 4:7], q[idx, 8:11]], axis=1)
    k = rng.integers(0, 3, n)
    w = rng.random(n, dtype=np.float32)
    w[: int(n * vertex_frac)] = 0.0
    a = v[np.arange(n), k]
    b = v[np.arange(n), (k + 1) % 3]
    target = (a + (b - a) * w[:, None]).astype(np.float32)
    o = np.array(desc.camera.origin, np.float32)[None, :] + (rng.random((n, 3), dtype=np.float32) - 0.5) * 0.2
    d = target - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = o
    r[:, 3] = np.inf
    r[:, 4:7] = d
    return r


def sphere_tangent_rays(desc, n, seed=5, rel=(-1e-6, 0.0, 1e-6)):
    """Rays from near the camera grazing the spheres' silhouettes: aimed at
    c + r (1 + s) u with u perpendicular to the view of the centre and s from
    `rel` (just inside, on, just outside the tangent)."""
    rng = np.random.default_rng(seed)
    q = _prims(desc)
    sph = np.nonzero((q[:, 3].view(np.uint32) >> 28) == 1)[0]
    idx = rng.choice(sph, n)
    c = q[idx, 0:3].astype(np.float64)
    r = q[idx, 4].astype(np.float64)
    o = np.array(desc.camera.origin, np.float64)[None, :] + (rng.random((n, 3)) - 0.5) * 0.2
    w = c - o
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    a = rng.normal(size=(n, 3))
    u = a - (a * w).sum(1, keepdims=True) * w
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    s = np.asarray(rel)[rng.integers(0, len(rel), n)]
    d = c + u * (r * (1.0 + s))[:, None] - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    out = np.zeros((n, 8), np.float32)
    out[:, :3] = o
    out[:, 3] = np.inf
    out[:, 4:7] = d
    return out
