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
