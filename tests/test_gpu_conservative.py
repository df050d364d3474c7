"""Box conservativeness: the traversal's fp32
slab test (approximate v_rcp_f32 reciprocal, rounded o * (1/d), FMA slabs) must
never cull a box whose primitives the exact test hits.  Every stored box carries
the guard band of scene_internal.h box_guard.  Adversarial rays -- aimed at the
vertices, edges and corners of the axis-aligned Cornell walls (flat boxes),
at edges of every triangle, and grazing sphere silhouettes -- through host SAH
trees and GPU-built (PLOC, radix) trees must give exactly the oracle's
brute-force closest hit (no boxes at all)."""
import numpy as np
import pytest

import ptrace
import pyoracle
import scenes
from conftest import load_fixture
from rays import axis_aligned_tris, edge_rays, interior_rays, sphere_tangent_rays

pytestmark = pytest.mark.gpu


def _adversarial(d, seed):
    parts = [edge_rays(d, 6000, seed=seed, vertex_frac=0.4, prims=axis_aligned_tris(d)),
             edge_rays(d, 6000, seed=seed + 1)]
    q = np.ctypeslib.as_array(ptrace.C.cast(d.prims, ptrace.C.POINTER(ptrace.C.c_float)), shape=(d.n_prims, 24))
    if ((q[:, 3].view(np.uint32) >> 28) == 1).any():
        parts.append(sphere_tangent_rays(d, 6000, seed=seed + 2))
    # shadow-like segments ending on the walls: tmax exactly at the hit
    seg = edge_rays(d, 3000, seed=seed + 3, prims=axis_aligned_tris(d))
    hits = pyoracle.intersect(d, seg, use_bvh=False)
    t = ptrace.hit_t(hits)
    seg[:, 3] = np.where(np.isfinite(t), t, 1.0)
    parts.append(seg)
    return np.concatenate(parts)


CASES = [("CBempty", None), ("CBspheres", None), ("CBbunny", None), ("CBcoil", None),
         ("CBbunny", "ploc"), ("CBbunny", "lbvh"), ("CBspheres", "ploc"), ("CBspheres", "lbvh"),
         ("CBcoil", "ploc")]


@pytest.mark.parametrize("name,builder", CASES)
def test_grazing_rays_match_brute_force(gpu_ctx, name, builder):
    sc = load_fixture(name) if builder is None else scenes.rebuilt(name, gpu_device=0, max_leaf=8, builder=builder)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    rays = _adversarial(d, seed=len(name))
    g = gpu_ctx.intersect(rays)
    o = pyoracle.intersect(d, rays, use_bvh=False)
    assert (o != ptrace.PT_HIT_NONE).sum() > len(rays) // 3
    bad = np.nonzero(g != o)[0]
    assert len(bad) == 0, f"{len(bad)} of {len(rays)} grazing rays differ, first {bad[:5]}: {g[bad[:5]]} vs {o[bad[:5]]}"
    if name != "CBspheres":  # the literal reference test too (triangles only)
        g = gpu_ctx.intersect(rays, flags=ptrace.PT_FLAG_REF_ARITH)
        o = pyoracle.intersect(d, rays, use_bvh=False, flags=ptrace.PT_FLAG_REF_ARITH)
        assert np.array_equal(g, o)


def test_guard_band_in_gpu_built_boxes(gpu_ctx):
    """GPU-built leaf boxes enclose their primitives with the guard band: no
    vertex lies within G = 2^-17 M of a box face from the inside."""
    sc = scenes.rebuilt("CBbunny", gpu_device=0, max_leaf=8, builder="ploc")
    d = sc.desc()
    a = scenes.fixture_arrays("CBbunny")
    M = max(np.abs(a["positions"]).max(), np.abs(np.array(d.camera.origin)).max(),
            np.abs(np.array(d.light.position)).max())
    G = np.ldexp(M, -17)
    prims = sc.prims()
    for i in range(d.n_nodes):
        n = d.nodes[i]
        for k in range(4):
            c = n.child[k]
            if c < 0 or d.nodes[c].prim_count == 0:
                continue
            m = d.nodes[c]
            q = prims[m.prim_start:m.prim_start + m.prim_count]
            v = q[:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].reshape(-1, 3).astype(np.float64)
            lo = np.array([n.bmin_x[k], n.bmin_y[k], n.bmin_z[k]], np.float64)
            hi = np.array([n.bmax_x[k], n.bmax_y[k], n.bmax_z[k]], np.float64)
            assert (v.min(0) - lo >= G * 0.999).all() and (hi - v.max(0) >= G * 0.999).all()
