"""GPU BVH build: the device-built 4-wide tree is a valid
layout for the traversal, and closest hits / images over it are bit-identical
to the oracle on the same flattened scene (closest hits do not depend on the
tree; ties break on the tree's own sorted primitive order)."""
import time

import numpy as np
import pytest

import ptrace
import pyoracle
import scenes
from rays import camera_rays, interior_rays

pytestmark = pytest.mark.gpu


def _check_layout(sc, max_leaf):
    d = sc.desc()
    prims = sc.prims()
    covered = np.zeros(d.n_prims, np.int32)
    for i in range(d.n_nodes):
        n = d.nodes[i]
        assert d.level_start[n.level] <= i < d.level_start[n.level + 1]
        if n.prim_count > 0:
            assert n.prim_count <= max_leaf and all(c < 0 for c in n.child)
            covered[n.prim_start:n.prim_start + n.prim_count] += 1
            continue
        for k in range(4):
            c = n.child[k]
            if c < 0:
                continue
            assert c > i and d.nodes[c].level == n.level + 1
            # the child's box holds every primitive below it
            stack, ids = [c], []
            while stack:
                m = d.nodes[stack.pop()]
                if m.prim_count:
                    ids.extend(range(m.prim_start, m.prim_start + m.prim_count))
                else:
                    stack.extend(x for x in m.child if x >= 0)
            q = prims[ids]
            tri = (q[:, 3].view(np.uint32) >> 28) == 0
            v = q[tri][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].reshape(-1, 3)
            lo = np.array([n.bmin_x[k], n.bmin_y[k], n.bmin_z[k]], np.float32)
            hi = np.array([n.bmax_x[k], n.bmax_y[k], n.bmax_z[k]], np.float32)
            assert (v >= lo).all() and (v <= hi).all()
    assert (covered == 1).all()


@pytest.mark.parametrize("max_leaf,builder", [(4, "ploc"), (8, "ploc"), (32, "ploc"), (8, "lbvh"), (32, "lbvh"),
                                              (4, "sah"), (8, "sah"), (32, "sah")])
def test_gpu_build_dragon_proxy(gpu_ctx, max_leaf, builder):
    t = time.perf_counter()
    host = scenes.dragon_proxy()
    host_s = time.perf_counter() - t
    sc = scenes.dragon_proxy(gpu_device=0, max_leaf=max_leaf, builder=builder)
    d = sc.desc()
    assert d.n_prims == host.desc().n_prims
    # same primitive records, permuted
    perm_h, perm_g = host.sorted_to_input(), sc.sorted_to_input()
    assert sorted(perm_g.tolist()) == list(range(d.n_prims))
    ph, pg = host.prims(), sc.prims()
    inv_h = np.empty_like(perm_h)
    inv_h[perm_h] = np.arange(len(perm_h))
    assert np.array_equal(pg.view(np.uint32), ph[inv_h[perm_g]].view(np.uint32))
    if max_leaf >= 8:
        _check_layout(sc, max_leaf)
    gpu_ctx.load_scene(sc)
    rays = np.concatenate([camera_rays(d, 20000, seed=37), interior_rays(d, 20000, seed=38)])
    g = gpu_ctx.intersect(rays)
    assert np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=True))
    sub = rays[::7]
    assert np.array_equal(g[::7], pyoracle.intersect(d, sub, use_bvh=False))
    gpu_ctx.clear()
    gpu_ctx.render(24, 24, 2, max_bounces=6)
    gi = gpu_ctx.get_image()
    oi, _ = pyoracle.image(d, 24, 24, 2, max_bounces=6)
    assert np.array_equal(gi, oi)
    print(f"GPU build {sc.build_ms:.1f} ms (host SAH build {host_s * 1e3:.0f} ms incl. proxy assembly)")


def test_gpu_build_small_and_spheres(gpu_ctx):
    b = ptrace.pt_bsdf()
    b.type = ptrace.PT_BSDF_DIFFUSE
    for k in range(3):
        b.albedo[k] = 0.5
    rng = np.random.default_rng(9)
    cases = [(1, 0, False), (0, 1, False), (2, 3, False), (37, 5, False), (5000, 0, False), (300, 0, True)]
    for (n_tris, n_sph, dup), builder in [(c, bld) for c in cases for bld in ("ploc", "lbvh", "sah")]:
        tris = None
        if n_tris:  # small triangles scattered in the box (big ones only for the tiny cases)
            size = 2.0 if n_tris < 100 else 0.15
            v0 = rng.random((n_tris, 1, 3), dtype=np.float32) * 4 - 2
            tris = (v0 + (rng.random((n_tris, 3, 3), dtype=np.float32) - 0.5) * size).reshape(n_tris, 9)
            if dup:  # groups of identical triangles: equal boxes, equal merge costs
                tris = np.repeat(tris[: n_tris // 10], 10, axis=0)
        sph = np.concatenate([rng.random((n_sph, 3), dtype=np.float32) * 4 - 2,
                              rng.random((n_sph, 1), dtype=np.float32) * 0.3 + 0.05], axis=1) if n_sph else None
        sc = ptrace.Scene.from_mesh(tris, [b], spheres=sph, gpu_device=0, max_leaf=4, builder=builder)
        d = sc.desc()
        assert d.n_prims == n_tris + n_sph
        _check_layout(sc, 4)
        gpu_ctx.load_scene(sc)
        rays = interior_rays(d, 5000, seed=n_tris)
        assert np.array_equal(gpu_ctx.intersect(rays), pyoracle.intersect(d, rays, use_bvh=False))
