import sys
sys.path.insert(0, "cuda-raytracer_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
import numpy as np
import ptrace, pyoracle
from rays import interior_rays
b = ptrace.pt_bsdf(); b.type = 0
for k in range(3): b.albedo[k] = 0.5
rng = np.random.default_rng(9)
ctx = ptrace.Context(0)
for n_tris, n_sph in [(1, 0), (0, 1), (2, 3), (37, 5), (5000, 0)]:
    tris = None
    if n_tris:
        size = 2.0 if n_tris < 100 else 0.15
        v0 = rng.random((n_tris, 1, 3), dtype=np.float32) * 4 - 2
        tris = (v0 + (rng.random((n_tris, 3, 3), dtype=np.float32) - 0.5) * size).reshape(n_tris, 9)
    sph = np.concatenate([rng.random((n_sph, 3), dtype=np.float32) * 4 - 2,
                          rng.random((n_sph, 1), dtype=np.float32) * 0.3 + 0.05], axis=1) if n_sph else None
    for gpu in (None, 0):
        sc = ptrace.Scene.from_mesh(tris, [b], spheres=sph, gpu_device=gpu, max_leaf=4)
        d = sc.desc()
        print(n_tris, n_sph, 'gpu' if gpu is not None else 'host', 'nodes', d.n_nodes, 'levels', sc.level_counts(), flush=True)
        if gpu is not None:
            for i in range(min(d.n_nodes, 12)):
                nd = d.nodes[i]
                print('   node', i, 'lvl', nd.level, 'child', list(nd.child), 'prims', nd.prim_start, nd.prim_count)
        ctx.load_scene(sc)
        rays = interior_rays(d, 5000, seed=n_tris)
        ctx.reset_stats()
        try:
            g = ctx.intersect(rays)
            st = ctx.stats()
            print('   ok', np.array_equal(g, pyoracle.intersect(d, rays, use_bvh=False)), 'visits', st.visits, 'peakq', st.peak_queue_entries, flush=True)
        except Exception as e:
            st = ctx.stats()
            print('   FAIL', e, 'visits', st.visits, 'peakq', st.peak_queue_entries, [st.level_visits[l] for l in range(8)], flush=True)
