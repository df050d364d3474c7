"""Debug (GPU): closest hits with the two-level traversal on and off."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import ptrace  # noqa: E402
import pyoracle  # noqa: E402
from conftest import load_fixture  # noqa: E402
from rays import camera_rays, interior_rays  # noqa: E402

ctx = ptrace.Context(0)
for name in sys.argv[1:] or ["CBgems"]:
    sc = load_fixture(name)
    d = sc.desc()
    rays = np.concatenate([camera_rays(d, 20000, seed=7), interior_rays(d, 20000, seed=8),
                           interior_rays(d, 5000, seed=9, tmax=0.5)])
    o = pyoracle.intersect(d, rays, use_bvh=True)
    for tl in ("0", "1"):
        for qf in ("4", "64"):
            os.environ["PT_TWO_LEVEL"] = tl
            os.environ["PT_QFACTOR"] = qf
            c2 = ptrace.Context(0)
            c2.load_scene(sc)
            c2.reset_stats()
            g = c2.intersect(rays)
            st = c2.stats()
            bad = np.nonzero(g != o)[0]
            print(f"{name} two_level={tl} qfactor={qf}: mismatches {len(bad)} peakq {st.peak_queue_entries} "
                  f"qf {st.queue_factor} first {bad[:6]} R {st.rays} V {list(st.level_visits)[:st.n_levels]} "
                  f"leafV {list(st.level_leaf_visits)[:st.n_levels]} items {list(st.level_items)[:st.n_levels]}",
                  flush=True)
            if len(bad):
                gt, ot = ptrace.hit_t(g[bad[:3]]), ptrace.hit_t(o[bad[:3]])
                print("   gpu", gt, ptrace.hit_prim(g[bad[:3]]), "oracle", ot, ptrace.hit_prim(o[bad[:3]]))
            c2.close()
ctx.close()
