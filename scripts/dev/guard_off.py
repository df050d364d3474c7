"""Diagnostic (GPU): grazing-ray mismatches against the brute-force closest hit
with the box guard band on (default) and off (PT_BOX_GUARD=0), on host-built
and GPU-built trees.  Prints one line per case; used for DESIGN.md §3."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import ptrace  # noqa: E402
import pyoracle  # noqa: E402
import scenes  # noqa: E402
from test_gpu_conservative import _adversarial  # noqa: E402

ctx = ptrace.Context(0)
for guard in ("1", "0"):
    os.environ["PT_BOX_GUARD"] = guard
    for name, builder in [("CBempty", None), ("CBspheres", None), ("CBbunny", None), ("CBbunny", "ploc"),
                          ("CBbunny", "lbvh"), ("CBspheres", "ploc"), ("CBcoil", "ploc")]:
        sc = scenes.rebuilt(name) if builder is None else scenes.rebuilt(name, gpu_device=0, max_leaf=8,
                                                                          builder=builder)
        d = sc.desc()
        ctx.load_scene(sc)
        rays = _adversarial(d, seed=len(name))
        g = ctx.intersect(rays)
        o = pyoracle.intersect(d, rays, use_bvh=False)
        print(f"guard={guard} {name:10s} {builder or 'host-sah':8s} rays {len(rays)} hits {(o != ptrace.PT_HIT_NONE).sum()}"
              f" mismatches {(g != o).sum()}", flush=True)
ctx.close()
