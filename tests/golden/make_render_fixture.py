"""Regenerate tests/golden/render_CBgems_16x16x2.npz (oracle regression pin).

Prints the relative L2 distance of the new sums to the previous golden; every
regeneration is logged with that distance in tests/golden/REGENERATIONS.md.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle")]
import ptrace  # noqa: E402
import pyoracle  # noqa: E402

OUT = ROOT / "tests/golden/render_CBgems_16x16x2.npz"
sc = ptrace.ArrayScene.load(ROOT / "tests/golden/scenes/CBgems.npz")
sums, rays = pyoracle.render(sc.desc(), 16, 16, 2, max_bounces=8, seed=15618)
if OUT.exists():
    old = np.load(OUT, allow_pickle=False)
    rel = np.linalg.norm(sums[..., :3] - old["sums"][..., :3]) / np.linalg.norm(old["sums"][..., :3])
    print(f"relative L2 to the previous golden: {rel:.3e} (rays {int(old['rays'])} -> {rays})")
np.savez_compressed(OUT, sums=sums, rays=np.int64(rays))
