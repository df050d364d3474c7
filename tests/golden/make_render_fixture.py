"""Regenerate tests/golden/render_CBgems_16x16x2.npz (oracle regression pin)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle")]
import ptrace  # noqa: E402
import pyoracle  # noqa: E402

sc = ptrace.ArrayScene.load(ROOT / "tests/golden/scenes/CBgems.npz")
sums, rays = pyoracle.render(sc.desc(), 16, 16, 2, max_bounces=8, seed=15618)
np.savez_compressed(ROOT / "tests/golden/render_CBgems_16x16x2.npz", sums=sums, rays=np.int64(rays))
