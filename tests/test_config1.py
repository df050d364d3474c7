"""BASELINE config 1 (CPU plumbing through the Scotty3D surface): the Cornell
box at 256x256, 4 spp, the reference schedule, rendered by the CPU oracle
behind scotty::PathTracerT (32x32-tile work queue + worker threads,
src/pathtracer.cpp:183-213, 499-558), reproduces the committed golden images
(tests/golden/make_config1_golden.py) bit for bit, for any worker count, and
equals the oracle's own tile renderer."""
import numpy as np
import pytest

import pyoracle
from conftest import ROOT  # noqa: F401

import sys
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import make_config1_golden as G  # noqa: E402


@pytest.mark.parametrize("name", G.SCENES)
def test_scotty_surface_reproduces_golden(name):
    with np.load(G.path(name), allow_pickle=False) as z:
        gold, rays = z["rgb"], int(z["rays"])
    img, r, _, thr = G.render(name)
    assert thr >= 1 and r == rays
    assert np.array_equal(img[..., :3], gold)
    img1, r1, _, _ = G.render(name, threads=3)
    assert r1 == rays and np.array_equal(img1, img)
    d = pyoracle  # the oracle's own tile renderer (pto_render) gives the same frame
    ref, r2 = d.image(G.ptrace.ArrayScene.load(ROOT / "tests" / "golden" / "scenes" / f"{name}.npz").desc(),
                      G.W, G.H, G.SPP, max_bounces=G.BOUNCES, seed=G.SEED, flags=G.FLAGS)
    assert r2 == rays and np.array_equal(ref[..., :3], gold)
    assert np.isfinite(gold).all() and gold.mean() > 0.05
