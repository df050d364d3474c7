"""BASELINE config 1 on the HIP path: pt_render of the Cornell box at 256x256,
4 spp, the reference schedule in the full reference mode equals the golden
frame the CPU Scotty3D surface produced (tests/golden/make_config1_golden.py),
bit for bit, with the same number of rays cast."""
import sys

import numpy as np
import pytest

import ptrace
from conftest import ROOT, load_fixture

sys.path.insert(0, str(ROOT / "tests" / "golden"))
import make_config1_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", G.SCENES)
def test_gpu_matches_config1_golden(gpu_ctx, name):
    with np.load(G.path(name), allow_pickle=False) as z:
        gold, rays = z["rgb"], int(z["rays"])
    gpu_ctx.load_scene(load_fixture(name))
    gpu_ctx.reset_stats()
    gpu_ctx.clear()
    gpu_ctx.render(G.W, G.H, G.SPP, max_bounces=G.BOUNCES, seed=G.SEED, flags=G.FLAGS)
    img = gpu_ctx.get_image()
    assert gpu_ctx.stats().rays == rays
    bad = np.count_nonzero(img[..., :3] != gold)
    assert bad == 0, f"{bad} values differ, max |diff| {np.abs(img[..., :3] - gold).max()}"
