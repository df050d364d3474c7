"""BASELINE config 1 golden images: the Cornell box at 256x256, 4 spp, the
reference schedule (2 bounces; NEE 2, 2, 1 weighted 0.5, 0.5, 1), rendered on
the CPU through the Scotty3D PathTracer surface (scotty::PathTracerT: a work
queue of 32x32 tiles, hardware_concurrency workers, raytrace_tile ->
raytrace_pixel; src/pathtracer.cpp:183-213, 499-558) with the oracle's
per-pixel estimator, in the full reference mode (PT_FLAG_REF_SCHEDULE |
REF_DROP_ON_MISS | REF_ARITH | NO_EMISSION: the kernels' literal arithmetic,
REAL_TIME).  The GPU test (tests/test_gpu_config1.py) must reproduce them bit
for bit.

  python tests/golden/make_config1_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle")]
import ptrace  # noqa: E402
import pyoracle  # noqa: E402

W = H = 256
SPP, BOUNCES, SEED = 4, 2, 15618
FLAGS = (ptrace.PT_FLAG_REF_SCHEDULE | ptrace.PT_FLAG_REF_DROP_ON_MISS | ptrace.PT_FLAG_REF_ARITH
         | ptrace.PT_FLAG_NO_EMISSION)
SCENES = ["CBempty", "CBbunny"]


def path(name):
    return ROOT / "tests" / "golden" / f"config1_{name}_{W}x{H}x{SPP}.npz"


def render(name, threads=0):
    d = ptrace.ArrayScene.load(ROOT / "tests" / "golden" / "scenes" / f"{name}.npz").desc()
    return pyoracle.scotty_render(d, W, H, SPP, BOUNCES, seed=SEED, flags=FLAGS, threads=threads)


def main():
    for name in SCENES:
        img, rays, sec, thr = render(name)
        np.savez_compressed(path(name), rgb=img[..., :3], rays=np.uint64(rays), flags=np.uint32(FLAGS))
        print(f"{name}: {rays} rays, {sec:.2f} s on {thr} threads, mean {img[..., :3].mean():.5f}")


if __name__ == "__main__":
    main()
