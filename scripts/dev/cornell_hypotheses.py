"""the Cornell-box factor under each hypothesis.  Renders the
four Cornell files on the oracle at the reference's framing (the fixture's
cameras) with one reading changed and prints the global factor reference /
ours and every region's ratio after it (tests/refrender.py compare).

  python scripts/dev/cornell_hypotheses.py [spp]
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "cuda-raytracer_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import ptrace  # noqa: E402
import pyoracle  # noqa: E402
import refrender as rr  # noqa: E402
from test_reference_renders import course_scene  # noqa: E402

CORNELL = ["CBbunny", "CBspheres_lambertian", "CBspheres", "CBcoil"]


def light_swap(d):
    d.light.dim_x[0], d.light.dim_y[2] = 0.8, 0.6


def light_unit(area):
    def f(d):
        d.light.dim_x[0], d.light.dim_y[2] = 1.0, 1.0
        if area is not None:
            d.light.area = area
    return f


def light_centre(d):
    for k in range(3):
        d.light.dim_x[k] *= 1e-6
        d.light.dim_y[k] *= 1e-6


HYPOTHESES = {  # name -> (scene edit, render flags)
    "baseline": (None, 0),
    "no emission through specular bounces": (None, ptrace.PT_FLAG_NO_EMISSION),
    "light dims swapped": (light_swap, ptrace.PT_FLAG_NO_EMISSION),
    "light dims 1x1, area 1": (light_unit(1.0), ptrace.PT_FLAG_NO_EMISSION),
    "light dims 1x1, area 0.48": (light_unit(None), ptrace.PT_FLAG_NO_EMISSION),
    "light sampled at its centre": (light_centre, ptrace.PT_FLAG_NO_EMISSION),
}


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    fx_all = rr.load(ROOT / "tests" / "golden" / "reference_renders.npz")
    for hyp, (edit, flags) in HYPOTHESES.items():
        for name in CORNELL:
            fx = fx_all[name]
            d = course_scene(name).desc()
            d.camera = ptrace.pt_camera.from_buffer_copy(fx["camera"].tobytes())
            if edit is not None:
                edit(d)
            img, _ = pyoracle.image(d, rr.W, rr.H, spp, max_bounces=8, flags=flags)
            c = rr.compare(fx, np.asarray(img, np.float64))
            rel = " ".join(f"{rr.ROLE_NAMES[c['role'][r]]}:{np.round(v, 3).tolist()}" for r, v in c["rel"].items())
            spread = " ".join(f"{rr.ROLE_NAMES[c['role'][r]]}:{mx:.3f}" for r, (_, mx) in c["spread"].items())
            # the log-average tone map (image.h:143-167) would scale by key / (avg * white^2)
            ill = np.asarray(img, np.float64)[..., :3] @ np.array([0.2126, 0.7152, 0.0722])
            tm = 0.18 / (np.exp(np.mean(np.log(1e-7 + ill.astype(np.float32)))) * 25.0)
            print(f"[{hyp}] {name}: factor {c['scale']:.4f} (tone map would give {tm:.3g})\n"
                  f"    {rel}\n    profiles {spread}; blocks within 8 levels {(c['block_diff'] <= 8).mean():.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
