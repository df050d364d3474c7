"""CBspheres cost split (dev tool): the single-leaf path kernel's time per ray
on CBspheres with its glass / mirror spheres as they are and with either or
both made diffuse (albedo 0.5), beside CBempty -- separates the spheres'
geometry from the specular vertices' shading.

  python scripts/dev/sphere_bsdf_ab.py [frames]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "cuda-raytracer_amd"))
import ptrace  # noqa: E402
import scenes  # noqa: E402

W = H = 1024
SPP, B = 256, 8
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 3


def run(ctx, scene, label):
    ctx.load_scene(scene)
    ctx.clear()
    ctx.render(W, H, SPP, max_bounces=B)  # warm-up
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(frames):
        ctx.clear()
        ctx.render(W, H, SPP, max_bounces=B, flags=ptrace.PT_FLAG_STATS)
    ms = (time.perf_counter() - t0) * 1e3 / frames
    st = ctx.stats()
    rays = (st.rays - st.culled_rays) / frames
    print(f"{label:28s} {ms:7.2f} ms/frame  {rays / 1e6:8.1f} Mrays/frame  {ms * 1e6 / rays:6.3f} ns/ray", flush=True)


def main():
    ctx = ptrace.Context(0)
    run(ctx, scenes.load("CBempty"), "CBempty")
    for name, change in (("as is", ()), ("glass diffuse", (ptrace.PT_BSDF_GLASS,)),
                         ("mirror diffuse", (ptrace.PT_BSDF_MIRROR,)),
                         ("both diffuse", (ptrace.PT_BSDF_GLASS, ptrace.PT_BSDF_MIRROR))):
        sc = scenes.load("CBspheres")
        d = sc.desc()
        for i in range(d.n_bsdfs):
            b = d.bsdfs[i]
            if b.type in change:
                b.type = ptrace.PT_BSDF_DIFFUSE
                for k in range(3):
                    b.albedo[k] = 0.5
        run(ctx, sc, "CBspheres " + name)
    ctx.close()


if __name__ == "__main__":
    main()
