"""Time one rank's share of a multi-GPU frame on one GPU (what each of N ranks
renders): python scripts/dev/share_time.py <scene> <nranks> [steps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import torch  # noqa: E402  (HIP runtime first)
import ptrace  # noqa: E402
import scenes  # noqa: E402

name, n = sys.argv[1], int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ctx = ptrace.Context(0)
ctx.load_scene(scenes.load(name))
W = H = 1024
for share in ([(0, 1)] if n == 1 else [(0, 1), (0, n)]):
    r, k = share
    for _ in range(1):
        ctx.clear()
        ctx.render(W, H, 256, max_bounces=8, rank=r, nranks=k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        ctx.clear()
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.render(W, H, 256, max_bounces=8, rank=r, nranks=k)
        t1 = time.perf_counter()
        ctx.get_image()
        t2 = time.perf_counter()
        ts.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
    st = ctx.stats()
    best = min(ts)
    print(f"{name} share {r}/{k}: render {best[0]:.2f} ms  get_image {best[1]:.2f} ms  rays {st.rays}  "
          f"ideal {'' if k == 1 else f'{ts0 / k:.2f} ms'}", flush=True)
    if k == 1:
        ts0 = best[0]
