"""Per-rank share times of one frame (what each of N ranks renders):
python scripts/dev/rank_balance.py <scene> <nranks> [steps]"""
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
res = []
for r, k in [(0, 1)] + [(r, n) for r in range(n)]:
    ctx.clear()
    ctx.render(W, H, 256, max_bounces=8, rank=r, nranks=k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        ctx.clear()
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.render(W, H, 256, max_bounces=8, rank=r, nranks=k)
        ts.append((time.perf_counter() - t0) * 1e3)
    res.append((r, k, min(ts), ctx.stats().rays))
    print(f"{name} share {r}/{k}: render {min(ts):.2f} ms  rays {ctx.stats().rays}", flush=True)
full = res[0][2]
worst = max(x[2] for x in res[1:])
print(f"{name}: full {full:.2f} ms, ideal share {full / n:.2f}, worst share {worst:.2f} "
      f"(efficiency bound {full / n / worst:.3f}), rays max/mean "
      f"{max(x[3] for x in res[1:]) / (sum(x[3] for x in res[1:]) / n):.3f}")
