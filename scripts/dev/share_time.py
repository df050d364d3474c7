"""Time one rank's share of a multi-GPU frame on one GPU (what each of N ranks
renders): python scripts/dev/share_time.py <scene> <n1,n2,...> [steps]

Per share: the best render wall time (pt_render, host-measured, the frame's
kernels synchronised), the image copy to the host, and -- from one more,
instrumented frame (PT_FLAG_STATS) -- the path kernel's time and the GPU time
of the whole render, against the ideal (full frame / n)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import torch  # noqa: E402  (HIP runtime first)
import ptrace  # noqa: E402
import scenes  # noqa: E402

name = sys.argv[1]
shares = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = ptrace.Context(0)
ctx.load_scene(scenes.load(name))
W = H = 1024
host = torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True)
full = None
for k in [1] + [s for s in shares if s != 1]:
    ctx.clear()
    ctx.render(W, H, 256, max_bounces=8, rank=0, nranks=k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        ctx.clear()
        t0 = time.perf_counter()
        ctx.render(W, H, 256, max_bounces=8, rank=0, nranks=k)
        t1 = time.perf_counter()
        ctx.get_image(out=host)
        t2 = time.perf_counter()
        ts.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
    ctx.clear()
    ctx.reset_stats()
    ctx.render(W, H, 256, max_bounces=8, rank=0, nranks=k, flags=ptrace.PT_FLAG_STATS)
    st = ctx.stats()
    best = min(ts)
    if k == 1:
        full = best[0]
    print(f"{name} share 1/{k}: render {best[0]:.3f} ms (median {sorted(t[0] for t in ts)[len(ts) // 2]:.3f}) "
          f"get_image {best[1]:.3f} ms  path kernel {st.ms_path:.3f} ms  GPU total {st.ms_total:.3f} ms  "
          f"ideal {full / k:.3f} ms  ratio {best[0] / (full / k):.3f}", flush=True)
