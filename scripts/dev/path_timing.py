"""Per-wave timeline of k_path_leaf (diagnostic build: make variant NAME=tm
DEFS=-DPT_PATH_TIMING=1, run with PTCORE_LIB=lib/libptcore_tm.so):
python scripts/dev/path_timing.py <scene> <nranks>"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import torch  # noqa: E402,F401
import ptrace  # noqa: E402
import scenes  # noqa: E402

name, n = sys.argv[1], int(sys.argv[2])
ctx = ptrace.Context(0)
ctx.load_scene(scenes.load(name))
lib = ptrace.LIB
NW = 16384
buf = (C.c_ulonglong * (NW * 8))()
for r, k in [(0, 1), (0, n)]:
    for _ in range(2):
        ctx.clear()
        ctx.render(1024, 1024, 256, max_bounces=8, rank=r, nranks=k)
    assert lib.pt_dbg_path_timing(buf, NW) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(NW, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    st, dr, en, ch = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, (a[:, 2] - t0) / 100.0, a[:, 3]
    # wall_clock64: 100 MHz -> /100 = microseconds
    q = lambda x: " ".join(f"{v:8.1f}" for v in np.percentile(x, [0, 1, 10, 50, 90, 99, 100]))
    print(f"{name} share {r}/{k}: waves {len(a)} chunks/wave {ch.mean():.2f} (min {ch.min()} max {ch.max()})")
    print("   pct        0        1       10       50       90       99      100  (us)")
    print("   start ", q(st))
    print("   drain ", q(dr))
    print("   end   ", q(en))
    print("   end-drain", q(en - dr))
    print("   grab total", q(a[:, 4] / 100.0), " max", q(a[:, 5] / 100.0))
    # active-wave profile over time
    T = en.max()
    for f in (0.5, 0.8, 0.9, 0.95, 0.98):
        print(f"   waves alive at {f:.2f} T ({f * T:7.1f} us): {(en > f * T).sum()}  drained-not-done {((dr < f * T) & (en > f * T)).sum()}")
