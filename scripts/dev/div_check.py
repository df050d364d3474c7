"""Where the triangle test's division (div_rn) differs from IEEE (dev tool)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import numpy as np
import torch  # noqa (HIP runtime first)
import ptrace
ctx = ptrace.Context(0)
rng = np.random.default_rng(5)
n = 20_000_000
en = rng.integers(-60, 41, n); ed = rng.integers(-60, 5, n)
num = (rng.uniform(1, 2, n) * np.exp2(en) * rng.choice([-1, 1], n)).astype(np.float32)
den = (rng.uniform(1, 2, n) * np.exp2(ed) * rng.choice([-1, 1], n)).astype(np.float32)
q = ctx.check_division(num, den)
ref = num / den
bad = q.view(np.uint32) != ref.view(np.uint32)
print("mismatches", bad.sum(), "of", n)
if bad.any():
    eq = np.floor(np.log2(np.abs(ref[bad].astype(np.float64))))
    print("quotient exponent range of mismatches", eq.min(), eq.max())
    print("num exp", en[bad].min(), en[bad].max(), "den exp", ed[bad].min(), ed[bad].max())
    d = (q[bad].view(np.int32).astype(np.int64) - ref[bad].view(np.int32).astype(np.int64))
    print("ulp diffs", np.unique(d, return_counts=True))
    for i in np.nonzero(bad)[0][:8]:
        print(repr(num[i]), repr(den[i]), repr(q[i]), repr(ref[i]))
    # mismatch rate by quotient exponent bucket
    eall = np.floor(np.log2(np.abs(ref.astype(np.float64)) + 1e-300))
    for lo in range(-70, 110, 10):
        m = (eall >= lo) & (eall < lo + 10)
        if m.any():
            print(f"q exp [{lo},{lo+10}): {bad[m].sum()} / {m.sum()}")
