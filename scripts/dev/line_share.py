"""Distinct memory lines touched by the level items' ray-record gathers
(diagnostic build: make variant NAME=ln DEFS=-DPT_DBG_LINES=1, run with
PTCORE_LIB=lib/libptcore_ln.so):  python scripts/dev/line_share.py <scene>...
Per item kind (interior / leaf): rays gathered, and the lines they touch for
records of 32 B (as built), 16 B and 8 B -- what a smaller traversal record
would save on random gathers that each cost a whole 128-B line."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import torch  # noqa: E402,F401
import ptrace  # noqa: E402
import scenes  # noqa: E402

lib = ptrace.LIB
buf = (C.c_ulonglong * 8)()
for name in sys.argv[1:]:
    ctx = ptrace.Context(0)
    ctx.load_scene(scenes.load(name))
    ctx.clear()
    ctx.render(1024, 1024, 16, max_bounces=8)
    assert lib.pt_dbg_lines(buf) == 0
    for kind, o in (("interior", 0), ("leaf", 4)):
        rays, l32, l16, l8 = (buf[o + i] for i in range(4))
        if not rays:
            continue
        print(f"{name:20s} {kind:8s} rays {rays / 1e6:9.1f} M  rays per line: 32-B records {rays / l32:.3f}"
              f"  16-B {rays / l16:.3f}  8-B {rays / l8:.3f}  ->  B per ray of 128-B lines: "
              f"{128 * l32 / rays:.1f} / {128 * l16 / rays:.1f} / {128 * l8 / rays:.1f}", flush=True)
    del ctx
