"""Per-pass kernel times of the last frame in a rocprofv3 kernel trace (dev tool):
python scripts/dev/pass_trace.py gpurun_out/kt_1/run_kernel_trace.csv
A pass starts at each k_shade_push / k_camera_push dispatch; prints the shade
kernel's duration, the level kernels' and scans' sum and the gap (idle GPU
time between dispatches) per pass of the last frame."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
frames = [i for i, r in enumerate(rows) if "k_camera_push" in r["Kernel_Name"]]
# the first frame of the run (bench: the timed frame; later ones are the
# instrumented frame and other flag sets)
start = frames[0]
end = frames[1] if len(frames) > 1 else len(rows)
passes, cur = [], None
prev_end = None
for r in rows[start:end]:
    m = re.search(r"\b(k_\w+)", r["Kernel_Name"])
    k = m.group(1) if m else r["Kernel_Name"][:30]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if k in ("k_shade_push", "k_camera_push"):
        cur = {"shade": 0.0, "levels": 0.0, "scan": 0.0, "other": 0.0, "gap": 0.0, "n": 0}
        passes.append(cur)
    if cur is None:
        continue
    d = (e - s) / 1e6
    cur["n"] += 1
    if prev_end is not None and s > prev_end:
        cur["gap"] += (s - prev_end) / 1e6
    prev_end = max(prev_end or 0, e)
    if k in ("k_shade_push", "k_camera_push"):
        cur["shade"] += d
    elif k.startswith("k_trace"):
        cur["levels"] += d
    elif k.startswith("k_scan"):
        cur["scan"] += d
    else:
        cur["other"] += d
tot = {k: 0.0 for k in ("shade", "levels", "scan", "other", "gap")}
for i, p in enumerate(passes):
    print(f"pass {i:2d}: shade {p['shade']:6.3f}  levels {p['levels']:6.3f}  scan {p['scan']:6.3f}  other {p['other']:6.3f}  gap {p['gap']:6.3f} ms  ({p['n']} dispatches)")
    for k in tot:
        tot[k] += p[k]
print("total:", {k: round(v, 2) for k, v in tot.items()})
