"""BASELINE.md §2 table rows from a round's bench line (dev tool):

  python scripts/dev/baseline_rows.py profiles/r04/bench_default.json

Prints one markdown row per workload of the line (headline first, then
`configs` in order) with Mrays/s, ms/frame, the dominant kernel's algorithmic
rate and fraction, and the other kernel's where the line has one."""
import json
import sys

d = json.load(open(sys.argv[1]))


def rate(r):
    if not r:
        return "", ""
    unit = "TFLOP/s" if r.get("bound") == "valu" or r.get("kernel") == "k_path_leaf" else "GB/s"
    name = r.get("kernel", "").replace("k_trace_real+k_trace_leaves+k_trace_level", "levels")
    return f"`{name}` {r['achieved']:,.1f} {unit}" if unit == "TFLOP/s" else f"`{name}` {r['achieved']:,.0f} {unit}", \
        f"{r['frac']:.3f}"


rows = [dict(scene=d["config"].get("scene", "CBempty"), value=d["value"], ms_per_frame=d["ms_per_frame"],
             roofline=d["roofline"], roofline_other=None, config=d["config"].get("workload", ""))]
rows += d.get("configs", [])
for r in rows:
    a, fa = rate(r.get("roofline"))
    b, fb = rate(r.get("roofline_other"))
    extra = f"; {b}" if b else ""
    fextra = f"; {fb}" if fb else ""
    print(f"| {r['scene']} | {r.get('config', '')} | {r['value']:,.0f} | {r['ms_per_frame']:,.2f} | {a}{extra} | "
          f"{fa}{fextra} |")
cb = d.get("cpu_baseline")
if cb:
    print(f"\ncpu_baseline: {cb['value']} {cb['unit']} on {cb['cores']} cores ({cb['kind']}): {cb['sample']}")
