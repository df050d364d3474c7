"""Per-level bytes per visit (dev tool): joins one scene's PMC passes split by
level (gpurun_out/pmc_<scene>_<n>/, scripts/pmc.sh) with the per-level visit
counts of the bench's detail file, and prints a markdown table.

  python scripts/dev/level_table.py <scene> <levels> [detail.json] [frames]

<levels>: the launched levels of one traversal pass in launch order, e.g.
2,4,6,7,8 (a level runs only when it is real or holds leaves; the sequence of
k_trace_real / k_trace_leaves launches between two shade launches tells which).
The PMC run covers `frames` frames (default 2: bench.py's timed frame and its
instrumented one, same work); the detail file's visits are per frame.
Read bytes are 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import json
import sys

sc = sys.argv[1]
LEVELS = [int(x) for x in sys.argv[2].split(",")]
detail = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/bench_detail.json"
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 2
byts = collections.defaultdict(lambda: [0.0, 0.0])
launches = collections.Counter()
for f in sorted(glob.glob(f"gpurun_out/pmc_{sc}_[0-9]/**/*counter_collection.csv", recursive=True)):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    lvl, i = {}, 0
    for r in rows:
        d = int(r["Dispatch_Id"])
        if any(k in r["Kernel_Name"] for k in ("k_trace_level", "k_trace_real", "k_trace_leaves")) and d not in lvl:
            lvl[d] = LEVELS[i % len(LEVELS)]
            i += 1
    seen = set()
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d not in lvl:
            continue
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        if c == "FETCH_SIZE":
            byts[lvl[d]][0] += 2 * v * 1024
        elif c == "WRITE_SIZE":
            byts[lvl[d]][1] += v * 1024
        else:
            continue
        if (c, d) not in seen:
            seen.add((c, d))
            if c == "FETCH_SIZE":
                launches[lvl[d]] += 1
d = json.load(open(detail))
recs = [d["headline"]] + d.get("configs", [])
rec = next(r for r in recs if r.get("scene") == sc and "REF_ARITH" not in str(r.get("config", ""))
           and "config 5" not in str(r.get("config", "")))
tl = {l["level"]: l for l in rec["trace"]["levels"]}
print(f"{sc}: {rec['trace'].get('passes')} passes per frame, PMC over {frames} frames\n")
print("| level | kind | visits / frame | leaf visits | ms / frame | read GB / frame | written GB / frame | B / visit (read + written) | real TB/s |")
print("|---|---|---|---|---|---|---|---|---|")
tot = [0.0, 0.0, 0, 0.0]
for l in sorted(byts):
    rd, wr = byts[l][0] / frames, byts[l][1] / frames
    t = tl.get(l, {})
    v, lv, ms = t.get("visits", 0), t.get("leaf_visits", 0), t.get("ms", 0.0)
    kind = "real" if (l - LEVELS[0]) % 2 == 0 else "leaf-only"  # (two-level traversal)
    bpv = (rd + wr) / v if v else float("nan")
    print(f"| {l} | {kind} | {v / 1e6:,.1f} M | {lv / 1e6:,.1f} M | {ms:.2f} | {rd / 1e9:.2f} | {wr / 1e9:.2f} | "
          f"{bpv:.0f} | {(rd + wr) / (ms * 1e-3) / 1e12 if ms else 0:.2f} |")
    tot[0] += rd
    tot[1] += wr
    tot[2] += v
    tot[3] += ms
print(f"| all | | {tot[2] / 1e6:,.1f} M | | {tot[3]:.2f} | {tot[0] / 1e9:.2f} | {tot[1] / 1e9:.2f} | "
      f"{(tot[0] + tot[1]) / max(tot[2], 1):.0f} | {(tot[0] + tot[1]) / (tot[3] * 1e-3) / 1e12:.2f} |")
