"""Per-level PMC of k_trace_level (and k_shade_push) from one scene's pmc passes:
  python scripts/dev/level_pmc.py <scene> <first_level> <last_level>
  python scripts/dev/level_pmc.py <scene> 2,4,6,7,8     (the launched levels of a pass, in order)"""
import collections
import csv
import glob
import sys

sc = sys.argv[1]
if "," in sys.argv[2]:
    LEVELS = [int(x) for x in sys.argv[2].split(",")]
else:
    LEVELS = list(range(int(sys.argv[2]), int(sys.argv[3]) + 1))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in sorted(glob.glob(f"gpurun_out/pmc_{sc}_[0-9]/**/*counter_collection.csv", recursive=True)):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    lvl, i = {}, 0
    for r in rows:
        d = int(r["Dispatch_Id"])
        if any(k in r["Kernel_Name"] for k in ("k_trace_level", "k_trace_real", "k_trace_leaves")) and d not in lvl:
            lvl[d] = LEVELS[i % len(LEVELS)]
            i += 1
    for r in rows:
        d = int(r["Dispatch_Id"])
        k = "shade" if "k_shade_push" in r["Kernel_Name"] else (f"L{lvl[d]}" if d in lvl else None)
        if not k:
            continue
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        if c == "FETCH_SIZE":
            c, v = "rd", 2 * v * 1024
        elif c == "WRITE_SIZE":
            c, v = "wr", v * 1024
        agg[k][c] += v
        cnt[(k, f)].add(d)
for k in sorted(agg):
    a = agg[k]
    n = max(len(v) for (kk, f), v in cnt.items() if kk == k)
    wc = max(a["SQ_WAVE_CYCLES"], 1)
    print(f"{k:6s} n={n:4d} rd/launch {a['rd'] / n / 1e9:7.3f} GB  wr {a['wr'] / n / 1e9:6.3f} GB  "
          f"valu/launch {a['SQ_INSTS_VALU'] / n:9.3g}  salu {a['SQ_INSTS_SALU'] / n:9.3g}  "
          f"wait_any {a['SQ_WAIT_ANY'] / wc:.2f} wait_inst {a['SQ_WAIT_INST_ANY'] / wc:.2f} "
          f"active {a['SQ_ACTIVE_INST_ANY'] / wc:.2f}  vmem_rd {a['SQ_INSTS_VMEM_RD'] / n:8.3g} smem {a['SQ_INSTS_SMEM'] / n:8.3g}")
