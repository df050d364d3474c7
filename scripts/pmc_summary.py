#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes per kernel (and per traversal level).

  python scripts/pmc_summary.py <run_counter_collection.csv>... [--levels L]
                                 [--json OUT --config "what was run"]

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts 128-B
memory-side requests at 64 B (MI355X_MICROARCH.md, HBM section), so the
corrected read bytes are 2 x FETCH_SIZE; the table shows them as READ_GB and
WRITE_GB.  With --levels L, k_trace_level dispatches are split by level
(launch order cycles through levels F..L-1 in every traversal pass; F =
--first-level, default 1, 2 for trees whose root pass skips level 1).
"""
import csv
import sys
from collections import defaultdict


def short(name):
    """pt::k_shade_push<16, 1>(pt::ShadeArgs) -> k_shade_push (also for
    kernels in an anonymous namespace: "(anonymous namespace)::pt::...")"""
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0].strip().split("::")[-1]


def main():
    args = sys.argv[1:]
    opts = {}
    for o in ("--levels", "--first-level", "--json", "--config"):
        if o in args:
            i = args.index(o)
            opts[o] = args[i + 1]
            del args[i:i + 2]
    levels = int(opts.get("--levels", 0))
    first = int(opts.get("--first-level", 1))  # 2 when the root pass skips level 1
    agg = defaultdict(lambda: defaultdict(float))  # key -> counter -> value
    ndisp = defaultdict(set)
    per_file = defaultdict(dict)  # key -> path -> dispatch ids
    for path in args:
        rows = []
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append(r)
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        lvl_of = {}
        li = 0
        for r in rows:
            d = int(r["Dispatch_Id"])
            k = short(r["Kernel_Name"])
            if levels and k == "k_trace_level" and d not in lvl_of:
                lvl_of[d] = li % (levels - first) + first
                li += 1
        for r in rows:
            d = int(r["Dispatch_Id"])
            k = short(r["Kernel_Name"])
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            if c == "FETCH_SIZE":
                c, v = "READ_GB", 2 * v * 1024 / 1e9
            elif c == "WRITE_SIZE":
                c, v = "WRITE_GB", v * 1024 / 1e9
            keys = [k] + ([f"{k}[L{lvl_of[d]}]"] if d in lvl_of else [])
            for key in keys:
                agg[key][c] += v
                ndisp[key].add((path, d))
                per_file[key].setdefault(path, set()).add(d)
    counters = sorted({c for a in agg.values() for c in a})
    print(f"{'kernel':22s} {'disp':>5s} " + " ".join(f"{c[:16]:>16s}" for c in counters))
    for key in sorted(agg, key=lambda k: (k.split("[")[0], k)):
        a = agg[key]
        print(f"{key:22s} {len(ndisp[key]):5d} " + " ".join(f"{a.get(c, 0):16.4g}" for c in counters))
    if "--json" in opts:
        import json
        ker = {}
        for key, a in agg.items():
            n = max(len(v) for v in per_file[key].values())
            e = {"dispatches": n}
            if "READ_GB" in a and "WRITE_GB" in a:
                e["read_bytes_per_launch"] = int(a["READ_GB"] * 1e9 / n)
                e["write_bytes_per_launch"] = int(a["WRITE_GB"] * 1e9 / n)
                e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
            for c, v in a.items():
                if c not in ("READ_GB", "WRITE_GB"):
                    e[c] = v
            ker[key] = e
        with open(opts["--json"], "w") as f:
            json.dump({"config": opts.get("--config", ""), "files": [str(p) for p in args],
                       "correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; KiB -> bytes",
                       "kernels": ker}, f, indent=1)


if __name__ == "__main__":
    main()
