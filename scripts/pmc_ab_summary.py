"""Per-kernel mean of each PMC counter over dispatches (gpurun_out/pmcab_<variant>)."""
import csv, glob, sys
from collections import defaultdict
for v in sys.argv[1:]:
    files = glob.glob(f"gpurun_out/pmcab_{v}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-40:]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    print(f"== {v}")
    for k, c in acc.items():
        d = len(n[k])
        print(f"  {k}  dispatches={d}")
        for name, val in sorted(c.items()):
            print(f"     {name:24s} {val/d:16.4g}")
