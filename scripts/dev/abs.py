"""Summarise A/B bench logs (dev tool): python scripts/dev/abs.py gpurun_out/ab_*.log"""
import json, sys
for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        rows = [dict(scene=d["config"]["scene"], value=d["value"], ms_per_frame=d["ms_per_frame"], roofline=d["roofline"],
                     trace=d.get("trace"))] + d.get("configs", [])
        for r in rows:
            tr = r.get("trace") or {}
            lv = " ".join(f'L{l["level"]}:{l["ms"]:.1f}' for l in tr.get("levels", []))
            print(f'{f.split("/")[-1]:24s} {r["scene"]:18s} {r["value"]:9.1f} Mr/s {r["ms_per_frame"]:8.2f} ms  '
                  f'path {tr.get("ms_path")} shade {tr.get("ms_shade_push")} lv {tr.get("ms_levels")} scan {tr.get("ms_scan")} {lv}')
