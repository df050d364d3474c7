#!/bin/bash
# A/B of environment knobs on one workload: bash scripts/dev/ab_env.sh <scene> "<ENV=1 ...>" ...
# Prints the level breakdown per variant (bench line gpurun_out/ab_<n>.log, detail ab_<n>.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
sc=$1; shift
n=0
for v in "" "$@"; do
  env $v timeout -k 10 300 python bench.py --scene $sc --configs none --config5 off --no-cpu --steps 2 --warmup 1 \
    --detail-out gpurun_out/ab_$n.json > gpurun_out/ab_$n.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/ab_$n.log; exit 1; }
  python - "$v" gpurun_out/ab_$n.log gpurun_out/ab_$n.json <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
t = json.load(open(sys.argv[3]))["headline"]["trace"]
lv = " ".join(f"L{x['level']}:{x['ms']:.1f}/s{x.get('scan_ms', 0):.1f}" for x in t["levels"])
print(f"[{sys.argv[1] or 'base'}] {d['value']:.0f} Mrays/s {d['ms_per_frame']:.1f} ms  levels {t['ms_levels']:.1f} shade {t['ms_shade_push']:.1f} scan {t['ms_scan']:.1f} | {lv}", flush=True)
PY
  n=$((n+1))
done
