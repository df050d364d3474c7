#!/bin/bash
# A/B of bench.py arguments on one workload: bash scripts/dev/ab_args.sh <scene> "<args>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
sc=$1; shift
n=0
for v in "" "$@"; do
  timeout -k 10 300 python bench.py --scene $sc --configs none --config5 off --no-cpu --steps 2 --warmup 1 $v \
    --detail-out gpurun_out/aba_$n.json > gpurun_out/aba_$n.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/aba_$n.log; exit 1; }
  python - "$v" gpurun_out/aba_$n.log gpurun_out/aba_$n.json <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
t = json.load(open(sys.argv[3]))["headline"]["trace"]
lv = " ".join(f"L{x['level']}:{x['ms']:.1f}" for x in t["levels"])
print(f"[{sys.argv[1] or 'base'}] {d['value']:.0f} Mrays/s {d['ms_per_frame']:.1f} ms  levels {t['ms_levels']:.1f} shade {t['ms_shade_push']:.1f} scan {t['ms_scan']:.1f} passes {t['passes']} | {lv}", flush=True)
PY
  n=$((n+1))
done
