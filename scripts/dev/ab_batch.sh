#!/bin/bash
# Pool-size sweep: bench.py --batch B for the traversal workloads (one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || exit 3
for b in ${BATCHES:-0 4194304 8388608 16777216}; do
  timeout -k 10 300 python bench.py --scene ${SCENE:-dragon_proxy} --configs ${CONFIGS:-CBbunny} --config5 off --ref-arith none --no-cpu --no-1spp --steps 2 --warmup 1 --batch $b --detail-out gpurun_out/batch_$b.json > gpurun_out/batch_$b.log 2>&1 || { echo "batch $b failed"; tail -5 gpurun_out/batch_$b.log; exit 1; }
  python - "$b" <<'PY'
import json, sys
b = sys.argv[1]
d = [json.loads(l) for l in open(f"gpurun_out/batch_{b}.log") if l.startswith("{")][-1]
t = json.load(open(f"gpurun_out/batch_{b}.json"))
rows = [t["headline"]] + t["configs"]
print(b, " | ".join(f"{r['scene']} {r['value']:.0f} Mrays/s {r['ms_per_frame']:.1f} ms levels {r['trace']['ms_levels']} shade {r['trace']['ms_shade_push']} scan {r['trace']['ms_scan']} passes {r['trace']['passes']}" for r in rows), flush=True)
PY
done
