#!/bin/bash
# Quick GPU iteration: parity tests (optional filter), then a short bench.
#   K="path_leaf or render" BENCH_ARGS="--configs CBspheres" bash scripts/quick.sh   (TESTS=none: no tests)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
if [ "${TESTS:-all}" != none ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 ${K:+-k "$K"} > $OUT/quick_test.log 2>&1
  rc=$?; echo "=== tests rc=$rc: $(tail -1 $OUT/quick_test.log)"
  [ $rc -ne 0 ] && { tail -30 $OUT/quick_test.log; exit $rc; }
fi
timeout -k 10 600 python bench.py --no-cpu --steps ${STEPS:-2} ${BENCH_ARGS:-} > $OUT/quick_bench.log 2>&1
rc=$?; echo "=== bench rc=$rc"
[ $rc -ne 0 ] && { tail -20 $OUT/quick_bench.log; exit $rc; }
python - <<'PY'
import json
for line in open("gpurun_out/quick_bench.log"):
    if line.startswith("{"):
        d = json.loads(line)
        rows = [dict(scene=d["config"]["scene"], value=d["value"], ms_per_frame=d["ms_per_frame"], roofline=d["roofline"], trace=d.get("trace"))] + d.get("configs", [])
        for r in rows:
            rf = r["roofline"]; tr = r.get("trace") or {}
            print(f'{r["scene"]:20s} {r["value"]:10.1f} Mrays/s {r["ms_per_frame"]:8.2f} ms  {rf["kernel"]} {rf["frac"]:.4f}  path {tr.get("ms_path")} shade {tr.get("ms_shade")} levels {tr.get("ms_levels")} scan {tr.get("ms_scan")}')
            for l in tr.get("levels", []):
                print(f'    L{l["level"]}: {l["ms"]:7.2f} ms  {l["Gvisits_per_s"]:6.2f} Gv/s leaf {l["leaf_visits"]/max(1,l["visits"]):.2f}')
PY
