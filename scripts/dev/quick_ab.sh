#!/bin/bash
# Quick GPU check of the working tree: a test subset (K) then N bench runs of
# the headline + CONFIGS.   K="path_leaf or render" N=2 bash scripts/dev/quick_ab.sh
cd ${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || exit 3
if [ "${K:-all}" != none ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/t_q.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_q.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t_q.log | head -30; exit $rc; }
fi
for i in $(seq 1 ${N:-2}); do
timeout -k 10 300 python bench.py --no-cpu --configs ${CONFIGS:-CBspheres} --config5 off --ref-arith none --steps 10 > gpurun_out/b$i.log 2>&1 || { tail -20 gpurun_out/b$i.log; exit 1; }
python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/b$i.log') if l.startswith('{')][-1]
print(d['config']['scene'], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], [ (c['scene'], c['value'], c['ms_per_frame']) for c in d['configs']])"
done
