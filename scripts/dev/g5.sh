cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${K:-cull or bunny or fullsize or render or regress}" > gpurun_out/t_sub.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t_sub.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_sub.log; exit $rc; }
for v in ${VARS:-PT_CULL_CAMERA=0 PT_CULL_BLOCK=256 PT_CULL_BLOCK=1024 PT_CULL_BLOCK=2048}; do
for sc in ${SCENES:-bunny}; do
env $v timeout -k 10 300 python bench.py --scene $sc --configs none --config5 off --no-cpu --steps 2 --warmup 1 --ref-arith none > gpurun_out/b.log 2>&1 || exit 1
python - "$v $sc" <<'PY'
import json,sys
l=[x for x in open("gpurun_out/b.log") if x.startswith("{")][-1]; d=json.loads(l)
t=d['trace']; print(sys.argv[1], d['value'], d['ms_per_frame'], 'passes', t['passes'], 'shade', t['ms_shade_push'], 'lv', t['ms_levels'], 'scan', t['ms_scan'], 'sv', d['roofline'].get('shaded_vertices') or (d.get('roofline_other') or [{}])[0].get('shaded_vertices'), flush=True)
PY
done; done
