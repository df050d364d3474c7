# dev: parity subset on the base library, then library A/B per scene (LIBS="base x" SCENES="...")
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${K:-parity or bunny or fullsize or render or regress or progressive or scotty}" > gpurun_out/t_sub.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t_sub.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_sub.log; exit $rc; }; }
for sc in ${SCENES:-CBbunny dragon_proxy bunny}; do
  for rep in ${REPS:-1}; do
  for v in ${LIBS:-base x}; do
    if [ "$v" = base ]; then lib=$PWD/cuda-raytracer_amd/lib/libptcore.so; else lib=$PWD/cuda-raytracer_amd/lib/libptcore_$v.so; fi
    PTCORE_LIB=$lib timeout -k 10 300 python bench.py --scene $sc --configs none --config5 off --no-cpu --steps 2 --warmup 1 --ref-arith none > gpurun_out/ab.log 2>&1 || { echo "$v $sc failed"; tail -5 gpurun_out/ab.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/ab.log") if x.startswith("{")][-1])
t = d["trace"]
print(f"[{sys.argv[1]}] {d['config']['scene']:14s} {d['value']:8.0f} Mrays/s {d['ms_per_frame']:7.2f} ms  levels {t['ms_levels']:.1f} shade {t['ms_shade_push']:.1f} path {t['ms_path']:.1f} scan {t['ms_scan']:.1f}", flush=True)
PY
  done; done
done
