#!/bin/bash
# Generic A/B (dev tool): optional parity subset on the main lib (K), then
# alternating bench runs of the main lib and variants (VARIANTS), optional PMC
# passes of the main lib (PMC_PASSES, PMC_ARGS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -k "$K" > gpurun_out/abg_test.log 2>&1
  rc=$?; echo "=== tests rc=$rc: $(tail -1 gpurun_out/abg_test.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/abg_test.log; exit $rc; }
fi
for r in $(seq ${REPS:-2}); do
  for v in base ${VARIANTS}; do
    if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
    PTCORE_LIB=$PWD/$lib timeout -k 10 400 python bench.py --no-cpu --steps ${STEPS:-3} --config5 off --ref-arith none --no-1spp ${BENCH_ARGS} >> gpurun_out/abg_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/abg_$v.log; exit 1; }
    echo "=== $v ok"
  done
done
if [ -n "$PMC_PASSES" ]; then
  PASSES="$PMC_PASSES" TAG=abg PMC_ARGS="$PMC_ARGS" bash scripts/pmc.sh || exit 1
fi
exit 0
