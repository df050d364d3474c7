#!/bin/bash
# A/B of library variants with a filtered parity-test subset per variant:
#   VARIANTS="base x" K="render or parity" BENCH_ARGS="..." bash scripts/ab_k.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  if [ -n "$K" ]; then
    PTCORE_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -k "$K" > $OUT/abk_test_$v.log 2>&1
    rc=$?; echo "=== $v tests rc=$rc: $(tail -1 $OUT/abk_test_$v.log)"
    [ $rc -ne 0 ] && exit $rc
  fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-cpu --steps 3} > $OUT/ab_bench_$v.log 2>&1
  rc=$?; echo "=== $v bench rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/ab_bench_$v.log; exit $rc; }
done
exit 0
