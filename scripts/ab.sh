#!/bin/bash
# A/B timing of library variants on one GPU box:  VARIANTS="base lds" bash scripts/ab.sh
# base = lib/libptcore.so, x = lib/libptcore_x.so.  Each variant: GPU parity
# tests, then the bench (BENCH_ARGS).  Stops at the first fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  if [ -z "$NOTEST" ]; then
    PTCORE_LIB=$PWD/$lib timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/ab_test_$v.log 2>&1
    rc=$?; echo "=== $v tests rc=$rc: $(tail -1 $OUT/ab_test_$v.log)"
    [ $rc -gt 1 ] && exit $rc
  fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 600 python bench.py ${BENCH_ARGS:---spp 32 --steps 3 --no-cpu} > $OUT/ab_bench_$v.log 2>&1
  rc=$?; echo "=== $v bench rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/ab_bench_$v.log; exit $rc; }
done
exit 0
