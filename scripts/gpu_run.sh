#!/bin/bash
# One GPU-box session: GPU tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; after a fault/abort/timeout nothing
# else is started (test assertion failures, exit 1, do not stop the session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139|132|135|136) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc), stopping"; exit $rc; fi
  return 0
}
# the shipped libraries must be up to date with their sources
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 900 python bench.py ${BENCH_ARGS:-}
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu --no-1spp ${PROF_ARGS:-}
fi
