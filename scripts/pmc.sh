#!/bin/bash
# HBM traffic counters (separate --pmc passes, kernel dispatch only) for one
# bench frame: PMC_ARGS are bench.py arguments.  Output: gpurun_out/pmc_<tag>_<counter>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
TAG=${TAG:-run}
for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_$c -o run -- \
    python bench.py --steps 1 --warmup 0 --no-cpu ${PMC_ARGS:-} > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "=== pmc $c rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_${TAG}_$c.log; exit $rc; }
done
exit 0
