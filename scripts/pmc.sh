#!/bin/bash
# rocprofv3 --pmc passes (kernel dispatch counters only, one pass per entry of
# PASSES, ';'-separated) over one bench frame; PMC_ARGS are bench.py arguments.
# Output: gpurun_out/pmc_<TAG>_<n>/run_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
TAG=${TAG:-run}
IFS=';' read -ra P <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE}"
n=0
for c in "${P[@]}"; do
  timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_$n -o run -- \
    python bench.py --steps 1 --warmup 0 --no-cpu --no-1spp --no-executed --detail-out gpurun_out/pmc_${TAG}_$n.detail.json ${PMC_ARGS:-} > gpurun_out/pmc_${TAG}_$n.log 2>&1
  rc=$?; echo "=== pmc [$c] rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_${TAG}_$n.log; exit $rc; }
  n=$((n+1))
done
exit 0
