#!/bin/bash
# GPU tests, smoke, the default bench line and the rocprofv3 stats set of a round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "=== tests rc=$rc: $(tail -1 gpurun_out/t_all.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_all.log; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
echo "=== smoke ok"
NO_PMC=1 bash scripts/profile_round.sh
