#!/bin/bash
# GPU parity tests on a library variant, then an interleaved A/B bench:
#   V=cl K="parity or fullsize" bash scripts/dev/ab_variant.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || exit 3
lib=$PWD/cuda-raytracer_amd/lib/libptcore_$V.so
PTCORE_LIB=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/var_$V.log 2>&1
rc=$?; echo "=== $V tests rc=$rc: $(tail -1 gpurun_out/var_$V.log)"
[ $rc -ne 0 ] && { tail -30 gpurun_out/var_$V.log; exit $rc; }
VARIANTS="base $V" CONFIGS=${CONFIGS:-CBspheres} bash scripts/dev/ab_quick.sh
