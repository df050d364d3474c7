#!/bin/bash
# DFS cut A/B: parity subset with the cut on, then levels per cut (dev tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
[ "${TESTS:-1}" = 1 ] && { PT_DFS_LEVEL=${TEST_CUT:-0} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  -k "${K:-closest or dragon or bunny_dae or render_bit_exact or tmin or bvhaccel}" > gpurun_out/dfs_test.log 2>&1
rc=$?; echo "=== tests rc=$rc: $(tail -1 gpurun_out/dfs_test.log)"
[ $rc -ne 0 ] && { tail -30 gpurun_out/dfs_test.log; exit $rc; }; }
for sc in ${SCENES:-dragon_proxy CBbunny bunny}; do
  echo "--- $sc"
  bash scripts/dev/ab_env.sh $sc ${CUTS:-PT_DFS_LEVEL=0 PT_DFS_LEVEL=1 PT_DFS_LEVEL=2} || exit 1
done
