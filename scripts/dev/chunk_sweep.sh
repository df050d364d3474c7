#!/bin/bash
# k_path_leaf grab size and path regions against the launch size: the whole
# frame and one rank's 1/8 share of CBempty and CBspheres (share_time.py)
#   CHUNKS="512 256" REGIONS="8 16" bash scripts/dev/chunk_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in ${REGIONS:-8}; do
for c in ${CHUNKS:-512 256 128}; do
  for s in ${SCENES:-CBempty CBspheres}; do
    PT_PATH_REGIONS=$r PT_PATH_CHUNK=$c timeout -k 10 200 python scripts/dev/share_time.py $s 1,8 5 > gpurun_out/chunk_${r}_${c}_$s.log 2>&1 || exit $?
    echo "regions $r chunk $c: $(grep -h share gpurun_out/chunk_${r}_${c}_$s.log | sed 's/ (median[^)]*)//;s/get_image [0-9.]* ms//;s/GPU total [0-9.]* ms//' | tr '\n' ' ')"
  done
done
done
