#!/bin/bash
# Round profile set (run on the GPU box):  bash scripts/profile_round.sh
#   gpurun_out/bench.log, gpurun_out/prof/ (rocprofv3 kernel stats of the same
#   bench command), gpurun_out/pmc_<scene>_{0,1}/ (FETCH_SIZE, WRITE_SIZE passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "bench ok"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --steps 1 --warmup 0 --no-cpu --no-1spp > gpurun_out/prof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "rocprof ok"
for sc in ${PMC_SCENES:-CBempty CBspheres CBbunny dragon_proxy dragon_proxy_gpubvh}; do
  TAG=$sc PMC_ARGS="--scene $sc --configs none" PASSES="FETCH_SIZE;WRITE_SIZE" bash scripts/pmc.sh || exit 1
done
echo "pmc ok"
