#!/bin/bash
# Round profile set (run on the GPU box):  bash scripts/profile_round.sh
#   gpurun_out/bench.log                     the default bench line
#   gpurun_out/prof_<scene>/                 rocprofv3 --kernel-trace --stats of
#                                            one bench frame of that workload alone
#   gpurun_out/pmc_<scene>_<n>/              rocprofv3 --pmc passes (scripts/pmc.sh)
# Summaries for profiles/<round>/ are made locally afterwards
# (scripts/pmc_summary.py, scripts/collect_profiles.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
SCENES=${PMC_SCENES:-CBempty CBspheres CBbunny bunny dragon_proxy dragon_proxy_gpubvh}
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "bench ok"
fi
[ -z "$NO_PROF" ] && for sc in $SCENES; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$sc -o run --output-format csv -- \
    python bench.py --scene $sc --configs none --config5 off --ref-arith none --steps 1 --warmup 0 --no-cpu --no-1spp --no-executed --detail-out gpurun_out/prof_$sc.detail.json \
    > gpurun_out/prof_$sc.log 2>&1 || { echo "rocprof $sc rc=$?"; exit 1; }
  echo "rocprof $sc ok"
done
[ -n "$NO_PMC" ] && exit 0
PASSES=${PASSES:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"}
for sc in $SCENES; do
  TAG=$sc PMC_ARGS="--scene $sc --configs none --config5 off --ref-arith none" PASSES="$PASSES" bash scripts/pmc.sh || exit 1
done
echo "pmc ok"
