#!/bin/bash
# Instruction-level PMC pass per library variant (one rocprofv3 run each):
#   VARIANTS="base pair" CTRS="SQ_WAVES SQ_INSTS_VALU ..." PMC_ARGS="--scene CBempty --configs none --spp 32" bash scripts/pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"}
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  PTCORE_LIB=$PWD/$lib timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmcab_$v -o run -- \
    python bench.py --steps 1 --warmup 0 --no-cpu ${PMC_ARGS:---scene CBempty --configs none --spp 32} > gpurun_out/pmcab_$v.log 2>&1
  rc=$?; echo "=== pmc $v rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/pmcab_$v.log; exit $rc; }
done
python3 scripts/pmc_ab_summary.py ${VARIANTS:-base}
