cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
for v in base w7 base w7; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 4 --configs CBspheres --config5 off --ref-arith none --no-1spp >> gpurun_out/ab6_$v.log 2>&1 || exit $?
  echo "=== $v ok"
done
PTCORE_LIB=$PWD/cuda-raytracer_amd/lib/libptcore_w7.so PASSES="WRITE_SIZE;FETCH_SIZE" TAG=w7 PMC_ARGS="--configs none --config5 off --ref-arith none" bash scripts/pmc.sh
