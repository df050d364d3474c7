cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -k "render or path or fullsize or furnace or analytic or scotty" > gpurun_out/t7.log 2>&1
rc=$?; echo "=== tests rc=$rc: $(tail -1 gpurun_out/t7.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t7.log; exit $rc; }
for v in base old base old; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 4 --configs CBspheres --config5 off --ref-arith none --no-1spp >> gpurun_out/ab7_$v.log 2>&1 || exit $?
  echo "=== $v ok"
done
PTCORE_LIB=$PWD/cuda-raytracer_amd/lib/libptcore.so PASSES="WRITE_SIZE;FETCH_SIZE" TAG=new PMC_ARGS="--configs none --config5 off --ref-arith none" bash scripts/pmc.sh
