cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/t5.log 2>&1
rc=$?; echo "=== tests rc=$rc: $(tail -1 gpurun_out/t5.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t5.log; exit $rc; }
for v in base noselect base noselect; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 3 --configs CBbunny,dragon_proxy --config5 off --ref-arith none --no-1spp >> gpurun_out/ab5_$v.log 2>&1 || exit $?
  echo "=== $v ok"
done
PASSES="WRITE_SIZE;FETCH_SIZE" TAG=empty PMC_ARGS="--configs none --config5 off --ref-arith none" bash scripts/pmc.sh
