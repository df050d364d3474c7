# full GPU tests + smoke on the default library, then path-kernel share times
# (default vs the pre-guided library) and the default bench line
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_run.sh test || exit $?
for v in base old base; do
  lib=cuda-raytracer_amd/lib/libptcore.so; [ $v = old ] && lib=cuda-raytracer_amd/lib/libptcore_old.so
  echo "== $v"; PTCORE_LIB=$PWD/$lib timeout -k 10 120 python scripts/dev/share_time.py CBempty 8 5 || exit $?
done > gpurun_out/share.log 2>&1
cat gpurun_out/share.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
echo bench ok
