cd "${GRAFT_REPO_ROOT}"
for v in base old base old; do
  lib=cuda-raytracer_amd/lib/libptcore.so; [ $v = old ] && lib=cuda-raytracer_amd/lib/libptcore_old.so
  echo "== $v"; PTCORE_LIB=$PWD/$lib timeout -k 10 120 python scripts/dev/share_time.py CBempty 8 5 || exit $?
done > gpurun_out/share.log 2>&1
cat gpurun_out/share.log
VARIANTS="base s3 s3nd" K="render_bit_exact or dragon or bunny_dae or ray_count or batching or sharding" BENCH_ARGS="--scene CBbunny --configs dragon_proxy,bunny --config5 off --no-cpu --steps 3" bash scripts/ab_k.sh
