cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="base bestbf" K="test_render_bit_exact or fullsize or furnace" BENCH_ARGS="--no-cpu --steps 3 --configs CBspheres --config5 off --ref-arith none --no-1spp" bash scripts/ab_k.sh || exit $?
for v in base bestbf; do mv gpurun_out/ab_bench_$v.log gpurun_out/ab_empty_$v.log; done
VARIANTS="base rootbr1" K="test_render_bit_exact or dragon or bunny_dae or closest or fullsize" BENCH_ARGS="--no-cpu --steps 2 --scene dragon_proxy --configs CBbunny,bunny --config5 off --ref-arith none --no-1spp" bash scripts/ab_k.sh
