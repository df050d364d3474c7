cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out

VARIANTS="base br1 br2" K="test_render_bit_exact or fullsize or analytic and furnace" BENCH_ARGS="--no-cpu --steps 3 --configs CBspheres --config5 off --ref-arith none --no-1spp" bash scripts/ab_k.sh
