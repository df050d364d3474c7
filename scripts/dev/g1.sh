cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t_all.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_all.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke fail; tail gpurun_out/smoke.log; exit 1; }
echo smoke ok
TESTS=none STEPS=2 BENCH_ARGS="--config5 off" bash scripts/quick.sh || exit 1
TESTS=0 SCENES="dragon_proxy bunny" bash scripts/dev/ab_dfs.sh
