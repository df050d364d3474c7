# dev: parity subset, per-pass kernel trace of one scene, short bench of the configs
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${K:-cull or bunny or fullsize or render or regress or progressive}" > gpurun_out/t_sub.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t_sub.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_sub.log; exit $rc; }; }
for sc in ${SC:-bunny}; do timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_$sc -o run --output-format csv -- python bench.py --scene $sc --configs none --config5 off --no-cpu --steps 1 --warmup 0 --no-1spp --ref-arith none > gpurun_out/kt.log 2>&1 || exit 1; echo "== $sc"; python scripts/dev/pass_trace.py gpurun_out/kt_$sc/run_kernel_trace.csv | tail -${NP:-16}; done
[ "${BENCH:-1}" = 1 ] && TESTS=none STEPS=2 BENCH_ARGS="--config5 off --ref-arith none" bash scripts/quick.sh | grep -v "^    L"
