# dev: per-pass kernel traces of one scene under env variants: SC=CBbunny VARS="A=1 A=2" bash scripts/dev/g9.sh
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
n=0
for v in "PT_NONE=0" $VARS; do
  env $v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_$n -o run --output-format csv -- python bench.py --scene ${SC:-CBbunny} --configs none --config5 off --no-cpu --steps 1 --warmup 0 --no-1spp --ref-arith none > gpurun_out/kt.log 2>&1 || exit 1
  echo "== $v"; python scripts/dev/pass_trace.py gpurun_out/kt_$n/run_kernel_trace.csv | tail -${NP:-20}
  n=$((n+1))
done
