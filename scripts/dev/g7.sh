# dev: parity subset, then env-knob A/B per scene: VARS="PT_X=0 ..." SCENES="..." bash scripts/dev/g7.sh
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || { echo "rebuild before gpurun"; exit 3; }
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${K:-parity or bunny or fullsize or render or regress or progressive or scotty}" > gpurun_out/t_sub.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t_sub.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/t_sub.log; exit $rc; }; }
for sc in ${SCENES:-CBbunny dragon_proxy bunny}; do bash scripts/dev/ab_env.sh $sc $VARS || exit 1; done
