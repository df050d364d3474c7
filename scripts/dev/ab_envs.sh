#!/bin/bash
# Interleaved A/B of environment settings on the headline + CONFIGS:
#   ENVS="PT_COPY_BLOCKS=0 PT_COPY_BLOCKS=64" bash scripts/dev/ab_envs.sh
cd ${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || exit 3
for rep in 1 2; do
for e in $ENVS; do
  env $e timeout -k 10 300 python bench.py --no-cpu --configs ${CONFIGS:-none} --config5 off --ref-arith none --steps 10 > gpurun_out/abe.log 2>&1 || { tail -20 gpurun_out/abe.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/abe.log') if l.startswith('{')][-1]
print('$e', d['value'], d['ms_per_step'], [(c['scene'], c['value'], c['ms_per_frame']) for c in d['configs']], flush=True)"
done
done
