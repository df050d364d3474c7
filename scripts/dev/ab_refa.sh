#!/bin/bash
# The CBbunny PT_FLAG_REF_ARITH line with and without an environment knob, REPS times:
#   REPS=2 bash scripts/dev/ab_refa.sh PT_NO_ROOT_CLUSTER=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for rep in $(seq ${REPS:-2}); do
  for v in "" "$@"; do
    env $v timeout -k 10 300 python bench.py --scene CBempty --configs none --config5 off --ref-arith CBbunny --no-cpu \
      --no-1spp --steps 2 --warmup 1 > gpurun_out/refa.log 2>&1 || { echo "[$v] failed"; tail -5 gpurun_out/refa.log; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/refa.log') if l.startswith('{')][-1]
print('[${v:-base}]', [(c['scene'], c['value'], c['ms_per_frame'], c['config'][-16:]) for c in d['configs']], flush=True)"
  done
done
