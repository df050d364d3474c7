#!/bin/bash
# Interleaved A/B of environment knobs on several workloads, REPS times:
#   SCENES="CBbunny dragon_proxy" REPS=2 bash scripts/dev/ab_env_rep.sh "PT_NO_ROOT_CLUSTER=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for rep in $(seq ${REPS:-2}); do
  for sc in ${SCENES:-CBbunny}; do
    bash scripts/dev/ab_env.sh $sc "$@" || exit 1
  done
done
