#!/bin/bash
# One rank's 1/N share of CBempty under path-scheduling knobs:
#   N=8 bash scripts/dev/share_sweep.sh "PT_PATH_GUIDE=2" "PT_PATH_REGIONS=16"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in "" "$@"; do
  echo "== [${v:-base}]"
  env $v timeout -k 10 120 python scripts/dev/share_time.py ${SCENE:-CBempty} ${N:-8} 5 | grep "share 0/${N:-8}" || exit 1
done
