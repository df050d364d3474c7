#!/bin/bash
# A/B: CBempty + CBspheres headline frames per variant (no tests), twice interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
make -s -C cuda-raytracer_amd check || exit 3
for rep in 1 2; do
for v in $VARIANTS; do
  if [ "$v" = base ]; then lib=cuda-raytracer_amd/lib/libptcore.so; else lib=cuda-raytracer_amd/lib/libptcore_$v.so; fi
  PTCORE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --configs ${CONFIGS:-CBspheres} --config5 off --ref-arith none --no-cpu --no-1spp --steps 3 --warmup 1 --detail-out gpurun_out/ab_$v.json > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][-1]
print('$v', d['value'], d['ms_per_frame'], [(c['scene'], c['value'], c['ms_per_frame']) for c in d['configs']], flush=True)"
done
done
