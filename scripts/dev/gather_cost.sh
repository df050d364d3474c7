#!/bin/bash
# The frame gather's cost on one GPU: CBempty frames with and without the
# RCCL gather path (bench.py --force-gather: WORLD_SIZE=1 under
# torch.distributed.run, local_sums_tensor + gather_frame + the host copy)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
A="--configs none --ref-arith none --config5 off --no-cpu --no-1spp --steps ${STEPS:-10} --warmup 2 --detail-out="
timeout -k 10 300 python bench.py $A > gpurun_out/gc_plain.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py $A --force-gather > gpurun_out/gc_gather.log 2>&1 || exit $?
for f in plain gather; do python - "$f" <<'PY'
import json, sys
for l in open(f"gpurun_out/gc_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[1], d["ms_per_step"], "ms/frame", d["value"], "Mrays/s")
PY
done
