cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python scripts/dev/share_time.py CBempty 1,2,4,8 5 > gpurun_out/share_CBempty.log 2>&1 && cat gpurun_out/share_CBempty.log && \
timeout -k 10 300 python scripts/dev/share_time.py CBspheres 1,8 5 > gpurun_out/share_CBspheres.log 2>&1 && cat gpurun_out/share_CBspheres.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/share_prof -o tr -- python scripts/dev/share_time.py CBempty 8 3 > gpurun_out/share_prof.log 2>&1; echo rc=$?
