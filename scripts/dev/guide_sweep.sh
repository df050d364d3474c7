set -e
for g in 0 1 2 4; do echo "== guide $g"; PT_PATH_GUIDE=$g PTCORE_LIB=cuda-raytracer_amd/lib/libptcore_tm.so timeout -k 10 100 python scripts/dev/path_timing.py CBempty 8; done > gpurun_out/tm.log 2>&1
for g in 0 2 4; do echo "== guide $g"; PT_PATH_GUIDE=$g timeout -k 10 100 python scripts/dev/share_time.py CBempty 8 5; PT_PATH_GUIDE=$g timeout -k 10 100 python scripts/dev/share_time.py CBspheres 8 5; done > gpurun_out/st.log 2>&1
