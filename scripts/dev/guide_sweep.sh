# k_path_leaf grab schedule sweep (guide factor x path regions): per-wave
# timing build, then share and full-frame times with the default library
set -e
for cfg in "4 1" "4 8" "4 32" "8 8"; do set -- $cfg; echo "== guide $1 regions $2"
  PT_PATH_GUIDE=$1 PT_PATH_REGIONS=$2 PTCORE_LIB=cuda-raytracer_amd/lib/libptcore_tm.so timeout -k 10 100 python scripts/dev/path_timing.py CBempty 8; done > gpurun_out/tm.log 2>&1
for cfg in "4 1" "4 8" "4 32" "8 8"; do set -- $cfg; echo "== guide $1 regions $2"
  PT_PATH_GUIDE=$1 PT_PATH_REGIONS=$2 timeout -k 10 100 python scripts/dev/share_time.py CBempty 8 5
  PT_PATH_GUIDE=$1 PT_PATH_REGIONS=$2 timeout -k 10 100 python scripts/dev/share_time.py CBspheres 8 5; done > gpurun_out/st.log 2>&1
