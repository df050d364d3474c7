#!/bin/bash
# Register/occupancy lines of kernels whose symbol matches $2 in translation unit $1 (dev tool)
SRC=$1; PAT=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=/tmp/kres2_$$.s
/opt/rocm/bin/hipcc -std=c++17 -O3 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only -S \
  -I"$ROOT/include" -I"$ROOT/cuda-raytracer_amd/csrc" "$@" "$SRC" -o $OUT 2>/dev/null
awk '/^\t\.globl\t/ {k=$2} /; TotalNumSgprs:/ {s=$3} /; NumVgprs:/ {v=$3} /; ScratchSize:/ {sc=$3}
     /; Occupancy:/ {print k, "vgpr", v, "sgpr", s, "scratch", sc, "occ", $3}' $OUT | grep "$PAT"
rm -f $OUT
