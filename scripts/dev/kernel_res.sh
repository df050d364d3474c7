#!/bin/bash
# Per-kernel register / spill / occupancy summary of a device translation unit
# (dev tool): scripts/dev/kernel_res.sh <src.hip> [extra hipcc flags...]
set -e
SRC=$1; shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=/tmp/kres_$$.s
/opt/rocm/bin/hipcc -std=c++17 -O3 -ffp-contract=off --offload-arch=${ARCH:-gfx950} --cuda-device-only -S \
  -I"$ROOT/include" -I"$ROOT/cuda-raytracer_amd/csrc" "$@" "$SRC" -o $OUT 2>/dev/null
awk '/^\t\.globl\t/ {k=$2} /; TotalNumSgprs:/ {s=$3} /; NumVgprs:/ {v=$3} /; ScratchSize:/ {sc=$3}
     /; Occupancy:/ {print k, "vgpr", v, "sgpr", s, "scratch", sc, "occ", $3}' $OUT | c++filt |
  awk '{n=$0; sub(/ vgpr .*/, "", n); sub(/\(.*/, "", n); printf "%-60s %s\n", substr(n,1,60), substr($0, index($0," vgpr "))}' | sort
rm -f $OUT
