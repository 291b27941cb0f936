#!/bin/bash
# Build a variant of the library with extra compile flags into flipcomplexityempirical_amd/ab/:
#   bash scripts/build_variant.sh NAME "-DFW_VAR_X -DFW_VAR_Y"
set -e
cd "$(dirname "$0")/../flipcomplexityempirical_amd/csrc"
NAME=$1; FLAGS=$2
OUT=/tmp/fwvar_$NAME; mkdir -p $OUT ../../ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
for s in fw_api fw_kernels fw_grid16; do /opt/rocm/bin/hipcc $F -c -o $OUT/$s.o $s.hip & done
wait
/opt/rocm/bin/hipcc $F -shared -o ../../ab/lib_$NAME.so $OUT/fw_api.o $OUT/fw_kernels.o $OUT/fw_grid16.o
echo built ab/lib_$NAME.so
