#!/bin/bash
# Chain-kernel variant: compile only fw_kernels.hip from the working tree (or from
# SRC_DIR), link it with the product build's fw_api.o / fw_grid16*.o -> ab/lib_NAME.so
#   bash scripts/build_k.sh NAME ["-DFLAG ..."]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; FLAGS=${2:-}
CS=${SRC_DIR:-$ROOT/flipcomplexityempirical_amd/csrc}
B=$ROOT/flipcomplexityempirical_amd/csrc/build
OUT=/tmp/fwk_$NAME; mkdir -p $OUT $ROOT/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
/opt/rocm/bin/hipcc $F -c -o $OUT/fw_kernels.o $CS/fw_kernels.hip
(cd $ROOT/flipcomplexityempirical_amd/csrc && ./gen_build_info.sh $OUT/build_info.cpp "$F k:$NAME")
g++ -O2 -fPIC -c -o $OUT/build_info.o $OUT/build_info.cpp
/opt/rocm/bin/hipcc $F -shared -o $ROOT/ab/lib_$NAME.so $B/fw_api.o $OUT/fw_kernels.o $B/fw_grid16.o $B/fw_grid16_lean.o $B/fw_grid16_w2.o $OUT/build_info.o
echo built ab/lib_$NAME.so
