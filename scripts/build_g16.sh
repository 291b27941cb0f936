#!/bin/bash
# Fast grid-kernel variant: compile only fw_grid16{,_lean,_w2}.hip from the working tree (or
# from SRC_DIR) with the Makefile's scheduling flags (GRID16_FLAGS / GRID16LEAN_FLAGS /
# GRID16W2_FLAGS override them), link with the product build's fw_api.o / fw_kernels.o
# -> ab/lib_NAME.so
#   bash scripts/build_g16.sh NAME ["-DFLAG ..."]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; FLAGS=${2:-}
CS=${SRC_DIR:-$ROOT/flipcomplexityempirical_amd/csrc}
B=$ROOT/flipcomplexityempirical_amd/csrc/build
OUT=/tmp/fwg16_$NAME; mkdir -p $OUT $ROOT/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
/opt/rocm/bin/hipcc $F ${GRID16_FLAGS-} -c -o $OUT/fw_grid16.o $CS/fw_grid16.hip &
/opt/rocm/bin/hipcc $F ${GRID16LEAN_FLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp} -c -o $OUT/fw_grid16_lean.o $CS/fw_grid16_lean.hip &
/opt/rocm/bin/hipcc $F ${GRID16W2_FLAGS--mllvm -amdgpu-sched-strategy=max-ilp} -c -o $OUT/fw_grid16_w2.o $CS/fw_grid16_w2.hip &
wait
(cd $ROOT/flipcomplexityempirical_amd/csrc && ./gen_build_info.sh $OUT/build_info.cpp "$F g16:$NAME")
g++ -O2 -fPIC -c -o $OUT/build_info.o $OUT/build_info.cpp
/opt/rocm/bin/hipcc $F -shared -o $ROOT/ab/lib_$NAME.so $B/fw_api.o $B/fw_kernels.o $OUT/fw_grid16.o $OUT/fw_grid16_lean.o $OUT/fw_grid16_w2.o $OUT/build_info.o
echo built ab/lib_$NAME.so
