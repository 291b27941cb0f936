#!/bin/bash
# Build a diagnostic variant of the library into ab/lib_NAME.so from a copy of the sources:
#   bash scripts/build_variant.sh NAME "-DFLAG ..." [scripts/variants/X.sed ...]
# Each sed script is applied to the copied kernel sources (the product sources keep no
# variant switches); the variant's fw_build_info names its flags and sed scripts.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; FLAGS=$2; shift 2 || true
SRC=/tmp/fwvar_src_$NAME
rm -rf $SRC; mkdir -p $SRC/flipcomplexityempirical_amd $SRC/include $ROOT/ab
cp -r $ROOT/flipcomplexityempirical_amd/csrc $SRC/flipcomplexityempirical_amd/
rm -rf $SRC/flipcomplexityempirical_amd/csrc/build
cp $ROOT/include/flipwalk.h $SRC/include/
TAGS=""
for s in "$@"; do
  for f in $SRC/flipcomplexityempirical_amd/csrc/fw_*.hip $SRC/flipcomplexityempirical_amd/csrc/fw_*.h; do
    sed -i -f "$s" "$f"
  done
  TAGS="$TAGS sed:$(basename $s)"
done
cd $SRC/flipcomplexityempirical_amd/csrc
OUT=/tmp/fwvar_$NAME; mkdir -p $OUT
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
for s in fw_api fw_kernels; do /opt/rocm/bin/hipcc $F -c -o $OUT/$s.o $s.hip & done
/opt/rocm/bin/hipcc $F -c -o $OUT/fw_grid16.o fw_grid16.hip &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=iterative-ilp -c -o $OUT/fw_grid16_lean.o fw_grid16_lean.hip &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -c -o $OUT/fw_grid16_w2.o fw_grid16_w2.hip &
wait
./gen_build_info.sh $OUT/build_info.cpp "$F$TAGS"
g++ -O2 -fPIC -c -o $OUT/build_info.o $OUT/build_info.cpp
/opt/rocm/bin/hipcc $F -shared -o $ROOT/ab/lib_$NAME.so $OUT/fw_api.o $OUT/fw_kernels.o $OUT/fw_grid16.o $OUT/fw_grid16_lean.o $OUT/fw_grid16_w2.o $OUT/build_info.o
echo built ab/lib_$NAME.so
