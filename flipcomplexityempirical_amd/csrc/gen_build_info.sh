#!/bin/bash
# gen_build_info.sh OUT.cpp "FLAGS": writes the fw_build_info() translation unit (include/
# flipwalk.h) of a build: a hash over every kernel, header and ABI source plus the flags.
set -e
cd "$(dirname "$0")"
OUT=$1
FLAGS=$2
H=$(cat fw_api.hip fw_kernels.hip fw_grid16.hip fw_grid16_lean.hip fw_grid16_w2.hip fw_internal.h fw_device.h fw_math.h \
      ../../include/flipwalk.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* fw_build_info(void) { return "src=%s flags=%s"; }\n' \
  "$H" "$(echo $FLAGS)" > "$OUT.tmp"
# rewrite only on change, so make relinks only when the provenance changes
if ! cmp -s "$OUT.tmp" "$OUT" 2>/dev/null; then mv "$OUT.tmp" "$OUT"; else rm -f "$OUT.tmp"; fi
