#!/bin/bash
# Interleaved A/B of library builds on one box: ab_libs.sh "<bench args>" tag lib1 lib2 ...
# (each lib: ab/lib_<name>.so; FLIPWALK_LIB points the loader at it).  3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARGS=$1; TAG=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.jsonl
: > $OUT
for rep in 1 2 3; do
  for v in "$@"; do
    FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 200 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab_one.json 2> gpurun_out/ab_$TAG.err || { echo "$v failed"; tail -5 gpurun_out/ab_$TAG.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.json').read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms']}))" $v $rep | tee -a $OUT
  done
done
