#!/bin/bash
# Interleaved A/B of library builds over several bench configurations on one box:
#   ab_set.sh tag lib1 lib2 ...   (each lib: ab/lib_<name>.so), configs in $CONFIGS
# separated by ';'.  Output: gpurun_out/abset_<tag>.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/abset_$TAG.jsonl
: > $OUT
IFS=';' read -ra CFGS <<< "${CONFIGS:---chains 8192;--config c5 --shard 0/8}"
for rep in ${REPS:-1 2}; do
  for cfg in "${CFGS[@]}"; do
    for v in "$@"; do
      FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 200 python -u bench.py $cfg --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline > gpurun_out/abset_one.json 2> gpurun_out/abset_$TAG.err || { echo "$v $cfg failed"; tail -5 gpurun_out/abset_$TAG.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/abset_one.json').read().strip().splitlines()[-1]); print(json.dumps({'cfg': sys.argv[3], 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms']}))" $v $rep "$cfg" | tee -a $OUT
    done
  done
done
