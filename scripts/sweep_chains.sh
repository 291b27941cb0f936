#!/bin/bash
# Single-GPU rate of the C3 workload against the number of chains on the device:
# the strong-scaled shards of 65,536 chains (8,192 / 16,384 / 32,768 per GPU at 8 / 4 / 2
# GPUs) and the launch tail around 65,536 (61,440 / 73,728).  Output: gpurun_out/sweep_<tag>.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
mkdir -p gpurun_out
OUT=gpurun_out/sweep_$TAG.jsonl
: > $OUT
for C in ${CHAINS:-8192 16384 32768 61440 65536 73728}; do
  timeout -k 10 120 python -u bench.py --chains $C --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline $EXTRA \
      >> $OUT 2> gpurun_out/sweep_$TAG.err || { echo "chains=$C failed"; tail -5 gpurun_out/sweep_$TAG.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT').read().splitlines()[-1]); print($C, '%.4g' % d['value'], 'kernel_ms=%.3f' % d['kernel_ms'])"
done
