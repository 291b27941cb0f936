#!/bin/bash
# Kernel time per launch against the steps per launch (--inner) at shard-sized chain
# counts: separates the per-launch fixed cost (state load / write-back, the last wave's
# tail) from the per-step cost.  Output: gpurun_out/inner_sweep.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/inner_sweep.jsonl
: > $OUT
for C in ${CHAINS:-8192 12288 65536}; do
  for I in ${INNERS:-250 1000 4000}; do
    v=$(timeout -k 10 120 python -u bench.py --chains $C --inner $I --steps 4 --warmup 2 --no-cpu-baseline \
        2> gpurun_out/inner_sweep.err) || { echo "chains=$C inner=$I failed"; tail -5 gpurun_out/inner_sweep.err; exit 1; }
    echo "$v" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); \
print(json.dumps({'chains': $C, 'inner': $I, 'value': d['value'], 'kernel_ms': d['kernel_ms']}))" | tee -a $OUT
  done
done
