#!/bin/bash
# SURVEY.md 8d's steady-state protocol (10^4 warm-up steps, then 10^5 timed, per chain) on
# every BASELINE workload.  Output: gpurun_out/steady_all.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/steady_all.jsonl
: > $OUT
for a in "--config c3" "--config c2" "--config c4" "--config c5 --shard 0/8" "--config frank" "--config c3 --shard 0/8"; do
  timeout -k 10 300 python -u bench.py $a --warmup 10 --steps 100 --no-cpu-baseline >> $OUT 2> gpurun_out/steady_all.err || { echo "$a failed"; tail -5 gpurun_out/steady_all.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT').read().splitlines()[-1]); print('$a', '%.4g' % d['value'], 'kernel_ms=%.2f' % d['kernel_ms'], 'mean_cut=%.1f' % d['mean_cut'])"
done
