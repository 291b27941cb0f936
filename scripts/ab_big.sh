#!/bin/bash
# Large grids: the grid kernel's large-grid plan against the one-chain-per-wave kernel
# (FLIPWALK_NO_GRID16=1) on 200x200 k=4 (2-bit labels) and k=8 (3-bit), 8,192 chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_big.jsonl
: > $OUT
for args in "--config c3 --grid 200" "--config c5"; do
  for env in "" "FLIPWALK_NO_GRID16=1"; do
    env $env FLIPWALK_VERBOSE=1 timeout -k 10 200 python -u bench.py $args --chains 8192 --steps 6 --warmup 2 --no-cpu-baseline >> $OUT 2> gpurun_out/ab_big.err || { echo "failed: $args $env"; tail -5 gpurun_out/ab_big.err; exit 1; }
    grep flipwalk: gpurun_out/ab_big.err | tail -1
    python3 -c "import json; d=json.loads(open('$OUT').read().splitlines()[-1]); print('$args', '$env', '%.4g' % d['value'], d['kernel_ms'], round(d['valid_frac'],3), round(d['bfs_runs_per_step'],3))"
  done
done
