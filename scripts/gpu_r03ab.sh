#!/bin/bash
# C4 / Frankengraph at HEAD (padded-row walks bounded): steady state (10^4 warm-up + 10^5
# timed steps) and C4 stamps.  Output under gpurun_out/r03ab/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab
mkdir -p $O
: > $O/steady.jsonl
for cfg in c4 frank; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "steady $cfg failed"; tail -5 $O/one.err; exit 1; }
  tail -1 $O/one.json >> $O/steady.jsonl
  python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['kernel_ms'], d['parity_check']['equal'], d['parity_check']['chains'])"
done
timeout -k 10 300 python -u scripts/stamps.py c4 16384 2 > $O/stamps_c4.txt 2>&1 || { echo "stamps c4 failed"; tail -5 $O/stamps_c4.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c4.txt
