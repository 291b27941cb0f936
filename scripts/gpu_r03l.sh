#!/bin/bash
# C5 shard 0 stamps at a 10^5-step checkpoint (the verdict protocol's timed window).
# Output under gpurun_out/r03l/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l
mkdir -p $O
CK=/tmp/ck_c5_100k.npz
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 100 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck.json 2> $O/ck.err || { echo "checkpoint run failed"; tail -5 $O/ck.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/ck.json').read().splitlines()[-1]); print('c5 0..100k', '%.4g' % d['value'], 'mean_cut', d['mean_cut'])"
timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK > $O/stamps_100k.txt 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_100k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_100k.txt
