#!/bin/bash
# race_search_g3 (C5's HBM-marked list search rewritten): the 3-bit / large-grid parity
# tests, then the C5 shard at the verdict's protocol (--steps 100 --warmup 10) and the
# steady-state stamps.  Output under gpurun_out/r03f/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "large_grid or 3bit or search_list_spill or c5 or many_units" > $O/pytest_g3.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_g3.log | tail -2
grep -E "FAILED|^E " $O/pytest_g3.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --config c5 --shard 0/8 --steps 100 --warmup 10 --no-cpu-baseline --check-chains 4 > $O/bench_c5_steady.json 2> $O/bench_c5_steady.err || { echo "bench c5 failed"; tail -5 $O/bench_c5_steady.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c5_steady.json').read().splitlines()[-1]); print('c5 shard steady', '%.4g' % d['value'], 'kernel_ms=%.3f' % d['kernel_ms'], d['parity_check']['equal'], '/', d['parity_check']['chains'])"
timeout -k 10 300 python -u scripts/stamps.py c5 8192 60 > $O/stamps_c5_warm60.txt 2>&1 || { echo "stamps warm60 failed"; tail -5 $O/stamps_c5_warm60.txt; exit 1; }
cat $O/stamps_c5_warm60.txt
