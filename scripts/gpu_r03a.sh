#!/bin/bash
# Round 3 check pass: every -m gpu test, smoke() (C3 shape, oracle spot-check) and the
# default bench line (with its parity_check leg).  Output under gpurun_out/r03a/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "bench failed"; tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]); print('%.4g' % d['value'], d['parity_check'])"
