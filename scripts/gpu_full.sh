#!/bin/bash
# Full GPU validation: all gpu tests, smoke(), then the default bench (with cpu_baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full.log 2>&1
rc2=$?
tail -1 gpurun_out/bench_full.log
exit $(( rc > rc2 ? rc : rc2 ))
