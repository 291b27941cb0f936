#!/bin/bash
# One GPU session: parity tests, then (only if nothing faulted) a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --inner 1000 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc2=$?
tail -5 gpurun_out/bench_quick.log
exit $(( rc > rc2 ? rc : rc2 ))
