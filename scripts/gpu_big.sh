#!/bin/bash
# Large-grid plan of the grid kernel: its parity tests, then C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "${KSEL:-big or large_grid or c5 or ladder}" > gpurun_out/pytest_big.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_big.log | tail -3
grep -E "FAILED|Error|error" gpurun_out/pytest_big.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
FLIPWALK_VERBOSE=1 timeout -k 10 200 python -u bench.py --config c5 --chains 8192 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_8192.json 2> gpurun_out/bench_c5_8192.err || { echo "c5 bench failed"; tail -5 gpurun_out/bench_c5_8192.err; exit 1; }
cut -c1-250 gpurun_out/bench_c5_8192.json
