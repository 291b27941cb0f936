#!/bin/bash
# Round-2 validation pass: host probe, every -m gpu test, the C3 headline at SURVEY §8d's
# protocol (10^4 warm-up + 10^5 timed flip steps per chain), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/host_probe.sh > gpurun_out/host_probe.txt 2>&1; cat gpurun_out/host_probe.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_steady.json 2> gpurun_out/bench_steady.err || { echo "steady bench failed"; tail -5 gpurun_out/bench_steady.err; exit 1; }
cut -c1-300 gpurun_out/bench_steady.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "default bench failed"; tail -5 gpurun_out/bench_default.err; exit 1; }
cut -c1-300 gpurun_out/bench_default.json
exit $rc
