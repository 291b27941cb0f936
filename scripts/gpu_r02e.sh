#!/bin/bash
# One-chain-per-wave kernel after branch-free grid gathers and the lane-parallel window
# check: parity (wave64 + CSR cases), C5 shard rate, stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wave64 or sec11 or frank or tract or county or delaunay or large_grid or c5 or c4 or window or spill" > gpurun_out/pytest_r02e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02e.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_r02e.log | head; exit $rc; }
timeout -k 10 200 python -u bench.py --config c5 --shard 0/8 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/c5_s0.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c5_s0.json').read().splitlines()[-1]); print('c5 shard0', '%.4g' % d['value'], d['kernel_ms'])"
timeout -k 10 200 python -u bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/c4.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c4.json').read().splitlines()[-1]); print('c4', '%.4g' % d['value'], d['kernel_ms'])"
timeout -k 10 200 python -u scripts/stamps.py c5 8192 > gpurun_out/stamps_c5_csr2.txt 2>&1; tail -8 gpurun_out/stamps_c5_csr2.txt
