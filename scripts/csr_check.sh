#!/bin/bash
# CSR-kernel configs (C4, C5, Frankengraph) with the LDS plan printed, then the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in c4 c5 frank; do
  FLIPWALK_VERBOSE=1 timeout -k 10 150 python -u bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_$cfg.json 2>gpurun_out/b_$cfg.err || { tail -5 gpurun_out/b_$cfg.err; exit 1; }
  grep "flipwalk:" gpurun_out/b_$cfg.err | tail -1
  python -c "import json;d=json.loads(open('gpurun_out/b_$cfg.json').read().strip().splitlines()[-1]);print('$cfg',d['value']/1e9,d['kernel_ms'])"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
