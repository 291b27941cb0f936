#!/bin/bash
# HEAD check after the speculative-attempt kernels: every -m gpu test, smoke(), then A/B
# lines (FLIPWALK_SPEC=1 vs the host's pick) on the 8-GPU C3 shard, the 4-GPU shard and C2.
# Output under gpurun_out/r03e/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
: > $O/ab_spec.jsonl
for rep in 1 2; do
for cfg in "--shard 0/8" "--config c2" "--shard 0/4" "--config c3"; do
  for sp in 1 auto; do
    if [ $sp = auto ]; then unset FLIPWALK_SPEC; else export FLIPWALK_SPEC=$sp; fi
    FLIPWALK_VERBOSE=1 timeout -k 10 200 python -u bench.py $cfg --steps 20 --warmup 5 --no-cpu-baseline --check-chains 4 >> $O/ab_spec.jsonl 2> $O/ab_spec.err || { echo "bench $cfg $sp failed"; tail -5 $O/ab_spec.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab_spec.jsonl').read().splitlines()[-1]); print('$cfg spec=$sp', '%.4g' % d['value'], 'kernel_ms=%.3f' % d['kernel_ms'], d['parity_check']['equal'], '/', d['parity_check']['chains'])"
    grep "grid kernel" $O/ab_spec.err | tail -1
  done
done
done
