#!/bin/bash
# Full validation + measurement pass of the tree: every -m gpu test, smoke(), the default
# bench line (with the CPU baselines), the other BASELINE workloads, and the 8-GPU C5 job
# emulated shard by shard.  Output under gpurun_out/round/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/round
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
cut -c1-200 $O/bench_default.json
: > $O/bench_configs.jsonl
for a in "--config c2" "--config c4" "--config c5 --shard 0/8" "--config frank" "--config c3 --grid 200 --chains 8192"; do
  timeout -k 10 300 python -u bench.py $a --steps 6 --warmup 2 --no-cpu-baseline >> $O/bench_configs.jsonl 2> $O/bench_configs.err || { echo "bench $a failed"; tail -5 $O/bench_configs.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_configs.jsonl').read().splitlines()[-1]); print('$a', '%.4g' % d['value'], 'kernel_ms=%.2f' % d['kernel_ms'])"
done
# round 1's C5 line, like for like: shard 0 of the contiguous ladder (the 8 lowest bases),
# 5 timed launches after 1 (profiles/r01/bench_configs.jsonl)
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --ladder contiguous --steps 5 --warmup 1 \
    --no-cpu-baseline > $O/bench_c5_r01protocol.json 2> $O/bench_configs.err || { echo "c5 r01 protocol failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c5_r01protocol.json').read().splitlines()[-1]); print('c5 contiguous shard 0, r01 protocol', '%.4g' % d['value'])"
# the driver's own protocol (BENCH_r01.json: --steps 20 --warmup 5)
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_driver.json 2> $O/bench_configs.err || { echo "c3 driver protocol failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3_driver.json').read().splitlines()[-1]); print('c3 driver protocol 20/5', '%.4g' % d['value'])"
# SURVEY 8d's steady-state protocol: 10^4 warm-up steps, then 10^5 timed, per chain
timeout -k 10 300 python -u bench.py --warmup 10 --steps 100 --no-cpu-baseline > $O/bench_c3_steady.json 2> $O/bench_configs.err || { echo "c3 steady failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3_steady.json').read().splitlines()[-1]); print('c3 steady state', '%.4g' % d['value'])"
bash scripts/shards.sh 8 "--config c5 --steps 6 --warmup 2" c5 | tail -1
bash scripts/shards.sh 8 "--steps 6 --warmup 2" c3 | tail -1
