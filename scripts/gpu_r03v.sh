#!/bin/bash
# Validation at HEAD (after the C5 search and CSR local-test work): every -m gpu test, smoke(), the driver-protocol bench line (20/5),
# the steady-state protocol (10/100) on every workload, and the C5 8-GPU job emulated shard
# by shard at the steady-state protocol.  Output under gpurun_out/r03v/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${R03V_OUT:-gpurun_out/r03v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "bench failed"; tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]); print('driver line %.4g' % d['value'], d['parity_check']['equal'], '/', d['parity_check']['chains'])"
: > $O/steady.jsonl
for a in "--config c3" "--config c2" "--config c4" "--config frank" "--config c3 --shard 0/8"; do
  timeout -k 10 300 python -u bench.py $a --warmup 10 --steps 100 --no-cpu-baseline --check-chains 4 >> $O/steady.jsonl 2> $O/steady.err || { echo "$a failed"; tail -5 $O/steady.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/steady.jsonl').read().splitlines()[-1]); print('steady $a', '%.4g' % d['value'], 'kernel_ms=%.2f' % d['kernel_ms'], 'parity %d/%d' % (d['parity_check']['equal'], d['parity_check']['chains']))"
done
: > $O/c5_job.jsonl
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 300 python -u bench.py --config c5 --shard $r/8 --warmup 10 --steps 100 --no-cpu-baseline --check-chains 2 >> $O/c5_job.jsonl 2> $O/c5_job.err || { echo "c5 shard $r failed"; tail -5 $O/c5_job.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_job.jsonl').read().splitlines()[-1]); print('c5 shard $r', '%.4g' % d['value'], 'parity %d/%d' % (d['parity_check']['equal'], d['parity_check']['chains']))"
done
python3 - $O/c5_job.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
steps = sum(r["value"] * r["ms_per_step"] * r["steps"] / 1e3 for r in rows)
tmax = max(r["ms_per_step"] * r["steps"] / 1e3 for r in rows)
print(json.dumps({"c5_job_rate_emulated": steps / tmax, "slowest_shard_s": tmax, "per_shard": [r["value"] for r in rows]}))
PY
