#!/bin/bash
# HEAD check: every -m gpu test, smoke, the driver-protocol bench line; A/B of the CSR local
# test by ballot closure (csrl = HEAD) against wave_or64 closure (seed) on C4 and the
# Frankengraph.  Output under gpurun_out/r03t/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03t
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
: > $O/ab.jsonl
for rep in 1 2; do
  for cfg in c4 frank; do
    for v in seed csrl; do
      FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $cfg $v failed"; tail -5 $O/one.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'cfg': sys.argv[3], 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']]}; print(json.dumps(r))" $v $rep $cfg | tee -a $O/ab.jsonl
    done
  done
done
