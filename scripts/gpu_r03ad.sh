#!/bin/bash
# Local-test adjacency from the sources rows (rowadj = HEAD) vs the nbadj table (db): full gpu
# tests, then C4 / Frankengraph at the driver protocol (20 timed launches after 5).
# Output under gpurun_out/r03ad/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
: > $O/ab.jsonl
for rep in 1 2 3; do
  for cfg in c4 frank; do
    for v in db rowadj; do
      FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $cfg $v failed"; tail -5 $O/one.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'cfg': sys.argv[3], 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']]}; print(json.dumps(r))" $v $rep $cfg | tee -a $O/ab.jsonl
    done
  done
done
