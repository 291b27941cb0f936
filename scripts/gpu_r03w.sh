#!/bin/bash
# 32-bit label-set masks in the chain kernel (m32 = HEAD) vs dpp: full gpu tests, then C4 /
# Frankengraph lines and the C5 shard at the 10^5-step checkpoint.  Output under
# gpurun_out/r03w/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
: > $O/ab.jsonl
for rep in 1 2; do
  for cfg in c4 frank; do
    for v in dpp m32; do
      FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $cfg $v failed"; tail -5 $O/one.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'cfg': sys.argv[3], 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']]}; print(json.dumps(r))" $v $rep $cfg | tee -a $O/ab.jsonl
    done
  done
done
CK=/tmp/ck_c5_100k.npz
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 100 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck100.json 2> $O/ck100.err || { echo "checkpoint run failed"; tail -5 $O/ck100.err; exit 1; }
for rep in 1 2; do
  for v in dpp m32; do
    FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --resume $CK --warmup 1 --steps 4 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench c5 $v failed"; tail -5 $O/one.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'cfg': 'c5@1e5', 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']]}; print(json.dumps(r))" $v $rep | tee -a $O/ab.jsonl
  done
done
