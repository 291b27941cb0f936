#!/bin/bash
# C5 shard 0 at the 10^5-step checkpoint: batched restore (b3r) vs b3s A/B, stamps, and a
# kernel trace + PMC profile (resumed launches).  Output under gpurun_out/r03o/ and
# gpurun_out/prof_r03_c5steady/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03o
mkdir -p $O
CK=/tmp/ck_c5_100k.npz
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 100 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck100.json 2> $O/ck100.err || { echo "checkpoint run failed"; tail -5 $O/ck100.err; exit 1; }
: > $O/ab.jsonl
for rep in 1 2; do
  for v in b3s b3r; do
    FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --resume $CK --warmup 1 --steps 4 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $v failed"; tail -5 $O/one.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'ck': 100, 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']]}; print(json.dumps(r))" $v $rep | tee -a $O/ab.jsonl
  done
done
FLIPWALK_LIB=$PWD/ab/lib_b3r_st.so timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK > $O/stamps_b3r_100k.txt 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_b3r_100k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_b3r_100k.txt
export FLIPWALK_LIB=$PWD/ab/lib_b3r.so
PMC_ARGS="--config c5 --shard 0/8 --resume $CK --steps 1 --warmup 1 --inner 1000 --no-cpu-baseline --check-chains 0" BENCH_ARGS="--config c5 --shard 0/8 --resume $CK --steps 4 --warmup 1 --inner 1000 --no-cpu-baseline --check-chains 2" timeout -k 10 900 bash scripts/profile.sh r03_c5steady > $O/prof.log 2>&1 || { echo "profile failed"; tail -20 $O/prof.log; exit 1; }
tail -28 $O/prof.log
