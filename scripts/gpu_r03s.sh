#!/bin/bash
# the list search seeded by the bitboard escape state (seed) vs b3f2:
# large-grid parity tests, then A/B against race_search_g3 (lib_g3h) at 3*10^4- and
# 10^5-step C5 checkpoints, stamps, and the C5 shard at the verdict protocol.
# Output under gpurun_out/r03s/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "large_grid or 3bit or search_list_spill or c5 or bitboard or many_units" > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
grep -E "FAILED|^E " $O/pytest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for S in 30 100; do
  CK=/tmp/ck_c5_${S}k.npz
  timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps $S --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck$S.json 2> $O/ck$S.err || { echo "checkpoint run failed"; tail -5 $O/ck$S.err; exit 1; }
done
: > $O/ab.jsonl
for S in 30 100; do
for rep in 1 2; do
  for v in b3f2 seed; do
    FLIPWALK_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --resume /tmp/ck_c5_${S}k.npz --warmup 1 --steps 4 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $v failed"; tail -5 $O/one.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'ck': int(sys.argv[3]), 'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']], 'bfs_nodes_per_run': d['bfs_nodes_per_run']}; print(json.dumps(r))" $v $rep $S | tee -a $O/ab.jsonl
  done
done
done
FLIPWALK_LIB=$PWD/ab/lib_seed_st.so timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 /tmp/ck_c5_100k.npz > $O/stamps_seed_100k.txt 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_seed_100k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_seed_100k.txt
timeout -k 10 500 python -u bench.py --config c5 --shard 0/8 --steps 100 --warmup 10 --no-cpu-baseline --check-chains 4 > $O/bench_c5_steady.json 2> $O/bench_c5_steady.err || { echo "bench c5 failed"; tail -5 $O/bench_c5_steady.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c5_steady.json').read().splitlines()[-1]); print('c5 shard 100/10', '%.4g' % d['value'], 'kernel_ms=%.3f' % d['kernel_ms'], d['parity_check']['equal'], '/', d['parity_check']['chains'])"
