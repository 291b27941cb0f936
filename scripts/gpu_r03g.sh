#!/bin/bash
# C5 steady state from a checkpoint (30,000 steps of the 8-GPU job's shard 0): A/B of the
# list-search variants (g3: one-hot atomic claims; peek: read marks first, claim empty
# ones; old: race_search_gscr; lb4: 4-bit labels, in-place LDS marks, fewer chains per
# CU), then their stamps.  Output under gpurun_out/r03g/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03g
mkdir -p $O
CK=/tmp/ck_c5_30k.npz
FLIPWALK_LIB=$PWD/ab/lib_g3.so timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 30 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck.json 2> $O/ck.err || { echo "checkpoint run failed"; tail -5 $O/ck.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/ck.json').read().splitlines()[-1]); print('c5 0..30k', '%.4g' % d['value'])"
: > $O/ab.jsonl
for rep in 1 2; do
  for v in g3 peek old lb4; do
    L=$v; unset FLIPWALK_CSR_LB
    if [ $v = lb4 ]; then L=g3; export FLIPWALK_CSR_LB=4; fi
    FLIPWALK_LIB=$PWD/ab/lib_$L.so timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --resume $CK --warmup 1 --steps 4 --check-chains 2 --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "bench $v failed"; tail -5 $O/one.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); r={'lib': sys.argv[1], 'rep': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [d['parity_check']['equal'], d['parity_check']['chains']], 'bfs_nodes_per_run': d['bfs_nodes_per_run'], 'mean_cut': d['mean_cut']}; print(json.dumps(r))" $v $rep | tee -a $O/ab.jsonl
  done
done
unset FLIPWALK_CSR_LB
for v in g3 peek old; do
  FLIPWALK_LIB=$PWD/ab/lib_${v}_st.so timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK > $O/stamps_$v.txt 2>&1 || { echo "stamps $v failed"; tail -5 $O/stamps_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/stamps_$v.txt
done
