#!/bin/bash
# C5 steady state (checkpoint at 30,000 steps): stamps of the 4-bit-label plan (in-place LDS
# marks) and its LDS plan.  Output under gpurun_out/r03h/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03h
mkdir -p $O
CK=/tmp/ck_c5_30k.npz
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 30 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck.json 2> $O/ck.err || { echo "checkpoint run failed"; tail -5 $O/ck.err; exit 1; }
for lb in 4 3; do
  FLIPWALK_VERBOSE=1 FLIPWALK_CSR_LB=$lb FLIPWALK_LIB=$PWD/ab/lib_peek_st.so timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK > $O/stamps_lb$lb.txt 2>&1 || { echo "stamps lb$lb failed"; tail -5 $O/stamps_lb$lb.txt; exit 1; }
  echo "== lb$lb"; grep -v amdgpu.ids $O/stamps_lb$lb.txt
done
