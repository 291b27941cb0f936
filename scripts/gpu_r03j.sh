#!/bin/bash
# Profiles at HEAD: C4 (stamps, kernel trace + PMC), C3 at steady state (checkpoint after
# 10^4 steps, then kernel trace + PMC of launches resumed from it).  Output under
# gpurun_out/r03j/ and gpurun_out/prof_r03_*/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u scripts/stamps.py c4 16384 2 > $O/stamps_c4.txt 2>&1 || { echo "stamps c4 failed"; tail -5 $O/stamps_c4.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c4.txt
CFG_ARGS="--config c4" timeout -k 10 900 bash scripts/profile.sh r03_c4 > $O/prof_c4.log 2>&1 || { echo "c4 profile failed"; tail -20 $O/prof_c4.log; exit 1; }
tail -30 $O/prof_c4.log
CK=/tmp/ck_c3_10k.npz
timeout -k 10 300 python -u bench.py --warmup 0 --steps 10 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck_c3.json 2> $O/ck_c3.err || { echo "c3 checkpoint failed"; tail -5 $O/ck_c3.err; exit 1; }
PMC_ARGS="--resume $CK --steps 1 --warmup 1 --inner 1000 --no-cpu-baseline --check-chains 0" BENCH_ARGS="--resume $CK --steps 10 --warmup 2 --inner 1000 --no-cpu-baseline --check-chains 2" timeout -k 10 900 bash scripts/profile.sh r03_c3steady > $O/prof_c3steady.log 2>&1 || { echo "c3 steady profile failed"; tail -20 $O/prof_c3steady.log; exit 1; }
tail -30 $O/prof_c3steady.log
