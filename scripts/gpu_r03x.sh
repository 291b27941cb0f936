#!/bin/bash
# Final round-3 pass at HEAD: every -m gpu test, smoke, the driver-protocol bench line, the
# steady-state table and the emulated C5 job, the C3 rocprof kernel trace + PMC passes
# (traffic / issue rooflines of the bench line), C5 and C4 stamps.
# Output under gpurun_out/r03x/ and gpurun_out/prof_r03_final_c3/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03x
mkdir -p $O
R03V_OUT=$O bash scripts/gpu_r03v.sh > $O/validation.log 2>&1 || { echo "validation failed"; tail -30 $O/validation.log; exit 1; }
cat $O/validation.log
timeout -k 10 900 bash scripts/profile.sh r03_final_c3 > $O/prof_c3.log 2>&1 || { echo "c3 profile failed"; tail -20 $O/prof_c3.log; exit 1; }
tail -28 $O/prof_c3.log
CK=/tmp/ck_c5_100k.npz
timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 100 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK > $O/ck100.json 2> $O/ck100.err || { echo "checkpoint run failed"; tail -5 $O/ck100.err; exit 1; }
timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK > $O/stamps_c5_100k.txt 2>&1 || { echo "stamps c5 failed"; tail -5 $O/stamps_c5_100k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c5_100k.txt
timeout -k 10 300 python -u scripts/stamps.py c4 16384 2 > $O/stamps_c4.txt 2>&1 || { echo "stamps c4 failed"; tail -5 $O/stamps_c4.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c4.txt
