#!/bin/bash
# C3 phase stamps at HEAD (65,536 chains and the 8,192-chain shard) and the shard's per-unit
# wall times.  Output under gpurun_out/r03y/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 300 python -u scripts/stamps.py c3 65536 2 > $O/stamps_c3_65k.txt 2>&1 || { echo "stamps 65k failed"; tail -5 $O/stamps_c3_65k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c3_65k.txt
timeout -k 10 300 python -u scripts/stamps.py c3 8192 4 > $O/stamps_c3_8k.txt 2>&1 || { echo "stamps 8k failed"; tail -5 $O/stamps_c3_8k.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_c3_8k.txt
timeout -k 10 300 python -u scripts/unit_times.py 8192 4 > $O/unit_times_8k.txt 2>&1 || { echo "unit times failed"; tail -5 $O/unit_times_8k.txt; exit 1; }
grep -v amdgpu.ids $O/unit_times_8k.txt
