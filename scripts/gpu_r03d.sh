#!/bin/bash
# C5 steady-state stamps (diagnostic build): contiguity cycles by path after 10 and 60
# warm-up launches of 1000 steps (scripts/stamps.py).  Output under gpurun_out/r03d/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 200 python -u scripts/stamps.py c5 8192 10 > $O/stamps_c5_warm10.txt 2>&1 || { echo "stamps warm10 failed"; tail -5 $O/stamps_c5_warm10.txt; exit 1; }
cat $O/stamps_c5_warm10.txt
timeout -k 10 300 python -u scripts/stamps.py c5 8192 60 > $O/stamps_c5_warm60.txt 2>&1 || { echo "stamps warm60 failed"; tail -5 $O/stamps_c5_warm60.txt; exit 1; }
cat $O/stamps_c5_warm60.txt
