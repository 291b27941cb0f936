#!/bin/bash
# rocprofv3 passes over one bench protocol: kernel trace + stats, then PMC passes (separate
# runs; no --pmc together with any trace domain), every pass with the SAME bench.py
# arguments, so pmc_summary.py can keep the timed launches of each and bench.py can match
# the profile to a line of that protocol (pmc_key + identity).  Output: gpurun_out/prof_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift
CFG_ARGS=${CFG_ARGS:-}   # e.g. "--config c5" (default: the C3 bench line)
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5 --no-cpu-baseline --check-chains 0 --secondary-inner 0 $CFG_ARGS"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- python3 bench.py $BENCH_ARGS > $OUT/ktrace_bench.log 2>&1 || { echo "ktrace failed rc=$?"; tail -20 $OUT/ktrace_bench.log; exit 1; }
tail -1 $OUT/ktrace_bench.log
PB=${PMC_ARGS:-"$BENCH_ARGS --check-chains 0"}
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH" \
            "FETCH_SIZE GRBM_GUI_ACTIVE" \
            "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $PB > $OUT/pmc${i}_bench.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $OUT/pmc${i}_bench.log; exit 1; }
  echo "pmc pass $i ok"
done
PMC_BENCH_ARGS="$PB" python3 scripts/pmc_summary.py $OUT $OUT/pmc.json > $OUT/summary.txt && cat $OUT/summary.txt
