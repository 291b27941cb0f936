#!/bin/bash
# Workgroups-per-CU cap of the grid kernel on strong-scaled shards (fw_grid16_plan):
# interleaved runs of the automatic cap and of no cap (FLIPWALK_WG_PER_CU=0) at the chain
# counts of the 8- and 4-GPU shards and of one residency round.  Output: gpurun_out/wgcap.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/wgcap.jsonl
: > $OUT
for rep in 1 2; do
  for C in ${CHAINS:-8192 12288 16384}; do
    for CAP in auto 0 ${CAPS:-}; do
      if [ "$CAP" = auto ]; then E=""; else E="FLIPWALK_WG_PER_CU=$CAP"; fi
      v=$(env $E timeout -k 10 120 python -u bench.py --chains $C --steps 6 --warmup 2 --no-cpu-baseline \
          2> gpurun_out/wgcap.err) || { echo "chains=$C cap=$CAP failed"; tail -5 gpurun_out/wgcap.err; exit 1; }
      echo "$v" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); \
print(json.dumps({'chains': $C, 'cap': '$CAP', 'rep': $rep, 'value': d['value'], 'kernel_ms': d['kernel_ms']}))" | tee -a $OUT
    done
  done
done
