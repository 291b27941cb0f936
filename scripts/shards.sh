#!/bin/bash
# An N-GPU strong-scaled job emulated shard by shard on one GPU: rank r's shard of the
# global chain ids runs standalone (bench.py --shard r/N); the job's rate is the sum of the
# shards' counted steps over the slowest shard's time (the ranks share nothing but the final
# histogram all-reduce).  Usage: shards.sh N "<bench args>" tag
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-8}; ARGS=${2:-}; TAG=${3:-c3}
mkdir -p gpurun_out
OUT=gpurun_out/shards_${TAG}_n$N.jsonl
: > $OUT
for ((r=0; r<N; r++)); do
  timeout -k 10 300 python -u bench.py $ARGS --shard $r/$N --no-cpu-baseline >> $OUT 2> gpurun_out/shards_$TAG.err || { echo "shard $r failed"; tail -5 gpurun_out/shards_$TAG.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
steps = sum(r["value"] * r["ms_per_step"] * r["steps"] / 1e3 for r in rows)
tmax = max(r["ms_per_step"] * r["steps"] / 1e3 for r in rows)
for r in rows:
    print(r["config"]["parallelism"][:40], "%.4g" % r["value"], "kernel_ms=%.2f" % r["kernel_ms"])
print(json.dumps({"job_rate_flip_steps_per_s": steps / tmax, "shards": len(rows),
                  "slowest_shard_s": tmax, "per_shard": [r["value"] for r in rows]}))
PY
