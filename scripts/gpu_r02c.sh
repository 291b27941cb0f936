#!/bin/bash
# Large-grid parity tests after the routing change, then 8-GPU jobs emulated shard by shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
KSEL="big or large_grid or ladder" bash scripts/gpu_big.sh || exit 1
bash scripts/shards.sh 8 "--config c5 --steps 6 --warmup 2" c5_interleaved || exit 1
bash scripts/shards.sh 8 "--config c5 --ladder contiguous --steps 6 --warmup 2" c5_contiguous || exit 1
bash scripts/shards.sh 8 "--steps 10 --warmup 2" c3 || exit 1
