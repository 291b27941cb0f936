#!/bin/bash
# C4 and C5 after the padded group sums: kernel trace + PMC passes (scripts/profile.sh),
# C5 as one 8-GPU shard (8,192 chains spanning the ladder) and the 8,192-chain C3 shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG_ARGS="--config c4" bash scripts/profile.sh r02b_c4 || exit 1
CFG_ARGS="--config c5 --chains 8192" bash scripts/profile.sh r02b_c5 || exit 1
CFG_ARGS="--chains 8192" bash scripts/profile.sh r02b_c3s8 || exit 1
