#!/bin/bash
# Interleaved C3 timing of (library, environment) variants on one box, 2 rounds:
#   bash scripts/ab_env.sh "libA.so" "libB.so" "libB.so FLIPWALK_NW=4" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS=("$@")
for i in 1 2; do
  for V in "${VARIANTS[@]}"; do
    read -r L ENVS <<< "$V"
    v=$(env FLIPWALK_LIB=flipcomplexityempirical_amd/$L $ENVS timeout -k 10 120 python bench.py \
        --no-cpu-baseline --steps 10 ${BENCH_ARGS:-} \
        | python -c "import json,sys; print('%.4e' % json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 1
    echo "$V $v"
  done
done
