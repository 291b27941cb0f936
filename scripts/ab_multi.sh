#!/bin/bash
# Interleaved timing of several library builds on one box (2 rounds):
#   bash scripts/ab_multi.sh libA.so libB.so ... 
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for L in "$@"; do
    v=$(FLIPWALK_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 \
        | python -c "import json,sys; print('%.4e' % json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 1
    echo "$(basename $L) $v"
  done
done
