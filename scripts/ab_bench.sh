#!/bin/bash
# A/B timing of two builds of the library on the same GPU, interleaved (A B A B A B):
#   bash scripts/ab_bench.sh path/to/libA.so path/to/libB.so [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; shift 2
for i in 1 2 3; do
  for L in $A $B; do
    v=$(FLIPWALK_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 "$@" \
        | python -c "import json,sys; print('%.4e' % json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 1
    echo "$(basename $L) $v"
  done
done
