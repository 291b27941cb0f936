#!/bin/bash
# Every BASELINE workload on one GPU: the default C3 line (with cpu_baseline), then
# C2, C4, C5 and the Frankengraph.  Output: gpurun_out/bench_<config>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
tail -1 gpurun_out/bench_c3.json | cut -c1-200
for cfg in c2 c4 c5 frank; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
      > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/bench_$cfg.err; exit 1; }
  tail -1 gpurun_out/bench_$cfg.json | cut -c1-200
done
