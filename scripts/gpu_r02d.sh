#!/bin/bash
# Stats write-back as 16-byte stores: parity, A/B timing against the old scalar stores,
# and a PMC pass (WRITE_SIZE) of the default C3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bit_exact or checkpoint or full_size or fold or split" > gpurun_out/pytest_r02d.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r02d.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_r02d.log | head; exit $rc; }
bash scripts/ab_multi.sh flipcomplexityempirical_amd/ab/lib_oldstats.so flipcomplexityempirical_amd/ab/lib_newstats.so || exit 1
bash scripts/profile.sh r02d || exit 1
