#!/bin/bash
# Keep a profile.sh run: scripts/install_pmc.sh <gpurun_out/prof_TAG> <pmc key> <profiles/r04/dir>
# copies its summary, kernel stats and pmc.json under the round's profiles/ directory and
# installs pmc.json as profiles/pmc/<key>.json (bench.py pmc_key) for the bench lines.
set -e
SRC=$1; KEY=$2; DST=$3
mkdir -p "$DST" profiles/pmc
cp "$SRC/summary.txt" "$SRC/pmc.json" "$DST/"
cp "$SRC/ktrace/run_kernel_stats.csv" "$DST/kernel_stats.csv"
python3 - "$SRC/pmc.json" "$DST" "profiles/pmc/$KEY.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = sys.argv[2]
json.dump(d, open(sys.argv[3], "w"), indent=1)
PY
echo "installed profiles/pmc/$KEY.json from $SRC"
