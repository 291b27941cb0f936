"""Mean of each PMC counter over the last K chain-kernel dispatches of one rocprofv3 --pmc
run:  python scripts/pmc_one.py DIR K [label]   (prints one JSON line)."""
import collections
import csv
import glob
import json
import re
import sys

CHAIN_KERNEL = re.compile(r"fw_(grid16|grid16_spec|grid16_w2|grid16_full|run)_kernel")
d, k = sys.argv[1], int(sys.argv[2])
per = collections.defaultdict(dict)
name = None
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if CHAIN_KERNEL.search(r["Kernel_Name"]):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            name = r["Kernel_Name"]
ids = sorted(per)[-k:]
out = {"label": sys.argv[3] if len(sys.argv) > 3 else d, "kernel": name, "dispatches": len(ids)}
for c in sorted({c for i in ids for c in per[i]}):
    v = [per[i][c] for i in ids if c in per[i]]
    out[c] = sum(v) / len(v)
print(json.dumps(out))
