"""Summarise a profile.sh output directory: kernel stats + per-dispatch PMC means."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
ks = os.path.join(d, "ktrace", "run_kernel_stats.csv")
if os.path.exists(ks):
    for r in csv.DictReader(open(ks)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:9.3f}")
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "fw_" in r["Kernel_Name"] and "eval" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
