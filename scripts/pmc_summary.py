"""Summarise a profile.sh output directory: kernel stats + per-dispatch PMC means.

    python scripts/pmc_summary.py gpurun_out/prof_<tag> [traffic.json]

With a second argument, writes the per-launch HBM traffic of the chain kernel as JSON
(bench.py --traffic-json reads it): FETCH_SIZE and WRITE_SIZE are kilobytes; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM), so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the state write-back).
"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
ks = os.path.join(d, "ktrace", "run_kernel_stats.csv")
kern = {}
if os.path.exists(ks):
    for r in csv.DictReader(open(ks)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:9.3f}")
        if "fw_" in r["Name"]:
            kern = {"name": r["Name"], "avg_ms": float(r["AverageNs"]) / 1e6, "calls": int(r["Calls"])}
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "fw_" in r["Kernel_Name"] and "eval" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
def _mean(name):
    v = agg.get(name)
    return sum(v) / len(v) if v else None


if len(sys.argv) > 2 and "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
    fetch = sum(agg["FETCH_SIZE"]) / len(agg["FETCH_SIZE"]) * 1024.0
    write = sum(agg["WRITE_SIZE"]) / len(agg["WRITE_SIZE"]) * 1024.0
    out = {"hbm_bytes_per_launch": 2.0 * fetch + write, "fetch_bytes_raw": fetch,
           "fetch_bytes_corrected": 2.0 * fetch, "write_bytes": write,
           "source": os.path.basename(os.path.normpath(d)), "kernel_trace": kern,
           # instruction issue per launch (the kernel's binding resource), for bench.py's
           # issue roofline: wave-instructions, SQ_INSTS_* summed over the chip
           "valu_insts_per_launch": _mean("SQ_INSTS_VALU"), "salu_insts_per_launch": _mean("SQ_INSTS_SALU"),
           "lds_insts_per_launch": _mean("SQ_INSTS_LDS"), "waves": _mean("SQ_WAVES"),
           # achieved residency: SQ_WAVE_CYCLES counts wave-lifetime in units of 4 cycles
           # (calibrated on the C3 grid kernel, whose 3 waves per SIMD live the whole launch:
           # 2.47e10 x 4 / 3.31e7 cycles / 1024 SIMDs = 2.92), GRBM_GUI_ACTIVE the launch's
           # busy cycles summed over the 8 XCDs; 256 CUs x 4 SIMDs
           "achieved_waves_per_simd": (4.0 * _mean("SQ_WAVE_CYCLES") / (_mean("GRBM_GUI_ACTIVE") / 8.0)
                                       / 1024.0) if _mean("SQ_WAVE_CYCLES") and _mean("GRBM_GUI_ACTIVE") else None,
           "l2_hit": (_mean("TCC_HIT_sum") / (_mean("TCC_HIT_sum") + _mean("TCC_MISS_sum"))
                      if _mean("TCC_HIT_sum") is not None and _mean("TCC_MISS_sum") else None),
           "l2_requests_per_launch": (_mean("TCC_HIT_sum") + _mean("TCC_MISS_sum")
                                      if _mean("TCC_HIT_sum") is not None and _mean("TCC_MISS_sum") is not None else None),
           "bench_args": os.environ.get("PMC_BENCH_ARGS"),
           "note": "FETCH_SIZE x2 (gfx950 coalesced-read correction) + WRITE_SIZE, KB->B"}
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
    print("traffic ->", sys.argv[2], out["hbm_bytes_per_launch"])
