"""Summarise a profile.sh output directory: kernel stats + per-dispatch PMC means.

    python scripts/pmc_summary.py gpurun_out/prof_<tag> [pmc.json]

Only the chain kernel's TIMED dispatches count: the bench line of each pass (the last JSON
line of ktrace_bench.log / pmc<i>_bench.log) names its protocol (warm-up W, timed K
launches, the "identity" bench.py prints), and the last K chain-kernel dispatches of every
pass are the timed ones.  So the counters, the rocprof kernel time and the line's own
HIP-event kernel time describe the same launches.

With a second argument, writes the per-launch figures as JSON (bench.py reads it by
pmc_key and checks its identity): FETCH_SIZE and WRITE_SIZE are kilobytes; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM), so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the state write-back).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

CHAIN_KERNEL = re.compile(r"fw_(grid16|grid16_spec|grid16_w2|grid16_full|run)_kernel")

d = sys.argv[1]


def bench_line(path):
    try:
        lines = [x for x in open(path).read().splitlines() if x.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except OSError:
        return None


line = bench_line(os.path.join(d, "ktrace_bench.log"))
timed = int(line["steps"]) if line else None

# rocprof kernel time of the timed launches (the last K dispatches of the chain kernel)
kern = {}
ktr = os.path.join(d, "ktrace", "run_kernel_trace.csv")
if os.path.exists(ktr):
    rows = [r for r in csv.DictReader(open(ktr)) if CHAIN_KERNEL.search(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    sel = rows[-timed:] if timed else rows
    if sel:
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        kern = {"name": sel[-1]["Kernel_Name"], "avg_ms": sum(ms) / len(ms), "calls": len(sel),
                "dispatches_in_run": len(rows), "selection": f"last {len(sel)} (timed)"}
        print(f"{kern['name'][:70]:70s} timed={len(sel)} of {len(rows)} avg_ms={kern['avg_ms']:9.3f}")
ks = os.path.join(d, "ktrace", "run_kernel_stats.csv")
if os.path.exists(ks):
    for r in csv.DictReader(open(ks)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:9.3f} (all calls)")

agg = collections.defaultdict(list)
pmc_lines = []
for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
    pl = bench_line(os.path.join(d, os.path.basename(os.path.dirname(f)) + "_bench.log"))
    pmc_lines.append(pl)
    k = int(pl["steps"]) if pl else None
    per = collections.defaultdict(dict)  # dispatch -> counter -> value
    for r in csv.DictReader(open(f)):
        if CHAIN_KERNEL.search(r["Kernel_Name"]):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)
    for i in (ids[-k:] if k else ids):
        for name, v in per[i].items():
            agg[name].append(v)
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")


def _mean(name):
    v = agg.get(name)
    return sum(v) / len(v) if v else None


if len(sys.argv) > 2 and "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
    fetch = _mean("FETCH_SIZE") * 1024.0
    write = _mean("WRITE_SIZE") * 1024.0
    ident = (line or {}).get("identity")
    same = all(pl is not None and pl.get("identity") == ident for pl in pmc_lines)
    out = {"hbm_bytes_per_launch": 2.0 * fetch + write, "fetch_bytes_raw": fetch,
           "fetch_bytes_corrected": 2.0 * fetch, "write_bytes": write,
           "source": os.path.basename(os.path.normpath(d)), "kernel_trace": kern,
           # the protocol and build the profile describes (bench.py compares it with its own)
           "identity": ident if same else None,
           "identity_note": None if same else "PMC passes ran another protocol than the trace",
           "line_kernel_ms": (line or {}).get("kernel_ms"),
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
           "wait_any_frac": (_mean("SQ_WAIT_ANY") / _mean("SQ_WAVE_CYCLES")
                             if _mean("SQ_WAIT_ANY") and _mean("SQ_WAVE_CYCLES") else None),
           "wait_inst_any_frac": (_mean("SQ_WAIT_INST_ANY") / _mean("SQ_WAVE_CYCLES")
                                  if _mean("SQ_WAIT_INST_ANY") and _mean("SQ_WAVE_CYCLES") else None),
           "l2_hit": (_mean("TCC_HIT_sum") / (_mean("TCC_HIT_sum") + _mean("TCC_MISS_sum"))
                      if _mean("TCC_HIT_sum") is not None and _mean("TCC_MISS_sum") else None),
           "l2_requests_per_launch": (_mean("TCC_HIT_sum") + _mean("TCC_MISS_sum")
                                      if _mean("TCC_HIT_sum") is not None and _mean("TCC_MISS_sum") is not None else None),
           "bench_args": os.environ.get("PMC_BENCH_ARGS"),
           "note": "timed dispatches only; FETCH_SIZE x2 (gfx950 coalesced-read correction) + "
                   "WRITE_SIZE, KB->B"}
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
    print("traffic ->", sys.argv[2], out["hbm_bytes_per_launch"])
