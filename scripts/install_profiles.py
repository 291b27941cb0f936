#!/usr/bin/env python3
"""Install profile.sh outputs as bench.py's PMC profiles, keyed by the protocol they ran:

    python scripts/install_profiles.py profiles/r05/prof gpurun_out/prof_*

For each directory: pmc.json (with the bench line's identity, pmc_summary.py) ->
profiles/pmc/<pmc_key>.json, and summary.txt, pmc.json, the kernel stats and trace of the
timed launches -> <dest>/<tag>/ (the evidence a bench line's "pmc.source" names)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dest = sys.argv[1]
for d in sys.argv[2:]:
    pj = os.path.join(d, "pmc.json")
    if not os.path.exists(pj):
        print("skip (no pmc.json):", d)
        continue
    prof = json.load(open(pj))
    ident = prof.get("identity")
    if not ident:
        print("skip (no identity):", d, prof.get("identity_note"))
        continue
    tag = os.path.basename(os.path.normpath(d)).replace("prof_", "")
    out = os.path.join(dest, tag)
    os.makedirs(out, exist_ok=True)
    for f in ("summary.txt", "pmc.json"):
        shutil.copy(os.path.join(d, f), out)
    ks = os.path.join(d, "ktrace", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(out, "kernel_stats.csv"))
    prof["source"] = os.path.relpath(out, ROOT)
    key = bench.pmc_key(ident["config"], ident["order"], ident["chains"], ident["inner"],
                        ident["warmup"], ident["steps"], ident["chain_id0"], ident["resumed_steps"])
    os.makedirs(os.path.join(ROOT, "profiles", "pmc"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "pmc", key + ".json"), "w") as f:
        json.dump(prof, f, indent=1)
    print(f"{d} -> profiles/pmc/{key}.json ({prof['kernel_trace'].get('avg_ms'):.3f} ms rocprof, "
          f"{prof.get('line_kernel_ms') or 0:.3f} ms line)")
