#!/usr/bin/env python3
"""Per-kernel register use of one HIP source for gfx950 (compile-only, no GPU).

    python scripts/resource_usage.py flipcomplexityempirical_amd/csrc/fw_grid16.hip [filter]

Prints VGPRs, SGPRs, spills and the occupancy the compiler reports for every kernel
(-Rpass-analysis=kernel-resource-usage), demangled template arguments only.
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-Wno-unused-function", "-c", "-o", "/tmp/_ru.o", src,
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(.+?): (.+?) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt not in r["name"]:
        continue
    nm = r["name"]
    t = re.search(r"kernel(I.*E)Ev", nm)
    print(f"{nm[:48]:48s} {t.group(1) if t else '':24s} V={r.get('VGPRs','?'):>4s} "
          f"S={r.get('TotalSGPRs','?'):>4s} Sspill={r.get('SGPRs Spill','?'):>4s} "
          f"Vspill={r.get('VGPRs Spill','?'):>3s} occ={r.get('Occupancy [waves/SIMD]','?')}")
