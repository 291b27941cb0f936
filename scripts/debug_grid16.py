"""Find the first step where the grid16 kernel diverges from the oracle (GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from cases import cases  # noqa: E402
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph  # noqa: E402
from oracle import oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "grid10_k2_bi"
case = {c.name: c for c in cases()}[name]
g = case.graph
lo, hi = case.bounds
dg = DeviceGraph(g)
NC, S, seed, id0 = 7, 2000, 2024, 17
ch = Chains(dg, NC, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, base=case.base,
            seed=seed, chain_id0=id0)
tr = ch.run_traced(S)
labs = ch.labels()
st = ch.stats()
for i in range(NC):
    olab, ost, _, otr = O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, seed, id0 + i,
                                     S, trace=True)
    gtr = np.where(tr[i] >= 0, tr[i] // 64, tr[i])
    bad = np.flatnonzero(gtr != otr)
    print(f"chain {i}: labels_equal={np.array_equal(labs[i], olab)} first_trace_diff="
          f"{bad[0] if len(bad) else None} gpu_stats_att={st['attempts'][i]} orc_att={ost['attempts'][0]}"
          f" bfs gpu={st['bfs_runs'][i]} orc={ost['bfs_runs'][0]} stuck={st['stuck'][i]}")
    if len(bad):
        b = bad[0]
        print("   around:", gtr[max(0, b - 3):b + 3], otr[max(0, b - 3):b + 3], "raw", tr[i][b - 1:b + 2])
        # state just before the divergent step, replayed on the oracle
        plab, pst, _, _ = O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, seed,
                                      id0 + i, b)
        print("   oracle state before step:\n", plab.reshape(-1, g.grid_w or 1))
        print("   gpu final labels:\n", labs[i].reshape(-1, g.grid_w or 1))
