"""Replay one chain up to its first divergent step and print attempt-level detail."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from cases import cases  # noqa: E402
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, eval_flips  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.reference_proxy import PhiloxStream  # noqa: E402

name, cid_local = sys.argv[1], int(sys.argv[2])
case = {c.name: c for c in cases()}[name]
g = case.graph
lo, hi = case.bounds
NC, seed, id0 = 7, 2024, 17
dg = DeviceGraph(g)
ch = Chains(dg, NC, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, base=case.base,
            seed=seed, chain_id0=id0)
tr = ch.run_traced(2000)
gid = id0 + cid_local
_, _, _, otr = O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, seed, gid, 2000,
                           trace=True)
gtr = np.where(tr[cid_local] >= 0, tr[cid_local] // 64, tr[cid_local])
b = int(np.flatnonzero(gtr != otr)[0])
print("first divergent step", b, "gpu", tr[cid_local][b], "oracle", otr[b])
lab, st, pops, _ = O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, seed, gid, b)
print("oracle state before step b:\n", lab.reshape(-1, g.grid_w))
print("attempts so far", st["attempts"][0], "pops", pops)
# enumerate the oracle's attempts of step b
rng = PhiloxStream(seed, gid)
rng.attempt = int(st["attempts"][0])
w = []
for x in range(g.n):
    nb = g.neighbors(x)
    fl = sorted({int(lab[u]) for u in nb if lab[u] != lab[x]})
    w.append(fl)
pairs = [(x, d) for x in range(g.n) for d in w[x]]
for t in range(12):
    rng.next_block()
    v, d = pairs[rng.index(len(pairs))]
    dc, co, po, db = O.eval_flips(g, lab, case.k, [v], [d], lo, hi)
    gdc, gco, gpo, gdb = eval_flips(dg, lab, case.k, [v], [d], (lo, hi))
    print(f"attempt {rng.attempt - 1}: v={v} ({v // g.grid_w},{v % g.grid_w}) d={d} oracle(dcut={dc[0]} "
          f"contig={co[0]} pop={po[0]}) gpu_eval(dcut={gdc[0]} contig={gco[0]} pop={gpo[0]}) u={rng.random():.4f}")
# GPU state after b steps of a fresh run and after one more step
ch2 = Chains(dg, NC, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, base=case.base,
             seed=seed, chain_id0=id0)
ch2.run(b)
print("gpu labels equal oracle before step b:", np.array_equal(ch2.labels()[cid_local], lab))
s0 = ch2.stats()[cid_local]
t1 = ch2.run_traced(1)
s1 = ch2.stats()[cid_local]
print("gpu step b:", t1[cid_local], {f: int(s1[f]) - int(s0[f]) for f in
                                     ["attempts", "pop_fail", "contig_fail", "bfs_runs", "bfs_nodes"]})
