"""Generate the committed golden fixtures (run here, where /root/reference exists).

    python tests/golden/make_golden.py

Writes, next to this file:
* kansas_<unit>20.npz — CSR (rowptr, col), TOTPOP (cast with int() as
  All_States_Chain.py:227-230 does) and contiguous seed plans for k = 2 and 4 drawn by
  recursive_tree_part (All_States_Chain.py:232) with epsilon 0.05, from the reference's
  State_Data/<unit>20.json.
* wait_sec11.json — the reference's published per-run wait sums
  (New_plots/sec11/{alignment}B{int(100*base)}P{int(100*pop)}wait.txt, one integer each).
* wait_ks.json — the same for plots/KS2 and plots/States/20.
* wait_frank2.json — the same for plots/FRANK2 (Frankenstein_chain.py on the Frankengraph,
  k=2, 100,000 yields per run, bases .3 .35 .379 and their inverses, pops .1 .5 .9).
* flips_golden.npz — per-flip verdicts (Δcut, contiguity, population, Δboundary) on
  states drawn from oracle chains, each verdict checked here against independent
  networkx ground truth (nx.is_connected on the district subgraph, brute-force cut
  counts, brute-force boundary sets).
* chains_golden.json — oracle chain results (final-plan digest, counters, sums) for the
  shared test cases, pinning the oracle itself against regressions.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import re
import sys

import networkx as nx
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from flipcomplexityempirical_amd.graph import Graph  # noqa: E402
from flipcomplexityempirical_amd.seeds import recursive_tree_part  # noqa: E402
from oracle import oracle as O  # noqa: E402


def kansas_fixtures():
    from flipcomplexityempirical_amd.chain import population_bounds
    for unit in ["County20", "Tract20", "COUSUB20", "BG20"]:
        g = Graph.from_json(os.path.join(REF, "State_Data", f"{unit}.json"), pop_col="TOTPOP")
        out = dict(rowptr=g.rowptr, col=g.col, pop=g.pop,
                   node_ids=np.array(g.nodes, dtype=np.int64))
        for k in (2, 4):
            for s in range(100):
                lab = recursive_tree_part(g, list(range(k)), g.total_pop / k, 0.05, seed=s)
                lo, hi = population_bounds(g.total_pop, k, 0.10)
                if O.plan_valid(g, lab, k, lo, hi):
                    break
            else:
                raise RuntimeError(f"no valid seed for {unit} k={k}")
            out[f"seed_k{k}"] = lab.astype(np.int8)
        np.savez_compressed(os.path.join(HERE, f"kansas_{unit}.npz"), **out)
        print(unit, g.n, g.n_edges, g.maxdeg)


def wait_fixtures():
    pat = re.compile(r"^(\w+?)B(\d+)P(\d+)wait\.txt$")
    res = {}
    for sub in ["New_plots/sec11", "plots/KS2", "plots/States/20"]:
        rows = []
        for f in sorted(glob.glob(os.path.join(REF, sub, "*wait.txt"))):
            m = pat.match(os.path.basename(f))
            with open(f) as fh:
                rows.append(dict(unit=m.group(1), base_label=int(m.group(2)),
                                 pop_label=int(m.group(3)), wait_sum=int(fh.read().strip())))
        res[sub] = rows
    with open(os.path.join(HERE, "wait_sec11.json"), "w") as f:
        json.dump(res["New_plots/sec11"], f, indent=0)
    frank = []
    for f in sorted(glob.glob(os.path.join(REF, "plots/FRANK2", "*wait.txt"))):
        m = pat.match(os.path.basename(f))
        with open(f) as fh:
            frank.append(dict(alignment=int(m.group(1)), base_label=int(m.group(2)),
                              pop_label=int(m.group(3)), wait_sum=int(fh.read().strip())))
    with open(os.path.join(HERE, "wait_frank2.json"), "w") as f:
        json.dump(frank, f, indent=0)
    with open(os.path.join(HERE, "wait_ks.json"), "w") as f:
        json.dump({"KS2": res["plots/KS2"], "States20": res["plots/States/20"]}, f, indent=0)


def nx_graph(g):
    G = nx.Graph()
    G.add_nodes_from(range(g.n))
    G.add_edges_from(map(tuple, g.edges().tolist()))
    return G


def ground_truth(G, g, lab, k, v, b, lo, hi):
    a = lab[v]
    cut = lambda L: sum(1 for x, y in G.edges if L[x] != L[y])  # noqa: E731
    bset = lambda L: {x for x in G.nodes if any(L[y] != L[x] for y in G[x])}  # noqa: E731
    after = lab.copy()
    after[v] = b
    rest = [x for x in G.nodes if after[x] == a]
    contig = len(rest) > 0 and nx.is_connected(G.subgraph(rest))
    pops = np.bincount(after, weights=g.pop_array(), minlength=k)
    pop_ok = all(lo <= p <= hi for p in pops[[a, b]])
    return cut(after) - cut(lab), int(contig), int(pop_ok), len(bset(after)) - len(bset(lab))


def flip_fixtures():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cases as C
    rng = np.random.default_rng(1234)
    arrays = {}
    names = []
    for case in C.cases():
        if case.name not in ("grid10_k2_bi", "grid12_k4_pairs", "sec11_a2_k2", "county_k2",
                             "tract_k4", "grid16x24_k8"):
            continue
        g = case.graph
        G = nx_graph(g)
        lo, hi = case.bounds
        lab, _, _, _ = O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, 99, 5, 3000)
        # candidate flips: every boundary (node, foreign label) pair, subsampled
        pairs = [(v, int(lab[u])) for v in range(g.n) for u in g.neighbors(v) if lab[u] != lab[v]]
        pairs = sorted(set(pairs))
        idx = rng.choice(len(pairs), size=min(160, len(pairs)), replace=False)
        vs = np.array([pairs[i][0] for i in idx], np.int32)
        ts = np.array([pairs[i][1] for i in idx], np.int16)
        dcut, contig, pop_ok, db = O.eval_flips(g, lab, case.k, vs, ts, lo, hi)
        for i in range(len(vs)):
            gt = ground_truth(G, g, lab.astype(np.int64), case.k, int(vs[i]), int(ts[i]), lo, hi)
            got = (int(dcut[i]), int(contig[i]), int(pop_ok[i]), int(db[i]))
            assert gt == got, (case.name, i, gt, got)
        names.append(case.name)
        arrays[f"{case.name}__labels"] = lab
        arrays[f"{case.name}__v"] = vs
        arrays[f"{case.name}__target"] = ts
        arrays[f"{case.name}__expect"] = np.stack([dcut, contig, pop_ok, db], 1).astype(np.int32)
        print("flips", case.name, len(vs), "contig=0:", int((contig == 0).sum()))
    arrays["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "flips_golden.npz"), **arrays)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.int16).tobytes()).hexdigest()[:16]


def chain_fixtures():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cases as C
    out = {}
    for case in C.cases():
        lo, hi = case.bounds
        for cid in (0, 1):
            lab, st, pops, _ = O.run_chain(case.graph, case.init, case.k, case.mode, lo, hi,
                                           case.thr, 2024, cid, 5000)
            rec = {f: (float(st[f][0]) if f == "sum_invb" else int(st[f][0]))
                   for f in st.dtype.names}
            rec["sum_invb"] = float(st["sum_invb"][0]).hex()
            rec["labels_sha"] = digest(lab)
            rec["pops"] = [int(x) for x in pops]
            out[f"{case.name}/{cid}"] = rec
    with open(os.path.join(HERE, "chains_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["waits"]:
        wait_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["chains"]:
        chain_fixtures()
        sys.exit(0)
    kansas_fixtures()
    wait_fixtures()
    flip_fixtures()
    chain_fixtures()
