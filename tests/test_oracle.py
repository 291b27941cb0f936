"""The CPU oracle against known answers, networkx ground truth, the committed golden
fixtures and the independent GerryChain-equivalent proxy (CPU only)."""
import json
import math
import os

import networkx as nx
import numpy as np
import pytest

from cases import GOLDEN, cases
from oracle import oracle as O
from oracle.reference_proxy import ProxyChain, philox4x32_10

CASES = {c.name: c for c in cases()}


# ------------------------------------------------------------------ Philox
KAT = [  # Random123 philox4x32-10 known-answer vectors
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_philox_kat(ctr, key, out):
    assert list(O.philox4x32_10(ctr, key)) == out
    assert list(philox4x32_10(*ctr, *key)) == out  # the proxy's pure-Python copy


def test_rank_and_uniform_maps():
    L = O.lib()
    for x0, x1, P in [(0, 0, 7), (0xFFFFFFFF, 0xFFFFFFFF, 7), (123, 456, 1), (5, 1 << 31, 1000)]:
        want = (((x1 << 32) | x0) * P) >> 64
        assert L.orc_scale64(x0, x1, P) == want < P
    # CPython random(): (a*2^26 + b) / 2^53 with a = x2>>5, b = x3>>6
    assert L.orc_u53(0, 0) == 0.0
    u = L.orc_u53(0xFFFFFFFF, 0xFFFFFFFF)
    assert u < 1.0 and u == (((1 << 27) - 1) * 67108864.0 + ((1 << 26) - 1)) / 2**53


# ------------------------------------------------------------------ per-flip verdicts
def _nx(g):
    G = nx.Graph()
    G.add_nodes_from(range(g.n))
    G.add_edges_from(map(tuple, g.edges().tolist()))
    return G


@pytest.mark.parametrize("name", ["grid10_k2_bi", "grid12_k4_pairs", "sec11_a2_k2", "county_k2",
                                  "tract_k4", "grid16x24_k8"])
def test_eval_flips_matches_golden_and_networkx(name):
    case = CASES[name]
    gold = np.load(os.path.join(GOLDEN, "flips_golden.npz"), allow_pickle=False)
    lab, v, t = gold[f"{name}__labels"], gold[f"{name}__v"], gold[f"{name}__target"]
    got = np.stack(O.eval_flips(case.graph, lab, case.k, v, t, *case.bounds), 1).astype(np.int32)
    assert np.array_equal(got, gold[f"{name}__expect"])
    # independent ground truth on a subsample
    G = _nx(case.graph)
    lo, hi = case.bounds
    pop = case.graph.pop_array()
    cut = lambda L: sum(1 for x, y in G.edges if L[x] != L[y])  # noqa: E731
    bset = lambda L: sum(1 for x in G.nodes if any(L[y] != L[x] for y in G[x]))  # noqa: E731
    for i in range(0, len(v), 7):
        a, b = int(lab[v[i]]), int(t[i])
        after = lab.astype(np.int64).copy()
        after[v[i]] = b
        rest = [x for x in G.nodes if after[x] == a]
        contig = int(bool(rest) and nx.is_connected(G.subgraph(rest)))
        pops = np.bincount(after, weights=pop, minlength=case.k)
        assert got[i, 0] == cut(after) - cut(lab)
        assert got[i, 1] == contig
        assert got[i, 2] == int(lo <= pops[a] <= hi and lo <= pops[b] <= hi)
        assert got[i, 3] == bset(after) - bset(lab)


def test_plan_valid_matches_networkx():
    rng = np.random.default_rng(3)
    case = CASES["grid12_k4_pairs"]
    g = case.graph
    G = _nx(g)
    for _ in range(40):
        lab = case.init.copy()
        flips = rng.integers(0, g.n, 6)
        lab[flips] = rng.integers(0, 4, 6)
        ok = all(len([x for x in G if lab[x] == d]) and nx.is_connected(
            G.subgraph([x for x in G if lab[x] == d])) for d in range(4))
        pops = np.bincount(lab, minlength=4)
        ok = ok and pops.min() >= 0 and True
        assert O.plan_valid(g, lab, 4, 0, g.n) == ok


# ------------------------------------------------------------------ chains
def test_chains_match_committed_golden():
    gold = json.load(open(os.path.join(GOLDEN, "chains_golden.json")))
    import hashlib
    for key, rec in gold.items():
        name, cid = key.split("/")
        case = CASES[name]
        lab, st, pops, _ = O.run_chain(case.graph, case.init, case.k, case.mode, *case.bounds,
                                       case.thr, 2024, int(cid), 5000)
        assert hashlib.sha256(lab.astype(np.int16).tobytes()).hexdigest()[:16] == rec["labels_sha"]
        for f in st.dtype.names:
            want = rec[f]
            got = float(st[f][0]).hex() if f == "sum_invb" else int(st[f][0])
            assert got == want, (key, f)
        assert [int(x) for x in pops] == rec["pops"]


@pytest.mark.parametrize("name", ["grid10_k2_bi", "grid12_k4_pairs", "grid12_k4_cut",
                                  "grid7x9_k3_cut", "sec11_a2_k2", "county_k2"])
def test_proxy_follows_the_same_trajectory(name):
    """GerryChain-equivalent Python (dict copies, cut-edge sets, networkx Dijkstra)."""
    case = CASES[name]
    S = 400
    lab, st, _, _ = O.run_chain(case.graph, case.init, case.k, case.mode, *case.bounds, case.thr,
                                77, 3, S)
    ch = ProxyChain(case.graph, case.init, case.k, case.mode, case.percent, case.base, 77, 3)
    ch.run(S, bounds=case.bounds)
    assert np.array_equal(np.array(ch.labels()), lab)
    for f in ("attempts", "steps", "accepts", "pop_fail", "contig_fail"):
        assert ch.counters[f] == int(st[f][0]), f
    assert ch.obs["sum_cut"] == int(st["sum_cut"][0])
    assert ch.obs["sum_bnodes"] == int(st["sum_bnodes"][0])
    assert ch.obs["sum_invb"] == float(st["sum_invb"][0])  # same summation order: exact


@pytest.mark.parametrize("name", ["grid20_k4_mu", "tract_k4", "grid11x13_k4"])
def test_chain_invariants(name):
    case = CASES[name]
    g = case.graph
    hc = np.zeros(g.n_edges + 1, np.uint64)
    hb = np.zeros(g.n + 1, np.uint64)
    lab, st, pops, _ = O.run_chain(g, case.init, case.k, case.mode, *case.bounds, case.thr, 1, 2,
                                   3000, hist_cut=hc, hist_b=hb)
    s = st[0]
    assert O.plan_valid(g, lab, case.k, *case.bounds)
    e = g.edges()
    cut = int((lab[e[:, 0]] != lab[e[:, 1]]).sum())
    bnodes = len(set(e[lab[e[:, 0]] != lab[e[:, 1]]].ravel().tolist()))
    assert s["cut"] == cut and s["bnodes"] == bnodes
    assert np.array_equal(pops, np.bincount(lab, weights=g.pop_array(), minlength=case.k))
    assert s["steps"] == 3000 and s["yields"] == 3001 and hc.sum() == hb.sum() == 3001
    assert s["attempts"] == s["steps"] + s["pop_fail"] + s["contig_fail"]
    assert math.isclose(float((hb[1:] / np.arange(1, g.n + 1)).sum()), s["sum_invb"],
                        rel_tol=1e-12)
    assert int((hc * np.arange(len(hc))).sum()) == s["sum_cut"]


def test_stuck_instead_of_infinite_loop():
    from flipcomplexityempirical_amd.graph import grid_graph, stripe_seed
    g = grid_graph(6, 6)
    lab = stripe_seed(6, 6)
    D = g.maxdeg
    thr = np.ones(2 * D + 1)
    out, st, _, _ = O.run_chain(g, lab, 2, 0, 18, 18, thr, 0, 0, 10, max_retries=50)
    assert st["stuck"][0] == 1 and st["steps"][0] == 0 and st["attempts"][0] == 50
    assert np.array_equal(out, lab)


@pytest.mark.parametrize("name", ["grid10_k2_bi", "grid12_k4_pairs", "grid7x9_k3_cut",
                                  "sec11_a2_k2"])
def test_oracle_maps_follow_the_reference_driver(name):
    """orc maps == a literal replay of grid_chain_sec11.py:383-384,396-400 over the trace."""
    case = CASES[name]
    g = case.graph
    lo, hi = case.bounds
    vals = np.array([-1, 1] if case.k == 2 else [5 - 2 * d for d in range(case.k)], np.int64)
    S = 250
    M = O.Maps(g, case.init, vals)
    O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, 3, 1, S, maps=M)
    e = g.edges()
    lab, st = case.init.copy(), O.new_stats(1)
    ct = np.zeros(len(e), np.int64)
    nf = np.zeros(g.n, np.int64)
    lf = np.zeros(g.n, np.int64)
    ps = vals[case.init.astype(np.int64)].copy()
    f = None
    for t in range(S + 1):  # yield t: the initial state, then one state per counted step
        if t > 0:
            prev = lab
            lab, st, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, 3, 1, 1,
                                        stats=st)
            changed = np.flatnonzero(prev != lab)
            if len(changed):
                f = int(changed[0])
        cur = lab.astype(np.int64)
        ct += cur[e[:, 0]] != cur[e[:, 1]]
        if f is not None:  # part.flips is not None
            ps[f] -= vals[cur[f]] * (t - lf[f])
            lf[f] = t
            nf[f] += 1
    assert np.array_equal(ct, M.cut_times) and np.array_equal(nf, M.num_flips)
    assert np.array_equal(ps, M.part_sum) and np.array_equal(lf, M.last_flipped)


@pytest.mark.parametrize("name,rule", [("grid10_k2_bi", "bratio"), ("grid12_k4_pairs", "bratio"),
                                       ("sec11_a2_k2", "bratio"), ("grid10_k2_bi", "boundary"),
                                       ("sec11_a0_k2_mu", "boundary"),
                                       ("grid12_k4_cut", "boundary")])
def test_accept_rules_follow_the_reference_functions(name, rule):
    """Oracle FW_ACCEPT_BRATIO / FW_ACCEPT_BOUNDARY == the proxy running literal restatements
    of annealing_cut_accept_backwards (base .1, beta 5 as the reference) and
    uniform_accept + boundary_condition (grid_chain_sec11.py:43-52,81-110,159-165)."""
    from flipcomplexityempirical_amd.chain import annealing_table
    from flipcomplexityempirical_amd.graph import boundary_flags
    case = CASES[name]
    g = case.graph
    S = 300
    if rule == "bratio":
        base, beta, flags, r = 0.1, 5, None, 1
        thr = annealing_table(base, beta, g.maxdeg)
    else:
        base, beta, r = case.base, 1, 2
        flags = boundary_flags(g)
        thr = case.thr
    lab, st, _, _ = O.run_chain(g, case.init, case.k, case.mode, *case.bounds, thr, 13, 2, S,
                                accept_rule=r, flags=flags)
    ch = ProxyChain(g, case.init, case.k, case.mode, case.percent, base, 13, 2, accept=rule,
                    beta=beta, flags=flags)
    ch.run(S, bounds=case.bounds)
    assert np.array_equal(np.array(ch.labels()), lab)
    for f in ("attempts", "steps", "accepts"):
        assert ch.counters[f] == int(st[f][0]), f
    assert 0 < st["accepts"][0] < S or rule == "boundary"


def _ramp(t):
    if t < 30:
        return 0
    if t < 130:
        return (t - 30) / 50
    return 2


@pytest.mark.parametrize("name", ["grid10_k2_bi", "grid12_k4_pairs", "sec11_a2_k2"])
def test_beta_schedule_follows_step_num(name):
    """Oracle schedule rows (fw_chains_set_schedule) == the proxy evaluating
    annealing_cut_accept_backwards with beta = f(partition["step_num"]), the reference's
    commented schedule form (grid_chain_sec11.py:85-93, step_num :282-289)."""
    from flipcomplexityempirical_amd.chain import schedule_rows
    case = CASES[name]
    g = case.graph
    S = 700
    rows, t0 = schedule_rows(0.1, _ramp, 30, 130, g.maxdeg)
    lab, st, _, _ = O.run_chain(g, case.init, case.k, case.mode, *case.bounds, rows[0], 17, 3,
                                S, accept_rule=1, schedule=(rows, t0))
    ch = ProxyChain(g, case.init, case.k, case.mode, case.percent, 0.1, 17, 3, accept="bratio",
                    beta=_ramp)
    ch.run(S, bounds=case.bounds)
    assert np.array_equal(np.array(ch.labels()), lab)
    for f in ("attempts", "steps", "accepts"):
        assert ch.counters[f] == int(st[f][0]), f
    assert st["accepts"][0] > 130  # the run went past the end of the ramp


def test_reference_beta_schedule_rows():
    """reference_beta is the commented ramp (grid_chain_sec11.py:88-93); its rows are exact
    at both clamped ends."""
    from flipcomplexityempirical_amd.chain import annealing_table, reference_beta, schedule_rows
    assert reference_beta(99999) == 0 and reference_beta(100000) == 0.0
    assert reference_beta(250000) == 1.5 and reference_beta(400000) == 3
    rows, t0 = schedule_rows(0.1, reference_beta, 100000, 400000, 4)
    assert t0 == 100000 and rows.shape == (300001, 9)
    assert np.array_equal(rows[0], annealing_table(0.1, 0, 4))
    assert np.array_equal(rows[-1], annealing_table(0.1, 3, 4))
    assert np.array_equal(rows[150000], annealing_table(0.1, 1.5, 4))
