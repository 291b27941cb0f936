"""GPU parity: the HIP path through the C-ABI against the CPU oracle, bit for bit.

Every chain's final plan, every counter, the fp64 sum of 1/|B| (bitwise), the district
populations and the yield histograms must equal oracle/flipchain_oracle.c run on the
same (seed, global chain id).  The oracle's per-flip verdicts are themselves pinned to
networkx ground truth (tests/golden/flips_golden.npz, tests/test_oracle.py).
"""
import os

import numpy as np
import pytest

from cases import GOLDEN, cases
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, eval_flips
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = cases()
IDS = [c.name for c in CASES]


def oracle_chains(case, seed, ids, steps_list):
    g = case.graph
    lo, hi = case.bounds
    hc = np.zeros(g.n_edges + 1, np.uint64)
    hb = np.zeros(g.n + 1, np.uint64)
    labs, sts, pops = [], [], []
    for cid in ids:
        lab = case.init.copy()
        st = O.new_stats(1)
        for steps in steps_list:
            lab, st, p, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, seed, cid,
                                        steps, stats=st, hist_cut=hc, hist_b=hb)
        labs.append(lab)
        sts.append(st[0])
        pops.append(p)
    return np.stack(labs), np.array(sts), np.stack(pops), hc, hb


def assert_stats_equal(gpu, orc):
    for f in orc.dtype.names:
        a, b = gpu[f], orc[f]
        if f == "sum_invb":
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (f, a, b)
        else:
            assert np.array_equal(a, b), (f, a, b)


# auto: the four-chains-per-wave kernel on grids; wave64: force one chain per wave.
# CSR graphs always run the one-chain-per-wave kernel, so they appear once.
KERNEL_CASES = [(c, p) for c in CASES for p in ("auto", "wave64") if p == "auto" or c.graph.grid_w]


@pytest.mark.parametrize("case,kernel_path", KERNEL_CASES,
                         ids=[f"{p}-{c.name}" for c, p in KERNEL_CASES])
def test_chain_bit_exact(gpu_lib, case, kernel_path, monkeypatch):
    if kernel_path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    n_chains, seed, id0 = 7, 2024, 17
    dg = DeviceGraph(case.graph)
    assert dg.grid_w == case.graph.grid_w
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=seed, chain_id0=id0)
    steps_list = [700, 1300]  # two launches: state must persist exactly across them
    for s in steps_list:
        ch.run(s)
    labs, st, pops = ch.labels(), ch.stats(), ch.pops()
    olabs, ost, opops, ohc, ohb = oracle_chains(case, seed, range(id0, id0 + n_chains), steps_list)
    assert np.array_equal(labs, olabs)
    assert_stats_equal(st, ost)
    assert np.array_equal(pops, opops)
    assert np.array_equal(ch.hist_cut(), ohc)
    assert np.array_equal(ch.hist_b(), ohb)
    assert (st["steps"] == sum(steps_list)).all() and not st["stuck"].any()


@pytest.mark.parametrize("case", [c for c in CASES if c.name in
                                  ("grid12_k4_pairs", "sec11_a2_k2", "tract_k4")],
                         ids=lambda c: c.name)
def test_trace_matches_oracle(gpu_lib, case):
    dg = DeviceGraph(case.graph)
    ch = Chains(dg, 3, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=5, chain_id0=0)
    tr = ch.run_traced(500)
    lo, hi = case.bounds
    for cid in range(3):
        _, _, _, otr = O.run_chain(case.graph, case.init, case.k, case.mode, lo, hi, case.thr, 5,
                                   cid, 500, trace=True)
        acc = tr[cid] >= 0
        assert np.array_equal(np.where(acc, tr[cid] // 64, -1), otr)


@pytest.mark.parametrize("name", ["grid10_k2_bi", "grid12_k4_pairs", "sec11_a2_k2", "county_k2",
                                  "tract_k4", "grid16x24_k8"])
def test_eval_flips_golden(gpu_lib, name):
    case = {c.name: c for c in CASES}[name]
    gold = np.load(os.path.join(GOLDEN, "flips_golden.npz"), allow_pickle=False)
    lab = gold[f"{name}__labels"]
    dg = DeviceGraph(case.graph)
    dcut, contig, pop_ok, db = eval_flips(dg, lab, case.k, gold[f"{name}__v"],
                                          gold[f"{name}__target"], case.bounds)
    got = np.stack([dcut, contig, pop_ok, db], 1).astype(np.int32)
    assert np.array_equal(got, gold[f"{name}__expect"])


def test_invalid_initial_state_raises(gpu_lib):
    from flipcomplexityempirical_amd._lib import InvalidInitialState
    from flipcomplexityempirical_amd.graph import grid_graph
    g = grid_graph(6, 6)
    lab = np.zeros(36, np.int16)
    lab[[0, 35]] = 1  # district 1 disconnected
    dg = DeviceGraph(g)
    with pytest.raises(InvalidInitialState):
        Chains(dg, 2, 2, lab, proposal="bi", pop_bounds=(0, 36), base=1.0)
    with pytest.raises(ValueError):  # GerryChain raises ValueError here
        Chains(dg, 2, 2, lab, proposal="bi", pop_bounds=(0, 36), base=1.0)


def test_stuck_flag_instead_of_hang(gpu_lib):
    """Tight bounds leave no valid flip: the reference would loop forever."""
    from flipcomplexityempirical_amd.graph import grid_graph, stripe_seed
    g = grid_graph(6, 6)
    lab = stripe_seed(6, 6)
    dg = DeviceGraph(g)
    ch = Chains(dg, 4, 2, lab, proposal="bi", pop_bounds=(18, 18), base=1.0)
    ch.run(10, max_retries=50)
    st = ch.stats()
    assert st["stuck"].all() and (st["steps"] == 0).all() and (st["attempts"] == 50).all()
    assert (ch.labels() == lab).all()


def _run_vs_oracle(case, n_chains, steps_list, seed=99, id0=3):
    dg = DeviceGraph(case.graph)
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=seed, chain_id0=id0)
    for s in steps_list:
        ch.run(s)
    labs, st, pops = ch.labels(), ch.stats(), ch.pops()
    olabs, ost, opops, ohc, ohb = oracle_chains(case, seed, range(id0, id0 + n_chains), steps_list)
    assert np.array_equal(labs, olabs)
    assert_stats_equal(st, ost)
    assert np.array_equal(pops, opops)
    assert np.array_equal(ch.hist_cut(), ohc)
    assert np.array_equal(ch.hist_b(), ohb)
    return st


@pytest.mark.parametrize("name", ["grid20_k4_mu", "grid16x24_k8", "grid30x18_k2_bi"])
@pytest.mark.parametrize("bitboard", [True, False])
def test_many_chains_per_workgroup(gpu_lib, name, bitboard, monkeypatch):
    """77 chains: several waves and workgroups, a ragged last wave; exact searches in the
    bitboard form (2-bit labels) and as the list search under the contended lock."""
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    if bitboard:
        monkeypatch.delenv("FLIPWALK_NO_BITBOARD", raising=False)
    else:
        monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 77, [300, 500])
    assert st["bfs_runs"].sum() > 0


W2_GRIDS = ["grid10_k2_bi", "grid12_k4_pairs", "grid12_k4_cut", "grid20_k4_mu", "grid11x13_k4",
            "grid30x18_k2_bi"]


@pytest.mark.parametrize("w2", ["0", "1"])
@pytest.mark.parametrize("name", W2_GRIDS)
@pytest.mark.parametrize("bitboard", [True, False])
def test_grid_kernel_register_budgets(gpu_lib, name, w2, bitboard, monkeypatch):
    """Both register budgets of the lean grid kernel (fw_grid16_plan): the default one held to
    3 waves per SIMD (FLIPWALK_W2=0) and W2, 2 waves per SIMD, which the plan takes for
    launches with at most 2 waves of work per SIMD (every small test, the 8-GPU job's
    8,192-chain shards): plans, counters, sums and histograms equal the oracle's, with
    exact searches in the bitboard form (its two-class path included) and as the list
    search."""
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    monkeypatch.setenv("FLIPWALK_W2", w2)
    if bitboard:
        monkeypatch.delenv("FLIPWALK_NO_BITBOARD", raising=False)
    else:
        monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 45, [400, 300])
    assert (st["accepts"] > 0).all()


@pytest.mark.parametrize("name,path", [("grid20_k4_mu", "auto"), ("grid20_k4_mu", "wave64"),
                                       ("grid30x18_k2_bi", "auto"), ("sec11_a2_k2", "auto"),
                                       ("tract_k4", "auto"), ("hub_k3", "auto"),
                                       ("grid40x4_k2", "auto")])
def test_search_list_spill(gpu_lib, name, path, monkeypatch):
    """A 2-entry LDS visit list: every exact search spills to its HBM slice (the grid
    kernel's bitboard search is switched off so that its list search runs)."""
    monkeypatch.setenv("FLIPWALK_LIST_CAP", "2")
    monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 21, [400, 400])
    assert (st["bfs_nodes"] > 2 * st["bfs_runs"]).any()  # searches did outgrow the LDS list


ACCEPT_CASES = [("grid12_k4_pairs", "bratio", "auto"), ("grid20_k4_mu", "bratio", "wave64"),
                ("grid16x24_k8", "bratio", "auto"), ("sec11_a2_k2", "bratio", "auto"),
                ("tract_k4", "bratio", "auto"), ("grid10_k2_bi", "boundary", "auto"),
                ("grid30x18_k2_bi", "boundary", "wave64"), ("sec11_a0_k2_mu", "boundary", "auto"),
                ("frank_a2_k2", "boundary", "auto"), ("grid12_k4_cut", "boundary", "auto"),
                ("hub_k3", "bratio", "auto"), ("hub_k2_cut", "boundary", "auto")]


@pytest.mark.parametrize("name,rule,path", ACCEPT_CASES,
                         ids=[f"{p}-{r}-{n}" for n, r, p in ACCEPT_CASES])
def test_accept_rules_bit_exact(gpu_lib, name, rule, path, monkeypatch):
    """annealing_cut_accept_backwards (|B'|/|B| factor, base .1 beta 5) and uniform_accept
    with boundary_condition (grid_chain_sec11.py:43-52,81-110,159-165) against the oracle."""
    from flipcomplexityempirical_amd.chain import annealing_table
    from flipcomplexityempirical_amd.graph import boundary_flags
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    g = case.graph
    r = 1 if rule == "bratio" else 2
    thr = annealing_table(0.1, 5, g.maxdeg) if rule == "bratio" else case.thr
    flags = boundary_flags(g) if rule == "boundary" else None
    n_chains, seed, id0, steps_list = 9, 77, 40, [600, 900]
    dg = DeviceGraph(g)
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                seed=seed, chain_id0=id0, thr=thr)
    ch.set_accept(rule, flags)
    for s in steps_list:
        ch.run(s)
    labs, st = ch.labels(), ch.stats()
    lo, hi = case.bounds
    for i in range(n_chains):
        lab, ost = case.init.copy(), O.new_stats(1)
        for s in steps_list:
            lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, thr, seed, id0 + i, s,
                                         stats=ost, accept_rule=r, flags=flags)
        assert np.array_equal(labs[i], lab), (name, i)
        for f in ("attempts", "steps", "accepts", "sum_cut", "bnodes", "bfs_nodes"):
            assert st[f][i] == ost[f][0], (name, i, f)


@pytest.mark.parametrize("n,k,bw,variant", [(132, 8, 4, "auto"), (200, 8, 4, "auto"),
                                            (200, 8, 4, "lb4"), (200, 8, 4, "list")])
def test_large_grid_ladder_bit_exact(gpu_lib, n, k, bw, variant, monkeypatch):
    """C5 shape: grids past the four-chains-per-wave kernel's 16,384-node limit (one chain
    per wave, implicit grid neighbours, 16 group sums per lane) with per-chain Metropolis
    bases from the C5 ladder (thr_per_chain).  auto: 3-bit labels with the list search's
    marks in HBM; lb4: 4-bit labels with in-place marks; list: 3-bit labels, every exact
    search as the HBM-marked list search with a 2-entry LDS list (spill)."""
    from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
    from flipcomplexityempirical_amd.graph import block_seed, grid_graph
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    if variant == "lb4":
        monkeypatch.setenv("FLIPWALK_CSR_LB", "4")
    if variant == "list":
        monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
        monkeypatch.setenv("FLIPWALK_LIST_CAP", "2")
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, bw)
    bounds = population_bounds(g.total_pop, k, 0.05)
    bases = np.geomspace(0.1, 10.0, 5)
    dg = DeviceGraph(g)
    ch = Chains(dg, len(bases), k, init, proposal="pairs", pop_bounds=bounds, base=bases, seed=8,
                chain_id0=1000)
    for s in (500, 300):
        ch.run(s)
    labs, st = ch.labels(), ch.stats()
    for i, b in enumerate(bases):
        lab, ost = init.copy(), O.new_stats(1)
        for s in (500, 300):
            lab, ost, _, _ = O.run_chain(g, lab, k, 1, *bounds, metropolis_table(b, 4), 8, 1000 + i,
                                         s, stats=ost)
        assert np.array_equal(labs[i], lab), i
        assert_stats_equal(st[i:i + 1], ost)


@pytest.mark.parametrize("n,variant", [(200, "auto"), (200, "list"), (160, "list")])
def test_large_grid_deep_search_bit_exact(gpu_lib, n, variant, monkeypatch):
    """C5 past burn-in: n x n, k=8, low ladder bases (0.1 .. 1) for 40,000 steps, where the
    districts are fractal (cut ~ 30% of the edges) and the exact searches that leave the
    7x7 window run tens of levels over hundreds of cells (scripts/search_stats.c), against
    the oracle bit for bit.  auto: the 64 x 64 bitboard, then the list search past it;
    list: every exact search as the list search (race_search_b3: visit marks in the labels,
    levels staged in LDS; at n = 160 the stage holds fewer entries, so larger levels are
    read from the HBM list)."""
    from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
    from flipcomplexityempirical_amd.graph import block_seed, grid_graph
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    if variant == "list":
        monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
    k = 8
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 4)
    bounds = population_bounds(g.total_pop, k, 0.05)
    bases = np.array([0.1, 0.25, 0.5, 1.0])
    steps = (20000, 20000)
    dg = DeviceGraph(g)
    ch = Chains(dg, len(bases), k, init, proposal="pairs", pop_bounds=bounds, base=bases,
                seed=11, chain_id0=77)
    for s in steps:
        ch.run(s)
    labs, st = ch.labels(), ch.stats()
    assert st["bfs_nodes"].sum() > 20 * st["bfs_runs"].sum() > 0
    for i, b in enumerate(bases):
        lab, ost = init.copy(), O.new_stats(1)
        for s in steps:
            lab, ost, _, _ = O.run_chain(g, lab, k, 1, *bounds, metropolis_table(b, 4), 11,
                                         77 + i, s, stats=ost)
        assert np.array_equal(labs[i], lab), i
        assert_stats_equal(st[i:i + 1], ost)
    ch.close()
    dg.close()


def _ramp(t):
    """A short stand-in for the reference's commented beta ramp (grid_chain_sec11.py:88-93)."""
    if t < 40:
        return 0
    if t < 160:
        return (t - 40) / 40
    return 3


SCHED_CASES = [("grid12_k4_pairs", "bratio", "auto"), ("grid20_k4_mu", "bratio", "wave64"),
               ("sec11_a2_k2", "bratio", "auto"), ("tract_k4", "bratio", "auto"),
               ("grid12_k4_cut", "cut", "auto"), ("grid30x18_k2_bi", "cut", "wave64")]


@pytest.mark.parametrize("name,rule,path", SCHED_CASES,
                         ids=[f"{p}-{r}-{n}" for n, r, p in SCHED_CASES])
def test_step_schedule_bit_exact(gpu_lib, name, rule, path, monkeypatch):
    """fw_chains_set_schedule: bounds indexed by step_num (accepted flips + 1) against the
    oracle, across two runs (the schedule position carries over) and a schedule change."""
    from flipcomplexityempirical_amd.chain import schedule_rows
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    g = case.graph
    r = 1 if rule == "bratio" else 0
    base = 0.1 if rule == "bratio" else 1.0 / max(case.base, 1e-9)
    rows, t0 = schedule_rows(base, _ramp, 40, 160, g.maxdeg)
    rows2, t02 = schedule_rows(base, lambda t: 2 - t / 200, 0, 400, g.maxdeg)
    n_chains, seed, id0 = 7, 91, 5
    dg = DeviceGraph(g)
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                seed=seed, chain_id0=id0, thr=case.thr)
    if rule == "bratio":
        ch.set_accept(rule)
    ch.set_schedule(rows, t0)
    ch.run(150)
    ch.run(250)
    ch.set_schedule(rows2, t02)
    ch.run(200)
    labs, st = ch.labels(), ch.stats()
    lo, hi = case.bounds
    for i in range(n_chains):
        lab, ost = case.init.copy(), O.new_stats(1)
        for s, sch in ((150, (rows, t0)), (250, (rows, t0)), (200, (rows2, t02))):
            lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, seed,
                                         id0 + i, s, stats=ost, accept_rule=r, schedule=sch)
        assert np.array_equal(labs[i], lab), (name, i)
        for f in ("attempts", "steps", "accepts", "sum_cut", "bnodes"):
            assert st[f][i] == ost[f][0], (name, i, f)
    assert st["accepts"].min() > 50  # the chains did move through the schedule


def _corridor_plan(h, w, k, vertical):
    """District 1: two blobs joined by a one-cell corridor far longer than the bitboard
    window (32 columns / 64 rows); district 0 around them; districts 2.. as corner blocks."""
    H, W = h, w
    lab = np.zeros((H, W), np.int16)
    mid = H // 2
    lab[mid - 5:mid + 6, 2:10] = 1
    lab[mid - 5:mid + 6, W - 10:W - 2] = 1
    lab[mid, 10:W - 10] = 1
    for t in range(2, k):  # small blocks along the top edge
        lab[0:2, 4 * (t - 2) + 12:4 * (t - 2) + 15] = t
    return np.ascontiguousarray(lab.T if vertical else lab).reshape(-1)


@pytest.mark.parametrize("k,vertical,path", [(2, False, "auto"), (2, True, "auto"),
                                             (2, False, "wave64"), (6, True, "wave64"),
                                             (6, False, "auto")])
def test_bitboard_window_escape(gpu_lib, k, vertical, path, monkeypatch):
    """Searches along a corridor longer than the bitboard window leave it: the kernels fall
    back to the list search.  Verdicts (fw_eval_flips) and whole chains (plans, search
    counters) against the oracle."""
    from flipcomplexityempirical_amd.graph import grid_graph
    monkeypatch.delenv("FLIPWALK_NO_BITBOARD", raising=False)
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    h, w = 30, 120
    g = grid_graph(w, h) if vertical else grid_graph(h, w)
    init = _corridor_plan(h, w, k, vertical)
    assert O.plan_valid(g, init, k, 1, g.n)
    dg = DeviceGraph(g)
    # every corridor cell flipped to district 0
    v = np.flatnonzero(init == 1).astype(np.int32)
    t = np.zeros(len(v), np.int16)
    got = np.stack(eval_flips(dg, init, k, v, t, (1, g.n)), 1).astype(np.int32)
    want = np.stack(O.eval_flips(g, init, k, v, t, 1, g.n), 1).astype(np.int32)
    assert np.array_equal(got, want)
    assert (got[:, 1] == 0).sum() > 50  # corridor cells disconnect district 1
    # chains from the corridor plan: many searches run past the window
    from flipcomplexityempirical_amd.chain import metropolis_table
    thr = metropolis_table(1.0, g.maxdeg)
    n_chains, steps, seed = 21, 150, 5
    ch = Chains(dg, n_chains, k, init, proposal="pairs", pop_bounds=(1, g.n), base=1.0, seed=seed)
    ch.run(steps)
    labs, st = ch.labels(), ch.stats()
    for i in range(n_chains):
        olab, ost, _, _ = O.run_chain(g, init, k, 1, 1, g.n, thr, seed, i, steps)
        assert np.array_equal(labs[i], olab), i
        for f in ("attempts", "steps", "accepts", "contig_fail", "bfs_runs", "bfs_nodes", "bfs_deg"):
            assert int(st[f][i]) == int(ost[f][0]), (i, f, st[f][i], ost[f][0])
    assert (st["bfs_nodes"] > 40 * st["bfs_runs"]).any()  # searches far past the window


@pytest.mark.parametrize("vertical", [False, True])
def test_bitboard_128_escape_3bit(gpu_lib, vertical, monkeypatch):
    """3-bit labels (the C5 path): a race along a corridor longer than 128 cells leaves the
    64 x 64 bitboard, continues on the 128 x 128 stage (race_bb4), leaves that too and ends
    in the list search seeded with the 128 window's last two levels.  Plans and every search
    counter against the oracle, chain by chain."""
    from flipcomplexityempirical_amd.chain import metropolis_table
    from flipcomplexityempirical_amd.graph import grid_graph
    monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    monkeypatch.setenv("FLIPWALK_CSR_LB", "3")
    monkeypatch.delenv("FLIPWALK_NO_BITBOARD", raising=False)
    h, w, k = 30, 300, 6
    g = grid_graph(w, h) if vertical else grid_graph(h, w)
    init = _corridor_plan(h, w, k, vertical)
    assert O.plan_valid(g, init, k, 1, g.n)
    dg = DeviceGraph(g)
    thr = metropolis_table(1.0, g.maxdeg)
    n_chains, steps, seed = 21, 120, 9
    ch = Chains(dg, n_chains, k, init, proposal="pairs", pop_bounds=(1, g.n), base=1.0, seed=seed)
    ch.run(steps)
    labs, st = ch.labels(), ch.stats()
    for i in range(n_chains):
        olab, ost, _, _ = O.run_chain(g, init, k, 1, 1, g.n, thr, seed, i, steps)
        assert np.array_equal(labs[i], olab), i
        for f in ("attempts", "steps", "accepts", "contig_fail", "bfs_runs", "bfs_nodes", "bfs_deg"):
            assert int(st[f][i]) == int(ost[f][0]), (i, f, st[f][i], ost[f][0])
    assert (st["bfs_nodes"] > 150 * st["bfs_runs"]).any()  # searches far past 128 cells


@pytest.mark.parametrize("name,path", [("grid20_k4_mu", "auto"), ("grid20_k4_mu", "wave64"),
                                       ("sec11_a2_k2", "auto"), ("tract_k4", "auto")])
def test_counter_fold_bit_exact(gpu_lib, name, path, monkeypatch):
    """The 32-bit per-launch counters that grow with attempts (attempts, population and
    contiguity failures, summed proposal degrees) fold into the 64-bit totals at a Philox
    refill; FLIPWALK_FOLD_AT=64 folds every few refills instead of at 2^31.  Totals and
    trajectories must not change."""
    monkeypatch.setenv("FLIPWALK_FOLD_AT", "64")
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 13, [500, 700])
    assert (st["sum_deg"] > 20 * 64).all()  # many folds happened


@pytest.mark.parametrize("name,path", [("grid20_k4_mu", "auto"), ("sec11_a2_k2", "auto")])
def test_long_run_split_into_launches(gpu_lib, name, path, monkeypatch):
    """fw_chains_run splits a run into launches of at most FW_MAX_LAUNCH_STEPS counted steps
    (the kernels' per-launch 32-bit step counters); FLIPWALK_LAUNCH_STEPS=97 forces many
    launches per call.  Trajectories and totals equal one oracle run."""
    monkeypatch.setenv("FLIPWALK_LAUNCH_STEPS", "97")
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    _run_vs_oracle(case, 11, [1000, 333])


@pytest.mark.parametrize("name,lb,cap", [("delaunay3k_k18", "5", None), ("delaunay3k_k18", "5", "2"),
                                         ("delaunay3k_k18", "8", None), ("tract_k4", "5", None),
                                         ("frank_a2_k2", "5", "2")])
def test_chain_kernel_5bit_labels(gpu_lib, name, lb, cap, monkeypatch):
    """General graphs on padded rows: 5-bit labels (the default when k + maxdeg needs more
    than 4 bits, C4's k = 18) with the list search's visit marks in HBM; FLIPWALK_CSR_LB=5
    forces them for small k, =8 keeps the in-place 8-bit marks; cap=2 spills the list."""
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    monkeypatch.setenv("FLIPWALK_CSR_LB", lb)
    if cap:
        monkeypatch.setenv("FLIPWALK_LIST_CAP", cap)
    case = {c.name: c for c in CASES}.get(name)
    if case is None:
        pytest.skip(f"{name}: fixture data absent")
    st = _run_vs_oracle(case, 23, [300, 200])
    assert st["bfs_runs"].sum() > 0


@pytest.mark.parametrize("name", ["grid20_k4_mu", "grid16x24_k8", "grid30x18_k2_bi"])
@pytest.mark.parametrize("search", ["bitboard", "list"])
def test_chain_kernel_3bit_labels(gpu_lib, name, search, monkeypatch):
    """The one-chain-per-wave kernel with 3-bit labels (FLIPWALK_CSR_LB=3; the default on
    large grids with k <= 8): labels straddle bytes, and the list search (race_search_b3)
    keeps its visit marks in the labels as borrowed class codes, with no HBM mark array
    (list: forced for every exact search, with a 2-entry LDS list so the visit list spills
    too)."""
    monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    monkeypatch.setenv("FLIPWALK_CSR_LB", "3")
    if search == "list":
        monkeypatch.setenv("FLIPWALK_NO_BITBOARD", "1")
        monkeypatch.setenv("FLIPWALK_LIST_CAP", "2")
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 29, [400, 300])
    assert st["bfs_runs"].sum() > 0


@pytest.mark.parametrize("name,path,slices,cap", [
    ("grid20_k4_mu", "auto", None, "1"), ("sec11_a2_k2", "auto", None, "1"),
    ("grid16x24_k8", "auto", None, "1"), ("grid20_k4_mu", "wave64", None, "1"),
    ("grid20_k4_mu", "auto", "1", "1"), ("grid20_k4_mu", "auto", "3", "1"),
    ("grid16x24_k8", "auto", "7", "1"), ("sec11_a2_k2", "auto", "4", "1"),
    ("grid20_k4_mu", "wave64", "3", "1"), ("tract_k4", "auto", "5", "1"),
    # several waves: a slice waits on its unit's previous slice held by another wave
    ("grid20_k4_mu", "auto", "3", "2"), ("sec11_a2_k2", "auto", "4", "3"),
    ("tract_k4", "auto", "6", "5")])
def test_many_units_per_wave(gpu_lib, name, path, slices, cap, monkeypatch):
    """FLIPWALK_GRID_CAP=1 leaves one workgroup (more: a few), so every wave runs many chains (quads)
    one after another through the work counter, and the grid kernel's later launches load
    each chain's group sums from its record (the derived-state cache) instead of deriving
    them.  With more work units than waves both kernels also cut each unit's steps (a quad
    of the grid kernel, a chain of the chain kernel) into slices handed out slice-major
    (the host's pick, or FLIPWALK_SLICES), every slice waiting for its unit's previous one;
    trajectories and totals equal one oracle run."""
    monkeypatch.setenv("FLIPWALK_GRID_CAP", cap)
    if slices:
        monkeypatch.setenv("FLIPWALK_SLICES", slices)
    else:
        monkeypatch.delenv("FLIPWALK_SLICES", raising=False)
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    _run_vs_oracle(case, 37, [600, 250, 150])


@pytest.mark.parametrize("name,path", [("grid20_k4_mu", "auto"), ("grid20_k4_mu", "wave64"),
                                       ("sec11_a2_k2", "auto"), ("tract_k4", "auto")])
def test_checkpoint_resume_bit_exact(gpu_lib, name, path, monkeypatch, tmp_path):
    """SURVEY.md §5 checkpoint / resume: plans + stats (with the Philox attempt counter) +
    histograms saved to an .npz (no pickle) after 300 steps and loaded into a NEW handle;
    400 more steps there equal 400 more steps of the uninterrupted handle, bit for bit."""
    from flipcomplexityempirical_amd import shape
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    g = case.graph
    dg = DeviceGraph(g)
    ch = Chains(dg, 12, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=71, chain_id0=9)
    ring = name.startswith("sec11")
    if ring:
        ch.enable_ring(*shape.ring_edges(g, shape.sec11_on_ring(39)))
    ch.run(300)
    path_ck = str(tmp_path / "ck.npz")
    ch.save_checkpoint(path_ck)
    ch.run(400)
    ch2 = Chains.from_checkpoint(dg, path_ck, case.k, proposal=case.mode, pop_bounds=case.bounds)
    ch2.run(400)
    assert np.array_equal(ch.labels(), ch2.labels())
    assert ch.stats().tobytes() == ch2.stats().tobytes()
    assert np.array_equal(ch.pops(), ch2.pops())
    assert np.array_equal(ch.hist_cut(), ch2.hist_cut())
    assert np.array_equal(ch.hist_b(), ch2.hist_b())
    if ring:
        assert np.array_equal(ch.hist_ring(), ch2.hist_ring())
    # the resumed run is also the oracle's uninterrupted 700-step run
    _, ost = oracle_chains(case, 71, range(9, 21), [700])[:2]
    assert_stats_equal(ch2.stats(), ost)
    # the checkpoint carries the population bounds: resuming without them runs the same
    # chain, and a handle with other bounds refuses it
    ch3 = Chains.from_checkpoint(dg, path_ck, case.k, proposal=case.mode, percent=0.5)
    assert (ch3.pop_lo, ch3.pop_hi) == tuple(case.bounds)
    ch3.run(400)
    assert ch3.stats().tobytes() == ch2.stats().tobytes()
    ck = dict(np.load(path_ck, allow_pickle=False))
    ck["stats"] = ck["stats"].view(ch.stats().dtype)
    ch4 = Chains(dg, 12, case.k, case.init, proposal=case.mode,
                 pop_bounds=(case.bounds[0] - 1, case.bounds[1]), base=case.base, seed=71,
                 chain_id0=9)
    with pytest.raises(ValueError, match="population bounds"):
        ch4.restore(ck)
    # sampled waits on, but a checkpoint without them: refused instead of silently
    # restarting the sums
    ch5 = Chains(dg, 12, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                 base=case.base, seed=71, chain_id0=9)
    ch5.enable_sampled_waits()
    with pytest.raises(ValueError, match="sampled waits"):
        ch5.restore(ck)


@pytest.mark.parametrize("name,rule,path", [("grid10_k2_bi", "boundary", "auto"),
                                            ("grid30x18_k2_bi", "boundary", "wave64"),
                                            ("grid12_k4_pairs", "bratio", "auto")])
def test_checkpoint_carries_accept_rule(gpu_lib, name, rule, path, monkeypatch, tmp_path):
    """A checkpoint taken under uniform_accept + boundary_condition (or the |B'|/|B| rule with
    a bound schedule) resumes under the same rule in a new handle: the boundary rule's
    flagged-node counts are rebuilt from the restored plans, and the resumed chains equal the
    oracle's uninterrupted run.  A plan write under enabled spatial maps is refused."""
    from flipcomplexityempirical_amd._lib import InvalidInitialState
    from flipcomplexityempirical_amd.chain import annealing_table, schedule_rows
    from flipcomplexityempirical_amd.graph import boundary_flags
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    g = case.graph
    r = 1 if rule == "bratio" else 2
    thr = annealing_table(0.1, 5, g.maxdeg) if rule == "bratio" else case.thr
    flags = boundary_flags(g) if rule == "boundary" else None
    sched = schedule_rows(0.1, _ramp, 40, 160, g.maxdeg) if rule == "bratio" else None
    dg = DeviceGraph(g)
    ch = Chains(dg, 8, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, seed=13,
                chain_id0=2, thr=thr)
    ch.set_accept(rule, flags)
    if sched:
        ch.set_schedule(*sched)
    ch.run(350)
    path_ck = str(tmp_path / "ck.npz")
    ch.save_checkpoint(path_ck)
    ch2 = Chains.from_checkpoint(dg, path_ck, case.k, pop_bounds=case.bounds)
    ch2.run(450)
    labs, st = ch2.labels(), ch2.stats()
    lo, hi = case.bounds
    for i in range(8):
        lab, ost = case.init.copy(), O.new_stats(1)
        lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, thr, 13, 2 + i, 800,
                                     stats=ost, accept_rule=r, flags=flags, schedule=sched)
        assert np.array_equal(labs[i], lab), (name, i)
        assert_stats_equal(st[i:i + 1], ost)
    ch3 = Chains(dg, 2, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, seed=13)
    ch3.enable_maps()
    with pytest.raises(InvalidInitialState):
        ch3.restore({k2: v[:2] if k2 in ("labels", "stats") else v
                     for k2, v in ch.checkpoint().items()
                     if k2 not in ("seed", "chain_id0")} | {"seed": 13, "chain_id0": 0})


BIG_CASES = [  # (h, w, k, seed blocks or bands, proposal, base, env)
    ("big132_k8_pairs", 132, 132, 8, (2, 4), "pairs", 0.5, {"FLIPWALK_BIG_K8": "1"}),
    ("big132_k8_cut", 132, 132, 8, (2, 4), "cutedge", 1.5, {"FLIPWALK_BIG_K8": "1"}),
    ("big132_k8_norow", 132, 132, 8, (2, 4), "pairs", 0.3,
     {"FLIPWALK_BIG_K8": "1", "FLIPWALK_NO_ROWBB": "1"}),
    ("big130x135_k4", 130, 135, 4, "band", "pairs", 0.5, {}),
    ("big200_k4_cut", 200, 200, 4, (2, 2), "cutedge", 0.8, {}),
    ("big200_k2_cold", 200, 200, 2, "band", "bi", 0.2, {}),
    ("big132_k6_list", 132, 132, 6, "band", "pairs", 0.3,
     {"FLIPWALK_BIG_K8": "1", "FLIPWALK_NO_BITBOARD": "1"}),
    ("big132_k3_spill", 132, 132, 3, "band", "pairs", 0.3,
     {"FLIPWALK_NO_BITBOARD": "1", "FLIPWALK_LIST_CAP": "2"}),
    ("big256_k8", 256, 256, 8, (2, 4), "pairs", 1.0, {"FLIPWALK_BIG_K8": "1"}),
    ("big256_k4", 256, 256, 4, (2, 2), "pairs", 0.4, {}),
]


@pytest.mark.parametrize("name,h,w,k,seedspec,proposal,base,env", BIG_CASES,
                         ids=[c[0] for c in BIG_CASES])
def test_big_grid_kernel_bit_exact(gpu_lib, name, h, w, k, seedspec, proposal, base, env,
                                   monkeypatch):
    """The grid kernel's large-grid plan (more than 256 weight groups: supergroup level,
    3-bit labels for 5 <= k <= 8, 2-bit for k <= 4), 37 chains over several waves and
    workgroups, two launches, against the oracle: plans, every counter, the fp64 sum,
    histograms.  Also the list search (bitboard off) with the shared scratch, its HBM spill,
    widths that are not multiples of 4 and the 65,536-node maximum."""
    from flipcomplexityempirical_amd.chain import PROPOSALS, metropolis_table, population_bounds
    from flipcomplexityempirical_amd.graph import band_seed, block_seed, grid_graph
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    g = grid_graph(h, w)
    init = band_seed(h, w, k) if seedspec == "band" else block_seed(h, w, *seedspec)
    pct = 0.3 if seedspec == "band" else 0.05
    bounds = population_bounds(g.total_pop, k, pct)
    n_chains, seed, id0, steps = 37, 12, 100, [400, 250]
    dg = DeviceGraph(g)
    ch = Chains(dg, n_chains, k, init, proposal=proposal, pop_bounds=bounds, base=base, seed=seed,
                chain_id0=id0)
    for s in steps:
        ch.run(s)
    labs, st = ch.labels(), ch.stats()
    thr = metropolis_table(base, 4)
    hc = np.zeros(g.n_edges + 1, np.uint64)
    hb = np.zeros(g.n + 1, np.uint64)
    for i in range(n_chains):
        lab, ost = init.copy(), O.new_stats(1)
        for s in steps:
            lab, ost, _, _ = O.run_chain(g, lab, k, PROPOSALS[proposal], *bounds, thr, seed,
                                         id0 + i, s, stats=ost, hist_cut=hc, hist_b=hb)
        assert np.array_equal(labs[i], lab), (name, i)
        assert_stats_equal(st[i:i + 1], ost)
    assert np.array_equal(ch.hist_cut(), hc) and np.array_equal(ch.hist_b(), hb)
    assert st["bfs_runs"].sum() > 0


@pytest.mark.parametrize("feature", ["maps", "ring", "bratio"])
def test_big_grid_full_instantiation(gpu_lib, feature, monkeypatch):
    """The large-grid plan's FULL instantiation (spatial maps, the ring observable, the
    |B'|/|B| accept rule) against the oracle on a 150x150 k=2 grid."""
    from flipcomplexityempirical_amd import shape
    from flipcomplexityempirical_amd.chain import (annealing_table, metropolis_table,
                                                   population_bounds)
    from flipcomplexityempirical_amd.graph import grid_graph, stripe_seed
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    n = 150
    g = grid_graph(n, n)
    init = stripe_seed(n, n)
    bounds = population_bounds(g.total_pop, 2, 0.1)
    thr = annealing_table(0.9, 1, 4) if feature == "bratio" else metropolis_table(0.7, 4)
    dg = DeviceGraph(g)
    ch = Chains(dg, 6, 2, init, proposal="bi", pop_bounds=bounds, seed=3, chain_id0=0, thr=thr)
    ru, rw = shape.ring_edges(g, shape.grid_on_ring(n, n))
    if feature == "maps":
        ch.enable_maps([-1, 1])
    elif feature == "ring":
        ch.enable_ring(ru, rw)
    else:
        ch.set_accept("bratio")
    for s in (300, 200):
        ch.run(s)
    labs, st = ch.labels(), ch.stats()
    ring = O.Ring(ru, rw)
    for i in range(6):
        lab, ost = init.copy(), O.new_stats(1)
        maps = O.Maps(g, init, np.array([-1, 1], np.int64)) if feature == "maps" else None
        for s in (300, 200):
            lab, ost, _, _ = O.run_chain(g, lab, 2, 0, *bounds, thr, 3, i, s, stats=ost,
                                         maps=maps, ring=ring if feature == "ring" else None,
                                         accept_rule=1 if feature == "bratio" else 0)
        assert np.array_equal(labs[i], lab), i
        assert_stats_equal(st[i:i + 1], ost)
        if feature == "maps":
            assert np.array_equal(ch.read_map("cut_times", (i, i + 1))[0], maps.cut_times)
            assert np.array_equal(ch.read_map("num_flips", (i, i + 1))[0], maps.num_flips)
    if feature == "ring":
        assert np.array_equal(ch.hist_ring(), ring.hist)


WAIT_CASES = [("grid10_k2_bi", "auto"), ("grid12_k4_pairs", "auto"), ("grid20_k4_mu", "wave64"),
              ("grid16x24_k8", "auto"), ("sec11_a2_k2", "auto"), ("tract_k4", "auto"),
              ("frank_a2_k2", "auto"), ("grid12_k4_cut", "wave64")]


@pytest.mark.parametrize("name,path", WAIT_CASES, ids=[f"{p}-{n}" for n, p in WAIT_CASES])
def test_sampled_waits_bit_exact(gpu_lib, name, path, monkeypatch, tmp_path):
    """Sampled geom_wait (grid_chain_sec11.py:147-148: one geometric draw per state object,
    re-used on re-yield, summed over yields): the kernels' per-chain {sum, current draw}
    equal the oracle's bit for bit across launches and across a checkpoint / resume (the
    shared fw_log1p / orc_log1p operation sequence), on both kernels."""
    from flipcomplexityempirical_amd.chain import wait_prob_table
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = {c.name: c for c in CASES}[name]
    g = case.graph
    n_chains, seed, id0, steps_list = 9, 31, 6, [500, 300]
    dg = DeviceGraph(g)
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=seed, chain_id0=id0)
    ch.enable_sampled_waits()
    ch.run(steps_list[0])
    path_ck = str(tmp_path / "ck.npz")
    ch.save_checkpoint(path_ck)
    ch.run(steps_list[1])
    got, st = ch.waits(), ch.stats()
    ch2 = Chains.from_checkpoint(dg, path_ck, case.k, pop_bounds=case.bounds)
    ch2.run(steps_list[1])
    assert got.tobytes() == ch2.waits().tobytes()
    pt = wait_prob_table(g.n, case.k)
    lo, hi = case.bounds
    for i in range(n_chains):
        lab, ost, w = case.init.copy(), O.new_stats(1), O.Waits(pt)
        for s in steps_list:
            lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, seed, id0 + i,
                                         s, stats=ost, waits=w)
        assert np.array([w.sum, w.cur]).tobytes() == got[i].tobytes(), (name, i, w.sum, got[i])
        assert_stats_equal(st[i:i + 1], ost)
    assert (got[:, 0] > 0).all()


def test_sampled_waits_big_grids(gpu_lib, monkeypatch):
    """Sampled waits on the large-grid plans: the grid kernel's (200x200, k=4) and the
    one-chain-per-wave kernel's (200x200, k=8, C5's), where p = |B|/(N^8 - 1) ~ 1e-33 (the
    reference's int64 draw overflows there; the fp64 inversion does not)."""
    from flipcomplexityempirical_amd.chain import (metropolis_table, population_bounds,
                                                   wait_prob_table)
    from flipcomplexityempirical_amd.graph import block_seed, grid_graph
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    g = grid_graph(200, 200)
    for k, bw in ((4, 2), (8, 4)):
        init = block_seed(200, 200, 2, bw)
        bounds = population_bounds(g.total_pop, k, 0.05)
        dg = DeviceGraph(g)
        ch = Chains(dg, 5, k, init, proposal="pairs", pop_bounds=bounds, base=0.5, seed=4)
        ch.enable_sampled_waits()
        ch.run(400)
        got = ch.waits()
        pt = wait_prob_table(g.n, k)
        for i in range(5):
            w = O.Waits(pt)
            O.run_chain(g, init, k, 1, *bounds, metropolis_table(0.5, 4), 4, i, 400, waits=w)
            assert np.array([w.sum, w.cur]).tobytes() == got[i].tobytes(), (k, i)
        assert np.isfinite(got).all() and (got[:, 0] > 0).all()


SPEC_GRIDS = ["grid10_k2_bi", "grid12_k4_pairs", "grid12_k4_cut", "grid20_k4_mu", "grid16x24_k8",
              "grid7x9_k3_cut", "grid11x13_k4", "grid30x18_k2_bi"]
SPEC_ENVS = {"plain": {}, "units": {"FLIPWALK_GRID_CAP": "1", "FLIPWALK_SLICES": "3"},
             "fold": {"FLIPWALK_FOLD_AT": "64"}, "list": {"FLIPWALK_NO_BITBOARD": "1"},
             "split": {"FLIPWALK_LAUNCH_STEPS": "97"}}
SPEC_CASES = ([(n, r, "plain") for n in SPEC_GRIDS for r in ("2", "4")] +
              [(n, r, e) for n in ("grid20_k4_mu", "grid16x24_k8") for r in ("2", "4")
               for e in ("units", "fold", "list", "split")])


@pytest.mark.parametrize("name,rows,env", SPEC_CASES, ids=[f"R{r}-{e}-{n}" for n, r, e in SPEC_CASES])
def test_speculative_attempts_bit_exact(gpu_lib, name, rows, env, monkeypatch):
    """The grid kernel with R rows per chain (FLIPWALK_SPEC=R: speculative attempts t .. t+R-1
    on one state, consumed up to the first state change): plans, every counter, the fp64 sum
    and the histograms equal the oracle's sequential chain, also with many work units per
    wave and slices, early counter folds, list searches under the lock and split launches."""
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    monkeypatch.setenv("FLIPWALK_SPEC", rows)
    for kk, vv in SPEC_ENVS[env].items():
        monkeypatch.setenv(kk, vv)
    case = {c.name: c for c in CASES}[name]
    st = _run_vs_oracle(case, 37, [600, 250, 150])
    assert (st["accepts"] > 0).all()


@pytest.mark.parametrize("rows", ["2", "4"])
def test_speculative_plan_runs_full_features(gpu_lib, rows, monkeypatch, tmp_path):
    """A handle planned with R rows per chain that later switches on FULL features (the
    |B'|/|B| rule, the ring observable, sampled waits) runs the R = 1 FULL kernel in the same
    LDS slots; a stuck chain stops at exactly max_retries attempts under speculation."""
    from flipcomplexityempirical_amd import shape
    from flipcomplexityempirical_amd.chain import annealing_table, wait_prob_table
    from flipcomplexityempirical_amd.graph import grid_graph, stripe_seed
    monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    monkeypatch.setenv("FLIPWALK_SPEC", rows)
    case = {c.name: c for c in CASES}["grid20_k4_mu"]
    g = case.graph
    thr = annealing_table(0.9, 1, g.maxdeg)
    dg = DeviceGraph(g)
    ch = Chains(dg, 21, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds, seed=3,
                thr=thr)
    ch.run(300)  # lean, R rows per chain
    ru, rw = shape.ring_edges(g, shape.grid_on_ring(20, 20))
    ch.set_accept("bratio")
    ch.enable_ring(ru, rw)
    ch.run(200)  # FULL, one row per chain
    ring = O.Ring(ru, rw)
    labs, st = ch.labels(), ch.stats()
    lo, hi = case.bounds
    for i in range(21):
        lab, ost = case.init.copy(), O.new_stats(1)
        lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, thr, 3, i, 300, stats=ost)
        lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, thr, 3, i, 200, stats=ost,
                                     accept_rule=1, ring=ring)
        assert np.array_equal(labs[i], lab), i
        assert_stats_equal(st[i:i + 1], ost)
    assert np.array_equal(ch.hist_ring(), ring.hist)
    g6 = grid_graph(6, 6)
    lab6 = stripe_seed(6, 6)
    ch6 = Chains(DeviceGraph(g6), 4, 2, lab6, proposal="bi", pop_bounds=(18, 18), base=1.0)
    ch6.run(10, max_retries=50)
    st6 = ch6.stats()
    assert st6["stuck"].all() and (st6["steps"] == 0).all() and (st6["attempts"] == 50).all()
