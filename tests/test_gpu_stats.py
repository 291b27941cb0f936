"""GPU chain law at full size: SURVEY.md §8(d) acceptance criteria and size-independent
properties of the BASELINE configurations.

* Distribution: the across-chain marginals of |cut edges| and |B| of GPU chains (C2 shape:
  40x40, k=4, 4,096 chains) against >= 256 oracle chains on DISJOINT Philox streams
  (independent samples), at matched step counts S in {10^3, 10^4}: two-sample KS at
  alpha = 0.01 and means within 3 combined standard errors, plus the per-chain time
  averages (sum over yields / yields).  The same at the C3 shape (100x100, 65,536 GPU
  chains vs 256 oracle chains) at S in {10^3, 10^4, 10^5}; C2 also at 10^5.
* C3 (100x100, k=4, 65,536 chains, the bench workload): counters, histogram moments and
  recomputed cut/boundary/population/contiguity of a subsample of final plans, and a
  spread of chain ids re-run on the oracle bit for bit.
* Sharding: splitting the chain-id range over several handles (as ranks do) gives
  bit-identical merged histograms and stats.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
from scipy import stats as sps

from flipcomplexityempirical_amd.chain import (Chains, DeviceGraph, metropolis_table,
                                               population_bounds)
from flipcomplexityempirical_amd.graph import block_seed, grid_graph
from oracle import oracle as O

pytestmark = pytest.mark.gpu
MU = 2.63815853


def _oracle_marginals(g, init, k, mode, bounds, base, seed, ids, steps):
    thr = metropolis_table(base, g.maxdeg)
    # ctypes releases the GIL: independent oracle chains run on a thread pool
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        st = list(ex.map(lambda cid: O.run_chain(g, init, k, mode, *bounds, thr, seed, cid,
                                                 steps)[1][0], ids))
    return np.array(st)


def _compare(a, b, what):
    ks = sps.ks_2samp(a, b)
    se = np.sqrt(a.var(ddof=1) / len(a) + b.var(ddof=1) / len(b))
    assert ks.pvalue > 0.01, (what, ks)
    assert abs(a.mean() - b.mean()) < 3 * se + 1e-12, (what, a.mean(), b.mean(), se)


@pytest.mark.parametrize("steps", [1000, 10000, 100000])
@pytest.mark.parametrize("proposal,mode", [("pairs", 1), ("cutedge", 2)])
def test_c2_marginals_match_independent_oracle_chains(gpu_lib, steps, proposal, mode):
    n, k, seed = 40, 4, 5
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 2)
    bounds = population_bounds(g.total_pop, k, 0.05)
    dg = DeviceGraph(g)
    ch = Chains(dg, 4096, k, init, proposal=proposal, pop_bounds=bounds, base=MU, seed=seed)
    ch.run(steps)
    gst = ch.stats()
    ost = _oracle_marginals(g, init, k, mode, bounds, MU, seed, range(1 << 20, (1 << 20) + 256),
                            steps)
    for f in ("cut", "bnodes"):
        _compare(gst[f].astype(float), ost[f].astype(float), f)
    for f in ("sum_cut", "sum_bnodes"):
        _compare(gst[f] / gst["yields"], ost[f] / ost["yields"], f)
    # the yield histograms are the union of the per-chain yields
    assert ch.hist_cut().sum() == gst["yields"].sum() == 4096 * (steps + 1)


@pytest.mark.parametrize("steps", [1000, 10000, 100000])
def test_c3_marginals_match_independent_oracle_chains(gpu_lib, steps):
    """SURVEY.md §8(d) at the bench shape: 65,536 GPU chains vs 256 oracle chains."""
    n, k, seed = 100, 4, 7
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 2)
    bounds = population_bounds(g.total_pop, k, 0.05)
    ch = Chains(DeviceGraph(g), 65536, k, init, proposal="pairs", pop_bounds=bounds, base=MU,
                seed=seed)
    ch.run(steps)
    gst = ch.stats()
    assert not gst["stuck"].any()
    ost = _oracle_marginals(g, init, k, 1, bounds, MU, seed, range(1 << 20, (1 << 20) + 256),
                            steps)
    for f in ("cut", "bnodes"):
        _compare(gst[f].astype(float), ost[f].astype(float), f)
    for f in ("sum_cut", "sum_bnodes"):
        _compare(gst[f] / gst["yields"], ost[f] / ost["yields"], f)
    assert ch.hist_cut().sum() == gst["yields"].sum() == 65536 * (steps + 1)


def test_c3_full_size_properties(gpu_lib):
    n, k, C, S, seed = 100, 4, 65536, 300, 0
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 2)
    bounds = population_bounds(g.total_pop, k, 0.05)
    dg = DeviceGraph(g)
    ch = Chains(dg, C, k, init, proposal="pairs", pop_bounds=bounds, base=MU, seed=seed)
    ch.run(S)
    ch.run(S)
    st, hc, hb, pops = ch.stats(), ch.hist_cut(), ch.hist_b(), ch.pops()
    assert (st["steps"] == 2 * S).all() and (st["yields"] == 2 * S + 1).all()
    assert not st["stuck"].any()
    assert (st["attempts"] == st["steps"] + st["pop_fail"] + st["contig_fail"]).all()
    assert hc.sum() == hb.sum() == st["yields"].sum()
    assert int((hc * np.arange(len(hc), dtype=np.uint64)).sum()) == int(st["sum_cut"].sum())
    assert int((hb * np.arange(len(hb), dtype=np.uint64)).sum()) == int(st["sum_bnodes"].sum())
    assert (pops.sum(1) == n * n).all() and (pops >= bounds[0]).all() and (pops <= bounds[1]).all()
    labs = ch.labels()
    e = g.edges()
    rng = np.random.default_rng(1)
    sample = np.unique(np.concatenate([rng.integers(0, C, 400), [0, 1, C - 2, C - 1]]))
    for i in sample:
        lab = labs[i]
        m = lab[e[:, 0]] != lab[e[:, 1]]
        assert int(m.sum()) == st["cut"][i]
        assert len(np.unique(e[m].ravel())) == st["bnodes"][i]
        assert np.array_equal(np.bincount(lab, minlength=k), pops[i])
        assert O.plan_valid(g, lab, k, *bounds)
    thr = metropolis_table(MU, g.maxdeg)
    for i in sample[::25]:  # full-size bit-exact re-runs on the oracle
        olab = init.copy()
        ost = O.new_stats(1)
        for _ in range(2):
            olab, ost, opop, _ = O.run_chain(g, olab, k, 1, *bounds, thr, seed, int(i), S,
                                             stats=ost)
        assert np.array_equal(olab, labs[i])
        for f in ("attempts", "steps", "accepts", "bfs_runs", "bfs_nodes", "sum_cut",
                  "sum_bnodes", "cut", "bnodes"):
            assert ost[f][0] == st[f][i], (i, f)
        assert ost["sum_invb"][0] == st["sum_invb"][i]


def test_sharded_handles_merge_bit_identically(gpu_lib):
    """Chain ids split over 1, 2, 4 and 8 handles (as over ranks) merge to the same bits."""
    n, k, S, seed = 40, 4, 700, 11
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 2)
    bounds = population_bounds(g.total_pop, k, 0.05)
    dg = DeviceGraph(g)
    keys = []
    for splits in ([4096], [2048, 2048], [1000, 1000, 1000, 1096], [512] * 8):
        hc = np.zeros(g.n_edges + 1, np.uint64)
        hb = np.zeros(g.n + 1, np.uint64)
        sts = []
        lo = 0
        for c in splits:  # one handle per "rank", chain ids [lo, lo + c)
            ch = Chains(dg, c, k, init, proposal="pairs", pop_bounds=bounds, base=MU, seed=seed,
                        chain_id0=lo)
            ch.run(S)
            hc += ch.hist_cut()
            hb += ch.hist_b()
            sts.append(ch.stats())
            ch.close()
            lo += c
        keys.append((hc.tobytes(), hb.tobytes(), np.concatenate(sts).tobytes()))
    assert all(kk == keys[0] for kk in keys[1:])


def test_c2_time_averaged_histograms_batch_means(gpu_lib):
    """time-averaged histograms of |cut edges| and |B| (all yields of all
    chains) from the GPU against independent oracle chains, bin by bin with batch-means
    error bars (oracle: 16 batches of 16 chains; GPU: 8 handles of 512 chains on disjoint
    id ranges), plus a chi-square over the populated bins."""
    n, k, seed, steps = 40, 4, 11, 2000
    g = grid_graph(n, n)
    init = block_seed(n, n, 2, 2)
    bounds = population_bounds(g.total_pop, k, 0.05)
    thr = metropolis_table(MU, g.maxdeg)
    E = g.n_edges
    dg = DeviceGraph(g)
    gh = {"cut": [], "b": []}
    for b in range(8):
        ch = Chains(dg, 512, k, init, proposal="pairs", pop_bounds=bounds, base=MU, seed=seed,
                    chain_id0=b * 512)
        ch.run(steps)
        gh["cut"].append(ch.hist_cut()[:E + 1] / ch.hist_cut().sum())
        gh["b"].append(ch.hist_b()[:g.n + 1] / ch.hist_b().sum())
        ch.close()
    oh = {"cut": [], "b": []}
    for b in range(16):
        hc = np.zeros(E + 1 + 64, np.uint64)
        hb = np.zeros(g.n + 1 + 64, np.uint64)
        for cid in range((1 << 20) + 16 * b, (1 << 20) + 16 * b + 16):
            O.run_chain(g, init, k, 1, *bounds, thr, seed, cid, steps, hist_cut=hc, hist_b=hb)
        oh["cut"].append(hc[:E + 1] / hc.sum())
        oh["b"].append(hb[:g.n + 1] / hb.sum())
    for f in ("cut", "b"):
        G, Q = np.array(gh[f]), np.array(oh[f])
        pg, po = G.mean(0), Q.mean(0)
        se = np.sqrt(G.var(0, ddof=1) / len(G) + Q.var(0, ddof=1) / len(Q))
        live = (po > 0.002) & (se > 0)
        z = (pg[live] - po[live]) / se[live]
        assert live.sum() >= 20, f
        assert np.abs(z).max() < 5.0, (f, np.abs(z).max())
        chi2 = float((z ** 2).sum())
        assert sps.chi2.sf(chi2, int(live.sum())) > 1e-3, (f, chi2, int(live.sum()))


def _full_size_properties(g, k, bounds, init, labs, st, hc, hb, pops, sample, steps_total):
    """Size-independent checks of a batched run: counters, histogram moments, and the
    recomputed cut / boundary / populations / contiguity of a sample of final plans."""
    assert (st["steps"] == steps_total).all() and (st["yields"] == steps_total + 1).all()
    assert not st["stuck"].any()
    assert (st["attempts"] == st["steps"] + st["pop_fail"] + st["contig_fail"]).all()
    assert hc.sum() == hb.sum() == st["yields"].sum()
    assert int((hc * np.arange(len(hc), dtype=np.uint64)).sum()) == int(st["sum_cut"].sum())
    assert int((hb * np.arange(len(hb), dtype=np.uint64)).sum()) == int(st["sum_bnodes"].sum())
    total = int(g.total_pop)
    assert (pops.sum(1) == total).all() and (pops >= bounds[0]).all() and (pops <= bounds[1]).all()
    e = g.edges()
    w = g.pop_array()
    for i in sample:
        lab = labs[i]
        m = lab[e[:, 0]] != lab[e[:, 1]]
        assert int(m.sum()) == st["cut"][i]
        assert len(np.unique(e[m].ravel())) == st["bnodes"][i]
        assert np.array_equal(np.bincount(lab, weights=w, minlength=k).astype(np.int64), pops[i])
        assert O.plan_valid(g, lab, k, *bounds)


def _oracle_rerun(g, init, k, mode, bounds, thr, seed, cid, steps_list):
    olab, ost = init.copy(), O.new_stats(1)
    for s in steps_list:
        olab, ost, _, _ = O.run_chain(g, olab, k, mode, *bounds, thr, seed, int(cid), s, stats=ost)
    return olab, ost


def test_c4_full_size_properties(gpu_lib):
    """BASELINE configs[3] at its stated size: the 9,000-node Delaunay dual graph, k=18 tree
    seed, 16,384 chains, with the production LDS plan the host picks for it (5-bit labels,
    list-search marks in HBM, 20 chains per CU; no FLIPWALK_* overrides)."""
    from flipcomplexityempirical_amd.workloads import workload
    for var in ("FLIPWALK_LIST_CAP", "FLIPWALK_NO_BITBOARD", "FLIPWALK_NO_GRID16"):
        assert var not in os.environ
    w = workload("c4")
    g, init, k = w.graph, w.init, w.k
    C, S, seed = w.chains, 250, 3
    bounds = population_bounds(g.total_pop, k, w.percent)
    dg = DeviceGraph(g)
    assert dg.n == 9000 and dg.grid_w == 0
    ch = Chains(dg, C, k, init, proposal=w.proposal, pop_bounds=bounds, base=w.base, seed=seed)
    ch.run(S)
    ch.run(S)
    st, hc, hb, pops, labs = ch.stats(), ch.hist_cut(), ch.hist_b(), ch.pops(), ch.labels()
    rng = np.random.default_rng(4)
    sample = np.unique(np.concatenate([rng.integers(0, C, 200), [0, 1, C - 2, C - 1]]))
    _full_size_properties(g, k, bounds, init, labs, st, hc, hb, pops, sample, 2 * S)
    assert st["bfs_runs"].sum() > 0 and st["contig_fail"].sum() > 0
    thr = metropolis_table(w.base, g.maxdeg)
    for i in sample[::12]:  # full-size bit-exact re-runs on the oracle
        olab, ost = _oracle_rerun(g, init, k, 1, bounds, thr, seed, i, [S, S])
        assert np.array_equal(olab, labs[i]), i
        for f in ("attempts", "steps", "accepts", "contig_fail", "bfs_runs", "bfs_nodes",
                  "bfs_deg", "sum_cut", "sum_bnodes", "cut", "bnodes", "npairs"):
            assert ost[f][0] == st[f][i], (i, f)
        assert ost["sum_invb"][0] == st["sum_invb"][i]


def test_c5_ladder_shard_full_size_properties(gpu_lib):
    """BASELINE configs[4], one GPU's shard at 8 GPUs: global chain ids [0, 8192) of the
    200x200 k=8 workload = 8 whole 1,024-chain base groups of the 64-base ladder (per-chain
    Metropolis tables), run in one handle."""
    from flipcomplexityempirical_amd.distributed import shard_range
    from flipcomplexityempirical_amd.workloads import ladder, ladder_base_index, workload
    w = workload("c5")
    g, init, k = w.graph, w.init, w.k
    lo, hi = shard_range(w.chains, 8, 0)
    assert (lo, hi) == (0, 8192)
    bases = w.bases(lo, hi)
    assert len(np.unique(bases)) == 8 and np.unique(ladder_base_index(np.arange(lo, hi))).size == 8
    C, S, seed = hi - lo, 150, 21
    bounds = population_bounds(g.total_pop, k, w.percent)
    dg = DeviceGraph(g)
    ch = Chains(dg, C, k, init, proposal=w.proposal, pop_bounds=bounds, base=bases, seed=seed,
                chain_id0=lo)
    ch.run(S)
    ch.run(S)
    st, hc, hb, pops, labs = ch.stats(), ch.hist_cut(), ch.hist_b(), ch.pops(), ch.labels()
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([rng.integers(0, C, 120), [0, 1023, 1024, C - 1]]))
    _full_size_properties(g, k, bounds, init, labs, st, hc, hb, pops, sample, 2 * S)
    for i in sample[::10]:
        thr = metropolis_table(float(bases[i]), g.maxdeg)
        olab, ost = _oracle_rerun(g, init, k, 1, bounds, thr, seed, lo + i, [S, S])
        assert np.array_equal(olab, labs[i]), i
        for f in ("attempts", "steps", "accepts", "contig_fail", "bfs_runs", "bfs_nodes",
                  "sum_cut", "sum_bnodes", "cut", "bnodes", "npairs"):
            assert ost[f][0] == st[f][i], (i, f)
        assert ost["sum_invb"][0] == st["sum_invb"][i]
    # low ladder bases favour long boundaries (base < 1), high ones short ones
    lad = ladder()[ladder_base_index(np.arange(lo, hi))]
    assert st["cut"][lad < 0.5].mean() > st["cut"][lad > 2.0].mean()


def test_rccl_histogram_merge_on_device(gpu_lib):
    """The one collective of the multi-GPU path, on RCCL: a 1-rank "nccl" process group
    merges histograms and per-chain stats held as device tensors (distributed.py)."""
    import socket

    import torch
    import torch.distributed as dist

    from flipcomplexityempirical_amd.distributed import gather_stats, merge_histograms
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        g = grid_graph(20, 20)
        init = block_seed(20, 20, 2, 2)
        bounds = population_bounds(g.total_pop, 4, 0.05)
        ch = Chains(DeviceGraph(g), 64, 4, init, proposal="pairs", pop_bounds=bounds, base=MU,
                    seed=1)
        ch.run(200)
        hc, hb = ch.hist_cut(), ch.hist_b()
        mhc, mhb = merge_histograms(hc, hb, dist)
        assert np.array_equal(mhc, hc) and np.array_equal(mhb, hb)
        st = ch.stats()
        mst = gather_stats(st, 64, dist, 0)
        assert mst.tobytes() == st.tobytes()
    finally:
        dist.destroy_process_group()
