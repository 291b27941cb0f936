"""District-shape observable: boundary_slope's ring cut edges and the
driver's slope / angle (grid_chain_sec11.py:55-78,371-394; Frankenstein_chain.py:57-80).

CPU: the oracle's per-yield ring-pair histogram equals a literal replay of the reference's
updater (markov.boundary_slope on the yielded partitions) over the oracle's trajectory, and
the pair -> (slope, angle) conversion equals the reference's expressions on
``part["slope"]``.  GPU (marked): the kernels' ring histogram equals the oracle's bit for
bit, on both chain kernels.
"""
import numpy as np
import pytest

from cases import cases
from flipcomplexityempirical_amd import markov as gc
from flipcomplexityempirical_amd import shape
from flipcomplexityempirical_amd.graph import (frankenstein_graph, frankenstein_seed, grid_graph,
                                               sec11_graph, sec11_seed)
from oracle import oracle as O

CASES = {c.name: c for c in cases(include_kansas=False)}


def _ring_for(case):
    g = case.graph
    if case.name.startswith("sec11"):
        return shape.ring_edges(g, shape.sec11_on_ring(39))
    if case.name.startswith("frank"):
        return shape.ring_edges(g, shape.frank_on_ring(50))
    h = g.n // g.grid_w
    return shape.ring_edges(g, shape.grid_on_ring(h, g.grid_w))


def test_sec11_ring_is_boundary_slopes_edge_set():
    g = sec11_graph()
    u, w = shape.ring_edges(g, shape.sec11_on_ring(39))
    # the outer ring of the 40x40 grid minus its 4 corners, closed by the 4 diagonals
    assert len(u) == 4 * 37 + 4
    # every cut edge boundary_slope returns is a ring edge and vice versa
    lab = sec11_seed(g, 2)
    part = gc.Partition(g, assignment={k: int(lab[i]) for i, k in enumerate(g.nodes)},
                        updaters={"cut_edges": gc.cut_edges})
    ring = {(g.nodes[a], g.nodes[b]) for a, b in zip(u, w)}
    got = {tuple(sorted(e)) for e in gc.boundary_slope(part)}
    want = {tuple(sorted(e)) for e in part["cut_edges"] if tuple(sorted(e)) in ring}
    assert got == want and len(got) == 2


def test_frankengraph_ring():
    g = frankenstein_graph()
    u, w = shape.ring_edges(g, shape.frank_on_ring(50))
    on = shape.frank_on_ring(50)
    assert len(u) > 150 and all(on(g.nodes[a], g.nodes[b]) for a, b in zip(u, w))


@pytest.mark.parametrize("name", ["sec11_a2_k2", "sec11_a0_k2_mu", "grid10_k2_bi",
                                  "grid12_k4_pairs", "frank_a2_k2"])
def test_oracle_ring_follows_the_reference_updater(name):
    """Oracle ring histogram == replay of boundary_slope over every yielded state, taking
    the first two cut ring edges in ring order; and the (slope, angle) of each pair ==
    the reference's expressions on part["slope"] when it holds exactly two edges."""
    case = CASES[name]
    g = case.graph
    lo, hi = case.bounds
    ru, rw = _ring_for(case)
    R = len(ru)
    S = 300
    ring = O.Ring(ru, rw)
    O.run_chain(g, case.init, case.k, case.mode, lo, hi, case.thr, 13, 2, S, ring=ring)
    order = {(int(a), int(b)): r for r, (a, b) in enumerate(zip(ru, rw))}
    idx = g.index()
    on = (shape.sec11_on_ring(39) if name.startswith("sec11") else
          shape.frank_on_ring(50) if name.startswith("frank") else
          shape.grid_on_ring(g.n // max(g.grid_w, 1), g.grid_w))
    want = np.zeros(R * R + 1, np.uint64)
    lab, st = case.init.copy(), O.new_stats(1)
    n_two = 0
    for t in range(S + 1):
        if t > 0:
            lab, st, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, 13, 2, 1,
                                        stats=st)
        part = gc.Partition(g, assignment={k: int(lab[i]) for i, k in enumerate(g.nodes)},
                            updaters={"cut_edges": gc.cut_edges})
        temp = [e for e in part["cut_edges"] if on(e[0], e[1])]  # boundary_slope's edges
        rs = sorted(order[tuple(sorted((idx[a], idx[b])))] for a, b in temp)
        want[rs[0] * R + rs[1] if len(rs) >= 2 else R * R] += 1
        if len(temp) == 2:
            n_two += 1
            s_ref, a_ref = gc.slope_and_angle(temp)
            s_got, a_got = shape.slope_and_angle_of(g, ru, rw, rs[0], rs[1])
            assert s_ref == s_got and a_ref == a_got
    assert np.array_equal(ring.hist, want)
    assert n_two > S // 2 or case.k > 2  # k = 2 plans cross the ring twice
    slopes, angles, counts, short = shape.shape_samples(ring.hist, g, ru, rw)
    assert counts.sum() + short == S + 1 and np.all((angles >= 0) & (angles <= np.pi))


@pytest.mark.gpu
@pytest.mark.parametrize("name,path", [("sec11_a2_k2", "auto"), ("sec11_a0_k2_mu", "auto"),
                                       ("frank_a2_k2", "auto"), ("grid10_k2_bi", "auto"),
                                       ("grid12_k4_pairs", "auto"), ("grid12_k4_pairs", "wave64"),
                                       ("grid30x18_k2_bi", "auto")])
def test_gpu_ring_histogram_bit_exact(gpu_lib, name, path, monkeypatch):
    """fw_chains_enable_ring on both kernels (grid kernel: its FULL instantiation) against
    the oracle: ring histograms, current pairs, and unchanged trajectories, across two
    launches."""
    from flipcomplexityempirical_amd.chain import Chains, DeviceGraph
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = CASES[name]
    g = case.graph
    lo, hi = case.bounds
    ru, rw = _ring_for(case)
    n_chains, seed, id0, steps = 9, 31, 4, [400, 350]
    dg = DeviceGraph(g)
    ch = Chains(dg, n_chains, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=seed, chain_id0=id0)
    ch.enable_ring(ru, rw)
    for s in steps:
        ch.run(s)
    ring = O.Ring(ru, rw)
    labs = ch.labels()
    pairs = ch.ring_pairs()
    for i in range(n_chains):
        lab, st = case.init.copy(), O.new_stats(1)
        for s in steps:
            lab, st, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, seed, id0 + i,
                                        s, stats=st, ring=ring)
        assert np.array_equal(labs[i], lab), i
        cut = [r for r in range(len(ru)) if lab[ru[r]] != lab[rw[r]]]
        assert tuple(pairs[i]) == (tuple(cut[:2]) if len(cut) >= 2 else (-1, -1))
    assert np.array_equal(ch.hist_ring(), ring.hist)
    assert ch.hist_ring().sum() == n_chains * (sum(steps) + 1)
