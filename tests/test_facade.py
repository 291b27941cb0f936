"""GerryChain-shaped façade: host pieces on CPU, the lowered chain on the GPU."""
import numpy as np
import pytest

from cases import MU
from flipcomplexityempirical_amd import markov as gc
from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
from flipcomplexityempirical_amd.graph import sec11_graph, sec11_seed
from oracle import oracle as O


def sec11_partition(alignment=2, base=0.1):
    """The reference's set-up, grid_chain_sec11.py:186-342, through the façade."""
    g = sec11_graph()
    lab = sec11_seed(g, alignment)
    cddict = {node: (1 if lab[i] else -1) for i, node in enumerate(g.nodes)}
    updaters = {"population": gc.Tally("population"), "cut_edges": gc.cut_edges,
                "b_nodes": gc.b_nodes_bi, "base": lambda p: base, "geom": gc.geom_wait}
    return g, gc.Partition(g, assignment=cddict, updaters=updaters)


def test_partition_updaters_on_host():
    g, part = sec11_partition()
    assert part.parts == [-1, 1] and len(part) == 2
    assert part["population"] == {-1: 798, 1: 798}
    cut = part["cut_edges"]
    lab = part.labels
    e = g.edges()
    assert len(cut) == int((lab[e[:, 0]] != lab[e[:, 1]]).sum())
    assert part["b_nodes"] == {x for e_ in cut for x in e_}
    node = next(iter(part["b_nodes"]))
    child = part.flip({node: -part.assignment[node]})
    assert child.parent is part and child.flips == {node: -part.assignment[node]}
    assert child.assignment[node] == -part.assignment[node]


def test_bounds_and_validator():
    g, part = sec11_partition()
    pb = gc.within_percent_of_ideal_population(part, 0.01)
    assert pb.bounds == (0.99 * 798, 1.01 * 798) and pb(part)
    assert population_bounds(1596, 2, 0.01) == (791, 805)
    with pytest.raises(TypeError):
        gc.Validator([lambda p: 1])(part)
    assert gc.Validator([lambda p: True, lambda p: False, lambda p: 1])(part) is False


def test_unknown_plugins_are_refused():
    g, part = sec11_partition()
    pb = gc.within_percent_of_ideal_population(part, 0.05)
    with pytest.raises(NotImplementedError):
        gc.MarkovChain(lambda p: p, gc.Validator([gc.single_flip_contiguous, pb]),
                       gc.cut_accept, part, 10)
    with pytest.raises(NotImplementedError):
        gc.MarkovChain(gc.slow_reversible_propose_bi, [gc.single_flip_contiguous, pb],
                       lambda p: True, part, 10)
    with pytest.raises(NotImplementedError):
        gc.slow_reversible_propose_bi(part)


@pytest.mark.gpu
def test_reference_script_shape_runs_on_gpu(gpu_lib):
    g, part = sec11_partition(alignment=2, base=0.1)
    pb = gc.within_percent_of_ideal_population(part, 0.05)
    chain = gc.MarkovChain(gc.slow_reversible_propose_bi,
                           gc.Validator([gc.single_flip_contiguous, pb]), accept=gc.cut_accept,
                           initial_state=part, total_steps=1500, seed=5, chain_id=3, chunk=600)
    parts, child_ok = [], None
    for p in chain:
        if p.parent is not None:
            # GerryChain erases the parent of the previous state: history is not kept alive
            assert p.parent.parent is None
            if child_ok is None:  # single_flip_contiguous on a child, while its parent lives
                child_ok = gc.single_flip_contiguous(p)
        parts.append(p)
    assert len(parts) == 1500 and parts[0] is part
    assert child_ok is True
    assert sum(p.parent is not None for p in parts[:-1]) == 0
    # the reference re-yields the same object after a Metropolis rejection
    assert any(a is b for a, b in zip(parts, parts[1:]))
    lo, hi = population_bounds(g.n, 2, 0.05)
    olab, ost, _, otr = O.run_chain(g, sec11_seed(g, 2), 2, 0, lo, hi, metropolis_table(0.1, 4),
                                    5, 3, 1499, trace=True)
    assert np.array_equal(parts[-1].labels, olab)
    # the per-yield observables of grid_chain_sec11.py:367-369 agree with the oracle's sums
    assert sum(len(p["cut_edges"]) for p in parts) == int(ost["sum_cut"][0])
    assert sum(len(p["b_nodes"]) for p in parts) == int(ost["sum_bnodes"][0])


@pytest.mark.gpu
def test_run_batched_matches_oracle(gpu_lib):
    g, part = sec11_partition(alignment=0, base=MU)
    pb = gc.within_percent_of_ideal_population(part, 0.10)
    chain = gc.MarkovChain(gc.slow_reversible_propose_bi, [gc.single_flip_contiguous, pb],
                           gc.MetropolisCutAccept(MU), part, 1001, seed=9)
    res = chain.run_batched(5, chain_id0=100)
    lo, hi = population_bounds(g.n, 2, 0.10)
    for i in range(5):
        olab, _, _, _ = O.run_chain(g, sec11_seed(g, 0), 2, 0, lo, hi, metropolis_table(MU, 4), 9,
                                    100 + i, 1000)
        assert np.array_equal(res.labels[i], olab)


def test_boundary_slope_updater_on_host():
    """A15 (grid_chain_sec11.py:55-78, 371-394) through the façade's host updaters."""
    g, part = sec11_partition(alignment=0)  # rows >= 20 vs rows < 20: a horizontal cut
    part.updaters["slope"] = gc.boundary_slope
    temp = part["slope"]
    assert sorted(temp) == sorted([((19, 0), (20, 0)), ((19, 39), (20, 39))])
    slope, angle = gc.slope_and_angle(temp)
    assert slope == np.inf and np.isclose(angle, np.pi, atol=0.06)  # midpoints share row 19.5


@pytest.mark.gpu
def test_reference_driver_loop_matches_gpu_maps(gpu_lib):
    """grid_chain_sec11.py:366-419 run literally over the façade's yielded partitions
    (cut_times per edge, part_sum / last_flipped / num_flips per node, slope and angle)
    equals the GPU's spatial maps of the same chain (MarkovChain.run_batched(maps=True))."""
    g, part = sec11_partition(alignment=2, base=0.1)
    part.updaters["slope"] = gc.boundary_slope
    pb = gc.within_percent_of_ideal_population(part, 0.05)
    mk = lambda: gc.MarkovChain(gc.slow_reversible_propose_bi,  # noqa: E731
                                gc.Validator([gc.single_flip_contiguous, pb]),
                                accept=gc.cut_accept, initial_state=part, total_steps=1200,
                                seed=4, chain_id=0, chunk=500)
    idx = g.index()
    eid = {tuple(e): i for i, e in enumerate(g.edges().tolist())}
    cut_times = np.zeros(g.n_edges, np.int64)
    part_sum = np.array([part.assignment[x] for x in g.nodes], np.int64)
    last_flipped = np.zeros(g.n, np.int64)
    num_flips = np.zeros(g.n, np.int64)
    slopes, angles = [], []
    t = 0
    for p in mk():
        for a, b in p["cut_edges"]:
            i, j = idx[a], idx[b]
            cut_times[eid[(min(i, j), max(i, j))]] += 1
        temp = p["slope"]
        assert len(temp) == 2
        s_, a_ = gc.slope_and_angle(temp)
        slopes.append(s_)
        angles.append(float(a_))
        if p.flips is not None:
            f = idx[list(p.flips.keys())[0]]
            part_sum[f] -= p.assignment[g.nodes[f]] * (t - last_flipped[f])
            last_flipped[f] = t
            num_flips[f] += 1
        t += 1
    final = p
    never = last_flipped == 0
    part_sum[never] = t * np.array([final.assignment[g.nodes[x]] for x in np.flatnonzero(never)])
    res = mk().run_batched(1, chain_id0=0, maps=True)
    # A15 on the GPU: the chain's ring-pair histogram, turned into (slope, angle) with the
    # reference's expressions, is the multiset the literal loop recorded (every state here
    # crosses the ring exactly twice, so the pick of "the first two" is order-free)
    from flipcomplexityempirical_amd import shape
    ru, rw = shape.ring_edges(g, shape.sec11_on_ring(39))
    ch = mk()._make(1, 0)
    ch.enable_ring(ru, rw)
    ch.run(1199)
    s_g, a_g, c_g, short = shape.shape_samples(ch.hist_ring(), g, ru, rw)
    ch.close()
    assert short == 0 and c_g.sum() == t
    got = sorted(zip(np.repeat(s_g, c_g).tolist(), np.repeat(a_g, c_g).tolist()))
    want = sorted(zip(slopes, angles))
    assert len(got) == len(want) and all(x == y for x, y in zip(got, want))
    assert np.array_equal(res.maps["cut_times"][0], cut_times)
    assert np.array_equal(res.maps["num_flips"][0], num_flips)
    assert np.array_equal(res.maps["last_flipped"][0], last_flipped)
    assert np.array_equal(res.maps["part_sum"][0], part_sum)
    assert len(slopes) == t and np.all(np.isfinite(angles))


@pytest.mark.gpu
@pytest.mark.parametrize("accept", ["annealing", "uniform"])
def test_alternative_accepts_through_the_facade(gpu_lib, accept):
    """annealing_cut_accept_backwards / uniform_accept (grid_chain_sec11.py:81-110,159-165)
    recognised by name, lowered to FW_ACCEPT_BRATIO / FW_ACCEPT_BOUNDARY, equal to the
    oracle; uniform_accept takes the nodes of the partition's "boundary" updater."""
    from flipcomplexityempirical_amd.chain import annealing_table
    from flipcomplexityempirical_amd.graph import boundary_flags
    g, part = sec11_partition(alignment=1, base=0.1)
    bnodes = [x for x in g.nodes if 0 in x or 39 in x]  # grid_chain_sec11.py:225-233
    part.updaters["boundary"] = lambda p: bnodes
    pb = gc.within_percent_of_ideal_population(part, 0.10)
    fn = gc.annealing_cut_accept_backwards if accept == "annealing" else gc.uniform_accept
    chain = gc.MarkovChain(gc.slow_reversible_propose_bi, gc.Validator(
        [gc.single_flip_contiguous, pb]), accept=fn, initial_state=part, total_steps=801, seed=2)
    res = chain.run_batched(3, chain_id0=7)
    lo, hi = population_bounds(g.n, 2, 0.10)
    flags = boundary_flags(g)
    assert flags.sum() == len(bnodes)
    thr = annealing_table(0.1, 5, 4) if accept == "annealing" else metropolis_table(1.0, 4)
    for i in range(3):
        olab, ost, _, _ = O.run_chain(g, sec11_seed(g, 1), 2, 0, lo, hi, thr, 2, 7 + i, 800,
                                      accept_rule=1 if accept == "annealing" else 2, flags=flags)
        assert np.array_equal(res.labels[i], olab)
        assert res.stats["accepts"][i] == ost["accepts"][0]


def test_reference_beta_schedule_is_lowered():
    """AnnealingCutAccept.reference_schedule() (grid_chain_sec11.py:88-93) lowers to
    FW_ACCEPT_BRATIO with step_num-indexed rows (host side only; the kernels are checked
    in tests/test_gpu_parity.py::test_step_schedule_bit_exact)."""
    from flipcomplexityempirical_amd.chain import annealing_table
    g, part = sec11_partition()
    pb = gc.within_percent_of_ideal_population(part, 0.05)
    chain = gc.MarkovChain(gc.slow_reversible_propose_bi, [gc.single_flip_contiguous, pb],
                           gc.AnnealingCutAccept.reference_schedule(), part, 10)
    rows, t0 = chain.schedule
    assert chain.accept_rule == "bratio" and t0 == 100000 and rows.shape == (300001, 9)
    assert np.array_equal(rows[200000], annealing_table(0.1, 2.0, 4))


@pytest.mark.gpu
def test_scheduled_annealing_through_the_facade(gpu_lib):
    """A step_num schedule through the façade equals the oracle with the same rows."""
    from flipcomplexityempirical_amd.chain import schedule_rows
    g, part = sec11_partition(alignment=1, base=0.1)
    pb = gc.within_percent_of_ideal_population(part, 0.10)
    beta = lambda t: 0 if t < 50 else ((t - 50) / 100 if t < 250 else 2)  # noqa: E731
    acc = gc.AnnealingCutAccept(0.1, 2, (beta, 50, 250))
    chain = gc.MarkovChain(gc.slow_reversible_propose_bi, gc.Validator(
        [gc.single_flip_contiguous, pb]), accept=acc, initial_state=part, total_steps=801, seed=4)
    res = chain.run_batched(3, chain_id0=2)
    lo, hi = population_bounds(g.n, 2, 0.10)
    rows, t0 = schedule_rows(0.1, beta, 50, 250, 4)
    for i in range(3):
        olab, ost, _, _ = O.run_chain(g, sec11_seed(g, 1), 2, 0, lo, hi, rows[0], 4, 2 + i, 800,
                                      accept_rule=1, schedule=(rows, t0))
        assert np.array_equal(res.labels[i], olab)
        assert res.stats["accepts"][i] == ost["accepts"][0]
