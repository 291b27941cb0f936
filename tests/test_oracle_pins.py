"""Statistical pins of the chain law against the reference's own published outputs.

Each New_plots/sec11/{alignment}B{int(100*base)}P{int(100*pop)}wait.txt holds
sum_t geom_wait_t over 100,000 yields of grid_chain_sec11.py's chain (k=2, the 1,596-node
sec11 graph, slow_reversible_propose_bi, cut_accept).  E[geom_wait | |B|] =
(N^2-1)/|B| - 1, so each file pins the run's harmonic-mean boundary size.  The oracle
is run on the same configurations (same seeds, tolerances, bases, 100,000 yields) and
its Rao-Blackwellised mean wait per yield must agree with the reference's 15-run mean
within 3 combined standard errors.  Fixture: tests/golden/wait_sec11.json (extracted
by tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest

from cases import GOLDEN
from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
from flipcomplexityempirical_amd.graph import sec11_graph, sec11_seed
from oracle import oracle as O

MU = 2.63815853
POPS = (0.01, 0.05, 0.1, 0.5, 0.9)


def _ours(base, runs):
    g = sec11_graph()
    M = float(g.n ** 2 - 1)
    out = []
    for a, pop in runs:
        lo, hi = population_bounds(g.n, 2, pop)
        _, st, _, _ = O.run_chain(g, sec11_seed(g, a), 2, 0, lo, hi,
                                  metropolis_table(base, g.maxdeg), 7, a * 10 + int(pop * 100),
                                  99999)
        out.append((M * st["sum_invb"][0] - st["yields"][0]) / st["yields"][0])
    return np.array(out)


@pytest.mark.parametrize("base,label,runs", [
    (MU, 263, [(a, p) for a in (0, 1, 2) for p in POPS]),
    (10.0, 1000, [(a, p) for a in (0, 1, 2) for p in POPS]),
    (1.0, 100, [(0, 0.05), (1, 0.5), (2, 0.9), (0, 0.9)]),
    (0.1, 10, [(a, p) for a in (0, 1, 2) for p in POPS]),
])
def test_sec11_mean_wait_matches_reference(base, label, runs):
    ref = json.load(open(os.path.join(GOLDEN, "wait_sec11.json")))
    refv = np.array([r["wait_sum"] / 1e5 for r in ref if r["base_label"] == label])
    assert len(refv) == 15
    ours = _ours(base, runs)
    se = np.sqrt(refv.var(ddof=1) / len(refv) + ours.var(ddof=1) / len(ours))
    assert abs(ours.mean() - refv.mean()) < 3 * se + 1e-9, (ours.mean(), refv.mean(), se)


FRANK_BASES = {30: 0.3, 263: 1 / .379, 333: 1 / .3}  # Frankenstein_chain.py:32 bases


def _frank_runs(base):
    from flipcomplexityempirical_amd.graph import frankenstein_graph, frankenstein_seed
    g = frankenstein_graph()
    M = float(g.n ** 2 - 1)
    out = {}
    for a in (0, 1, 2):
        for pop in (0.1, 0.5, 0.9):
            lo, hi = population_bounds(g.n, 2, pop)
            _, st, _, _ = O.run_chain(g, frankenstein_seed(g, a), 2, 0, lo, hi,
                                      metropolis_table(base, g.maxdeg), 7,
                                      a * 10 + int(pop * 100), 99999)
            out[(a, int(round(pop * 100)))] = (M * st["sum_invb"][0] - st["yields"][0]) / 1e5
    return out


@pytest.mark.parametrize("label", sorted(FRANK_BASES))
def test_frankengraph_mean_wait_matches_reference(label):
    """plots/FRANK2/{a}B{b}P{p}wait.txt (Frankenstein_chain.py, the 5,000-node
    Frankengraph, k=2, 100,000 yields): per seed alignment, the mean over the three
    population tolerances must agree within 3 standard errors (within-alignment variance
    pooled over both samples).  The alignments differ systematically (the horizontal seed
    sits across the square/triangular seam), so they are compared separately."""
    ref = json.load(open(os.path.join(GOLDEN, "wait_frank2.json")))
    refd = {(r["alignment"], r["pop_label"]): r["wait_sum"] / 1e5 for r in ref
            if r["base_label"] == label}
    assert len(refd) == 9
    ours = _frank_runs(FRANK_BASES[label])
    groups = {a: (np.array([ours[(a, p)] for p in (10, 50, 90)]),
                  np.array([refd[(a, p)] for p in (10, 50, 90)])) for a in (0, 1, 2)}
    ss = sum(((o - o.mean()) ** 2).sum() + ((r - r.mean()) ** 2).sum() for o, r in groups.values())
    s2 = ss / (len(groups) * 2 * (3 - 1))
    se = np.sqrt(s2 * (1 / 3 + 1 / 3))
    for a, (o, r) in groups.items():
        assert abs(o.mean() - r.mean()) < 3 * se, (a, o, r, se)


# All_States_Chain.py:36-38: bases and population tolerances of the Kansas runs
KS_BASES = {10: .1, 14: 1 / MU ** 2, 20: .2, 37: 1 / MU, 80: .8, 100: 1.0}
KS_POPS = {5: .05, 10: .1, 50: .5, 90: .9}
KS_UNITS = {"BG": "BG20", "COUSUB": "COUSUB20", "Tract": "Tract20", "County": "County20"}


def _ks_ours(unit, base_label, T):
    """The oracle on one (unit, base) cell of All_States_Chain.py: k=2 on the Kansas dual
    graph, slow_reversible_propose_bi, cut_accept, T yields, a fresh recursive_tree_part
    seed (epsilon .05, :232) per run as the reference draws one per run; mean wait per
    yield of each of the four population tolerances."""
    from cases import kansas
    from flipcomplexityempirical_amd.seeds import recursive_tree_part
    g = kansas(KS_UNITS[unit])
    M = float(g.n ** 2 - 1)
    b = KS_BASES[base_label]
    out = []
    for pl, p in KS_POPS.items():
        lab = recursive_tree_part(g, [0, 1], g.total_pop / 2, 0.05, seed=1000 * base_label + pl)
        lo, hi = population_bounds(g.total_pop, 2, p)
        _, st, _, _ = O.run_chain(g, lab, 2, 0, lo, hi, metropolis_table(b, g.maxdeg), 7,
                                  100 * base_label + pl, T - 1)
        out.append((M * st["sum_invb"][0] - st["yields"][0]) / T)
    return np.array(out)


@pytest.mark.parametrize("key,T", [("States20", 10000), ("KS2", 100000)])
def test_kansas_mean_wait_matches_reference(key, T):
    """plots/States/20/*wait.txt (All_States_Chain.py with fips 20: Kansas BG / COUSUB /
    Tract / County dual graphs, k=2, total_steps 10,000) and plots/KS2/*wait.txt (the same
    chain at 100,000 yields): for every unit and every base <= 1 (short burn-in; the
    reference's seed plan is a random tree partition, ours another draw of the same
    procedure), the oracle's mean wait per yield over the four population tolerances
    against the reference's four runs.  Each of the 24 cells within 3.5 combined standard
    errors (4 + 4 runs), and the mean squared z within what two 4-run samples give
    (t-tails: E[z^2] ~ 1.5).  Fixture: tests/golden/wait_ks.json."""
    from concurrent.futures import ThreadPoolExecutor
    ref = json.load(open(os.path.join(GOLDEN, "wait_ks.json")))[key]
    cells = [(u, bl) for u in KS_UNITS for bl in KS_BASES]
    # ctypes releases the GIL: the oracle chains of the cells run on a thread pool
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        ours = list(ex.map(lambda c: _ks_ours(c[0], c[1], T), cells))
    zs = []
    for (u, bl), o in zip(cells, ours):
        r = np.array([x["wait_sum"] / T for x in ref if x["unit"] == u and x["base_label"] == bl])
        assert len(r) == 4
        se = np.sqrt(r.var(ddof=1) / len(r) + o.var(ddof=1) / len(o))
        z = (o.mean() - r.mean()) / se
        zs.append(z)
        assert abs(z) < 3.5, (key, u, bl, o.mean(), r.mean(), se)
    assert float(np.mean(np.square(zs))) < 2.5, (key, zs)


@pytest.mark.parametrize("base,label", [(1.0, 100), (0.1, 10)])
def test_sec11_sampled_wait_spread_matches_reference(base, label):
    """The sampled form of geom_wait (one geometric inversion draw per state object,
    re-used on re-yield: grid_chain_sec11.py:147-148,368,410-411; oracle wait_draw) on the
    reference's own 15 sec11 runs (3 seed alignments x 5 tolerances, 100,000 yields): the
    mean wait per yield within 3 combined standard errors of New_plots/sec11/*wait.txt, and
    the run-to-run spread by a two-sided F test (alpha 0.002, 14 / 14 df).  At these bases
    most of the reference's spread (CV 0.5-1.4%) is the geometric draws' own noise, which the
    Rao-Blackwellised sum removes; the sampled sums must carry it."""
    from concurrent.futures import ThreadPoolExecutor

    from scipy import stats as S

    from flipcomplexityempirical_amd.chain import wait_prob_table
    ref = json.load(open(os.path.join(GOLDEN, "wait_sec11.json")))
    refv = np.array([r["wait_sum"] / 1e5 for r in ref if r["base_label"] == label])
    assert len(refv) == 15
    g = sec11_graph()
    pt = wait_prob_table(g.n, 2)

    def one(run):
        a, pop = run
        lo, hi = population_bounds(g.n, 2, pop)
        w = O.Waits(pt)
        _, st, _, _ = O.run_chain(g, sec11_seed(g, a), 2, 0, lo, hi,
                                  metropolis_table(base, g.maxdeg), 7, a * 10 + int(pop * 100),
                                  99999, waits=w)
        return w.sum / st["yields"][0]

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        ours = np.array(list(ex.map(one, [(a, p) for a in (0, 1, 2) for p in POPS])))
    se = np.sqrt(refv.var(ddof=1) / 15 + ours.var(ddof=1) / 15)
    assert abs(ours.mean() - refv.mean()) < 3 * se, (ours.mean(), refv.mean(), se)
    F = ours.var(ddof=1) / refv.var(ddof=1)
    assert S.f.ppf(0.001, 14, 14) < F < S.f.ppf(0.999, 14, 14), (F, ours.std(), refv.std())
