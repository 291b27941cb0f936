"""Spatial observables on the GPU against the oracle, bit for bit.

The reference driver updates, once per yield, cut_times of every cut edge and
part_sum / last_flipped / num_flips of the node whose flip created the yielded state
(grid_chain_sec11.py:383-384, 396-400; finalised at :416-419).  The oracle does exactly
that per yield (its maps are themselves checked against a replay of the driver loop in
tests/test_oracle.py); the kernels keep the same maps lazily (fire-and-forget atomics on
state changes) and must agree per chain, per element, across launches.
"""
import numpy as np
import pytest

from cases import cases
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = {c.name: c for c in cases()}
MAP_CASES = [("grid12_k4_pairs", "auto"), ("grid16x24_k8", "auto"), ("grid10_k2_bi", "auto"),
             ("grid7x9_k3_cut", "auto"), ("grid20_k4_mu", "wave64"), ("sec11_a2_k2", "auto"),
             ("frank_a2_k2", "auto"), ("tract_k4", "auto"), ("delaunay3k_k18", "auto"),
             ("hub_k3", "auto"), ("grid40x4_k2", "auto")]


def label_values(k):
    return np.array([-1, 1]) if k == 2 else np.array([7 - 3 * d for d in range(k)])


@pytest.mark.parametrize("name,path", MAP_CASES, ids=[f"{p}-{n}" for n, p in MAP_CASES])
def test_maps_match_oracle(gpu_lib, name, path, monkeypatch):
    if path == "wave64":
        monkeypatch.setenv("FLIPWALK_NO_GRID16", "1")
    else:
        monkeypatch.delenv("FLIPWALK_NO_GRID16", raising=False)
    case = CASES[name]
    g = case.graph
    vals = label_values(case.k)
    nc, seed, id0, steps_list = 7, 31, 5, [700, 1300]
    dg = DeviceGraph(g)
    ch = Chains(dg, nc, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds,
                base=case.base, seed=seed, chain_id0=id0)
    ch.enable_maps(vals)
    for s in steps_list:
        ch.run(s)
    got = {w: ch.read_map(w) for w in ("cut_times", "num_flips", "part_sum", "last_flipped")}
    fin = ch.read_map("part_sum", finalize=True)
    labs, st = ch.labels(), ch.stats()
    lo, hi = case.bounds
    tot = {w: 0 for w in got}
    for i in range(nc):
        M = O.Maps(g, case.init, vals)
        lab, ost = case.init.copy(), O.new_stats(1)
        for s in steps_list:
            lab, ost, _, _ = O.run_chain(g, lab, case.k, case.mode, lo, hi, case.thr, seed,
                                         id0 + i, s, stats=ost, maps=M)
        assert np.array_equal(lab, labs[i])
        for w in got:
            assert np.array_equal(got[w][i], getattr(M, w)), (name, i, w)
            tot[w] = tot[w] + getattr(M, w)
        assert np.array_equal(fin[i], M.finalized_part_sum(lab, int(ost["yields"][0])))
        # every yield after the first accepted flip is counted once in num_flips
        assert 0 < M.num_flips.sum() < st["yields"][i]
        assert M.cut_times.sum() == st["sum_cut"][i]  # sum over yields of |cut edges|
    for w in got:  # device-side sum over chains
        assert np.array_equal(ch.read_map(w, total=True), tot[w])
    assert np.array_equal(ch.read_map("cut_times", chains=(2, 5)), got["cut_times"][2:5])


def test_maps_are_refused_after_the_first_run(gpu_lib):
    from flipcomplexityempirical_amd._lib import FlipwalkError
    case = CASES["grid12_k4_pairs"]
    dg = DeviceGraph(case.graph)
    ch = Chains(dg, 2, case.k, case.init, proposal=case.mode, pop_bounds=case.bounds)
    ch.run(5)
    with pytest.raises(FlipwalkError):
        ch.enable_maps()
