"""Host-side logic: graph construction, seeds, bounds and Metropolis tables (CPU only)."""
import math
import os

import numpy as np
import pytest

from cases import GOLDEN, kansas, kansas_seed
from flipcomplexityempirical_amd.chain import (expected_wait_sum, metropolis_table,
                                               population_bounds)
from flipcomplexityempirical_amd.graph import (Graph, band_seed, block_seed, detect_grid,
                                               grid_graph, sec11_graph, sec11_seed)
from flipcomplexityempirical_amd.seeds import recursive_tree_part
from oracle import oracle as O


def test_sec11_graph_matches_reference_construction():
    g = sec11_graph()  # grid_chain_sec11.py:191,236,252-260
    assert (g.n, g.n_edges, g.maxdeg, g.grid_w) == (1596, 3116, 4, 0)
    idx = g.index()
    assert idx[(1, 0)] in g.neighbors(idx[(0, 1)])  # the added corner diagonal
    for a in (0, 1, 2):
        lab = sec11_seed(g, a)
        assert lab.sum() == 798 and O.plan_valid(g, lab, 2, 790, 806)


def test_grid_detection():
    assert grid_graph(7, 9).grid_w == 9 and detect_grid(grid_graph(100, 100)) == 100
    assert sec11_graph().grid_w == 0
    g = grid_graph(5, 5)
    g2 = Graph.from_adjacency(list(range(25)), {i: list(g.neighbors(i)) for i in range(25)})
    assert g2.grid_w == 5


def test_population_bounds_equal_gerrychain_float_semantics():
    for total, k, p in [(1596, 2, 0.01), (10000, 4, 0.05), (2853118, 18, 0.05), (100, 2, 0.1),
                        (40000, 8, 0.05), (1530, 2, 0.9)]:
        lo_i, hi_i = population_bounds(total, k, p)
        ideal = total / k
        lo, hi = (1 - p) * ideal, (1 + p) * ideal
        for pop in range(max(0, lo_i - 50), hi_i + 50):
            assert (lo <= pop <= hi) == (lo_i <= pop <= hi_i)


def test_metropolis_table_is_python_pow():
    for base in (0.1, 2.63815853, 1.0, 10.0, 1 / 2.63815853 ** 2):
        thr = metropolis_table(base, 4)
        for d in range(-4, 5):
            assert thr[d + 4] == base ** (-d)  # cut_accept: base**(c_old - c_new)


def test_expected_wait_sum():
    st = np.zeros(2, O.STATS_DTYPE)
    st["sum_invb"] = [0.5, 0.25]
    st["yields"] = [3, 4]
    got = expected_wait_sum(st, 10, 2)
    assert np.allclose(got, [99 * 0.5 - 3, 99 * 0.25 - 4])


def test_block_and_band_seeds():
    b = block_seed(100, 100, 2, 2)
    assert np.bincount(b).tolist() == [2500] * 4
    assert np.bincount(band_seed(11, 13, 4)).sum() == 143
    g = grid_graph(100, 100)
    assert O.plan_valid(g, b, 4, *population_bounds(10000, 4, 0.05))


@pytest.mark.parametrize("unit,n,e,md", [("County20", 105, 263, 8), ("Tract20", 770, 2005, 13),
                                         ("COUSUB20", 1530, 3808, 16), ("BG20", 2351, 6252, 15)])
def test_kansas_fixtures(unit, n, e, md):
    g = kansas(unit)
    g.validate()
    assert (g.n, g.n_edges, g.maxdeg) == (n, e, md)
    assert g.total_pop == 2853118  # Kansas 2010 TOTPOP (All_States_Chain.py:226-230)
    for k in (2, 4):
        lab = kansas_seed(unit, k)
        assert O.plan_valid(g, lab, k, *population_bounds(g.total_pop, k, 0.10))


def test_recursive_tree_part_gives_balanced_contiguous_plans():
    g = kansas("Tract20")
    for seed in range(3):
        lab = recursive_tree_part(g, [0, 1, 2], g.total_pop / 3, 0.05, seed=seed)
        lo, hi = population_bounds(g.total_pop, 3, 0.10)
        pops = np.bincount(lab, weights=g.pop, minlength=3)
        # the first k-1 districts are within epsilon of the target by construction
        assert all(abs(p - g.total_pop / 3) < 0.05 * g.total_pop / 3 for p in pops[:2])
        assert O.plan_valid(g, lab, 3, 0, g.total_pop)


def test_json_loader_casts_string_totpop():
    p = os.path.join(GOLDEN, "..", "..", "tests", "golden")
    assert os.path.isdir(p)
    import json
    import tempfile
    data = {"directed": False, "multigraph": False, "graph": [],
            "nodes": [{"id": 0, "TOTPOP": "5"}, {"id": 1, "TOTPOP": "7"}],
            "adjacency": [[{"id": 1}], [{"id": 0}]]}
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(data, f)
    g = Graph.from_json(f.name)
    os.unlink(f.name)
    assert g.pop.tolist() == [5, 7] and g.n_edges == 1
    assert math.isclose(g.total_pop, 12)


def test_frankengraph_matches_reference_construction():
    """Frankenstein_chain.py:188-248: 50x50 grid composed with triangular_lattice_graph(50, 98)."""
    from flipcomplexityempirical_amd.graph import (boundary_flags, frankenstein_graph,
                                                   frankenstein_seed)
    g = frankenstein_graph()
    assert (g.n, g.n_edges, g.maxdeg, g.grid_w) == (5000, 12300, 6, 0)
    idx = g.index()
    assert idx[(0, 1)] in g.neighbors(idx[(0, 0)]) and idx[(0, -1)] in g.neighbors(idx[(0, 0)])
    flags = boundary_flags(g)
    rim = [k for k in g.nodes if k[0] in (0, 49) or k[1] in (50, -49)]
    assert flags.sum() == len(rim) and all(flags[idx[k]] for k in rim)
    sizes = [int(frankenstein_seed(g, a).sum()) for a in (0, 1, 2)]
    assert sizes == [2450, 2500, 2450]  # diagonal, vertical, horizontal (construct_FRANK.py)
    for a in (0, 1, 2):
        assert O.plan_valid(g, frankenstein_seed(g, a), 2, *population_bounds(g.n, 2, 0.1))


def test_delaunay_c4_graph_and_tree_seed():
    """C4: ~9k-node Delaunay dual graph, lognormal populations, k=18 tree seed within 5%."""
    from flipcomplexityempirical_amd.graph import delaunay_graph
    g = delaunay_graph()
    assert g.n == 9000 and 3 * g.n - 6 >= g.n_edges > 2.9 * g.n and 8 < g.maxdeg < 32
    assert g.pop.min() >= 1 and 500 < np.median(g.pop) < 2000
    k = 18
    lab = recursive_tree_part(g, list(range(k)), g.total_pop / k, 0.05, seed=0)
    lo, hi = population_bounds(g.total_pop, k, 0.05)
    assert O.plan_valid(g, lab, k, lo, hi)  # the debt rule keeps the remainder in bounds too


def test_write_wait_txt(tmp_path):
    from flipcomplexityempirical_amd.chain import write_wait_txt
    st = np.zeros(1, O.STATS_DTYPE)
    st["sum_invb"], st["yields"] = [250.5], [100000]
    w = expected_wait_sum(st, 1596, 2)[0]
    p = tmp_path / "2B10P5wait.txt"  # grid_chain_sec11.py:410 naming
    write_wait_txt(str(p), w)
    assert p.read_text() == str(int(round(w))) and "\n" not in p.read_text()


def test_bench_refuses_maps_with_resume():
    """bench.py --maps --resume cannot work (plan writes are refused under maps, maps cannot
    be enabled after a restore): argparse rejects the pair before anything is built."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--maps", "--resume",
                        "x.npz"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "--maps cannot be combined with --resume" in r.stderr


def test_hilbert_numbering_is_the_same_graph():
    """delaunay_graph(order="hilbert") renumbers the C4 graph along the Hilbert curve of its
    points: the same graph up to isomorphism (the same points, populations and triangles),
    with neighbours mostly in the same 64-node weight group."""
    from flipcomplexityempirical_amd.graph import delaunay_graph, hilbert_index
    g0, g1 = delaunay_graph(2000, seed=3), delaunay_graph(2000, seed=3, order="hilbert")
    assert (g0.n, g0.n_edges, g0.total_pop) == (g1.n, g1.n_edges, g1.total_pop)
    # map by point coordinates: the edge sets agree
    pos0 = {(a["x"], a["y"]): i for i, a in enumerate(g0.node_attrs)}
    perm = np.array([pos0[(a["x"], a["y"])] for a in g1.node_attrs])
    e1 = {tuple(sorted((int(perm[u]), int(perm[v])))) for u, v in g1.edges()}
    e0 = {tuple(map(int, e)) for e in g0.edges()}
    assert e0 == e1
    assert np.array_equal(g1.pop, g0.pop[perm])
    src = np.repeat(np.arange(g1.n), g1.degrees)
    assert ((src // 64) == (g1.col // 64)).mean() > 0.6
    # the curve visits a 4 x 4 lattice cell by cell
    side = 4
    xy = np.array([[(i + .5) / side, (j + .5) / side] for i in range(side) for j in range(side)])
    walk = (xy[np.argsort(hilbert_index(xy, 2))] * side).astype(int)
    assert all(np.abs(walk[i] - walk[i + 1]).sum() == 1 for i in range(15))


def test_boundary_flags_needs_attributes_or_coordinate_keys():
    """boundary_condition's flags come from the boundary_node attribute, else from (x, y)
    keys; a graph with neither (or with keys of mixed kinds) is refused by name."""
    import networkx as nx
    import pytest as _pytest
    from flipcomplexityempirical_amd.graph import Graph, boundary_flags
    G = nx.grid_2d_graph(3, 4)
    f = boundary_flags(Graph.from_networkx(G))
    assert f.sum() == 10 and f[[k for k in G.nodes].index((1, 1))] == 0
    G.add_edge("hub", (1, 1))
    with _pytest.raises(ValueError, match="boundary_node"):
        boundary_flags(Graph.from_networkx(G))
    for v in G.nodes:
        G.nodes[v]["boundary_node"] = v == "hub"
    assert boundary_flags(Graph.from_networkx(G)).sum() == 1
