"""Shared test configurations (graphs, seed plans, chain parameters).

Graphs follow the reference's constructions: the plain grid (nx.grid_graph,
grid_chain_sec11.py:191), the sec11 grid with corner diagonals and corners removed
(:191-260), and the Kansas dual graphs (State_Data/*.json, All_States_Chain.py:208,221)
from the committed CSR fixtures in tests/golden (the reference tree does not travel
to the GPU box).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
from flipcomplexityempirical_amd.graph import (Graph, band_seed, block_seed, delaunay_graph,
                                               frankenstein_graph, frankenstein_seed, grid_graph,
                                               sec11_graph, sec11_seed, stripe_seed)
from flipcomplexityempirical_amd.seeds import tree_seed

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MU = 2.63815853


def kansas(name: str) -> Graph:
    """Kansas dual graph from the committed CSR fixture (TOTPOP populations)."""
    d = np.load(os.path.join(GOLDEN, f"kansas_{name}.npz"), allow_pickle=False)
    g = Graph(rowptr=d["rowptr"], col=d["col"], pop=d["pop"], nodes=list(range(len(d["pop"]))))
    return g


def kansas_seed(name: str, k: int) -> np.ndarray:
    d = np.load(os.path.join(GOLDEN, f"kansas_{name}.npz"), allow_pickle=False)
    return d[f"seed_k{k}"].astype(np.int16)


@dataclass
class Case:
    name: str
    graph: Graph
    init: np.ndarray
    k: int
    mode: int
    percent: float
    base: float

    @property
    def bounds(self):
        return population_bounds(self.graph.total_pop, self.k, self.percent)

    @property
    def thr(self):
        return metropolis_table(self.base, self.graph.maxdeg)


def hub_graph(n: int = 15) -> Graph:
    """An n x n grid plus two hub nodes: one joined to every cell of the two middle rows
    (degree 2n = 30), one to the middle column and to seven cells of row 0 (degree 22), so
    the graph has no 16-wide padded-row table and runs the CSR-walking chain kernel."""
    import networkx as nx
    G = nx.grid_2d_graph(n, n)
    G.add_node("hub")
    for c in range(n):
        G.add_edge("hub", (n // 2, c))
        G.add_edge("hub", (n // 2 + 1, c))
    G.add_node("hub2")
    for r in range(n):
        G.add_edge("hub2", (r, n // 2))
    for c in range(7):
        G.add_edge("hub2", (0, c))
    for v in G.nodes:  # the grid's outer ring (boundary_condition); the hubs are interior
        G.nodes[v]["boundary_node"] = isinstance(v, tuple) and (min(v) == 0 or max(v) == n - 1)
    return Graph.from_networkx(G)


def c4_seed(g: Graph, k: int, percent: float = 0.05) -> np.ndarray:
    return tree_seed(g, k, percent)


def cases(include_kansas: bool = True):
    out = [
        Case("grid10_k2_bi", grid_graph(10, 10), stripe_seed(10, 10), 2, 0, 0.10, MU),
        Case("grid12_k4_pairs", grid_graph(12, 12), block_seed(12, 12, 2, 2), 4, 1, 0.10, 0.5),
        Case("grid12_k4_cut", grid_graph(12, 12), block_seed(12, 12, 2, 2), 4, 2, 0.10, 1.5),
        Case("grid20_k4_mu", grid_graph(20, 20), block_seed(20, 20, 2, 2), 4, 1, 0.05, MU),
        Case("grid16x24_k8", grid_graph(16, 24), block_seed(16, 24, 2, 4), 8, 1, 0.10, 1.0),
        # widths that are not multiples of 4 (node windows wrap into the next grid row)
        Case("grid7x9_k3_cut", grid_graph(7, 9), band_seed(7, 9, 3), 3, 2, 0.30, 0.7),
        Case("grid11x13_k4", grid_graph(11, 13), band_seed(11, 13, 4), 4, 1, 0.30, MU),
        Case("grid30x18_k2_bi", grid_graph(30, 18), band_seed(30, 18, 2), 2, 0, 0.10, 0.4),
        # edge shapes: the narrowest grid of the four-chains-per-wave kernel (W = 4), one
        # below it (W = 3: the one-chain-per-wave kernel on the grid), three rows only
        Case("grid40x4_k2", grid_graph(40, 4), band_seed(40, 4, 2), 2, 1, 0.20, 0.8),
        Case("grid40x3_k2_cut", grid_graph(40, 3), band_seed(40, 3, 2), 2, 2, 0.20, MU),
        Case("grid3x40_k2_bi", grid_graph(3, 40), band_seed(3, 40, 2), 2, 0, 0.40, 0.6),
    ]
    g11 = sec11_graph()
    out.append(Case("sec11_a2_k2", g11, sec11_seed(g11, 2), 2, 0, 0.05, 0.1))
    out.append(Case("sec11_a0_k2_mu", g11, sec11_seed(g11, 0), 2, 0, 0.10, MU))
    gf = frankenstein_graph()
    out.append(Case("frank_a2_k2", gf, frankenstein_seed(gf, 2), 2, 0, 0.5, 1 / .379))
    out.append(Case("frank_a0_k2_cold", gf, frankenstein_seed(gf, 0), 2, 0, 0.1, 0.3))
    gd = delaunay_graph(3000, seed=1)
    out.append(Case("delaunay3k_k18", gd, c4_seed(gd, 18), 18, 1, 0.05, MU))
    # k = 31: every 5-bit label code but one in use
    out.append(Case("delaunay3k_k31", gd, c4_seed(gd, 31, 0.10), 31, 1, 0.10, MU))
    # hubs of degree 30 and 22: rows past the 16-wide padded table, the CSR-walking kernel
    gh = hub_graph()
    out.append(Case("hub_k3", gh, c4_seed(gh, 3, 0.10), 3, 1, 0.10, 1.2))
    out.append(Case("hub_k2_cut", gh, c4_seed(gh, 2, 0.10), 2, 2, 0.10, MU))
    if include_kansas:
        out.append(Case("county_k2", kansas("County20"), kansas_seed("County20", 2), 2, 0, 0.10,
                        1.0))
        out.append(Case("tract_k4", kansas("Tract20"), kansas_seed("Tract20", 4), 4, 1, 0.20,
                        0.8))
        out.append(Case("tract_k2_cut", kansas("Tract20"), kansas_seed("Tract20", 2), 2, 2, 0.20,
                        MU))
    return out
