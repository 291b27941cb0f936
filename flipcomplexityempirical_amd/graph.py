"""Graphs as canonical CSR (host side).

Replaces the networkx / ``gerrychain.Graph`` objects the reference builds:

* ``grid_graph(h, w)``      — ``nx.grid_graph([k*gn, k*gn])`` (grid_chain_sec11.py:191),
  node (i, j) -> id i*w + j, row-major; the HIP library detects this layout and
  uses implicit neighbours.
* ``sec11_graph()``         — the 40x40 grid with the four corner diagonals added and the
  corners removed (grid_chain_sec11.py:191,236,252-260): 1,596 nodes, 3,116 edges.
* ``Graph.from_json(path)`` — ``gerrychain.Graph.from_json`` (All_States_Chain.py:208,221),
  networkx adjacency-JSON, including the TOTPOP str->int cast (All_States_Chain.py:227-230).
* ``Graph.from_networkx(G)``.
* ``frankenstein_graph()`` — the "Frankengraph" of Frankenstein_chain.py:188-197 /
  construct_FRANK.py: a 50x50 square grid glued along one row to a triangular lattice
  (5,000 nodes, 12,300 edges, max degree 6), with the three seed plans of :209-248.
* ``delaunay_graph()``      — the C4 benchmark graph: Delaunay triangulation
  of 9,000 uniform points, lognormal integer populations (a VTD-style dual graph).

Canonical form (what every other component assumes): node ids 0..n-1 in sorted order
of the original node keys, neighbour lists strictly ascending, no self loops,
symmetric.  Proposal order "(v, u) in CSR order" is therefore "(v, u) ascending".
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, Hashable, List, Optional, Sequence

import numpy as np


@dataclass
class Graph:
    rowptr: np.ndarray  # int32 [n+1]
    col: np.ndarray  # int32 [nnz]
    pop: Optional[np.ndarray] = None  # int64 [n] or None (= all ones)
    nodes: List[Hashable] = field(default_factory=list)  # original node keys, by id
    grid_w: int = 0  # >0: this is the row-major grid_w-wide grid
    node_attrs: Optional[List[Dict[str, Any]]] = None

    # ------------------------------------------------------------------ basics
    @property
    def n(self) -> int:
        return int(len(self.rowptr) - 1)

    @property
    def n_edges(self) -> int:
        return int(len(self.col) // 2)

    @property
    def degrees(self) -> np.ndarray:
        return np.diff(self.rowptr).astype(np.int32)

    @property
    def maxdeg(self) -> int:
        return int(self.degrees.max()) if self.n else 0

    @property
    def total_pop(self) -> int:
        return int(self.n if self.pop is None else int(self.pop.sum()))

    def neighbors(self, v: int) -> np.ndarray:
        return self.col[self.rowptr[v]:self.rowptr[v + 1]]

    def index(self) -> Dict[Hashable, int]:
        return {k: i for i, k in enumerate(self.nodes)}

    def edges(self) -> np.ndarray:
        """Undirected edges (u < v) as an int32 [m, 2] array, in CSR order."""
        src = np.repeat(np.arange(self.n, dtype=np.int32), self.degrees)
        keep = src < self.col
        return np.stack([src[keep], self.col[keep]], axis=1)

    def pop_array(self) -> np.ndarray:
        return np.ones(self.n, np.int64) if self.pop is None else self.pop

    def validate(self) -> None:
        rp, col = self.rowptr, self.col
        if rp[0] != 0 or rp[-1] != len(col) or np.any(np.diff(rp) < 0):
            raise ValueError("malformed rowptr")
        for v in range(self.n):
            nb = col[rp[v]:rp[v + 1]]
            if len(nb) and (np.any(np.diff(nb) <= 0) or nb[0] < 0 or nb[-1] >= self.n or v in nb):
                raise ValueError(f"row {v}: neighbours must be ascending, in range, no self loop")
        e = self.edges()
        if 2 * len(e) != len(col):
            raise ValueError("adjacency is not symmetric")

    # ------------------------------------------------------------ constructors
    @classmethod
    def from_adjacency(cls, nodes: Sequence[Hashable], adj: Dict[Hashable, Sequence[Hashable]],
                       pop: Optional[Sequence[int]] = None, node_attrs=None) -> "Graph":
        try:
            order = sorted(nodes)
        except TypeError:
            order = list(nodes)
        idx = {k: i for i, k in enumerate(order)}
        n = len(order)
        nbrs = [sorted({idx[u] for u in adj[k] if u != k}) for k in order]
        rowptr = np.zeros(n + 1, np.int32)
        rowptr[1:] = np.cumsum([len(x) for x in nbrs])
        col = np.array([u for x in nbrs for u in x], dtype=np.int32)
        p = None
        if pop is not None:
            pmap = dict(zip(nodes, pop))
            p = np.array([int(pmap[k]) for k in order], dtype=np.int64)
        attrs = None
        if node_attrs is not None:
            amap = dict(zip(nodes, node_attrs))
            attrs = [amap[k] for k in order]
        g = cls(rowptr=rowptr, col=col, pop=p, nodes=list(order), node_attrs=attrs)
        g.validate()
        g.grid_w = detect_grid(g)
        return g

    @classmethod
    def from_networkx(cls, G, pop_col: Optional[str] = None) -> "Graph":
        nodes = list(G.nodes())
        adj = {k: list(G.neighbors(k)) for k in nodes}
        pop = None
        if pop_col is not None:
            pop = [int(G.nodes[k][pop_col]) for k in nodes]
        return cls.from_adjacency(nodes, adj, pop, [dict(G.nodes[k]) for k in nodes])

    @classmethod
    def from_json(cls, path: str, pop_col: Optional[str] = "TOTPOP") -> "Graph":
        """networkx ``adjacency_data`` JSON (the State_Data/*.json format).

        ``pop_col`` values are cast with ``int()`` as All_States_Chain.py:227-230 does
        (BG20 stores TOTPOP as strings).
        """
        with open(path) as f:
            data = json.load(f)
        nodes = [d["id"] for d in data["nodes"]]
        adj = {nid: [e["id"] for e in data["adjacency"][i]] for i, nid in enumerate(nodes)}
        pop = None
        if pop_col is not None:
            pop = [int(d[pop_col]) for d in data["nodes"]]
        return cls.from_adjacency(nodes, adj, pop, data["nodes"])


def detect_grid(g: Graph) -> int:
    """Width w if ``g`` is exactly the row-major h x w grid graph (h, w >= 2), else 0."""
    n = g.n
    if n < 4:
        return 0
    nb0 = g.neighbors(0)
    if len(nb0) != 2 or nb0[0] != 1:
        return 0
    w = int(nb0[1])
    if w < 2 or n % w or n // w < 2:
        return 0
    ref = grid_graph(n // w, w, detect=False)
    if len(ref.col) == len(g.col) and np.array_equal(ref.rowptr, g.rowptr) and np.array_equal(
            ref.col, g.col):
        return w
    return 0


def grid_graph(h: int, w: int, detect: bool = True) -> Graph:
    """Row-major h x w grid (4-neighbour), node (i, j) -> i*w + j, unit populations."""
    ids = np.arange(h * w, dtype=np.int64).reshape(h, w)
    rows = []
    for i in range(h):
        for j in range(w):
            nb = []
            if i > 0:
                nb.append(ids[i - 1, j])
            if j > 0:
                nb.append(ids[i, j - 1])
            if j < w - 1:
                nb.append(ids[i, j + 1])
            if i < h - 1:
                nb.append(ids[i + 1, j])
            rows.append(nb)
    rowptr = np.zeros(h * w + 1, np.int32)
    rowptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.array([u for r in rows for u in r], dtype=np.int32)
    g = Graph(rowptr=rowptr, col=col, pop=None, nodes=[(i, j) for i in range(h) for j in range(w)])
    g.grid_w = w if detect else 0
    return g


def sec11_graph() -> Graph:
    """The grid_chain_sec11.py graph: 40x40 grid, corner diagonals, corners removed."""
    n = 40
    nodes = [(i, j) for i in range(n) for j in range(n)]
    adj: Dict[Hashable, set] = {x: set() for x in nodes}
    for i in range(n):
        for j in range(n):
            for di, dj in ((1, 0), (0, 1)):
                a, b = (i, j), (i + di, j + dj)
                if b[0] < n and b[1] < n:
                    adj[a].add(b)
                    adj[b].add(a)
    for a, b in [((0, 1), (1, 0)), ((0, 38), (1, 39)), ((38, 0), (39, 1)), ((38, 39), (39, 38))]:
        adj[a].add(b)
        adj[b].add(a)
    for c in [(0, 0), (0, 39), (39, 0), (39, 39)]:
        for u in adj.pop(c):
            adj[u].discard(c)
        nodes.remove(c)
    return Graph.from_adjacency(nodes, {k: sorted(v) for k, v in adj.items()})


def sec11_seed(g: Graph, alignment: int) -> np.ndarray:
    """Seed plans of grid_chain_sec11.py:194-214, labels {-1, 1} mapped to {0, 1}."""
    lab = np.zeros(g.n, np.int16)
    for i, (a, b) in enumerate(g.nodes):
        if alignment == 0:
            v = 1 if a > 19 else -1
        elif alignment == 1:
            v = 1 if b > 19 else -1
        elif alignment == 2:
            v = 1 if (a > b or (a == b and a > 19)) else -1
        else:
            raise ValueError("alignment must be 0, 1 or 2")
        lab[i] = 1 if v == 1 else 0
    return lab


def block_seed(h: int, w: int, brows: int, bcols: int) -> np.ndarray:
    """Row-major grid split into brows x bcols equal rectangles, labelled row-major.

    quadrants (C2/C3, k=4) = block_seed(h, w, 2, 2); C5 (k=8) = block_seed(200, 200, 2, 4).
    """
    if h % brows or w % bcols:
        raise ValueError("grid must divide evenly into blocks")
    i = np.arange(h)[:, None] // (h // brows)
    j = np.arange(w)[None, :] // (w // bcols)
    return (i * bcols + j).astype(np.int16).reshape(-1)


def band_seed(h: int, w: int, k: int) -> np.ndarray:
    """Rows split into k horizontal bands of (nearly) equal height, labelled 0..k-1."""
    if k > h:
        raise ValueError("need at least one row per band")
    band = (np.arange(h) * k) // h
    return np.repeat(band[:, None], w, axis=1).astype(np.int16).reshape(-1)


def stripe_seed(h: int, w: int) -> np.ndarray:
    """Rows i >= h/2 -> 1, else 0 (the sec11 'alignment 0' analogue used for C1)."""
    return (np.arange(h)[:, None] >= h // 2).repeat(w, axis=1).astype(np.int16).reshape(-1)


# ---------------------------------------------------------------- Frankengraph
def frankenstein_graph(m: int = 50) -> Graph:
    """Frankenstein_chain.py:188-197: nx.compose(relabelled m x m grid, triangular lattice).

    Node keys are the reference's (x, y) tuples; node attributes carry ``boundary_node``
    (:259-265: x == 0, x == m-1, y == m or y == -m+1) for the boundary_condition rule.
    """
    import networkx as nx
    G = nx.grid_graph([m, m])
    H = nx.triangular_lattice_graph(m, 2 * m - 2)
    G = nx.relabel_nodes(G, {x: (x[0], x[1] - m + 1) for x in G.nodes()})
    F = nx.compose(G, H)
    nodes = list(F.nodes())
    adj = {x: list(F.neighbors(x)) for x in nodes}
    attrs = [{"population": 1,
              "boundary_node": bool(x[0] == 0 or x[0] == m - 1 or x[1] == m or x[1] == -m + 1)}
             for x in nodes]
    return Graph.from_adjacency(nodes, adj, None, attrs)


def frankenstein_seed(g: Graph, alignment: int, m: int = 50) -> np.ndarray:
    """Seed plans of Frankenstein_chain.py:209-248 (start_plans = [diagonal, vertical,
    horizontal]; members -> 1, others -> -1), labels {-1, 1} mapped to {0, 1}."""
    lab = np.zeros(g.n, np.int16)
    for i, (x, y) in enumerate(g.nodes):
        if alignment == 0:
            inside = 2 * x - y <= m - 3
        elif alignment == 1:
            inside = x < m / 2
        elif alignment == 2:
            inside = y < 0
        else:
            raise ValueError("alignment must be 0, 1 or 2")
        lab[i] = 1 if inside else 0
    return lab


def boundary_flags(g: Graph) -> np.ndarray:
    """uint8 per node: the ``boundary_node`` attribute (grid_chain_sec11.py:225-233 marks
    the outer ring of the grid; Frankenstein_chain.py:259-265 the Frankengraph rim)."""
    if g.node_attrs is not None and g.node_attrs and "boundary_node" in g.node_attrs[0]:
        return np.array([1 if a["boundary_node"] else 0 for a in g.node_attrs], np.uint8)
    if g.nodes and all(isinstance(k, tuple) and len(k) == 2 for k in g.nodes):
        xs = np.array([k[0] for k in g.nodes])
        ys = np.array([k[1] for k in g.nodes])
        return ((xs == xs.min()) | (xs == xs.max()) | (ys == ys.min()) |
                (ys == ys.max())).astype(np.uint8)
    raise ValueError("graph has no boundary_node attribute and no coordinate keys")


# ---------------------------------------------------------------- C4 dual graph
def hilbert_index(xy: np.ndarray, bits: int = 16) -> np.ndarray:
    """Position of each point of the unit square (rows of ``xy``) along the Hilbert curve of
    a 2^bits x 2^bits lattice (the classic xy -> d rotation walk, vectorised)."""
    side = 1 << bits
    x = np.minimum((xy[:, 0] * side).astype(np.int64), side - 1)
    y = np.minimum((xy[:, 1] * side).astype(np.int64), side - 1)
    d = np.zeros(len(xy), np.int64)
    s = side >> 1
    while s > 0:
        rx = (x & s) > 0
        ry = (y & s) > 0
        d += s * s * ((3 * rx) ^ ry)
        # rotate the quadrant so the sub-curve has the canonical orientation
        flip = ~ry
        swap_x = np.where(flip & rx, s - 1 - x, x)
        swap_y = np.where(flip & rx, s - 1 - y, y)
        x = np.where(flip, swap_y, x)
        y = np.where(flip, swap_x, y)
        s >>= 1
    return d


def delaunay_graph(n_points: int = 9000, seed: int = 0, pop_median: float = 1000.0,
                   pop_sigma: float = 0.8, order: str = "random") -> Graph:
    """Delaunay triangulation of ``n_points`` points drawn by
    ``np.random.default_rng(seed).random((n, 2))``, node populations
    ``max(1, round(lognormal(ln pop_median, pop_sigma)))`` from the same generator.

    ``order``: node ids in the points' draw order ("random": unrelated to position), or
    along the Hilbert curve of the points ("hilbert": the same graph up to isomorphism,
    numbered so that neighbours get nearby ids, as census units in a shapefile's
    geographic order do — a node's neighbours then share its 64-node weight group and
    nearby rows of the padded adjacency table)."""
    from scipy.spatial import Delaunay
    rng = np.random.default_rng(seed)
    pts = rng.random((n_points, 2))
    tri = Delaunay(pts)
    indptr, indices = tri.vertex_neighbor_vertices
    pop = np.maximum(1, np.rint(rng.lognormal(np.log(pop_median), pop_sigma, n_points))).astype(
        np.int64)
    if order == "random":
        key = np.arange(n_points)
    elif order == "hilbert":
        key = np.empty(n_points, np.int64)
        key[np.argsort(hilbert_index(pts), kind="stable")] = np.arange(n_points)
    else:
        raise ValueError("order must be 'random' or 'hilbert'")
    nodes = [int(key[v]) for v in range(n_points)]
    adj = {int(key[v]): [int(key[u]) for u in indices[indptr[v]:indptr[v + 1]]]
           for v in range(n_points)}
    attrs = [{"x": float(pts[v, 0]), "y": float(pts[v, 1])} for v in range(n_points)]
    return Graph.from_adjacency(nodes, adj, pop.tolist(), attrs)
