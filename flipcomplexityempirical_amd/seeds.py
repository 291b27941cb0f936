"""Seed plans (host side).

``recursive_tree_part`` restates gerrychain.tree.recursive_tree_part [ext], which the
reference calls as ``recursive_tree_part(graph, [-1, 1], totpop/2, "TOTPOP", .05, 1)``
(All_States_Chain.py:232): split off one district at a time by drawing a random
spanning tree (minimum spanning tree under i.i.d. uniform edge weights), rooting it,
and cutting a uniformly chosen tree edge whose side has population within
``epsilon * pop_target`` of ``pop_target``; redraw the tree when no edge qualifies.
The last district takes the remainder.  As in GerryChain 0.2.x's recursive_tree_part, a
running population "debt" narrows each split's window so that the remainder, too, ends
within ``epsilon`` of ``pop_target``.  GerryChain is not installed, so the draw
sequence is our own (numpy ``default_rng``); the law over plans follows the
published algorithm.  Grid seeds (grid_chain_sec11.py:194-214) live in ``graph``.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import breadth_first_order, minimum_spanning_tree

from .graph import Graph


def _balanced_cut(rowptr, col, pop, nodes, target, eps, rng, max_tries=10000):
    """One bipartition_tree draw on the induced subgraph ``nodes`` -> subset (global ids)."""
    nodes = np.asarray(nodes, np.int64)
    local = -np.ones(len(rowptr) - 1, np.int64)
    local[nodes] = np.arange(len(nodes))
    src, dst = [], []
    for i, x in enumerate(nodes):
        nb = col[rowptr[x]:rowptr[x + 1]]
        nb = local[nb]
        nb = nb[nb > i]
        src.extend([i] * len(nb))
        dst.extend(nb.tolist())
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    m = len(nodes)
    p = pop[nodes].astype(np.float64)
    total = p.sum()
    for _ in range(max_tries):
        w = rng.random(len(src)) + 1e-9
        A = csr_matrix((w, (src, dst)), shape=(m, m))
        T = minimum_spanning_tree(A)
        T = T + T.T
        deg = np.diff(T.indptr)
        inner = np.flatnonzero(deg > 1)
        root = int(rng.choice(inner)) if len(inner) else 0
        order, pred = breadth_first_order(T, root, directed=False, return_predecessors=True)
        if len(order) != m:
            raise ValueError("subgraph is disconnected")
        sub = p.copy()
        for x in order[::-1][:-1]:
            sub[pred[x]] += sub[x]
        cands = []
        for x in order[1:]:
            if abs(sub[x] - target) < eps * target:
                cands.append((x, False))
            if abs((total - sub[x]) - target) < eps * target:
                cands.append((x, True))
        if not cands:
            continue
        x, comp = cands[int(rng.integers(len(cands)))]
        # subtree of x in the rooted tree
        children = [[] for _ in range(m)]
        for y in order[1:]:
            children[pred[y]].append(y)
        stack, inside = [x], np.zeros(m, bool)
        while stack:
            y = stack.pop()
            inside[y] = True
            stack.extend(children[y])
        if comp:
            inside = ~inside
        return nodes[inside]
    raise RuntimeError("no balanced cut found")


def recursive_tree_part(graph: Graph, parts: Sequence, pop_target: float, epsilon: float,
                        seed: Optional[int] = 0, node_repeats: int = 1) -> np.ndarray:
    """District labels (index into ``parts``) for every node; see the module docstring."""
    rng = np.random.default_rng(seed)
    pop = graph.pop_array()
    remaining = np.arange(graph.n)
    lab = np.full(graph.n, len(parts) - 1, np.int16)
    debt = 0.0
    for i in range(len(parts) - 1):
        min_pop = max(pop_target * (1 - epsilon), pop_target * (1 - epsilon) - debt)
        max_pop = min(pop_target * (1 + epsilon), pop_target * (1 + epsilon) - debt)
        target = (min_pop + max_pop) / 2
        subset = _balanced_cut(graph.rowptr, graph.col, pop, remaining, target,
                               (max_pop - min_pop) / (2 * target), rng)
        lab[subset] = i
        debt += float(pop[subset].sum()) - pop_target
        remaining = np.setdiff1d(remaining, subset)
    return lab


def tree_seed(graph: Graph, k: int, percent: float = 0.05, seed: int = 0,
              tries: int = 50) -> np.ndarray:
    """A recursive_tree_part plan (labels 0..k-1) that is valid for the chain's
    within_percent_of_ideal_population(percent) bounds; tries successive seeds."""
    from .chain import population_bounds
    lo, hi = population_bounds(graph.total_pop, k, percent)
    pop = graph.pop_array()
    for s in range(seed, seed + tries):
        lab = recursive_tree_part(graph, list(range(k)), graph.total_pop / k, percent, seed=s)
        p = np.bincount(lab, weights=pop, minlength=k)
        if p.min() >= lo and p.max() <= hi:
            return lab  # tree cuts leave every district connected
    raise RuntimeError(f"no plan within {percent:.0%} after {tries} tree draws")
