"""TEST INFRASTRUCTURE ONLY — GerryChain-equivalent Python proxy of the reference chain.

GerryChain (the library that owns the reference's hot loop) is not vendored in
/root/reference and is not installed, so it cannot be run here or on the GPU box.
This module restates, in plain Python over networkx, the same per-proposal work
classes the reference performs, so that it can be timed as the "reference CPU
path" (bench.py cpu_baseline, kind "port") and used as an independent second
implementation of the chain semantics:

* ``Partition.flip``  — O(N) assignment-dict copy per proposal, parent link, flips
  (gerrychain.Partition [ext]; called grid_chain_sec11.py:145)
* ``cut_edges``       — incremental set update (parent cut set | new - obsolete)
  (gerrychain.updaters.cut_edges [ext], registered grid_chain_sec11.py:302)
* ``Tally``           — incremental district populations (grid_chain_sec11.py:299)
* ``b_nodes_bi`` / ``b_nodes`` — endpoint / (node, foreign label) sets rebuilt from
  the cut set (grid_chain_sec11.py:151-156)
* proposals           — ``random.choice(list(b_nodes))`` (grid_chain_sec11.py:128,143) and
  ``propose_random_flip`` [ext]; the draw is the canonical Philox mapping of
  include/flipwalk.h over the SORTED set (the reference's unseeded MT19937 +
  set-iteration order cannot be replayed)
* ``single_flip_contiguous`` — networkx Dijkstra from each old-district neighbour
  with a weight function that hides edges whose endpoints differ
  (gerrychain.constraints [ext], grid_chain_sec11.py:340)
* ``within_percent_of_ideal_population`` — float bounds from the initial plan
  (grid_chain_sec11.py:319)
* ``cut_accept``      — random() < base**(c_old - c_new) (grid_chain_sec11.py:171-179)
* ``MarkovChain``     — retry invalid proposals uncounted; count and yield valid ones
  (gerrychain.MarkovChain [ext], grid_chain_sec11.py:340-342,366)
* per-yield observables rce / rbn / waits (grid_chain_sec11.py:367-369)

With the same seed it follows the same trajectory as oracle/flipchain_oracle.c and
the HIP path (tests/test_oracle.py::test_proxy_follows_the_same_trajectory checks this).
"""
from __future__ import annotations

import math
import time

import networkx as nx

MASK32 = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & MASK32
            k1 = (k1 + 0xBB67AE85) & MASK32
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0, p1 & MASK32, (p0 >> 32) ^ c3 ^ k1, p0 & MASK32)
    return c0, c1, c2, c3


class PhiloxStream:
    """One Philox block per proposal attempt (include/flipwalk.h, 'Randomness')."""

    def __init__(self, seed, chain_id):
        self.k0, self.k1 = seed & MASK32, (seed >> 32) & MASK32
        self.g0, self.g1 = chain_id & MASK32, (chain_id >> 32) & MASK32
        self.attempt = 0
        self.block = None

    def next_block(self):
        t = self.attempt
        self.block = philox4x32_10(t & MASK32, (t >> 32) & MASK32, self.g0, self.g1, self.k0,
                                   self.k1)
        self.attempt += 1
        return self.block

    def index(self, size):
        x0, x1 = self.block[0], self.block[1]
        return (((x1 << 32) | x0) * size) >> 64

    def random(self):
        x2, x3 = self.block[2], self.block[3]
        return ((x2 >> 5) * 67108864.0 + (x3 >> 6)) * (1.0 / 9007199254740992.0)


class Partition:
    """Minimal gerrychain.Partition: assignment copy on flip, cached updaters."""

    def __init__(self, graph, assignment=None, updaters=None, parent=None, flips=None):
        self.graph = graph
        if parent is None:
            self.assignment = dict(assignment)
            self.updaters = updaters
            self.parent = None
            self.flips = None
        else:
            self.assignment = dict(parent.assignment)  # O(N) copy, as GerryChain does
            self.assignment.update(flips)
            self.updaters = parent.updaters
            self.parent = parent
            self.flips = flips
        self.parts = sorted(set(self.assignment.values()))
        self._cache = {}

    def flip(self, flips):
        return Partition(self.graph, parent=self, flips=flips)

    def __getitem__(self, key):
        if key not in self._cache:
            self._cache[key] = self.updaters[key](self)
        return self._cache[key]

    def __len__(self):
        return len(self.parts)


# ------------------------------------------------------------------ updaters
def cut_edges(partition):
    parent = partition.parent
    a = partition.assignment
    if parent is None:
        return {tuple(sorted(e)) for e in partition.graph.edges if a[e[0]] != a[e[1]]}
    cut = set(parent["cut_edges"])
    for node in partition.flips:
        for nb in partition.graph.neighbors(node):
            e = (node, nb) if node < nb else (nb, node)
            if a[node] != a[nb]:
                cut.add(e)
            else:
                cut.discard(e)
    return cut


def population(partition):
    parent = partition.parent
    if parent is None:
        tot = {}
        for v, d in partition.assignment.items():
            tot[d] = tot.get(d, 0) + partition.graph.nodes[v]["population"]
        return tot
    tot = dict(parent["population"])
    for v, d in partition.flips.items():
        p = partition.graph.nodes[v]["population"]
        tot[parent.assignment[v]] -= p
        tot[d] = tot.get(d, 0) + p
    return tot


def b_nodes_bi(partition):
    return {x[0] for x in partition["cut_edges"]}.union({x[1] for x in partition["cut_edges"]})


def b_nodes(partition):
    a = partition.assignment
    return {(x[0], a[x[1]]) for x in partition["cut_edges"]}.union(
        {(x[1], a[x[0]]) for x in partition["cut_edges"]})


def step_num(partition):
    """grid_chain_sec11.py:282-289: 0 for the initial plan, else the parent's + 1."""
    parent = partition.parent
    if not parent:
        return 0
    return parent["step_num"] + 1


UPDATERS = {"cut_edges": cut_edges, "population": population, "b_nodes_bi": b_nodes_bi,
            "b_nodes": b_nodes, "step_num": step_num}


# ----------------------------------------------------------------- proposals
def propose_pairs(partition, rng):
    """slow_reversible_propose, grid_chain_sec11.py:117-130.  For k=2 the (node, label)
    pairs and the boundary nodes of slow_reversible_propose_bi coincide."""
    pairs = sorted(partition["b_pairs"])
    node, label = pairs[rng.index(len(pairs))]
    return partition.flip({node: label})


def propose_cutedge(partition, rng):
    """gerrychain propose_random_flip: uniform cut edge, uniform endpoint."""
    directed = sorted([(u, v) for (u, v) in partition["cut_edges"]] +
                      [(v, u) for (u, v) in partition["cut_edges"]])
    v, u = directed[rng.index(len(directed))]
    return partition.flip({v: partition.assignment[u]})


# --------------------------------------------------------------- constraints
def single_flip_contiguous(partition):
    """gerrychain.constraints.single_flip_contiguous (0.2.x behaviour)."""
    graph = partition.graph
    assignment = partition.assignment

    def edge_avoid(u, v, attrs):
        return None if assignment[u] != assignment[v] else 1

    for changed in partition.flips:
        old = partition.parent.assignment[changed]
        old_neighbors = [n for n in graph.neighbors(changed) if assignment[n] == old]
        if not old_neighbors:
            return False
        start = old_neighbors[0]
        for nb in old_neighbors[1:]:
            try:
                nx.multi_source_dijkstra(graph, [nb], target=start, weight=edge_avoid)
            except nx.NetworkXNoPath:
                return False
    return True


class PopBound:
    """within_percent_of_ideal_population(initial, percent) -> Bounds."""

    def __init__(self, initial, percent):
        pops = initial["population"]
        ideal = sum(pops.values()) / len(pops)
        self.lo = (1 - percent) * ideal
        self.hi = (1 + percent) * ideal

    def __call__(self, partition):
        vals = partition["population"].values()
        return self.lo <= min(vals) and max(vals) <= self.hi


# ----------------------------------------------------------------- accept rules
def annealing_cut_accept_bound(partition, base, beta):
    """annealing_cut_accept_backwards, grid_chain_sec11.py:81-110 (its bound; the Validator
    already enforced its inline popbound / single_flip_contiguous checks).  A callable
    ``beta`` is the commented schedule (:85-93): beta = beta(partition["step_num"])."""
    t = partition["step_num"]
    if callable(beta):
        beta = beta(t)
    boundaries1 = {x[0] for x in partition["cut_edges"]}.union(
        {x[1] for x in partition["cut_edges"]})
    boundaries2 = {x[0] for x in partition.parent["cut_edges"]}.union(
        {x[1] for x in partition.parent["cut_edges"]})
    return (base ** (beta * (-len(partition["cut_edges"]) + len(partition.parent["cut_edges"])))
            ) * (len(boundaries1) / len(boundaries2))


def boundary_condition(partition, blist):
    """grid_chain_sec11.py:43-52 over blist = partition["boundary"] (boundary_node == 1)."""
    o_part = partition.assignment[blist[0]]
    for x in blist:
        if partition.assignment[x] != o_part:
            return True
    return False


# ----------------------------------------------------------------- the chain
class ProxyChain:
    """MarkovChain with cut_accept; yields (state, observables) per counted step."""

    def __init__(self, graph_csr, labels, k, mode, percent, base, seed, chain_id,
                 pop=None, accept="cut", beta=1, flags=None):
        G = nx.Graph()
        n = graph_csr.n
        pops = graph_csr.pop_array() if pop is None else pop
        for v in range(n):
            G.add_node(v, population=int(pops[v]))
        for u, v in graph_csr.edges():
            G.add_edge(int(u), int(v))
        self.graph = G
        self.mode = mode
        self.k = k
        upd = dict(UPDATERS)
        upd["b_nodes"] = b_nodes_bi if mode == 0 else b_nodes
        upd["b_pairs"] = b_nodes
        self.state = Partition(G, {v: int(labels[v]) for v in range(n)}, upd)
        self.popbound = PopBound(self.state, percent) if percent is not None else None
        self.base = base
        self.rng = PhiloxStream(seed, chain_id)
        self.propose = propose_cutedge if mode == 2 else propose_pairs
        self.counters = dict(attempts=0, steps=0, accepts=0, pop_fail=0, contig_fail=0)
        self.obs = dict(yields=0, sum_cut=0, sum_bnodes=0, sum_invb=0.0)
        self.n = n
        self.accept, self.beta = accept, beta
        self.blist = None if flags is None else [v for v in range(n) if flags[v]]

    def _yield(self):
        s = self.state
        c = len(s["cut_edges"])
        b = len(s["b_nodes_bi"])
        self.obs["yields"] += 1
        self.obs["sum_cut"] += c
        self.obs["sum_bnodes"] += b
        self.obs["sum_invb"] += 1.0 / b

    def run(self, steps, max_retries=1 << 20, bounds=None):
        """Advance by ``steps`` counted steps; ``bounds`` overrides (lo, hi) ints."""
        if self.obs["yields"] == 0:
            self._yield()
        C = self.counters
        for _ in range(steps):
            retries = 0
            while True:
                if retries >= max_retries:
                    raise RuntimeError("stuck: no valid proposal")
                self.rng.next_block()
                C["attempts"] += 1
                proposed = self.propose(self.state, self.rng)
                self.state.parent = None  # MarkovChain erases the parent's parent
                if bounds is not None:
                    vals = proposed["population"].values()
                    pop_ok = bounds[0] <= min(vals) and max(vals) <= bounds[1]
                else:
                    pop_ok = self.popbound(proposed)
                if not pop_ok:
                    C["pop_fail"] += 1
                    retries += 1
                    continue
                if not single_flip_contiguous(proposed):
                    C["contig_fail"] += 1
                    retries += 1
                    continue
                break
            C["steps"] += 1
            if self.accept == "bratio":
                bound = annealing_cut_accept_bound(proposed, self.base, self.beta)
            elif self.accept == "boundary":  # uniform_accept, grid_chain_sec11.py:159-165
                bound = 1 if boundary_condition(proposed, self.blist) else 0
            else:  # cut_accept, grid_chain_sec11.py:171-179
                bound = self.base ** (-len(proposed["cut_edges"]) +
                                      len(proposed.parent["cut_edges"]))
            if self.rng.random() < bound:
                C["accepts"] += 1
                self.state = proposed
            self._yield()

    def labels(self):
        return [self.state.assignment[v] for v in range(self.n)]


def time_steps(graph_csr, labels, k, mode, percent, base, seed, chain_id, steps,
               bounds=None):
    """Wall time of ``steps`` counted steps of one proxy chain (for cpu_baseline)."""
    ch = ProxyChain(graph_csr, labels, k, mode, percent, base, seed, chain_id)
    t0 = time.perf_counter()
    ch.run(steps, bounds=bounds)
    return time.perf_counter() - t0, ch
