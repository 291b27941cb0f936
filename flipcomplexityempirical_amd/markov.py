"""GerryChain-shaped façade over the batched GPU flip walk.

The reference builds its chain from GerryChain plug-ins (grid_chain_sec11.py:299-342):

    updaters = {'population': Tally('population'), 'cut_edges': cut_edges,
                'b_nodes': b_nodes_bi, 'base': new_base, 'geom': geom_wait, ...}
    grid_partition = Partition(graph, assignment=cddict, updaters=updaters)
    popbound = within_percent_of_ideal_population(grid_partition, pop1)
    exp_chain = MarkovChain(slow_reversible_propose_bi,
                            Validator([single_flip_contiguous, popbound]),
                            accept=cut_accept, initial_state=grid_partition, total_steps=100000)
    for part in exp_chain: ...

The same code runs against this module: ``MarkovChain`` recognises the reference's
plug-ins (by identity, or by the GerryChain name of a user-defined function) and lowers
them to one GPU chain configuration; iteration yields ``Partition`` objects rebuilt on
the host from the kernel's per-step trace, with the reference's semantics (the initial
state first, one yield per counted step, the same object re-yielded after a Metropolis
rejection).  ``MarkovChain.run_batched`` runs ``n_chains`` independent copies instead.
Plug-ins that are not the reference's are refused (NotImplementedError): there is no
CPU fallback for the chain.
"""
from __future__ import annotations

import math
import random
from typing import Any, Callable, Dict, Hashable, Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from .chain import (DEFAULT_MAX_RETRIES, Chains, DeviceGraph, RunResult, annealing_table,
                    eval_flips, population_bounds, read_maps, reference_beta, schedule_rows)
from .graph import Graph, boundary_flags


# ===================================================================== Partition
class Partition:
    """Minimal gerrychain.Partition: assignment, parts, flips, parent, cached updaters."""

    def __init__(self, graph: Graph, assignment=None, updaters: Optional[Dict] = None,
                 parent: "Partition" = None, flips: Optional[Dict] = None, _labels=None,
                 _label_values=None):
        self.graph = graph
        if parent is None:
            if isinstance(assignment, dict):
                keys = graph.nodes
                vals = sorted({assignment[k] for k in keys})
                self._label_values = list(vals)
                idx = {v: i for i, v in enumerate(vals)}
                self._labels = np.array([idx[assignment[k]] for k in keys], np.int16)
            else:
                lab = np.asarray(assignment, np.int16)
                self._label_values = sorted(int(v) for v in np.unique(lab))
                remap = {v: i for i, v in enumerate(self._label_values)}
                self._labels = np.array([remap[int(v)] for v in lab], np.int16)
            self.updaters = dict(updaters or {})
            self.parent = None
            self.flips = None
        else:
            self._label_values = parent._label_values
            self._labels = parent._labels.copy() if _labels is None else _labels
            self.updaters = parent.updaters
            self.parent = parent
            self.flips = dict(flips)
            vidx = {v: i for i, v in enumerate(self._label_values)}
            nidx = graph.index()
            for node, lab in self.flips.items():
                self._labels[nidx[node]] = vidx[lab]
        self._cache: Dict[str, Any] = {}

    # --- gerrychain surface
    @property
    def assignment(self) -> Dict[Hashable, Any]:
        vals = self._label_values
        return {k: vals[int(l)] for k, l in zip(self.graph.nodes, self._labels)}

    @property
    def parts(self):
        return list(self._label_values)

    def __len__(self):
        return len(self._label_values)

    def flip(self, flips: Dict) -> "Partition":
        return Partition(self.graph, parent=self, flips=flips)

    def __getitem__(self, key: str):
        if key not in self._cache:
            self._cache[key] = self.updaters[key](self)
        return self._cache[key]

    # --- internal
    @property
    def labels(self) -> np.ndarray:
        """District index (0..k-1) per node id."""
        return self._labels


# ===================================================================== updaters
def cut_edges(partition: Partition):
    """gerrychain.updaters.cut_edges: set of (u, v) node-key pairs with differing labels."""
    g, lab = partition.graph, partition.labels
    e = g.edges()
    m = lab[e[:, 0]] != lab[e[:, 1]]
    nodes = g.nodes
    return {(nodes[a], nodes[b]) for a, b in e[m].tolist()}


class Tally:
    """gerrychain.updaters.Tally(field, alias): per-district sum of a node attribute."""

    def __init__(self, field: str = "population", alias: Optional[str] = None):
        self.field, self.alias = field, alias or field

    def __call__(self, partition: Partition):
        g = partition.graph
        if g.pop is not None:
            w = g.pop
        elif g.node_attrs is not None and self.field in (g.node_attrs[0] or {}):
            w = np.array([int(a[self.field]) for a in g.node_attrs], np.int64)
        else:
            w = np.ones(g.n, np.int64)
        sums = np.bincount(partition.labels, weights=w, minlength=len(partition))
        return {v: int(s) for v, s in zip(partition.parts, sums)}


def b_nodes_bi(partition: Partition):
    """grid_chain_sec11.py:155-156: endpoints of cut edges."""
    return {x for e in partition["cut_edges"] for x in e}


def b_nodes(partition: Partition):
    """grid_chain_sec11.py:151-153: (node, label of a cut-edge neighbour) pairs."""
    a = partition.assignment
    out = set()
    for x, y in partition["cut_edges"]:
        out.add((x, a[y]))
        out.add((y, a[x]))
    return out


def geom_wait(partition: Partition):
    """grid_chain_sec11.py:147-148 (numpy geometric draw, as the reference)."""
    p = len(list(partition["b_nodes"])) / (len(partition.graph.nodes) ** len(partition.parts) - 1)
    return int(np.random.geometric(p, 1)) - 1


def boundary_slope(partition: Partition, last: int = 39):
    """grid_chain_sec11.py:55-78 ("slope" updater): the cut edges that lie on the outer
    ring of the sec11 grid (both endpoints in row 0, column 0, row 39 or column 39) or
    are one of its four corner diagonals, as a list (of a set, as the reference)."""
    diag = {((0, 1), (1, 0)), ((0, last - 1), (1, last)), ((last - 1, 0), (last, 1)),
            ((last - 1, last), (last, last - 1))}
    diag |= {(b, a) for a, b in diag}
    out = set()
    for x in partition["cut_edges"]:
        if (x[0][0] == 0 and x[1][0] == 0) or (x[0][1] == 0 and x[1][1] == 0) or \
                (x[0][0] == last and x[1][0] == last) or (x[0][1] == last and x[1][1] == last) or \
                x in diag:
            out.add(x)
    return list(out)


def slope_and_angle(temp, centre=(20, 20)):
    """grid_chain_sec11.py:371-394: slope between the midpoints of the first two ring cut
    edges, and the angle they subtend at the grid centre (np.inf for a vertical pair)."""
    enda = ((temp[0][0][0] + temp[0][1][0]) / 2, (temp[0][0][1] + temp[0][1][1]) / 2)
    endb = ((temp[1][0][0] + temp[1][1][0]) / 2, (temp[1][0][1] + temp[1][1][1]) / 2)
    slope = (endb[1] - enda[1]) / (endb[0] - enda[0]) if endb[0] != enda[0] else np.inf
    anga = np.array((enda[0] - centre[0], enda[1] - centre[1]))
    angb = np.array((endb[0] - centre[0], endb[1] - centre[1]))
    angle = np.arccos(np.clip(np.dot(anga / np.linalg.norm(anga), angb / np.linalg.norm(angb)),
                              -1, 1))
    return slope, angle


# ===================================================================== proposals
def _not_direct(name):
    def f(partition):
        raise NotImplementedError(
            f"{name} is lowered to the GPU kernel by MarkovChain; it is not evaluated on the host")
    f.__name__ = name
    return f


propose_random_flip = _not_direct("propose_random_flip")
slow_reversible_propose = _not_direct("slow_reversible_propose")
slow_reversible_propose_bi = _not_direct("slow_reversible_propose_bi")

_PROPOSALS = {"propose_random_flip": _lib.PROPOSE_CUTEDGE,
              "slow_reversible_propose": _lib.PROPOSE_PAIRS,
              "slow_reversible_propose_bi": _lib.PROPOSE_BI}


# ===================================================================== constraints
class Bounds:
    """gerrychain.constraints.Bounds(func, bounds): lower <= min(values) and max <= upper."""

    def __init__(self, func: Callable, bounds):
        self.func, self.bounds = func, tuple(bounds)

    def __call__(self, partition: Partition) -> bool:
        vals = list(self.func(partition))
        return self.bounds[0] <= min(vals) and max(vals) <= self.bounds[1]


def within_percent_of_ideal_population(initial_partition: Partition, percent: float = 0.01,
                                       pop_key: str = "population") -> Bounds:
    """Bounds from the INITIAL plan: ideal = total / k, ((1-p) ideal, (1+p) ideal)."""
    pops = initial_partition[pop_key]
    ideal = sum(pops.values()) / len(pops)
    b = Bounds(lambda part: part[pop_key].values(), ((1 - percent) * ideal, (1 + percent) * ideal))
    b.percent, b.total, b.k = percent, sum(pops.values()), len(pops)
    return b


def single_flip_contiguous(partition: Partition) -> bool:
    """gerrychain.constraints.single_flip_contiguous, evaluated by the GPU eval kernel."""
    if partition.parent is None or not partition.flips:  # full check: every district
        return _all_contiguous(partition)
    parent = partition.parent
    nidx = partition.graph.index()
    vidx = {v: i for i, v in enumerate(partition._label_values)}
    vs = [nidx[n] for n in partition.flips]
    ts = [vidx[l] for l in partition.flips.values()]
    dg = _device_graph(partition.graph)
    _, contig, _, _ = eval_flips(dg, parent.labels, len(partition), vs, ts, (0, 2**62))
    return bool(contig.all())


def _all_contiguous(partition: Partition) -> bool:
    g, lab = partition.graph, partition.labels
    for d in range(len(partition)):
        nodes = np.flatnonzero(lab == d)
        if len(nodes) == 0:
            return False
        seen = {int(nodes[0])}
        stack = [int(nodes[0])]
        while stack:
            x = stack.pop()
            for y in g.neighbors(x):
                if lab[y] == d and int(y) not in seen:
                    seen.add(int(y))
                    stack.append(int(y))
        if len(seen) != len(nodes):
            return False
    return True


class Validator:
    """gerrychain.constraints.Validator: all constraints, in order, first False wins."""

    def __init__(self, constraints: Sequence[Callable]):
        self.constraints = list(constraints)

    def __call__(self, partition: Partition) -> bool:
        for c in self.constraints:
            r = c(partition)
            if r is False:
                return False
            if r is not True:
                raise TypeError(f"constraint {c} returned a non-boolean {r!r}")
        return True


# ===================================================================== accept
def cut_accept(partition: Partition) -> bool:
    """grid_chain_sec11.py:171-179: random() < base ** (len(parent cut) - len(cut))."""
    bound = 1
    if partition.parent is not None:
        bound = partition["base"] ** (-len(partition["cut_edges"]) +
                                      len(partition.parent["cut_edges"]))
    return random.random() < bound


def always_accept(partition: Partition) -> bool:
    return True


def annealing_cut_accept_backwards(partition: Partition) -> bool:
    """grid_chain_sec11.py:81-110 (base .1, beta 5): lowered to FW_ACCEPT_BRATIO."""
    raise NotImplementedError("annealing_cut_accept_backwards is lowered to the GPU kernel")


def uniform_accept(partition: Partition) -> bool:
    """grid_chain_sec11.py:159-165 (boundary_condition): lowered to FW_ACCEPT_BOUNDARY."""
    raise NotImplementedError("uniform_accept is lowered to the GPU kernel")


class AnnealingCutAccept:
    """annealing_cut_accept_backwards with explicit base / beta (the reference fixes
    base = .1, beta = 5): random() < base**(beta*(c_old - c_new)) * |B'| / |B|."""

    def __init__(self, base: float = 0.1, beta: float = 5, schedule=None):
        """``schedule`` = (beta_of_t, t_start, t_stop): beta as a function of
        partition["step_num"], constant outside [t_start, t_stop] — e.g.
        ``AnnealingCutAccept.reference_schedule()``, the reference's commented ramp."""
        self.base, self.beta, self.schedule = float(base), beta, schedule

    @classmethod
    def reference_schedule(cls, base: float = 0.1) -> "AnnealingCutAccept":
        """grid_chain_sec11.py:88-93: beta 0 until step 100,000, ramp to 3 at 400,000."""
        return cls(base, 3, (reference_beta, 100000, 400000))

    def __call__(self, partition: Partition) -> bool:
        raise NotImplementedError("AnnealingCutAccept is lowered to the GPU kernel")


class MetropolisCutAccept:
    """cut_accept with an explicit base (no 'base' updater needed)."""

    def __init__(self, base: float):
        self.base = float(base)

    def __call__(self, partition: Partition) -> bool:
        bound = 1
        if partition.parent is not None:
            bound = self.base ** (-len(partition["cut_edges"]) + len(partition.parent["cut_edges"]))
        return random.random() < bound


# ===================================================================== the chain
_DGRAPHS: Dict[int, DeviceGraph] = {}


def _device_graph(graph: Graph, device: int = 0) -> DeviceGraph:
    key = (id(graph), device)
    if key not in _DGRAPHS:
        _DGRAPHS[key] = DeviceGraph(graph, device)
    return _DGRAPHS[key]


def _fname(f) -> str:
    return getattr(f, "__name__", type(f).__name__)


class MarkovChain:
    """gerrychain.MarkovChain(proposal, constraints, accept, initial_state, total_steps)."""

    def __init__(self, proposal: Callable, constraints, accept: Callable,
                 initial_state: Partition, total_steps: int, *, seed: int = 0, device: int = 0,
                 chain_id: int = 0, chunk: int = 4096, max_retries: int = DEFAULT_MAX_RETRIES):
        self.initial_state = initial_state
        self.total_steps = int(total_steps)
        self.seed, self.device, self.chain_id = seed, device, chain_id
        self.chunk, self.max_retries = chunk, max_retries
        # ---- lower the plug-ins
        name = _fname(proposal)
        if name not in _PROPOSALS:
            raise NotImplementedError(f"proposal {name!r} is not one the GPU path implements")
        self.mode = _PROPOSALS[name]
        cons = constraints.constraints if isinstance(constraints, Validator) else (
            list(constraints) if isinstance(constraints, (list, tuple)) else [constraints])
        bounds = [c for c in cons if isinstance(c, Bounds)]
        others = [c for c in cons if not isinstance(c, Bounds)]
        if len(bounds) != 1 or len(others) != 1 or _fname(others[0]) != "single_flip_contiguous":
            raise NotImplementedError(
                "constraints must be [single_flip_contiguous, within_percent_of_ideal_population]")
        lo, hi = bounds[0].bounds
        self.pop_bounds = (int(math.ceil(lo)), int(math.floor(hi)))
        self.accept_rule, self.thr, self.flags = "cut", None, None
        self.schedule = None
        if isinstance(accept, MetropolisCutAccept):
            self.base = accept.base
        elif isinstance(accept, AnnealingCutAccept) or \
                _fname(accept) == "annealing_cut_accept_backwards":
            a = accept if isinstance(accept, AnnealingCutAccept) else AnnealingCutAccept()
            self.base, self.accept_rule = a.base, "bratio"
            self.thr = annealing_table(a.base, a.beta, initial_state.graph.maxdeg)
            if a.schedule is not None:
                fn, t_start, t_stop = a.schedule
                self.schedule = schedule_rows(a.base, fn, t_start, t_stop,
                                              initial_state.graph.maxdeg)
        elif _fname(accept) == "uniform_accept":
            # boundary_condition reads partition["boundary"] (grid_chain_sec11.py:44), the
            # boundary_node nodes; without that updater the graph's attribute is used
            self.base, self.accept_rule = 1.0, "boundary"
            g = initial_state.graph
            if "boundary" in initial_state.updaters:
                idx = g.index()
                self.flags = np.zeros(g.n, np.uint8)
                self.flags[[idx[x] for x in initial_state["boundary"]]] = 1
            else:
                self.flags = boundary_flags(g)
        elif _fname(accept) == "always_accept":
            self.base = 1.0
        elif _fname(accept) == "cut_accept":
            if "base" not in initial_state.updaters:
                raise ValueError("cut_accept reads partition['base']: add a 'base' updater")
            self.base = float(initial_state["base"])
        else:
            raise NotImplementedError(f"accept {_fname(accept)!r} is not one the GPU path implements")
        self.k = len(initial_state)
        self.graph = initial_state.graph
        # GerryChain raises ValueError for an invalid initial state (Chains does too)
        self._chains: Optional[Chains] = None

    def _make(self, n_chains=1, chain_id0=None) -> Chains:
        dg = _device_graph(self.graph, self.device)
        ch = Chains(dg, n_chains, self.k, self.initial_state.labels, proposal=self.mode,
                    pop_bounds=self.pop_bounds, base=self.base, seed=self.seed,
                    chain_id0=self.chain_id if chain_id0 is None else chain_id0, thr=self.thr)
        if self.accept_rule != "cut":
            ch.set_accept(self.accept_rule, self.flags)
        if self.schedule is not None:
            ch.set_schedule(*self.schedule)
        return ch

    def __iter__(self):
        ch = self._make()
        state = self.initial_state
        yield state
        remaining = self.total_steps - 1
        vals = state._label_values
        nodes = self.graph.nodes
        while remaining > 0:
            s = min(self.chunk, remaining)
            tr = ch.run_traced(s, self.max_retries)[0]
            for code in tr:
                if code < -1:
                    raise RuntimeError("chain stuck: no valid proposal within max_retries")
                # GerryChain's MarkovChain erases the current state's parent link once the
                # next proposal exists, so a yielded state's grandparent is None and the
                # chain's history is not kept alive (a re-yielded state loses its parent)
                prev = state
                if code >= 0:
                    v, d = divmod(int(code), 64)
                    state = state.flip({nodes[v]: vals[d]})
                prev.parent = None
                yield state
            remaining -= s
        ch.close()

    def __len__(self):
        return self.total_steps

    def run_batched(self, n_chains: int, chain_id0: int = 0, maps: bool = False,
                    waits: bool = False) -> RunResult:
        """n_chains independent copies for total_steps yields each (no per-state objects).

        ``maps`` adds the driver's spatial observables per chain, keyed by node / edge
        index (grid_chain_sec11.py:383-400, finalised as :416-419), with the initial
        partition's own label values (e.g. -1/+1) in part_sum.  ``waits`` adds the sampled
        sum(waits) of each chain (geom_wait, :147-148, written at :410-411), the value the
        reference's wait.txt holds.
        """
        ch = self._make(n_chains, chain_id0)
        if maps:
            ch.enable_maps(np.asarray(self.initial_state._label_values, np.int64))
        if waits:
            ch.enable_sampled_waits()
        ch.run(self.total_steps - 1, self.max_retries)
        res = RunResult(ch.labels(), ch.stats(), ch.hist_cut(), ch.hist_b(), ch.pops(),
                        ch.last_kernel_ms(), read_maps(ch) if maps else None,
                        ch.sampled_waits() if waits else None)
        ch.close()
        return res
