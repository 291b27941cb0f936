"""Batched flip-walk chains on MI355X (host side of the drop-in boundary).

``Chains`` is the batched form of the reference's

    MarkovChain(slow_reversible_propose_bi, Validator([single_flip_contiguous, popbound]),
                accept=cut_accept, initial_state=grid_partition, total_steps=100000)

(grid_chain_sec11.py:340-342): thousands of independent chains, one per Philox
stream, advanced by the HIP kernel through the C-ABI.  Host-side numerics that
the kernels take as inputs are computed here exactly as the reference computes
them in Python:

* ``population_bounds`` — ``within_percent_of_ideal_population`` (grid_chain_sec11.py:319):
  ideal = sum(pops)/k, (1-p)*ideal <= pop <= (1+p)*ideal with Python floats, turned
  into the equivalent integer interval [ceil(lo), floor(hi)].
* ``metropolis_table`` — ``cut_accept`` (grid_chain_sec11.py:171-179): bound =
  base ** (len(parent cut) - len(cut)) = base ** (-Δcut) with Python's float pow.
"""
from __future__ import annotations

import math
import warnings
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import STATS_DTYPE, check, ptr
from .graph import Graph

DEFAULT_MAX_RETRIES = 1 << 20

PROPOSALS = {"bi": _lib.PROPOSE_BI, "pairs": _lib.PROPOSE_PAIRS, "cutedge": _lib.PROPOSE_CUTEDGE}


def population_bounds(total_pop: int, k: int, percent: float):
    """Integer bounds equivalent to GerryChain's Bounds((1-p)*ideal, (1+p)*ideal)."""
    ideal = total_pop / k
    lo = (1 - percent) * ideal
    hi = (1 + percent) * ideal
    return int(math.ceil(lo)), int(math.floor(hi))


def metropolis_table(base: float, maxdeg: int) -> np.ndarray:
    """thr[d + maxdeg] = base ** (-d): cut_accept's bound for Δcut = d."""
    b = float(base)
    return np.array([b ** (-d) for d in range(-maxdeg, maxdeg + 1)], dtype=np.float64)


def annealing_table(base: float, beta: float, maxdeg: int) -> np.ndarray:
    """thr[d + maxdeg] = base ** (beta * (-d)): the power of annealing_cut_accept_backwards
    (grid_chain_sec11.py:101), base**(beta*(-len(cut)+len(parent cut))), for Δcut = d."""
    b = float(base)
    return np.array([b ** (beta * (-d)) for d in range(-maxdeg, maxdeg + 1)], dtype=np.float64)


def reference_beta(t: int):
    """The commented beta schedule of annealing_cut_accept_backwards
    (grid_chain_sec11.py:88-93) at step_num t: 0 before 100,000, a linear ramp to 3 at
    400,000, then 3 (Python int / float values as the reference writes them)."""
    if t < 100000:
        return 0
    if t < 400000:
        return (t - 100000) / 100000
    return 3


def schedule_rows(base: float, beta_of_t, t_start: int, t_stop: int,
                  maxdeg: int) -> tuple[np.ndarray, int]:
    """Rows for ``Chains.set_schedule``: row i = annealing_table(base, beta_of_t(t_start+i))
    for step_num t_start..t_stop; returns (rows, t0 = t_start).  Exact when beta_of_t is
    constant for t <= t_start and for t >= t_stop (the kernel clamps to the end rows).
    Each power is CPython's float pow, as in the reference."""
    rows = np.empty((t_stop - t_start + 1, 2 * maxdeg + 1), np.float64)
    cache = {}
    for i in range(rows.shape[0]):
        beta = beta_of_t(t_start + i)
        key = (type(beta), beta)
        if key not in cache:
            cache[key] = annealing_table(base, beta, maxdeg)
        rows[i] = cache[key]
    return rows, t_start


ACCEPT_RULES = {"cut": _lib.ACCEPT_CUT, "bratio": _lib.ACCEPT_BRATIO,
                "boundary": _lib.ACCEPT_BOUNDARY}


def expected_wait_sum(stats, n_nodes: int, k: int) -> np.ndarray:
    """Σ_t E[geom_wait_t] = (N^k - 1) * Σ 1/|B_t| - T (geom_wait, grid_chain_sec11.py:147-148)."""
    M = float(n_nodes ** k - 1)
    return M * stats["sum_invb"] - stats["yields"].astype(np.float64)


def wait_prob_table(n_nodes: int, k: int) -> np.ndarray:
    """p_b = len(b_nodes) / (N**k - 1) for every boundary size b = 0..N, divided as
    geom_wait divides (grid_chain_sec11.py:148: Python int / int, correctly rounded)."""
    M = int(n_nodes) ** int(k) - 1
    return np.array([b / M for b in range(int(n_nodes) + 1)], np.float64)


def write_wait_txt(path: str, wait_sum: float) -> None:
    """The reference's only text output (grid_chain_sec11.py:410-411):
    ``wfile.write(str(sum(waits)))``.  ``wait_sum`` is either the sampled sum
    (``Chains.sampled_waits``, the reference's own kind of value: a sum of integer draws)
    or the Rao-Blackwellised expectation (expected_wait_sum), written as the nearest
    integer."""
    with open(path, "w") as f:
        f.write(str(int(round(float(wait_sum)))))


class DeviceGraph:
    """A CSR graph uploaded to one HIP device (fw_graph)."""

    def __init__(self, graph: Graph, device: int = 0):
        L = _lib.require_device()
        self.graph = graph
        self.device = device
        h = _lib.ctypes.c_void_p()
        rowptr = np.ascontiguousarray(graph.rowptr, np.int32)
        col = np.ascontiguousarray(graph.col, np.int32)
        pop = None if graph.pop is None else np.ascontiguousarray(graph.pop, np.int64)
        check(L.fw_graph_create(ptr(rowptr), ptr(col), ptr(pop), graph.n, len(col), device,
                                _lib.ctypes.byref(h)))
        self._h = h
        info = np.zeros(5, np.int64)
        check(L.fw_graph_info(self._h, ptr(info)))
        self.n, self.n_edges, self.maxdeg, self.grid_w, self.grid_h = (int(x) for x in info)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().fw_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Chains:
    """n_chains independent flip walks resident on one device (fw_chains)."""

    def __init__(self, dgraph: DeviceGraph, n_chains: int, k: int, init_labels,
                 proposal: str | int = "pairs", pop_bounds=None, percent: float = 0.05,
                 base: float | Sequence[float] = 1.0, seed: int = 0, chain_id0: int = 0,
                 thr: Optional[np.ndarray] = None):
        L = _lib.require_device()
        self.dgraph = dgraph
        g = dgraph.graph
        self.n_chains, self.k = int(n_chains), int(k)
        self.mode = PROPOSALS[proposal] if isinstance(proposal, str) else int(proposal)
        lab = np.ascontiguousarray(init_labels, np.int16)
        if lab.ndim == 2 and lab.shape[0] not in (1, n_chains):
            raise ValueError(f"init_labels has {lab.shape[0]} rows: need 1 or n_chains={n_chains}")
        if lab.ndim not in (1, 2) or lab.shape[-1] != g.n:
            raise ValueError(f"init_labels must be [{g.n}] or [rows, {g.n}], got {lab.shape}")
        per_chain = 1 if lab.ndim == 2 and lab.shape[0] == n_chains and n_chains > 1 else 0
        if lab.ndim == 2 and not per_chain:
            lab = np.ascontiguousarray(lab[0])
        if pop_bounds is None:
            pop_bounds = population_bounds(g.total_pop, k, percent)
        self.pop_lo, self.pop_hi = int(pop_bounds[0]), int(pop_bounds[1])
        D = dgraph.maxdeg
        if thr is not None:  # an explicit bound table [2*maxdeg+1] or [n_chains][2*maxdeg+1]
            thr = np.asarray(thr, np.float64)
            thr_per = 1 if thr.ndim == 2 else 0
        elif np.ndim(base) == 0:
            thr = metropolis_table(float(base), D)
            thr_per = 0
        else:
            bases = np.asarray(base, np.float64)
            if len(bases) != n_chains:
                raise ValueError("per-chain bases need one base per chain")
            thr = np.stack([metropolis_table(float(b), D) for b in bases])
            thr_per = 1
        self.thr = np.ascontiguousarray(thr)
        self.seed, self.chain_id0 = int(seed), int(chain_id0)
        # the configuration a checkpoint must carry besides the state (set_accept,
        # set_schedule change it after creation)
        self.accept_rule, self.node_flags = _lib.ACCEPT_CUT, None
        self._sched, self._sched_t0 = None, 0
        self.waits_on = False
        h = _lib.ctypes.c_void_p()
        check(L.fw_chains_create(dgraph.handle, self.n_chains, self.k, ptr(lab), per_chain,
                                 self.mode, self.pop_lo, self.pop_hi, ptr(self.thr), thr_per,
                                 self.seed & (2**64 - 1), self.chain_id0, _lib.ctypes.byref(h)))
        self._h = h

    # ------------------------------------------------------------- stepping
    def run(self, steps: int, max_retries: int = DEFAULT_MAX_RETRIES) -> None:
        check(_lib.load().fw_chains_run(self._h, int(steps), int(max_retries)))

    def run_async(self, steps: int, max_retries: int = DEFAULT_MAX_RETRIES) -> None:
        check(_lib.load().fw_chains_run_async(self._h, int(steps), int(max_retries)))

    def sync(self) -> None:
        check(_lib.load().fw_chains_sync(self._h))

    def run_traced(self, steps: int, max_retries: int = DEFAULT_MAX_RETRIES) -> np.ndarray:
        tr = np.empty((self.n_chains, int(steps)), np.int32)
        check(_lib.load().fw_chains_run_traced(self._h, int(steps), int(max_retries), ptr(tr),
                                               tr.nbytes))
        return tr

    def last_kernel_ms(self) -> float:
        return float(_lib.load().fw_chains_last_kernel_ms(self._h))

    def launch_info(self) -> dict:
        """The launch plan (fw_chains_launch_info) and the residency it gives: waves per SIMD
        and chains per CU of the persistent grid (4 SIMDs per CU)."""
        info = np.zeros(8, np.int64)
        check(_lib.load().fw_chains_launch_info(self._h, ptr(info)))
        wgs, nw, cpw, lds, vgpr, scratch, cus, per_cu = (int(x) for x in info)
        resident = min(wgs, per_cu * cus)
        return {"workgroups": wgs, "waves_per_workgroup": nw, "chains_per_wave": cpw,
                "lds_bytes_per_workgroup": lds, "vgprs": vgpr, "scratch_bytes_per_lane": scratch,
                "cus": cus, "workgroups_per_cu": per_cu,
                "waves_per_simd_limit": per_cu * nw / 4.0,
                "waves_per_simd": resident * nw / (4.0 * cus),
                "chains_per_cu": resident * nw * cpw / cus}

    def reset_observables(self) -> None:
        check(_lib.load().fw_chains_reset_observables(self._h))

    # ------------------------------------------------------------- reading
    def _read(self, what, arr):
        check(_lib.load().fw_chains_read(self._h, what, ptr(arr), arr.nbytes))
        return arr

    def labels(self) -> np.ndarray:
        return self._read(_lib.READ_LABELS, np.empty((self.n_chains, self.dgraph.n), np.int16))

    def stats(self) -> np.ndarray:
        return self._read(_lib.READ_STATS, np.empty(self.n_chains, STATS_DTYPE))

    def hist_cut(self) -> np.ndarray:
        return self._read(_lib.READ_HIST_CUT, np.empty(self.dgraph.n_edges + 1, np.uint64))

    def hist_b(self) -> np.ndarray:
        return self._read(_lib.READ_HIST_B, np.empty(self.dgraph.n + 1, np.uint64))

    def pops(self) -> np.ndarray:
        return self._read(_lib.READ_POPS, np.empty((self.n_chains, self.k), np.int64))

    def set_accept(self, rule: str | int, node_flags=None) -> None:
        """Accept rule: "cut" (cut_accept), "bratio" (annealing_cut_accept_backwards' |B'|/|B|
        factor on the tabulated power) or "boundary" (uniform_accept + boundary_condition
        over ``node_flags``, the boundary_node attribute); see include/flipwalk.h."""
        r = ACCEPT_RULES[rule] if isinstance(rule, str) else int(rule)
        fl = None if node_flags is None else np.ascontiguousarray(node_flags, np.uint8)
        check(_lib.load().fw_chains_set_accept(self._h, r, ptr(fl)))
        self.accept_rule, self.node_flags = r, fl

    def set_schedule(self, rows=None, t0: int = 0) -> None:
        """Step-dependent bounds shared by every chain (fw_chains_set_schedule): a proposal
        with step_num t (accepted flips + 1, grid_chain_sec11.py:282-289) uses row
        clamp(t - t0, 0, len(rows) - 1) in place of the thr table.  ``rows=None`` removes
        it.  See ``schedule_rows``."""
        if rows is None:
            check(_lib.load().fw_chains_set_schedule(self._h, None, 0, 0))
            self._sched, self._sched_t0 = None, 0
            return
        r = np.ascontiguousarray(rows, np.float64)
        if r.ndim != 2 or r.shape[1] != self.thr.shape[-1]:
            raise ValueError(f"schedule rows must be [n][{self.thr.shape[-1]}]")
        check(_lib.load().fw_chains_set_schedule(self._h, ptr(r), r.shape[0], int(t0)))
        self._sched, self._sched_t0 = r, int(t0)

    # ------------------------------------------------------------- sampled waits
    def enable_sampled_waits(self) -> None:
        """Draw geom_wait per state object (grid_chain_sec11.py:147-148, cached and re-used
        on re-yield) and sum it over yields (:368, :410-411); see fw_chains_enable_waits.
        Call before the first run."""
        pt = np.ascontiguousarray(wait_prob_table(self.dgraph.n, self.k))
        check(_lib.load().fw_chains_enable_waits(self._h, ptr(pt)))
        self.waits_on = True

    def waits(self) -> np.ndarray:
        """float64 [n_chains, 2]: {sum of the sampled waits over yields, the current
        state's draw}."""
        return self._read(_lib.READ_WAITS, np.empty((self.n_chains, 2), np.float64))

    def sampled_waits(self) -> np.ndarray:
        """Per chain, sum(waits) of grid_chain_sec11.py:410 (integer-valued floats)."""
        return self.waits()[:, 0].copy()

    # ------------------------------------------------------------- district shapes
    def enable_ring(self, ring_u, ring_w) -> None:
        """Count yields per pair of first two cut ring edges (boundary_slope and the
        driver's slope / angle, grid_chain_sec11.py:55-78,371-394); ``shape.ring_edges``
        builds the ring of a graph from the reference's predicates.  Zeroes the histogram.

        Parity holds for plans whose cut crosses the ring at most twice (k = 2 with both
        districts connected: the reference's sec11 and Frankenstein runs).  With more
        crossings the reference picks temp[0], temp[1] of ``list(set(...))`` (hash order),
        this handle the first two in ring order, so k > 2 shape histograms are not
        comparable with the reference's; a RuntimeWarning says so."""
        if self.k > 2:
            warnings.warn(f"enable_ring with k = {self.k}: plans can cut the ring more than "
                          "twice, where the pair kept (first two in ring order) differs from "
                          "the reference's set-order pick; shape parity holds for k = 2 only",
                          RuntimeWarning, stacklevel=2)
        u = np.ascontiguousarray(ring_u, np.int32)
        w = np.ascontiguousarray(ring_w, np.int32)
        if u.shape != w.shape or u.ndim != 1:
            raise ValueError("ring_u and ring_w must be equal-length 1-D arrays")
        check(_lib.load().fw_chains_enable_ring(self._h, ptr(u), ptr(w), len(u)))
        self.ring = (u, w)

    def hist_ring(self) -> np.ndarray:
        """uint64 [R*R+1]: yields per ring pair (i*R + j, i < j); [R*R]: fewer than two."""
        R = len(self.ring[0])
        return self._read(_lib.READ_HIST_RING, np.empty(R * R + 1, np.uint64))

    def ring_pairs(self) -> np.ndarray:
        """int32 [n_chains, 2]: each chain's current first two cut ring edges (-1: none)."""
        return self._read(_lib.READ_RING_PAIR, np.empty((self.n_chains, 2), np.int32))

    # ------------------------------------------------------------- checkpoint / resume
    def checkpoint(self) -> dict:
        """Everything a resumed chain needs: plans, the stats records (with the Philox
        attempt counter: the counter-based RNG makes resume exact) and the histograms."""
        ck = {"labels": self.labels(), "stats": self.stats(), "hist_cut": self.hist_cut(),
              "hist_b": self.hist_b(), "seed": np.uint64(self.seed),
              "chain_id0": np.int64(self.chain_id0), "thr": self.thr,
              "mode": np.int32(self.mode), "accept_rule": np.int32(self.accept_rule),
              "pop_lo": np.int64(self.pop_lo), "pop_hi": np.int64(self.pop_hi)}
        if self.node_flags is not None:
            ck["node_flags"] = self.node_flags
        if self._sched is not None:
            ck["sched_rows"], ck["sched_t0"] = self._sched, np.int64(self._sched_t0)
        if self.waits_on:
            ck["waits"] = self.waits()
        if getattr(self, "ring", None) is not None:
            ck["hist_ring"] = self.hist_ring()
            ck["ring_u"], ck["ring_w"] = self.ring
        return ck

    def restore(self, ck: dict) -> None:
        """Load a ``checkpoint`` into this handle (same graph, chain count, seed and chain
        ids): the chains continue exactly where the checkpointed ones stopped."""
        if int(ck["seed"]) != self.seed or int(ck["chain_id0"]) != self.chain_id0:
            raise ValueError("checkpoint of another seed / chain-id range")
        if "mode" in ck and int(ck["mode"]) != self.mode:
            raise ValueError(f"checkpoint of proposal mode {int(ck['mode'])}, handle has "
                             f"{self.mode}")
        if "pop_lo" in ck and (int(ck["pop_lo"]), int(ck["pop_hi"])) != (self.pop_lo, self.pop_hi):
            raise ValueError(f"checkpoint of population bounds [{int(ck['pop_lo'])}, "
                             f"{int(ck['pop_hi'])}], handle has [{self.pop_lo}, {self.pop_hi}]")
        if self.waits_on and "waits" not in ck:
            raise ValueError("sampled waits are enabled but the checkpoint carries none: the "
                             "resumed sums would miss every earlier yield")
        L = _lib.load()
        if "waits" in ck and not self.waits_on:
            self.enable_sampled_waits()
        for what, key in ((_lib.READ_LABELS, "labels"), (_lib.READ_STATS, "stats"),
                          (_lib.READ_HIST_CUT, "hist_cut"), (_lib.READ_HIST_B, "hist_b")):
            a = np.ascontiguousarray(ck[key])
            if key == "stats":
                a = np.ascontiguousarray(a, STATS_DTYPE)
                if a.shape != (self.n_chains,):
                    raise ValueError("checkpoint of another chain count")
            check(L.fw_chains_write(self._h, what, ptr(a), a.nbytes))
        if "waits" in ck:
            a = np.ascontiguousarray(ck["waits"], np.float64)
            check(L.fw_chains_write(self._h, _lib.READ_WAITS, ptr(a), a.nbytes))
        if "hist_ring" in ck:
            self.enable_ring(ck["ring_u"], ck["ring_w"])
            a = np.ascontiguousarray(ck["hist_ring"], np.uint64)
            check(L.fw_chains_write(self._h, _lib.READ_HIST_RING, ptr(a), a.nbytes))
        # the accept rule and the bound schedule the checkpointed chains ran under (after the
        # plans: the boundary rule's flagged-node counts are taken from them)
        if "accept_rule" in ck:
            rule, fl = int(ck["accept_rule"]), ck.get("node_flags")
            same = rule == self.accept_rule and (
                (fl is None and self.node_flags is None) or
                (fl is not None and self.node_flags is not None and
                 np.array_equal(np.asarray(fl, np.uint8), self.node_flags)))
            # the labels write above already re-derived the boundary rule's flagged-node
            # counts for the handle's own flags; only a different rule or flag set needs them
            # recounted
            if not same:
                self.set_accept(rule, fl)
        if "sched_rows" in ck:
            self.set_schedule(ck["sched_rows"], int(ck["sched_t0"]))
        elif "accept_rule" in ck:
            self.set_schedule(None)

    def save_checkpoint(self, path: str) -> None:
        ck = self.checkpoint()
        ck["stats"] = ck["stats"].view(np.uint8)  # plain bytes: loadable without pickle
        np.savez(path, **ck)

    @classmethod
    def from_checkpoint(cls, dgraph: "DeviceGraph", path: str, k: int, proposal=None,
                        pop_bounds=None, percent: float = 0.05) -> "Chains":
        """A new handle resumed from ``save_checkpoint`` output (numpy, no pickle), with the
        proposal mode, population bounds, accept rule and bound schedule the checkpointed
        chains ran under (``pop_bounds`` / ``percent`` only for checkpoints without bounds)."""
        d = np.load(path, allow_pickle=False)
        labels = d["labels"]
        if proposal is None:
            proposal = int(d["mode"]) if "mode" in d.files else "pairs"
        if pop_bounds is None and "pop_lo" in d.files:
            pop_bounds = (int(d["pop_lo"]), int(d["pop_hi"]))
        ch = cls(dgraph, labels.shape[0], k, labels, proposal=proposal, pop_bounds=pop_bounds,
                 percent=percent, seed=int(d["seed"]), chain_id0=int(d["chain_id0"]),
                 thr=d["thr"])
        ck = {key: d[key] for key in d.files}
        ck["stats"] = d["stats"].view(STATS_DTYPE)
        ch.restore(ck)
        return ch

    # ------------------------------------------------------------- spatial maps
    def enable_maps(self, label_values: Optional[Sequence[int]] = None) -> None:
        """Track the reference driver's per-edge / per-node maps on every chain
        (grid_chain_sec11.py:383-384, 396-400).  ``label_values``: the GerryChain
        assignment value of each district index (default 0..k-1; {-1, 1} for the
        reference's k=2 plans).  Call before the first run."""
        lv = None
        if label_values is not None:
            lv = np.ascontiguousarray(label_values, np.int64)
            if len(lv) != self.k:
                raise ValueError(f"need {self.k} label values")
        check(_lib.load().fw_chains_enable_maps(self._h, ptr(lv)))
        self.label_values = (np.arange(self.k, dtype=np.int64) if lv is None else lv)

    MAPS = {"cut_times": _lib.MAP_CUT_TIMES, "num_flips": _lib.MAP_NUM_FLIPS,
            "part_sum": _lib.MAP_PART_SUM, "last_flipped": _lib.MAP_LAST_FLIPPED}

    def read_map(self, what: str, chains=None, total: bool = False,
                 finalize: bool = False) -> np.ndarray:
        """int64 map ``what`` (cut_times [E], num_flips / part_sum / last_flipped [n]) of
        chains ``range(*chains)`` (default all) as [n_chains, len], or summed over them
        (``total``).  ``finalize`` applies grid_chain_sec11.py:416-419 to part_sum."""
        lo, hi = (0, self.n_chains) if chains is None else (int(chains[0]), int(chains[1]))
        m = self.dgraph.n_edges if what == "cut_times" else self.dgraph.n
        out = np.empty(m if total else (hi - lo, m), np.int64)
        flags = (_lib.MAP_SUM if total else 0) | (_lib.MAP_FINALIZE if finalize else 0)
        check(_lib.load().fw_chains_read_map(self._h, self.MAPS[what], lo, hi - lo, flags,
                                             ptr(out), out.nbytes))
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().fw_chains_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def eval_flips(dgraph: DeviceGraph, labels, k: int, v, target, pop_bounds):
    """Batched per-flip verdicts on one state (fw_eval_flips)."""
    L = _lib.require_device()
    lab = np.ascontiguousarray(labels, np.int16)
    v = np.ascontiguousarray(v, np.int32)
    t = np.ascontiguousarray(target, np.int16)
    m = len(v)
    dcut = np.zeros(m, np.int32)
    contig = np.zeros(m, np.uint8)
    pop_ok = np.zeros(m, np.uint8)
    db = np.zeros(m, np.int32)
    check(L.fw_eval_flips(dgraph.handle, ptr(lab), int(k), ptr(v), ptr(t), m, int(pop_bounds[0]),
                          int(pop_bounds[1]), ptr(dcut), ptr(contig), ptr(pop_ok), ptr(db)))
    return dcut, contig, pop_ok, db


@dataclass
class RunResult:
    labels: np.ndarray      # [n_chains, n] final plans
    stats: np.ndarray       # [n_chains] STATS_DTYPE
    hist_cut: np.ndarray    # yields per |cut edges|
    hist_b: np.ndarray      # yields per |B|
    pops: np.ndarray        # [n_chains, k]
    kernel_ms: float
    maps: Optional[dict] = None  # spatial observables (Chains.read_map), per chain
    waits: Optional[np.ndarray] = None  # sampled geom_wait sums per chain (Chains.sampled_waits)

    def expected_wait_sums(self, n_nodes: int, k: int) -> np.ndarray:
        return expected_wait_sum(self.stats, n_nodes, k)


def read_maps(ch: "Chains", finalize: bool = True) -> dict:
    """All four spatial maps of every chain; part_sum finalised as the reference's
    end-of-run loop does (grid_chain_sec11.py:416-419) unless ``finalize`` is False."""
    return {"cut_times": ch.read_map("cut_times"), "num_flips": ch.read_map("num_flips"),
            "part_sum": ch.read_map("part_sum", finalize=finalize),
            "last_flipped": ch.read_map("last_flipped")}


def run_chains(graph: Graph, init_labels, k: int, n_chains: int, steps: int,
               proposal: str | int = "pairs", percent: float = 0.05, base=1.0, seed: int = 0,
               chain_id0: int = 0, device: int = 0, pop_bounds=None,
               max_retries: int = DEFAULT_MAX_RETRIES, total_steps: Optional[int] = None,
               maps: bool = False, label_values=None, waits: bool = False) -> RunResult:
    """Run ``n_chains`` chains for ``steps`` counted steps each and read everything back.

    ``total_steps`` (GerryChain's meaning: yields including the initial state) may be
    given instead of ``steps``; then steps = total_steps - 1.  ``maps`` also returns the
    driver's spatial observables (``label_values``: GerryChain values of districts 0..k-1);
    ``waits`` the sampled geom_wait sums (grid_chain_sec11.py:147-148,410-411).
    """
    if total_steps is not None:
        steps = int(total_steps) - 1
    dg = DeviceGraph(graph, device)
    ch = Chains(dg, n_chains, k, init_labels, proposal=proposal, pop_bounds=pop_bounds,
                percent=percent, base=base, seed=seed, chain_id0=chain_id0)
    if maps:
        ch.enable_maps(label_values)
    if waits:
        ch.enable_sampled_waits()
    ch.run(steps, max_retries)
    res = RunResult(ch.labels(), ch.stats(), ch.hist_cut(), ch.hist_b(), ch.pops(),
                    ch.last_kernel_ms(), read_maps(ch) if maps else None,
                    ch.sampled_waits() if waits else None)
    ch.close()
    dg.close()
    return res
