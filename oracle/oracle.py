"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (flipchain_oracle.c).

Each function cites the reference behaviour it restates; see the C file header.
Builds ``oracle/liboracle.so`` with ``make -C oracle`` when it is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

STATS_DTYPE = np.dtype(
    [
        ("attempts", "<u8"),
        ("steps", "<u8"),
        ("accepts", "<u8"),
        ("pop_fail", "<u8"),
        ("contig_fail", "<u8"),
        ("bfs_runs", "<u8"),
        ("bfs_nodes", "<u8"),
        ("bfs_deg", "<u8"),
        ("sum_deg", "<u8"),
        ("acc_deg", "<u8"),
        ("n_bchg", "<u8"),
        ("yields", "<u8"),
        ("sum_cut", "<i8"),
        ("sum_bnodes", "<i8"),
        ("sum_invb", "<f8"),
        ("cut", "<i4"),
        ("bnodes", "<i4"),
        ("npairs", "<i4"),
        ("stuck", "<i4"),
    ]
)

_P = ctypes.c_void_p


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "flipchain_oracle.c")
    if (not os.path.exists(path)) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(build())
        L.orc_philox4x32_10.argtypes = [_P, _P, _P]
        L.orc_philox4x32_10.restype = None
        L.orc_scale64.argtypes = [ctypes.c_uint32] * 3
        L.orc_scale64.restype = ctypes.c_uint32
        L.orc_u53.argtypes = [ctypes.c_uint32] * 2
        L.orc_u53.restype = ctypes.c_double
        L.orc_run_chain.argtypes = [
            _P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int64, ctypes.c_int64, _P, ctypes.c_uint64, ctypes.c_uint64, _P, _P,
            ctypes.c_int64, ctypes.c_int32, _P, _P, _P, _P,
        ]
        L.orc_run_chain.restype = ctypes.c_int
        L.orc_run_chain_ex.argtypes = L.orc_run_chain.argtypes + [
            _P, ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_int64, _P, _P]
        L.orc_log1p.argtypes = [ctypes.c_double]
        L.orc_log1p.restype = ctypes.c_double
        L.orc_run_chain_ex.restype = ctypes.c_int
        L.orc_eval_flips.argtypes = [
            _P, _P, _P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P,
            ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _P, _P, _P, _P,
        ]
        L.orc_eval_flips.restype = ctypes.c_int
        L.orc_plan_valid.argtypes = [
            _P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int64, ctypes.c_int64,
        ]
        L.orc_plan_valid.restype = ctypes.c_int
        L.orc_stats_size.restype = ctypes.c_int32
        assert L.orc_stats_size() == STATS_DTYPE.itemsize
        _LIB = L
    return _LIB


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def philox4x32_10(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().orc_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def new_stats(n=1):
    return np.zeros(n, dtype=STATS_DTYPE)


class _OrcMaps(ctypes.Structure):
    _fields_ = [("cut_times", _P), ("num_flips", _P), ("part_sum", _P), ("last_flipped", _P),
                ("label_value", _P), ("cur_f", ctypes.c_int32), ("pad", ctypes.c_int32)]


class Maps:
    """The reference driver's per-edge / per-node observables of one chain
    (grid_chain_sec11.py:383-384, 396-400), updated per yield by the C oracle."""

    def __init__(self, graph, init_labels, label_values):
        self.label_value = np.ascontiguousarray(label_values, np.int64)
        self.cut_times = np.zeros(graph.n_edges, np.int64)
        self.num_flips = np.zeros(graph.n, np.int64)
        # part_sum starts at the initial assignment (grid_chain_sec11.py:219)
        self.part_sum = self.label_value[np.asarray(init_labels, np.int64)].copy()
        self.last_flipped = np.zeros(graph.n, np.int64)
        self._s = _OrcMaps(_ptr(self.cut_times), _ptr(self.num_flips), _ptr(self.part_sum),
                           _ptr(self.last_flipped), _ptr(self.label_value), -1, 0)

    @property
    def cur_f(self):
        return self._s.cur_f

    def finalized_part_sum(self, labels, n_yields):
        """grid_chain_sec11.py:416-419: never-flipped nodes get t * final label."""
        ps = self.part_sum.copy()
        never = self.last_flipped == 0
        ps[never] = n_yields * self.label_value[np.asarray(labels, np.int64)[never]]
        return ps


class _OrcRing(ctypes.Structure):
    _fields_ = [("u", _P), ("w", _P), ("n_ring", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("hist", _P)]


class Ring:
    """The district-shape observable (boundary_slope, grid_chain_sec11.py:55-78 and the
    driver's :371-394): yields per pair of first two cut ring edges, ring order."""

    def __init__(self, ring_u, ring_w):
        self.u = np.ascontiguousarray(ring_u, np.int32)
        self.w = np.ascontiguousarray(ring_w, np.int32)
        n = len(self.u)
        self.hist = np.zeros(n * n + 1, np.uint64)
        self._s = _OrcRing(_ptr(self.u), _ptr(self.w), n, 0, _ptr(self.hist))


class _OrcWaits(ctypes.Structure):
    _fields_ = [("lp", _P), ("sum", ctypes.c_double), ("cur", ctypes.c_double)]


def log1p(x):
    return lib().orc_log1p(float(x))


class Waits:
    """Sampled geometric waits of one chain (geom_wait, grid_chain_sec11.py:147-148): one
    inversion draw per state object, re-used on re-yield; ``p_table`` [n+1] holds
    b / (N**k - 1) as the reference divides (chain.wait_prob_table)."""

    def __init__(self, p_table):
        self.lp = np.array([log1p(-float(p)) for p in p_table], np.float64)
        self._s = _OrcWaits(_ptr(self.lp), 0.0, 0.0)

    @property
    def sum(self):
        return self._s.sum

    @property
    def cur(self):
        return self._s.cur


def run_chain(graph, labels, k, mode, pop_lo, pop_hi, thr, seed, chain_id, steps,
              max_retries=1 << 20, stats=None, hist_cut=None, hist_b=None, trace=False,
              maps=None, accept_rule=0, flags=None, schedule=None, ring=None, waits=None):
    """Run one chain on the CPU oracle.  ``graph`` needs rowptr/col/pop/n/grid_w.

    Returns (labels, stats, pops, trace-or-None); ``labels`` is a new int16 array.
    ``maps`` (an oracle ``Maps``) accumulates the per-yield spatial observables;
    ``accept_rule`` is FW_ACCEPT_* (0 cut_accept, 1 the |B'|/|B| rule, 2 uniform_accept
    with boundary_condition over the uint8 ``flags``).  ``schedule`` = (rows, t0): the
    step-dependent bounds of fw_chains_set_schedule; ``ring`` (an oracle ``Ring``)
    accumulates the district-shape observable; ``waits`` (an oracle ``Waits``) the sampled
    geometric waits (its ``sum`` / ``cur`` carry over between calls, like ``stats``).
    """
    srows, st0 = (None, 0) if schedule is None else schedule
    if srows is not None:
        srows = np.ascontiguousarray(srows, np.float64)
    fl = None if flags is None else np.ascontiguousarray(flags, np.uint8)
    lab = np.array(labels, dtype=np.int16, copy=True)
    st = new_stats(1) if stats is None else stats
    thr = np.ascontiguousarray(thr, dtype=np.float64)
    tr = np.full(int(steps), -2, dtype=np.int32) if trace else None
    pops = np.zeros(k, dtype=np.int64)
    rc = lib().orc_run_chain_ex(
        _ptr(graph.rowptr), _ptr(graph.col), _ptr(graph.pop), graph.n, graph.grid_w, k, mode,
        int(pop_lo), int(pop_hi), _ptr(thr), int(seed), int(chain_id), _ptr(lab), _ptr(st),
        int(steps), int(max_retries), _ptr(hist_cut), _ptr(hist_b), _ptr(tr), _ptr(pops),
        None if maps is None else ctypes.byref(maps._s), int(accept_rule), _ptr(fl),
        _ptr(srows), 0 if srows is None else int(srows.shape[0]), int(st0),
        None if ring is None else ctypes.byref(ring._s),
        None if waits is None else ctypes.byref(waits._s),
    )
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return lab, st, pops, tr


def eval_flips(graph, labels, k, v, target, pop_lo, pop_hi):
    lab = np.ascontiguousarray(labels, dtype=np.int16)
    v = np.ascontiguousarray(v, dtype=np.int32)
    t = np.ascontiguousarray(target, dtype=np.int16)
    m = len(v)
    dcut = np.zeros(m, np.int32)
    contig = np.zeros(m, np.uint8)
    pop_ok = np.zeros(m, np.uint8)
    dbound = np.zeros(m, np.int32)
    rc = lib().orc_eval_flips(
        _ptr(graph.rowptr), _ptr(graph.col), _ptr(graph.pop), graph.n, graph.grid_w, k, _ptr(lab),
        _ptr(v), _ptr(t), m, int(pop_lo), int(pop_hi), _ptr(dcut), _ptr(contig), _ptr(pop_ok),
        _ptr(dbound),
    )
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return dcut, contig, pop_ok, dbound


def plan_valid(graph, labels, k, pop_lo, pop_hi):
    lab = np.ascontiguousarray(labels, dtype=np.int16)
    return bool(lib().orc_plan_valid(_ptr(graph.rowptr), _ptr(graph.col), _ptr(graph.pop),
                                     graph.n, k, _ptr(lab), int(pop_lo), int(pop_hi)))
