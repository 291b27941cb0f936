"""ctypes binding of ``libflipwalk.so`` (the C-ABI in include/flipwalk.h).

The HIP library is the only compute path: if it is missing or no GPU is visible,
every compute entry point raises ``FlipwalkUnavailable`` — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLIPWALK_LIB", os.path.join(_HERE, "libflipwalk.so"))

FW_OK = 0
FW_EINVAL, FW_EHIP, FW_ESTATE, FW_EUNSUPPORTED, FW_ENOMEM = -1, -2, -3, -4, -5
PROPOSE_BI, PROPOSE_PAIRS, PROPOSE_CUTEDGE = 0, 1, 2
READ_LABELS, READ_STATS, READ_HIST_CUT, READ_HIST_B, READ_POPS = 0, 1, 2, 3, 4
READ_HIST_RING, READ_RING_PAIR, READ_WAITS = 5, 6, 7
MAP_CUT_TIMES, MAP_NUM_FLIPS, MAP_PART_SUM, MAP_LAST_FLIPPED = 0, 1, 2, 3
MAP_SUM, MAP_FINALIZE = 1, 2
ACCEPT_CUT, ACCEPT_BRATIO, ACCEPT_BOUNDARY = 0, 1, 2

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

# Every symbol include/flipwalk.h declares: (name, restype, argtypes).
_P = ctypes.c_void_p
_I32, _I64, _U64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
SIGNATURES = [
    ("fw_last_error", ctypes.c_char_p, []),
    ("fw_version", _I32, []),
    ("fw_build_info", ctypes.c_char_p, []),
    ("fw_device_count", _I32, []),
    ("fw_graph_create", ctypes.c_int, [_P, _P, _P, _I32, _I32, ctypes.c_int, _P]),
    ("fw_graph_destroy", None, [_P]),
    ("fw_graph_info", ctypes.c_int, [_P, _P]),
    ("fw_chains_create", ctypes.c_int,
     [_P, _I32, _I32, _P, _I32, _I32, _I64, _I64, _P, _I32, _U64, _I64, _P]),
    ("fw_chains_destroy", None, [_P]),
    ("fw_chains_run", ctypes.c_int, [_P, _I64, _I32]),
    ("fw_chains_run_async", ctypes.c_int, [_P, _I64, _I32]),
    ("fw_chains_sync", ctypes.c_int, [_P]),
    ("fw_chains_run_traced", ctypes.c_int, [_P, _I64, _I32, _P, ctypes.c_size_t]),
    ("fw_chains_last_kernel_ms", ctypes.c_double, [_P]),
    ("fw_chains_launch_info", ctypes.c_int, [_P, _P]),
    ("fw_chains_read", ctypes.c_int, [_P, _I32, _P, ctypes.c_size_t]),
    ("fw_chains_write", ctypes.c_int, [_P, _I32, _P, ctypes.c_size_t]),
    ("fw_chains_reset_observables", ctypes.c_int, [_P]),
    ("fw_chains_set_accept", ctypes.c_int, [_P, _I32, _P]),
    ("fw_chains_set_schedule", ctypes.c_int, [_P, _P, _I32, _I64]),
    ("fw_chains_enable_maps", ctypes.c_int, [_P, _P]),
    ("fw_chains_enable_ring", ctypes.c_int, [_P, _P, _P, _I32]),
    ("fw_chains_enable_waits", ctypes.c_int, [_P, _P]),
    ("fw_chains_read_map", ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _P, ctypes.c_size_t]),
    ("fw_eval_flips", ctypes.c_int,
     [_P, _P, _I32, _P, _P, _I32, _I64, _I64, _P, _P, _P, _P]),
]


class FlipwalkUnavailable(RuntimeError):
    """The HIP library could not be loaded or no MI355X is visible."""


class FlipwalkError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class InvalidInitialState(FlipwalkError, ValueError):
    """GerryChain's MarkovChain raises ValueError for an invalid initial state."""


_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """Load the library (no device needed) and bind every declared symbol."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise FlipwalkUnavailable(
                f"{path} not found: build it with `make -C flipcomplexityempirical_amd/csrc` "
                "or __graft_entry__.build()")
        try:
            # import torch first when it is present so one HIP runtime serves both
            import torch  # noqa: F401
        except Exception:
            pass
        L = ctypes.CDLL(path)
        in_tree = os.path.join(_HERE, "libflipwalk.so")
        is_in_tree = os.path.exists(in_tree) and os.path.samefile(path, in_tree)
        skipped = []
        for name, res, args in SIGNATURES:
            try:
                fn = getattr(L, name)
            except AttributeError:
                # an older build pointed at by FLIPWALK_LIB (A/B runs) may predate an entry
                # point; the in-tree library (by any path or symlink) must export them all
                if is_in_tree:
                    raise
                skipped.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        if skipped:
            import sys
            print(f"flipwalk: {path} lacks {', '.join(skipped)} (an older build)", file=sys.stderr)
        L.skipped_symbols = tuple(skipped)
        _lib = L
        return L


def build_info() -> str:
    """fw_build_info() of the loaded library ("src=<hash> flags=<...>"), or a note when the
    library predates it."""
    L = load()
    if "fw_build_info" in getattr(L, "skipped_symbols", ()):
        return "unknown (library predates fw_build_info)"
    return L.fw_build_info().decode()


def check(rc: int) -> None:
    if rc == FW_OK:
        return
    msg = load().fw_last_error().decode(errors="replace")
    if rc == FW_ESTATE:
        raise InvalidInitialState(rc, msg)
    raise FlipwalkError(rc, msg)


def require_device():
    L = load()
    if L.fw_device_count() <= 0:
        raise FlipwalkUnavailable("no HIP device visible: the flip walk runs only on the GPU")
    return L


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)
