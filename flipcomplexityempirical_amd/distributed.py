"""Multi-GPU sharding of independent chains (one process per GPU).

Chains are independent, so the data path has no collective: rank r of R owns global
chain ids [shard_range(C, R, r)), and its Philox streams depend only on those ids, so
every chain's trajectory is the same at 1, 2, 4 or 8 GPUs.  The only exchange is one
all-reduce(sum) of the yield histograms and per-chain sums at the end of a run
(SURVEY.md §8e), over RCCL ("nccl" backend on ROCm) between GPUs, or gloo on CPU.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of global chain ids owned by ``rank`` (balanced to within one)."""
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device_for(dist):
    import torch
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def allreduce_sum_int64(arr: np.ndarray, dist=None) -> np.ndarray:
    """Sum an int64/uint64 array over all ranks (identity without a process group)."""
    if dist is None or not dist.is_initialized():
        return arr
    import torch
    t = torch.from_numpy(np.ascontiguousarray(arr).astype(np.int64)).to(_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(arr.dtype)


def merge_histograms(hist_cut: np.ndarray, hist_b: np.ndarray, dist=None):
    """One all-reduce of the concatenated histograms (the run's only collective)."""
    if dist is None or not dist.is_initialized():
        return hist_cut, hist_b
    both = allreduce_sum_int64(np.concatenate([hist_cut, hist_b]), dist)
    return both[:len(hist_cut)], both[len(hist_cut):]


def gather_stats(stats: np.ndarray, n_total: int, dist=None, lo: int = 0) -> np.ndarray:
    """Assemble per-chain stats records of all ranks into one [n_total] array (sum-merge)."""
    if dist is None or not dist.is_initialized():
        return stats
    full = np.zeros(n_total, stats.dtype)
    full[lo:lo + len(stats)] = stats
    raw = full.view(np.int64).reshape(n_total, -1)
    merged = allreduce_sum_int64(raw.reshape(-1), dist).reshape(raw.shape)
    return np.ascontiguousarray(merged).view(stats.dtype).reshape(n_total)


def _local_device(device: Optional[int]) -> int:
    """The GPU of this process: explicit, else LOCAL_RANK (one process per GPU per node)."""
    if device is not None:
        return int(device)
    import os
    return int(os.environ.get("LOCAL_RANK", "0"))


def _shard_rows(x, n_total: int, lo: int, hi: int):
    """Rows [lo, hi) of a per-chain array ([n_total, ...]); shared values pass through."""
    if x is None or np.ndim(x) == 0:
        return x
    a = np.asarray(x)
    if a.shape[0] == n_total and (a.ndim == 2 or (a.ndim == 1 and a.dtype.kind == "f")):
        return a[lo:hi]
    return a


def run_sharded(graph, init_labels, k: int, n_total: int, steps: int, dist=None,
                device: Optional[int] = None, engine=None, **kw):
    """Strong-scaling run: ``n_total`` chains split over the process group.

    Rank r runs global chain ids ``shard_range(n_total, world, r)`` on its node-local GPU
    (LOCAL_RANK unless ``device`` is given).  Per-chain inputs (``init_labels`` of shape
    [n_total, n], ``base`` of length n_total) are sliced to the rank's rows; shared ones
    are passed as they are.  ``engine`` (default ``chain.run_chains``, the GPU path) has
    run_chains' signature; tests substitute a CPU engine to check the sharding alone.
    Returns (local RunResult, merged hist_cut, merged hist_b, merged stats[n_total]).
    """
    from .chain import run_chains
    engine = engine or run_chains
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    lo, hi = shard_range(n_total, world, rank)
    init = np.asarray(init_labels)
    if init.ndim == 2 and init.shape[0] == n_total and n_total > 1:
        init = init[lo:hi]
    kw = dict(kw)
    if "base" in kw:
        kw["base"] = _shard_rows(kw["base"], n_total, lo, hi)
    res = engine(graph, init, k, hi - lo, steps, chain_id0=lo, device=_local_device(device),
                 **kw)
    hc, hb = merge_histograms(res.hist_cut, res.hist_b, dist)
    st = gather_stats(res.stats, n_total, dist, lo)
    return res, hc, hb, st
