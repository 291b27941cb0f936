"""The BASELINE.json configurations as chain workloads.

Shared by bench.py and the full-size GPU tests, so the benched workload is the tested one.

    C2  configs[1]  40x40 grid, k=4 quadrants, 4,096 chains
    C3  configs[2]  100x100 grid, k=4 quadrants, 65,536 chains (the headline)
    C4  configs[3]  9,000-node Delaunay dual graph, lognormal populations, k=18 tree seed,
                    16,384 chains
    C5  configs[4]  200x200 grid, k=8 (2x4 blocks), 64 Metropolis bases log-spaced in
                    [0.1, 10] (grid_chain_sec11.py:34's range) x 1,024 chains = 65,536
    frank           the 5,000-node Frankengraph of Frankenstein_chain.py, k=2, bi proposal

Every workload is a fixed set of global chain ids [0, chains): chain g's plan, base and
Philox stream depend on g alone, so sharding the ids over GPUs (distributed.shard_range)
changes nothing about any chain.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

MU = 2.63815853  # the reference's transition base, grid_chain_sec11.py:33
LADDER_GROUP = 1024  # chains per base of the C5 ladder


def ladder(n_bases: int = 64, lo: float = 0.1, hi: float = 10.0) -> np.ndarray:
    """C5: Metropolis bases log-spaced over the reference's range (grid_chain_sec11.py:34)."""
    return np.geomspace(lo, hi, n_bases)


def ladder_base_index(cid, n_bases: int = 64, n_gpus_hint: int = 8,
                      interleave: bool = True) -> np.ndarray:
    """Ladder index of global chain id(s) ``cid``: base group b = cid // 1024 of block
    s = b // 8 (one GPU's 8,192-id shard at 8 GPUs) runs, at position i = b % 8, an entry
    of ladder octave i: 8 i + s for even i, 8 i + 7 - s for odd i.  Every shard thus holds
    8 whole base groups spread over the ladder, and the snake order gives every shard the
    same mix of cheap and dear bases (the low bases grow fractal boundaries that make steps
    several times dearer; adjacent groups put them all on one GPU, and the plain
    interleave 8 i + s still left shard 0 with the lowest base of every octave: 0.39 vs
    0.44 x 10^9 flip steps/s for shard 7, profiles/r02/round_d/shards_c5_n8.jsonl).
    A fixed function of the id, independent of the GPU count."""
    b = np.asarray(cid, np.int64) // LADDER_GROUP
    per = n_bases // n_gpus_hint
    b = b % n_bases
    if not interleave:  # round 1's assignment: adjacent groups, ladder entry b
        return b
    i, s = b % per, b // per
    return i * n_gpus_hint + np.where(i % 2 == 0, s, n_gpus_hint - 1 - s)


@dataclass
class Workload:
    name: str
    graph: object
    init: np.ndarray
    k: int
    proposal: str
    percent: float
    chains: int             # total chains of the configuration (all GPUs)
    base: Optional[float]   # shared Metropolis base, or None for the C5 ladder
    desc: str

    interleave: bool = True  # C5: ladder_base_index's spread of base groups over shards

    def bases(self, lo: int, hi: int):
        """Base(s) of global chain ids [lo, hi): a float, or a per-chain array (ladder)."""
        if self.base is not None:
            return self.base
        return ladder()[ladder_base_index(np.arange(lo, hi), interleave=self.interleave)]

    def base_desc(self, lo: int, hi: int) -> str:
        if self.base is not None:
            return f"base {self.base:.9g}"
        idx = np.unique(ladder_base_index(np.arange(lo, hi), interleave=self.interleave))
        return (f"{len(idx)} ladder bases x {LADDER_GROUP} chains "
                f"({', '.join(f'{b:.3g}' for b in ladder()[idx][:8])}"
                f"{', ...' if len(idx) > 8 else ''})")


C4_ORDER = "hilbert"  # node numbering of the C4 Delaunay graph (graph.delaunay_graph)


def workload(name: str, grid: Optional[int] = None, k: Optional[int] = None,
             order: Optional[str] = None) -> Workload:
    from .graph import (block_seed, delaunay_graph, frankenstein_graph, frankenstein_seed,
                        grid_graph)
    from .seeds import tree_seed
    if name in ("c3", "c2"):
        n = grid or (100 if name == "c3" else 40)
        kk = k or 4
        g = grid_graph(n, n)
        init = block_seed(n, n, 2, 2) if kk == 4 else block_seed(n, n, 2, kk // 2)
        return Workload(name, g, init, kk, "pairs", 0.05, 65536 if name == "c3" else 4096, MU,
                        f"{name.upper()}: {n}x{n} grid, k={kk} block seed")
    if name == "c4":
        order = order or C4_ORDER
        g = delaunay_graph(9000, seed=0, order=order)
        kk = k or 18
        return Workload(name, g, tree_seed(g, kk, 0.05), kk, "pairs", 0.05, 16384, MU,
                        f"C4: 9000-node Delaunay dual graph (lognormal pops, {order} node "
                        f"order), k={kk} tree seed")
    if name == "c5":
        n = grid or 200
        g = grid_graph(n, n)
        return Workload(name, g, block_seed(n, n, 2, 4), 8, "pairs", 0.05, 64 * LADDER_GROUP,
                        None, f"C5: {n}x{n} grid, k=8 2x4 blocks, 64-base ladder [0.1,10] "
                              f"x {LADDER_GROUP} chains")
    if name == "frank":
        g = frankenstein_graph()
        return Workload(name, g, frankenstein_seed(g, 0), 2, "bi", 0.5, 16384, 1 / .379,
                        "Frankengraph (Frankenstein_chain.py), k=2 diagonal seed, bi proposal")
    raise ValueError(f"unknown workload {name}")
