"""Spread of per-chain work in one C3 launch (grid kernel, four chains per wave).

With fewer chains than resident waves hold (a strong-scaled shard), a launch lasts as long
as its slowest quad, so the per-quad spread of attempts (iterations) and exact-search work
sets the launch time.  Prints, for one 1000-step launch after `warm` launches: attempts per
chain and per quad (max over the four rows), exact searches and dequeued search nodes per
quad (summed: a wave runs its rows' searches one after another), as mean / p99 / max.

    python scripts/quad_spread.py [chains] [warm]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds  # noqa: E402
from flipcomplexityempirical_amd.workloads import workload  # noqa: E402

chains = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 4
w = workload("c3")
dg = DeviceGraph(w.graph)
ch = Chains(dg, chains, w.k, w.init, proposal=w.proposal,
            pop_bounds=population_bounds(w.graph.total_pop, w.k, w.percent), base=w.base)
for _ in range(warm):
    ch.run(1000)
s0 = ch.stats()
ch.run(1000)
s1 = ch.stats()
print(f"chains {chains}, launch after {warm} warm launches: kernel {ch.last_kernel_ms():.3f} ms")


def d(key):
    return (s1[key].astype(np.int64) - s0[key].astype(np.int64))


def q(x):
    return f"mean {x.mean():9.1f}  p99 {np.percentile(x, 99):9.1f}  max {x.max():9.1f}"


att = d("attempts")
nq = chains // 4
print("attempts / chain      ", q(att))
print("attempts / quad (max) ", q(att[:nq * 4].reshape(nq, 4).max(1)))
for key in ("bfs_runs", "bfs_nodes", "contig_fail", "pop_fail", "accepts"):
    x = d(key)
    print(f"{key:10s} / chain     ", q(x))
    print(f"{key:10s} / quad (sum)", q(x[:nq * 4].reshape(nq, 4).sum(1)))
cut = s1["cut"].astype(np.int64) if "cut" in s1.dtype.names else None
if cut is not None:
    print("cut edges / chain     ", q(cut))
