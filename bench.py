#!/usr/bin/env python3
"""bench.py — flip steps/sec of the batched single-node flip walk on MI355X.

Workload (BASELINE.json configs[2], SURVEY.md §8d "C3"): 100x100 grid, k=4 districts
seeded as 50x50 quadrants, 65,536 independent chains per GPU, proposal
slow_reversible_propose over (node, foreign label) pairs (grid_chain_sec11.py:117-130),
single_flip_contiguous + 5% population bound, Metropolis cut_accept with base
mu = 2.63815853 (grid_chain_sec11.py:33,171-179).

A bench "step" is one kernel launch that advances every chain by --inner counted flip
steps (valid proposals, MarkovChain counter increments); value = counted flip steps of
all chains on all ranks / max-over-ranks wall time of the K timed launches.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Extra fields: "roofline" (dominant kernel, algorithmic bytes of SURVEY.md §8d per launch /
mean HIP-event launch time vs 8 TB/s) and "cpu_baseline" (the GerryChain-equivalent
Python proxy, oracle/reference_proxy.py, one chain per process on the host cores, rank 0
at N=1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MU = 2.63815853
METRIC = "flip steps/sec (whole node), 100×100 grid k=4 batched chains; % HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(d):
    """SURVEY.md §8d byte model over counter deltas ``d`` (int32 CSR, int16 labels).

    B_prop = 30 + 6*d_v + sum over dequeued search nodes (8 + 6*d_u)
    B_acc  = 10 + 2*(1 + d_v) + 12*n_bchg
    """
    return (30 * d["attempts"] + 6 * d["sum_deg"] + 8 * d["bfs_nodes"] + 6 * d["bfs_deg"]
            + 12 * d["accepts"] + 2 * d["acc_deg"] + 12 * d["n_bchg"])


def totals(st):
    keys = ["attempts", "steps", "accepts", "pop_fail", "contig_fail", "bfs_runs", "bfs_nodes",
            "bfs_deg", "sum_deg", "acc_deg", "n_bchg"]
    return {k: int(st[k].astype(np.uint64).sum()) for k in keys}


# ------------------------------------------------------------------ workloads
def ladder(n_bases=64, lo=0.1, hi=10.0):
    """C5: Metropolis bases log-spaced over the reference's range (grid_chain_sec11.py:34)."""
    return np.geomspace(lo, hi, n_bases)


def workload(name, grid=None, k=None):
    """(graph, seed plan, k, proposal, base, percent, default chains/GPU, description).

    c3 (default, BASELINE configs[2]) 100x100 grid, k=4 quadrants, 65,536 chains/GPU
    c2 (configs[1])   40x40 grid, k=4 quadrants, 4,096 chains
    c4 (configs[3])   9,000-node Delaunay dual graph, lognormal pops, k=18 tree seed
    c5 (configs[4])   200x200 grid, k=8 (2x4 blocks), 1,024 chains per base of a 64-base
                      ladder in [0.1, 10]; 8 bases (8,192 chains) per GPU
    frank             the 5,000-node Frankengraph of Frankenstein_chain.py, k=2, bi proposal
    """
    from flipcomplexityempirical_amd.graph import (block_seed, delaunay_graph, frankenstein_graph,
                                                   frankenstein_seed, grid_graph)
    from flipcomplexityempirical_amd.seeds import tree_seed
    if name in ("c3", "c2"):
        n = grid or (100 if name == "c3" else 40)
        kk = k or 4
        g = grid_graph(n, n)
        init = block_seed(n, n, 2, 2) if kk == 4 else block_seed(n, n, 2, kk // 2)
        chains = 65536 if name == "c3" else 4096
        return (g, init, kk, "pairs", MU, 0.05, chains,
                f"{name.upper()}: {n}x{n} grid, k={kk} block seed")
    if name == "c4":
        g = delaunay_graph(9000, seed=0)
        kk = k or 18
        return (g, tree_seed(g, kk, 0.05), kk, "pairs", MU, 0.05, 16384,
                f"C4: 9000-node Delaunay dual graph (lognormal pops), k={kk} tree seed")
    if name == "c5":
        n = grid or 200
        g = grid_graph(n, n)
        return (g, block_seed(n, n, 2, 4), 8, "pairs", None, 0.05, 8192,
                f"C5: {n}x{n} grid, k=8 2x4 blocks, 64-base ladder [0.1,10] x 1024 chains")
    if name == "frank":
        g = frankenstein_graph()
        return (g, frankenstein_seed(g, 0), 2, "bi", 1 / .379, 0.5, 16384,
                "Frankengraph (Frankenstein_chain.py), k=2 diagonal seed, bi proposal")
    raise ValueError(f"unknown workload {name}")


# ------------------------------------------------------------------ CPU baseline
def _proxy_worker(args):
    name, percent, base, seed, cid, seconds = args
    sys.path.insert(0, ROOT)
    from flipcomplexityempirical_amd.chain import PROPOSALS
    from oracle.reference_proxy import ProxyChain
    g, lab, k, proposal, _, _, _, _ = workload(name)
    ch = ProxyChain(g, lab, k, PROPOSALS[proposal], percent, base, seed, cid)
    ch.run(1)  # builds caches
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < seconds:
        ch.run(5)
        steps += 5
    return steps, time.perf_counter() - t0


def cpu_baseline(name, desc, percent, base, seed, seconds=10.0, workers=None):
    workers = workers or min(16, os.cpu_count() or 1)
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        res = pool.map(_proxy_worker, [(name, percent, base, seed, i, seconds)
                                       for i in range(workers)])
    rate = sum(s / t for s, t in res)
    return {"value": rate, "unit": "flip steps/s", "cores": workers, "kind": "port",
            "sample": f"GerryChain-equivalent Python proxy (oracle/reference_proxy.py): "
                      f"{workers} chains x ~{seconds:.0f}s, one chain per process, same "
                      f"workload ({desc}, base {base:.6g}, {percent:.0%} pop); "
                      f"{sum(s for s, _ in res)} steps total"}


def native_cpu_rate(g, init, k, mode, percent, base, seed, steps=20000):
    from flipcomplexityempirical_amd.chain import metropolis_table, population_bounds
    from oracle import oracle as O
    lo, hi = population_bounds(g.total_pop, k, percent)
    t0 = time.perf_counter()
    O.run_chain(g, init, k, mode, lo, hi, metropolis_table(base, g.maxdeg), seed, 0, steps)
    return steps / (time.perf_counter() - t0)


# ------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inner", type=int, default=1000, help="flip steps per chain per launch")
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c4", "c5", "frank"],
                    help="workload (see workload()); the driver's line is the default c3")
    ap.add_argument("--chains", type=int, default=None, help="chains per GPU (weak scaling)")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--base", type=float, default=None)
    ap.add_argument("--percent", type=float, default=None)
    ap.add_argument("--proposal", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo for rehearsals)")
    ap.add_argument("--same-device", action="store_true",
                    help="put every rank on GPU 0 (multi-rank rehearsal on a one-GPU box)")
    ap.add_argument("--maps", action="store_true",
                    help="also keep the spatial observables (cut_times, part_sum, ...) per chain")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c3.json"),
                    help="per-launch HBM bytes from a rocprofv3 PMC pass of the default C3 "
                         "command (scripts/profile.sh -> scripts/pmc_summary.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = 0 if args.same_device else local_rank
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    tdev = "cuda" if args.backend == "nccl" else "cpu"
    from flipcomplexityempirical_amd.chain import (PROPOSALS, Chains, DeviceGraph,
                                                   population_bounds)
    from flipcomplexityempirical_amd.distributed import merge_histograms

    g, init, k, proposal, base, percent, chains, desc = workload(args.config, args.grid, args.k)
    proposal = args.proposal or proposal
    percent = args.percent if args.percent is not None else percent
    chains = args.chains or chains
    cid0 = rank * chains
    if args.config == "c5" and args.base is None:
        # whole 1,024-chain base groups per GPU: global chain id g runs ladder[g // 1024]
        lad = ladder()
        base = lad[(np.arange(cid0, cid0 + chains) // 1024) % len(lad)]
        base_desc = f"ladder bases {lad[(cid0 // 1024) % 64]:.4g}..{base[-1]:.4g}"
    else:
        base = args.base if args.base is not None else base
        base_desc = f"base {base:.9g}"
    bounds = population_bounds(g.total_pop, k, percent)
    dg = DeviceGraph(g, device=device)
    ch = Chains(dg, chains, k, init, proposal=proposal, pop_bounds=bounds, base=base,
                seed=args.seed, chain_id0=cid0)
    if args.maps:
        ch.enable_maps([-1, 1] if k == 2 else None)

    def barrier():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        ch.run(args.inner)
    st0 = totals(ch.stats())
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        ch.run_async(args.inner)
        ch.sync()
        kms.append(ch.last_kernel_ms())
    barrier()
    dt = time.perf_counter() - t0
    st1_arr = ch.stats()
    st1 = totals(st1_arr)
    d = {kk: st1[kk] - st0[kk] for kk in st1}
    steps_local = d["steps"]
    if dist is not None:
        t = torch.tensor([dt, float(steps_local)], dtype=torch.float64, device=tdev)
        dist.all_reduce(t[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        dt, steps_all = float(t[0]), float(t[1])
    else:
        steps_all = float(steps_local)
    hist_cut, hist_b = merge_histograms(ch.hist_cut(), ch.hist_b(), dist)

    kernel_ms = float(np.mean(kms))
    bytes_per_launch = algorithmic_bytes(d) / args.steps
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    traffic = None
    issue = None
    default_c3 = (args.config, g.n, k, chains, args.inner, proposal) == (
        "c3", 10000, 4, 65536, 1000, "pairs")
    if default_c3 and args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        traffic = tj.get("hbm_bytes_per_launch")
        if tj.get("valu_insts_per_launch"):
            # what binds this kernel: VALU issue.  Peak: every SIMD takes one wave64 VALU
            # instruction per 2 cycles (SIMD-32, MI355X_MICROARCH.md) -> 256 CUs x 4 SIMDs
            # x 2.4 GHz / 2; achieved: the PMC pass's VALU wave-instructions per launch
            # over this run's mean launch time.
            peak = 256 * 4 * 2.4e9 / 2
            ach = tj["valu_insts_per_launch"] / (kernel_ms * 1e-3)
            issue = {"bound": "valu-issue", "achieved": ach, "peak": peak,
                     "unit": "wave-instr/s", "frac": ach / peak,
                     "source": tj.get("source"),
                     # rocprofv3 --kernel-trace --stats mean of the same kernel, same command
                     "rocprof_kernel_ms": (tj.get("kernel_trace") or {}).get("avg_ms")}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": steps_all / dt,
            "unit": "flip steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": f"{desc}, {chains} chains/GPU, {proposal} proposal, {base_desc}, "
                            f"{percent:.0%} pop bound, contiguity",
                "chains_per_gpu": chains,
                "spatial_maps": bool(args.maps),
                "flip_steps_per_chain_per_step": args.inner,
                "parallelism": f"chains sharded over {world} GPU(s), RCCL histogram merge",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
            },
            "issue_roofline": issue,
            "kernel_ms": kernel_ms,
            "proposals_per_s": d["attempts"] * world / dt,
            "accepts_per_s": d["accepts"] * world / dt,
            "valid_frac": d["steps"] / max(1, d["attempts"]),
            "accept_frac": d["accepts"] / max(1, d["steps"]),
            "bfs_runs_per_step": d["bfs_runs"] / max(1, d["steps"]),
            "bfs_nodes_per_run": d["bfs_nodes"] / max(1, d["bfs_runs"]),
            "alg_bytes_per_proposal": algorithmic_bytes(d) / max(1, d["attempts"]),
            "mean_cut": float(st1_arr["cut"].mean()),
            "mean_bnodes": float(st1_arr["bnodes"].mean()),
            "hist_yields": int(hist_cut.sum()),
        }
        if world == 1 and not args.no_cpu_baseline:
            b0 = float(np.ravel(base)[0])
            out["cpu_baseline"] = cpu_baseline(args.config, desc, percent, b0, args.seed,
                                               seconds=args.cpu_seconds)
            out["cpu_native_1core"] = native_cpu_rate(g, init, k, PROPOSALS[proposal], percent,
                                                      b0, args.seed)
        print(json.dumps(out), flush=True)
    ch.close()
    dg.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
