#!/usr/bin/env python3
"""bench.py — flip steps/sec of the batched single-node flip walk on MI355X.

Workload (BASELINE.json configs[2], SURVEY.md §8d "C3"): 100x100 grid, k=4 districts
seeded as 50x50 quadrants, 65,536 independent chains IN TOTAL, sharded over the GPUs of
the run (strong scaling: global chain ids distributed.shard_range(65536, N, rank), so at
N = 1/2/4/8 each GPU runs 65,536 / 32,768 / 16,384 / 8,192 chains); proposal
slow_reversible_propose over (node, foreign label) pairs (grid_chain_sec11.py:117-130),
single_flip_contiguous + 5% population bound, Metropolis cut_accept with base
mu = 2.63815853 (grid_chain_sec11.py:33,171-179).  ``--scaling weak`` gives every GPU
``--chains`` chains instead.

A bench "step" is one kernel launch that advances every chain by --inner counted flip
steps (valid proposals, MarkovChain counter increments); value = counted flip steps of
all chains on all ranks / max-over-ranks wall time of the K timed launches.  The default
--inner 5000 makes every protocol SURVEY.md §8d's: the defaults (--warmup 2 --steps 20)
time 10^5 steps per chain after 10^4 of warm-up, and the driver's --warmup 5 --steps 20
time 10^5 after 2.5 x 10^4.  (The reference runs its 10^5 steps per chain as one loop,
grid_chain_sec11.py:342, which the library runs as one launch; a launch lasts as long as
its slowest chain, a wait that shrinks with longer launches: profiles/r05/launch_length/.)
At N = 1 the line also carries "secondary": the same warm-up and timed launch COUNTS at
1,000 steps per launch (the protocol of rounds 1-5, chains earlier in their burn-in and
therefore faster), on a fresh set of chains after the headline measurement.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Extra fields: "roofline" (dominant kernel, algorithmic bytes of SURVEY.md §8d per launch /
mean HIP-event launch time vs 8 TB/s), "cpu_baseline" (the GerryChain-equivalent Python
proxy, oracle/reference_proxy.py, one chain per process on every usable host core) and
"cpu_native" (the C oracle, one chain per thread on the same cores), rank 0 at N=1 only,
bounded samples of the same workload.
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from flipcomplexityempirical_amd.workloads import MU, ladder, workload  # noqa: E402,F401

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


# ------------------------------------------------------------------ host description
def host_cores():
    """(usable cores, affinity cores, cgroup CPU quota in cores or None, os.cpu_count())."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return usable, aff, quota, os.cpu_count()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------ CPU baselines
def _proxy_worker(args):
    name, percent, base, seed, cid, seconds = args
    sys.path.insert(0, ROOT)
    from flipcomplexityempirical_amd.chain import PROPOSALS
    from oracle.reference_proxy import ProxyChain
    w = workload(name)
    ch = ProxyChain(w.graph, w.init, w.k, PROPOSALS[w.proposal], percent, base, seed, cid)
    ch.run(1)  # builds caches
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < seconds:
        ch.run(5)
        steps += 5
    return steps, time.perf_counter() - t0


def _host_fields(workers):
    usable, aff, quota, total = host_cores()
    return {"cores": workers, "cpu_model": cpu_model(), "cpu_count": total,
            "affinity_cores": aff, "cgroup_quota_cores": quota}


def cpu_baseline(name, desc, percent, base, seed, seconds=10.0, workers=None):
    """The GerryChain-equivalent Python proxy, one chain per process on every usable core."""
    workers = workers or host_cores()[0]
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        res = pool.map(_proxy_worker, [(name, percent, base, seed, i, seconds)
                                       for i in range(workers)])
    rate = sum(s / t for s, t in res)
    out = {"value": rate, "unit": "flip steps/s", "kind": "port",
           "sample": f"GerryChain-equivalent Python proxy (oracle/reference_proxy.py): "
                     f"{workers} chains x ~{seconds:.0f}s, one chain per process on every usable "
                     f"host core, same workload ({desc}, base {base:.6g}, {percent:.0%} pop); "
                     f"{sum(s for s, _ in res)} steps total"}
    out.update(_host_fields(workers))
    out["per_core"] = rate / workers
    out["extrapolated_all_cpus"] = rate / workers * out["cpu_count"]
    return out


def native_cpu_baseline(w, bounds, base, seed, seconds=10.0, workers=None, lo=0, chains=1):
    """The C oracle (oracle/flipchain_oracle.c), one chain per thread on every usable core
    (ctypes releases the GIL), each chain advanced in 5,000-step calls until the deadline.
    Worker k runs the benched chain lo + i_k, i_k spread evenly over the line's ``chains``,
    with that chain's own base (``base``: one value or one per benched chain), so a base
    ladder (C5) is sampled across its bases."""
    from concurrent.futures import ThreadPoolExecutor

    from flipcomplexityempirical_amd.chain import PROPOSALS, metropolis_table
    from oracle import oracle as O
    workers = workers or host_cores()[0]
    bases = np.broadcast_to(np.asarray(base, np.float64), (max(1, chains),))
    mode = PROPOSALS[w.proposal] if isinstance(w.proposal, str) else int(w.proposal)
    init = np.asarray(w.init, np.int16)
    pick = np.linspace(0, max(1, chains) - 1, workers).round().astype(int)

    def one(k):
        i = int(pick[k])
        cid = lo + i
        thr = metropolis_table(float(bases[i]), w.graph.maxdeg)
        lab = (init if init.ndim == 1 else init[i]).copy()
        st = O.new_stats(1)
        lab, st, _, _ = O.run_chain(w.graph, lab, w.k, mode, *bounds, thr, seed, cid, 100, stats=st)
        t0 = time.perf_counter()
        s0 = int(st["steps"][0])
        while time.perf_counter() - t0 < seconds:
            lab, st, _, _ = O.run_chain(w.graph, lab, w.k, mode, *bounds, thr, seed, cid, 5000,
                                        stats=st)
        return int(st["steps"][0]) - s0, time.perf_counter() - t0

    with ThreadPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(one, range(workers)))
    rate = sum(s / t for s, t in res)
    out = {"value": rate, "unit": "flip steps/s", "kind": "port",
           "sample": f"C oracle (oracle/flipchain_oracle.c, the bit-exact restatement), "
                     f"{workers} chains x ~{seconds:.0f}s, one chain per thread on every usable "
                     f"host core, same workload (chains spread over the line's {chains}, each "
                     f"with its own base, from the seed plan); {sum(s for s, _ in res)} steps "
                     f"total"}
    out.update(_host_fields(workers))
    out["per_core"] = rate / workers
    out["extrapolated_all_cpus"] = rate / workers * out["cpu_count"]
    return out


# ------------------------------------------------------------------ parity spot-check
STAT_FIELDS = ("attempts", "steps", "accepts", "pop_fail", "contig_fail", "bfs_runs", "bfs_nodes",
               "bfs_deg", "sum_deg", "acc_deg", "n_bchg", "yields", "sum_cut", "sum_bnodes",
               "sum_invb", "cut", "bnodes", "npairs", "stuck")


def check_ids(chains, n_check):
    """Local chain indices to re-run on the oracle: both ends, the middle and an even spread."""
    ids = {0, chains - 1, chains // 2, min(1, chains - 1)}
    ids.update(int(x) for x in np.linspace(0, chains - 1, max(2, n_check)).round())
    return sorted(ids)[:max(n_check, 4)]


def parity_check(w, ch, bounds, base, seed, chain_id0, total_steps, n_check, workers):
    """Checker leg (outside the timed region): re-run a spread of the benched chains on the C
    oracle (oracle/flipchain_oracle.c) from the same initial plan for the same number of
    counted steps, and compare the final plan, the populations and every stats field (the
    fp64 sum bitwise) with what the GPU holds.  Trajectories do not depend on how the steps
    were split into launches, so one oracle call covers warm-up plus timed launches."""
    from concurrent.futures import ThreadPoolExecutor

    from flipcomplexityempirical_amd.chain import PROPOSALS, metropolis_table
    from oracle import oracle as O
    ids = check_ids(ch.n_chains, n_check)
    labs, st, pops = ch.labels(), ch.stats(), ch.pops()
    mode = PROPOSALS[w.proposal] if isinstance(w.proposal, str) else int(w.proposal)
    bases = np.broadcast_to(np.asarray(base, np.float64), (ch.n_chains,))
    init = np.asarray(w.init, np.int16)

    def one(i):
        thr = metropolis_table(float(bases[i]), ch.dgraph.maxdeg)
        lab0 = init if init.ndim == 1 else init[i]
        olab, ost, opops, _ = O.run_chain(w.graph, lab0, w.k, mode, *bounds, thr, seed,
                                          chain_id0 + i, total_steps)
        bad = [f for f in STAT_FIELDS
               if ost[f][0].tobytes() != np.asarray(st[f][i], ost[f].dtype).tobytes()]
        if not np.array_equal(olab, labs[i]):
            bad.append("labels")
        if not np.array_equal(opops, pops[i]):
            bad.append("pops")
        return i, bad

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        res = list(ex.map(one, ids))
    mism = {str(chain_id0 + i): bad for i, bad in res if bad}
    return {"chains": len(ids), "equal": len(ids) - len(mism),
            "global_ids": [chain_id0 + i for i in ids], "steps_per_chain": int(total_steps),
            "compared": "final plan, populations, all 19 stats fields (sum_invb bitwise)",
            "mismatches": mism, "oracle_s": round(time.perf_counter() - t0, 2)}


def secondary_line(dg, w, chains, init, proposal, bounds, base, seed, lo, inner, warmup, steps):
    """The same warm-up and timed launch counts at ``inner`` steps per launch on a fresh set
    of the same chains (the round 1-5 driver protocol at inner = 1,000): chains earlier in
    their burn-in, reported beside the headline, never as it."""
    import torch

    from flipcomplexityempirical_amd.chain import Chains
    ch = Chains(dg, chains, w.k, init, proposal=proposal, pop_bounds=bounds, base=base,
                seed=seed, chain_id0=lo)
    for _ in range(warmup):
        ch.run(inner)
    s0 = int(ch.stats()["steps"].astype(np.uint64).sum())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    for _ in range(steps):
        ch.run_async(inner)
        ch.sync()
        kms.append(ch.last_kernel_ms())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s1 = int(ch.stats()["steps"].astype(np.uint64).sum())
    ch.close()
    return {"value": (s1 - s0) / dt, "unit": "flip steps/s",
            "flip_steps_per_chain_per_step": inner, "warmup": warmup, "steps": steps,
            "ms_per_step": dt * 1e3 / steps, "kernel_ms": float(np.mean(kms)),
            "protocol": f"{warmup} + {steps} launches of {inner} steps per chain on fresh chains "
                        f"(timed steps {warmup * inner}-{(warmup + steps) * inner} of each chain: "
                        f"earlier in the burn-in than the headline)"}


def flipwalk_env():
    """FLIPWALK_* overrides active in this process (they change launch plans, not trajectories)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("FLIPWALK_")}


# ------------------------------------------------------------------ PMC profiles
def pmc_key(config, order, chains, inner, warmup, steps, chain_id0=0, resumed=0):
    """Name of the PMC summary of one bench protocol (profiles/pmc/<key>.json): workload,
    chains on this GPU (and the first global id when it is a shard other than the first),
    steps per launch, warm-up and timed launches, and the counted steps per chain a
    --resume checkpoint already held (the steady state)."""
    from flipcomplexityempirical_amd.workloads import C4_ORDER
    name = config
    if config == "c4" and (order or C4_ORDER) != "hilbert":
        name += "r"
    key = f"{name}_{chains}_{inner}_w{warmup}_s{steps}"
    if chain_id0:
        key += f"_id{chain_id0}"
    if resumed:
        key += f"_r{resumed}"
    return key


def load_pmc(pmc_dir, key):
    path = os.path.join(pmc_dir, key + ".json")
    if not pmc_dir or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def pmc_mismatch(prof, identity, kernel_ms, tol=0.10):
    """Why a stored PMC profile does not describe this line (None when it does): it must
    come from the same workload, protocol, FLIPWALK_* settings and library build, and its
    timed launches' rocprof kernel time must be within ``tol`` of this line's HIP-event
    kernel time (otherwise its per-launch counters describe other launches)."""
    if prof is None:
        return "no PMC profile of this protocol (profiles/pmc, scripts/profile.sh)"
    pid = prof.get("identity")
    if not pid:
        return f"profile {prof.get('source')} carries no identity (an older protocol)"
    diff = sorted(k for k in set(pid) | set(identity) if pid.get(k) != identity.get(k))
    if diff:
        return (f"profile {prof.get('source')} is of another configuration: "
                + ", ".join(f"{k}={pid.get(k)!r} here {identity.get(k)!r}" for k in diff))
    pms = (prof.get("kernel_trace") or {}).get("avg_ms")
    if not pms or abs(pms - kernel_ms) > tol * kernel_ms:
        return (f"profile {prof.get('source')} timed launches at {pms} ms (rocprof) vs this "
                f"line's {kernel_ms:.4g} ms: more than {tol:.0%} apart")
    return None


# ------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inner", type=int, default=5000,
                    help="flip steps per chain per launch (see the module docstring)")
    ap.add_argument("--secondary-inner", type=int, default=1000,
                    help="N=1: also time the same launch counts at this many steps per launch "
                         "(the round 1-5 protocol) on fresh chains -> \"secondary\" (0 = off)")
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c4", "c5", "frank"],
                    help="workload (flipcomplexityempirical_amd/workloads.py); the driver's line "
                         "is the default c3")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: --chains (default: the configuration's) in total, sharded; "
                         "weak: --chains per GPU")
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="run only rank R's shard of an N-GPU job, standalone on this GPU (one "
                         "line per shard; the N-GPU job's rate is total steps / max shard time: "
                         "scripts/shards.sh)")
    ap.add_argument("--ladder", default="interleaved", choices=["interleaved", "contiguous"],
                    help="C5: base groups spread over the shards in snake order of the ladder octaves "
                         "(default, workloads.ladder_base_index) or adjacent (round 1)")
    ap.add_argument("--order", default=None, choices=["random", "hilbert"],
                    help="C4: node numbering of the Delaunay graph (workloads.C4_ORDER by default)")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--base", type=float, default=None)
    ap.add_argument("--percent", type=float, default=None)
    ap.add_argument("--proposal", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check-chains", type=int, default=16,
                    help="chains per rank re-run on the C oracle after the timed region and "
                         "compared bit for bit (parity_check; 0 = off)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo for rehearsals)")
    ap.add_argument("--same-device", action="store_true",
                    help="put every rank on GPU 0 (multi-rank rehearsal on a one-GPU box)")
    ap.add_argument("--maps", action="store_true",
                    help="also keep the spatial observables (cut_times, part_sum, ...) per chain")
    ap.add_argument("--resume", default=None, metavar="NPZ",
                    help="continue the chains of a --save-checkpoint file (same workload, seed "
                         "and shard) instead of starting from the seed plan: steady-state "
                         "timing and profiling without the burn-in launches")
    ap.add_argument("--save-checkpoint", default=None, metavar="NPZ",
                    help="write the chains (Chains.save_checkpoint) after the timed launches")
    ap.add_argument("--save-hist", default=None, metavar="NPZ",
                    help="rank 0 writes the merged histograms (hist_cut, hist_b) and the "
                         "gathered per-chain final cut / |B| to this file")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles", "pmc"),
                    help="per-workload rocprofv3 PMC summaries (scripts/profile.sh -> "
                         "scripts/pmc_summary.py), named by pmc_key(): per-launch HBM traffic, "
                         "VALU issue and achieved occupancy for the roofline fields")
    args = ap.parse_args()
    if args.maps and args.resume:
        # fw_chains_write refuses plan writes while maps are on, and maps cannot be enabled
        # after a restore (the handle has run): checkpoints do not carry the per-node maps
        ap.error("--maps cannot be combined with --resume (checkpoints carry no spatial maps)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # a process group whenever torch.distributed.run launched us, also at world 1 (the RCCL
    # path then runs its collectives over one rank: tests/test_distributed.py)
    launched = "MASTER_ADDR" in os.environ and "WORLD_SIZE" in os.environ
    if world > 1 and not launched:
        # every rank would run its shard unsynchronised and rank 0 would report a 1-GPU line
        raise SystemExit("WORLD_SIZE > 1 without MASTER_ADDR: launch bench.py through "
                         "torch.distributed.run (or set the rendezvous variables)")
    shard_rank, shard_world = rank, world
    if args.shard:
        if launched:
            raise SystemExit("--shard emulates one rank of a job: run it as a single process")
        shard_rank, shard_world = (int(x) for x in args.shard.split("/"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = 0 if args.same_device else local_rank
    import torch
    dist = None
    if launched:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    tdev = "cuda" if args.backend == "nccl" else "cpu"
    from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds
    from flipcomplexityempirical_amd.distributed import merge_histograms, shard_range

    w = workload(args.config, args.grid, args.k, args.order)
    w.interleave = args.ladder == "interleaved"
    g, init, k = w.graph, w.init, w.k
    proposal = args.proposal or w.proposal
    percent = args.percent if args.percent is not None else w.percent
    if args.scaling == "strong":
        total = args.chains or w.chains
        lo, hi = shard_range(total, shard_world, shard_rank)
    else:
        per = args.chains or w.chains
        total = per * shard_world
        lo, hi = shard_rank * per, (shard_rank + 1) * per
    chains = hi - lo
    if args.base is not None:
        base, base_desc = args.base, f"base {args.base:.9g}"
    else:
        base, base_desc = w.bases(lo, hi), w.base_desc(0, total)
    bounds = population_bounds(g.total_pop, k, percent)
    dg = DeviceGraph(g, device=device)
    ch = Chains(dg, chains, k, init, proposal=proposal, pop_bounds=bounds, base=base,
                seed=args.seed, chain_id0=lo)
    if args.maps:
        ch.enable_maps([-1, 1] if k == 2 else None)
    resumed = 0  # counted steps per chain already in the checkpoint
    if args.resume:
        from flipcomplexityempirical_amd.chain import STATS_DTYPE
        ckf = np.load(args.resume, allow_pickle=False)
        ck = {key: ckf[key] for key in ckf.files}
        ck["stats"] = ckf["stats"].view(STATS_DTYPE)
        ch.restore(ck)
        resumed = int(ck["stats"]["steps"].max())

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
        t = torch.tensor([dt, float(steps_local), float(d["attempts"]), float(d["accepts"])],
                         dtype=torch.float64, device=tdev)
        dist.all_reduce(t[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:4], op=dist.ReduceOp.SUM)
        dt, steps_all, att_all, acc_all = (float(x) for x in t)
    else:
        steps_all, att_all, acc_all = float(steps_local), float(d["attempts"]), float(d["accepts"])
    hist_cut, hist_b = merge_histograms(ch.hist_cut(), ch.hist_b(), dist)

    # checker leg, after the timed region: every rank re-runs a spread of its chains on the
    # C oracle; the line carries the totals over ranks
    pc = None
    if args.check_chains > 0:
        pc = parity_check(w, ch, bounds, base, args.seed, lo,
                          resumed + (args.warmup + args.steps) * args.inner, args.check_chains,
                          host_cores()[0])
        yields_local = int(st1_arr["yields"].astype(np.uint64).sum())
        if dist is not None:
            t = torch.tensor([pc["chains"], pc["equal"], yields_local], dtype=torch.int64,
                             device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            pc["chains"], pc["equal"], yields_all = (int(x) for x in t)
            pc["ranks"] = world
        else:
            yields_all = yields_local
        # every yield of every chain lands in exactly one bin of each merged histogram
        pc["hist_yields_equal"] = bool(int(hist_cut.sum()) == yields_all ==
                                       int(hist_b.sum()))

    if args.save_checkpoint:
        ch.save_checkpoint(args.save_checkpoint)
    if args.save_hist:
        fin = np.stack([st1_arr["cut"], st1_arr["bnodes"]]).astype(np.int64)
        if dist is not None:
            parts = [None] * world
            dist.all_gather_object(parts, fin)
            fin = np.concatenate(parts, axis=1)
        if rank == 0:
            np.savez(args.save_hist, hist_cut=hist_cut, hist_b=hist_b, final=fin)
    kernel_ms = float(np.mean(kms))
    bytes_per_launch = algorithmic_bytes(d) / args.steps
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    from flipcomplexityempirical_amd._lib import build_info
    identity = {
        "config": args.config, "order": args.order, "grid": args.grid, "k": k,
        "proposal": proposal, "base": base_desc, "percent": percent, "seed": args.seed,
        "chains": chains, "chain_id0": lo, "inner": args.inner,
        "warmup": args.warmup, "steps": args.steps, "resumed_steps": resumed,
        "maps": bool(args.maps), "flipwalk_env": flipwalk_env(), "build": build_info(),
    }
    prof = load_pmc(args.pmc_dir, pmc_key(args.config, args.order, chains, args.inner,
                                          args.warmup, args.steps, lo, resumed))
    why = pmc_mismatch(prof, identity, kernel_ms)
    pmc_from = prof.get("source") if prof else None
    if why:
        prof = None  # its counters would describe other launches: every PMC field null
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    issue = None
    if prof and prof.get("valu_insts_per_launch"):
        # what binds this kernel: VALU issue.  Peak: every SIMD takes one wave64 VALU
        # instruction per 2 cycles (SIMD-32, MI355X_MICROARCH.md) -> 256 CUs x 4 SIMDs
        # x 2.4 GHz / 2; achieved: the PMC pass's VALU wave-instructions per timed launch
        # over this run's mean launch time (the same protocol, pmc_mismatch).
        peak = 256 * 4 * 2.4e9 / 2
        ach = prof["valu_insts_per_launch"] / (kernel_ms * 1e-3)
        issue = {"bound": "valu-issue", "achieved": ach, "peak": peak,
                 "unit": "wave-instr/s", "frac": ach / peak, "source": prof.get("source"),
                 # rocprofv3 --kernel-trace mean of the same timed launches, same command
                 "rocprof_kernel_ms": (prof.get("kernel_trace") or {}).get("avg_ms"),
                 "wait_any_frac": prof.get("wait_any_frac"),
                 "wait_inst_any_frac": prof.get("wait_inst_any_frac")}
    try:
        occupancy = dict(ch.launch_info())
    except AttributeError:  # an A/B library older than fw_chains_launch_info
        occupancy = {}
    occupancy["achieved_waves_per_simd"] = prof.get("achieved_waves_per_simd") if prof else None
    occupancy["source"] = prof.get("source") if prof else None
    l2 = None
    if prof and prof.get("l2_requests_per_launch") is not None:
        l2 = {"requests_per_launch": prof["l2_requests_per_launch"], "hit": prof.get("l2_hit"),
              "requests_per_attempt": prof["l2_requests_per_launch"] / max(1.0, d["attempts"] / args.steps)}
    pmc_info = {"key": pmc_key(args.config, args.order, chains, args.inner, args.warmup,
                               args.steps, lo, resumed),
                "source": pmc_from, "used": why is None, "reason_null": why}

    if rank == 0:
        if args.shard:
            par = (f"shard {shard_rank} of {shard_world} (global chain ids [{lo}, {hi})) run "
                   f"standalone on 1 GPU: one rank of the {shard_world}-GPU job")
        elif dist is None:
            par = "1 GPU"
        elif args.same_device:
            par = (f"REHEARSAL: {world} ranks on ONE device (same device, {args.backend} "
                   f"process group); chain ids sharded by shard_range, histograms merged by one "
                   f"{args.backend} all-reduce")
        else:
            par = (f"{world} GPUs, one process each: chain ids sharded by shard_range (no "
                   f"data-path collective), histograms merged by one "
                   f"{'RCCL (nccl) all-reduce over xGMI' if args.backend == 'nccl' else 'gloo all-reduce'}")
        out = {
            "metric": METRIC,
            "value": steps_all / dt,
            "unit": "flip steps/s",
            "n_gpus": 1 if args.same_device else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": f"{w.desc}, {total} chains in total ({chains} on rank 0), "
                            f"{proposal} proposal, {base_desc}, {percent:.0%} pop bound, "
                            f"contiguity",
                "chains_total": total,
                "chains_per_gpu": chains,
                "shard": args.shard,
                "ladder": args.ladder if w.base is None else None,
                "spatial_maps": bool(args.maps),
                "flip_steps_per_chain_per_step": args.inner,
                "resumed_steps_per_chain": resumed,
                "parallelism": par,
                "flipwalk_env": flipwalk_env(),
            },
            "parity_check": pc,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_null_reason": None if traffic is not None else why,
            },
            "issue_roofline": issue,
            "occupancy": occupancy,
            "l2": l2,
            "pmc": pmc_info,
            "identity": identity,
            "kernel_ms": kernel_ms,
            "proposals_per_s": att_all / dt,
            "accepts_per_s": acc_all / dt,
            "valid_frac": d["steps"] / max(1, d["attempts"]),
            "accept_frac": d["accepts"] / max(1, d["steps"]),
            "bfs_runs_per_step": d["bfs_runs"] / max(1, d["steps"]),
            "bfs_nodes_per_run": d["bfs_nodes"] / max(1, d["bfs_runs"]),
            "alg_bytes_per_proposal": algorithmic_bytes(d) / max(1, d["attempts"]),
            "mean_cut": float(st1_arr["cut"].mean()),
            "mean_bnodes": float(st1_arr["bnodes"].mean()),
            "hist_yields": int(hist_cut.sum()),
        }
        if world == 1 and not args.shard and args.secondary_inner > 0 and not args.resume \
                and not args.maps and args.secondary_inner != args.inner:
            out["secondary"] = secondary_line(dg, w, chains, init, proposal, bounds, base,
                                              args.seed, lo, args.secondary_inner, args.warmup,
                                              args.steps)
        if world == 1 and not args.no_cpu_baseline:
            b0 = float(np.ravel(base)[0])
            if not args.shard:
                out["cpu_baseline"] = cpu_baseline(args.config, w.desc, percent, b0, args.seed,
                                                   seconds=args.cpu_seconds)
            # every line (shards too): the native C path on the host cores, and the GPU's
            # rate over it extrapolated to every hardware thread of the host
            out["cpu_native"] = native_cpu_baseline(w, bounds, base, args.seed,
                                                    seconds=args.cpu_seconds, lo=lo,
                                                    chains=chains)
            out["cpu_native"]["gpu_over_all_cpus"] = (
                out["value"] / out["cpu_native"]["extrapolated_all_cpus"])
        print(json.dumps(out), flush=True)
    ch.close()
    dg.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
