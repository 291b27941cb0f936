"""Multi-process sharding on CPU (gloo, world_size 2).

The GPU path shards global chain ids over ranks with no data-path collective and
merges histograms with one all-reduce (flipcomplexityempirical_amd/distributed.py).  Here
each rank runs its shard on the CPU oracle (the per-rank engine is irrelevant to the
sharding logic under test), and the merged histograms/stats must be bit-identical to a
single-process run of all chains: the per-chain Philox key is the global id.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from flipcomplexityempirical_amd.distributed import (gather_stats, merge_histograms,
                                                     shard_range)

N_TOTAL, STEPS, SEED = 10, 300, 99


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_shard(case, lo, hi):
    from oracle import oracle as O
    g = case.graph
    hc = np.zeros(g.n_edges + 1, np.uint64)
    hb = np.zeros(g.n + 1, np.uint64)
    st = np.zeros(hi - lo, O.STATS_DTYPE)
    for i, cid in enumerate(range(lo, hi)):
        _, s, _, _ = O.run_chain(g, case.init, case.k, case.mode, *case.bounds, case.thr, SEED, cid,
                                 STEPS, hist_cut=hc, hist_b=hb)
        st[i] = s[0]
    return hc, hb, st


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from cases import cases
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    case = {c.name: c for c in cases(include_kansas=False)}["grid12_k4_pairs"]
    lo, hi = shard_range(N_TOTAL, world, rank)
    hc, hb, st = _run_shard(case, lo, hi)
    mhc, mhb = merge_histograms(hc, hb, dist)
    mst = gather_stats(st, N_TOTAL, dist, lo)
    if rank == 0:
        np.savez(out, hc=mhc, hb=mhb, st=mst.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (1, 7, 65536):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_two_rank_merge_is_bit_identical(tmp_path):
    from cases import cases
    case = {c.name: c for c in cases(include_kansas=False)}["grid12_k4_pairs"]
    out = str(tmp_path / "merged.npz")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    hc, hb, st = _run_shard(case, 0, N_TOTAL)
    assert np.array_equal(got["hc"], hc) and np.array_equal(got["hb"], hb)
    assert np.array_equal(got["st"], st.view(np.uint8))


def test_merge_without_process_group_is_identity():
    a, b = np.arange(5, dtype=np.uint64), np.arange(3, dtype=np.uint64)
    x, y = merge_histograms(a, b, None)
    assert x is a and y is b


def oracle_engine(graph, init_labels, k, n_chains, steps, chain_id0=0, device=0, proposal="pairs",
                  pop_bounds=None, base=1.0, seed=0, **_):
    """run_chains' signature and result on the CPU oracle (test stand-in for the GPU)."""
    from flipcomplexityempirical_amd.chain import (PROPOSALS, RunResult, metropolis_table)
    from oracle import oracle as O
    hc = np.zeros(graph.n_edges + 1, np.uint64)
    hb = np.zeros(graph.n + 1, np.uint64)
    st = np.zeros(n_chains, O.STATS_DTYPE)
    init = np.asarray(init_labels)
    bases = np.broadcast_to(np.asarray(base, np.float64), (n_chains,))
    labs = []
    for i in range(n_chains):
        lab0 = init[i] if init.ndim == 2 else init
        lab, s, _, _ = O.run_chain(graph, lab0, k, PROPOSALS[proposal], *pop_bounds,
                                   metropolis_table(bases[i], graph.maxdeg), seed, chain_id0 + i,
                                   steps, hist_cut=hc, hist_b=hb)
        st[i] = s[0]
        labs.append(lab)
    return RunResult(np.stack(labs), st, hc, hb, None, 0.0)


def _sharded_worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from test_distributed import _sharded_inputs, oracle_engine
    from flipcomplexityempirical_amd.distributed import run_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, init, bases, bounds = _sharded_inputs()
    res, hc, hb, st = run_sharded(g, init, 4, N_TOTAL, STEPS, dist, engine=oracle_engine,
                                  proposal="pairs", pop_bounds=bounds, base=bases, seed=SEED)
    lo, hi = shard_range(N_TOTAL, world, rank)
    assert len(res.stats) == hi - lo
    if rank == 0:
        np.savez(out, hc=hc, hb=hb, st=st.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


def _sharded_inputs():
    from flipcomplexityempirical_amd.chain import population_bounds
    from flipcomplexityempirical_amd.graph import block_seed, grid_graph
    g = grid_graph(12, 12)
    init = np.stack([block_seed(12, 12, 2, 2)] * N_TOTAL)
    init[N_TOTAL // 2:] = np.ascontiguousarray(
        block_seed(12, 12, 2, 2).reshape(12, 12).T).reshape(-1)  # per-chain plans differ
    bases = np.geomspace(0.5, 2.0, N_TOTAL)  # per-chain bases
    return g, init, bases, population_bounds(g.n, 4, 0.10)


def test_run_sharded_two_ranks_slices_per_chain_inputs(tmp_path):
    """run_sharded over gloo, world 2: each rank runs its id range with ITS rows of the
    per-chain plans and bases; the merged result equals one process running all chains."""
    out = str(tmp_path / "sharded.npz")
    mp.start_processes(_sharded_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    g, init, bases, bounds = _sharded_inputs()
    ref = oracle_engine(g, init, 4, N_TOTAL, STEPS, proposal="pairs", pop_bounds=bounds,
                        base=bases, seed=SEED)
    assert np.array_equal(got["hc"], ref.hist_cut) and np.array_equal(got["hb"], ref.hist_b)
    assert np.array_equal(got["st"], ref.stats.view(np.uint8))


def _gpu_sharded_worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from test_distributed import _sharded_inputs
    from flipcomplexityempirical_amd.distributed import run_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, init, bases, bounds = _sharded_inputs()
    # the real engine (chain.run_chains -> libflipwalk.so), every rank on device 0
    res, hc, hb, st = run_sharded(g, init, 4, N_TOTAL, STEPS, dist, device=0,
                                  proposal="pairs", pop_bounds=bounds, base=bases, seed=SEED)
    lo, hi = shard_range(N_TOTAL, world, rank)
    assert len(res.stats) == hi - lo
    np.savez(out + f".{rank}.npz", labels=res.labels)
    if rank == 0:
        np.savez(out, hc=hc, hb=hb, st=st.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_run_sharded_two_ranks_bit_identical(tmp_path, gpu_lib):
    """run_sharded with the GPU engine in 2 gloo ranks (both on device 0): each rank's
    handle runs its id range with its rows of the per-chain plans and bases; the merged
    histograms and stats equal ONE handle running all chains, and the oracle, bit for bit."""
    from flipcomplexityempirical_amd.chain import run_chains
    out = str(tmp_path / "gpu_sharded.npz")
    mp.start_processes(_gpu_sharded_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    g, init, bases, bounds = _sharded_inputs()
    one = run_chains(g, init, 4, N_TOTAL, STEPS, proposal="pairs", pop_bounds=bounds, base=bases,
                     seed=SEED)
    assert np.array_equal(got["hc"], one.hist_cut) and np.array_equal(got["hb"], one.hist_b)
    assert np.array_equal(got["st"], one.stats.view(np.uint8))
    labs = np.concatenate([np.load(out + f".{r}.npz")["labels"] for r in range(2)])
    assert np.array_equal(labs, one.labels)
    ref = oracle_engine(g, init, 4, N_TOTAL, STEPS, proposal="pairs", pop_bounds=bounds,
                        base=bases, seed=SEED)
    assert np.array_equal(one.hist_cut, ref.hist_cut) and np.array_equal(one.hist_b, ref.hist_b)
    assert np.array_equal(one.stats.view(np.uint8), ref.stats.view(np.uint8))


@pytest.mark.gpu
def test_bench_under_torchrun_two_ranks(tmp_path, gpu_lib):
    """bench.py itself under torch.distributed.run at world 2 (gloo process group, both ranks
    on device 0): the max-over-ranks timing, the checker all-reduce and the histogram merge
    of the multi-rank path.  Every checked chain equals the oracle, every yield lands in one
    bin of each merged histogram, and the merged histograms and the final per-chain cut / |B|
    equal a world-1 run of the same 8,192 chains bit for bit."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--config", "c3", "--chains", "8192", "--steps", "2", "--warmup", "1",
            "--inner", "300", "--no-cpu-baseline", "--check-chains", "4"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    h2, h1 = str(tmp_path / "w2.npz"), str(tmp_path / "w1.npz")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--same-device", "--save-hist", h2] + args,
                       capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    pc = line["parity_check"]
    assert pc["ranks"] == 2 and pc["equal"] == pc["chains"] >= 8, pc
    assert pc["hist_yields_equal"]
    assert line["hist_yields"] == 8192 * (3 * 300 + 1)
    r1 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--save-hist", h1] + args,
                        capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads(r1.stdout.strip().splitlines()[-1])
    assert one["hist_yields"] == line["hist_yields"]
    a, b = np.load(h2), np.load(h1)
    for key in ("hist_cut", "hist_b", "final"):
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.gpu
def test_bench_rccl_branch_under_torchrun(tmp_path, gpu_lib):
    """bench.py's RCCL path itself: launched by torch.distributed.run (one rank, a fresh
    child process), it opens the "nccl" process group and runs its device-tensor
    all-reduces (max-over-ranks time, step / attempt sums, the checker totals, the
    histogram merge) over RCCL.  Every checked chain equals the oracle and every yield
    lands in exactly one bin of each merged histogram."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "1",
                        "--backend", "nccl", "--config", "c3", "--chains", "8192", "--steps", "2",
                        "--warmup", "1", "--inner", "300", "--no-cpu-baseline",
                        "--check-chains", "4"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    pc = line["parity_check"]
    assert pc["ranks"] == 1 and pc["equal"] == pc["chains"] >= 4, pc
    assert pc["hist_yields_equal"]
    assert line["hist_yields"] == 8192 * (3 * 300 + 1)
    assert "RCCL" in line["config"]["parallelism"], line["config"]["parallelism"]
