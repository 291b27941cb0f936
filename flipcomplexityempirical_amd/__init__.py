"""flipcomplexityempirical_amd — MI355X-native batched single-node flip walk.

The hot path of drdeford/FlipComplexityEmpirical (GerryChain's MarkovChain with
slow_reversible_propose[_bi] / propose_random_flip, single_flip_contiguous, a population
bound and the cut_accept Metropolis rule; grid_chain_sec11.py:340-342) as hand-written
HIP kernels for gfx950 behind the C-ABI in include/flipwalk.h.
"""
from .graph import Graph, block_seed, grid_graph, sec11_graph, sec11_seed, stripe_seed  # noqa: F401
from .chain import (Chains, DeviceGraph, RunResult, eval_flips, expected_wait_sum,  # noqa: F401
                    metropolis_table, population_bounds, run_chains)

__version__ = "0.1.0"
