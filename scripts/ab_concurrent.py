"""A/B: one fw_chains object over all chains vs P objects over equal slices, launched
concurrently on their own streams (do other kernels' waves fill a launch's tail?).

    python scripts/ab_concurrent.py [workload] [chains] [steps_per_launch] [launches]
"""
import json
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds  # noqa: E402
from flipcomplexityempirical_amd.workloads import workload  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    launches = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    w = workload(name)
    dg = DeviceGraph(w.graph, 0)
    bounds = population_bounds(w.graph.total_pop, w.k, w.percent)
    for P in (1, 2, 3, 4, 1):
        part = [chains // P + (1 if i < chains % P else 0) for i in range(P)]
        objs, lo = [], 0
        for n in part:
            objs.append(Chains(dg, n, w.k, w.init, proposal=w.proposal, pop_bounds=bounds,
                               base=w.bases(lo, lo + n), seed=0, chain_id0=lo))
            lo += n
        for o in objs:
            o.run_async(steps)
        for o in objs:
            o.sync()
        t0 = time.perf_counter()
        for _ in range(launches):
            for o in objs:
                o.run_async(steps)
            for o in objs:
                o.sync()
        dt = time.perf_counter() - t0
        rate = chains * steps * launches / dt
        print(json.dumps({"workload": name, "chains": chains, "P": P, "steps": steps,
                          "launches": launches, "s": round(dt, 4), "steps_per_s": rate,
                          "kernel_ms": [round(o.last_kernel_ms(), 2) for o in objs]}), flush=True)
        for o in objs:
            o.close()


if __name__ == "__main__":
    main()
