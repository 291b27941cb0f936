"""Per-phase cycle shares of the grid16 kernel (diagnostic stamps build)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["FLIPWALK_LIB"] = os.path.join(ROOT, "flipcomplexityempirical_amd", "libflipwalk_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from flipcomplexityempirical_amd import _lib  # noqa: E402
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds  # noqa: E402
from flipcomplexityempirical_amd.graph import block_seed, grid_graph  # noqa: E402

L = _lib.load()
L.fw_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
g = grid_graph(n, n)
dg = DeviceGraph(g)
ch = Chains(dg, 65536, 4, block_seed(n, n, 2, 2), proposal="pairs",
            pop_bounds=population_bounds(n * n, 4, 0.05), base=2.63815853, seed=0)
ch.run(1000)
ch.run(1000)
buf = np.zeros(8, np.uint64)
L.fw_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
for _ in range(3):
    ch.run(1000)
L.fw_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), 0)
names = ["draw", "select L1", "select L2", "gather+pop", "ring+search", "commit+observe",
         "loop exit", "-"]
tot = buf[:7].sum()
st = ch.stats()
print("kernel ms/launch (stamped):", ch.last_kernel_ms())
iters = st["attempts"].sum() / 4  # rough: 4 chains per wave iteration
for nm, v in zip(names, buf):
    if v:
        print(f"{nm:16s} {v / tot * 100:6.2f} %")
