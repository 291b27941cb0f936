"""Per-phase cycle shares of the grid16 kernel (diagnostic stamps build)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FLIPWALK_LIB", os.path.join(ROOT, "flipcomplexityempirical_amd", "libflipwalk_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from flipcomplexityempirical_amd import _lib  # noqa: E402
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds  # noqa: E402

L = _lib.load()
L.fw_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
# usage: stamps.py [config] [chains] [warm launches]   (config c3 default; c5 = the 64-base
# ladder workload; warm launches of 1000 steps before the stamped ones, default 2; an
# optional checkpoint to resume from first)
from flipcomplexityempirical_amd.workloads import workload  # noqa: E402
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
w = workload("c4", order="random") if cfg == "c4r" else workload(cfg)
nch = int(sys.argv[2]) if len(sys.argv) > 2 else w.chains
g = w.graph
dg = DeviceGraph(g)
ch = Chains(dg, nch, w.k, w.init, proposal=w.proposal,
            pop_bounds=population_bounds(g.total_pop, w.k, w.percent), base=w.bases(0, nch), seed=0)
if len(sys.argv) > 4:  # a bench.py --save-checkpoint file of the same workload and chains
    from flipcomplexityempirical_amd.chain import STATS_DTYPE  # noqa: E402
    ckf = np.load(sys.argv[4], allow_pickle=False)
    ck = {key: ckf[key] for key in ckf.files}
    ck["stats"] = ckf["stats"].view(STATS_DTYPE)
    ch.restore(ck)
for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 2):
    ch.run(1000)
buf = np.zeros(16, np.uint64)
L.fw_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
L.fw_debug_stamps_csr.argtypes = [ctypes.c_void_p, ctypes.c_int]
cz = np.zeros(24, np.uint64)
L.fw_debug_stamps_csr(cz.ctypes.data_as(ctypes.c_void_p), 1)
att0 = int(ch.stats()["attempts"].sum())
for _ in range(3):
    ch.run(1000)
L.fw_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), 0)
names = ["draw", "select L1", "select L2", "gather+pop", "exact search", "counters+observe",
         "loop exit", "ring+7x7 window", "outcome+accept", "commit"]
tot = buf[:10].sum()
st = ch.stats()
print("kernel ms/launch (stamped):", ch.last_kernel_ms())
iters = (int(st["attempts"].sum()) - att0) / 4  # rough: 4 chains per wave iteration
print(f"7x7 window runs per wave-iter {buf[12] / iters:.3f}, flood iterations per run {buf[13] / max(buf[12], 1):.2f}")
for nm, v in zip(names, buf):
    if v:
        print(f"{nm:16s} {v / tot * 100:6.2f} %  {v / iters:8.1f} clk/wave-iter")

# the one-chain-per-wave kernel's stamps (configurations routed to it, e.g. C4, C5)
L.fw_debug_stamps_csr.argtypes = [ctypes.c_void_p, ctypes.c_int]
cb = np.zeros(24, np.uint64)
L.fw_debug_stamps_csr(cb.ctypes.data_as(ctypes.c_void_p), 0)
if cb[:6].sum():
    att = int(st["attempts"].sum()) - att0
    cn = ["draw", "select", "gather+target+pop", "contiguity", "accept+commit", "observe"]
    tot = cb[:6].sum()
    print("one-chain-per-wave kernel, attempts timed:", att)
    for nm, v in zip(cn, cb[:6]):
        print(f"{nm:18s} {v / tot * 100:6.2f} %  {v / att:8.1f} clk/attempt")
    print(f"contiguity decided by: 7x7 window {cb[8] / att:.3f}/attempt, bitboard search "
          f"{cb[9] / att:.3f}, list search {cb[10] / att:.3f}")
    if cb[6]:
        print(f"list search: {cb[6] / max(cb[10], 1):.1f} levels per run, "
              f"{cb[7] / max(cb[10], 1):.2f} of the runs seeded by the bitboard, "
              f"map-test rounds {cb[15] / cb[6]:.2f} per level, "
              f"restore {cb[14] / max(cb[10], 1):.0f} clk per run")
    if cb[11] + cb[12] + cb[13]:
        print(f"contiguity cycles by path (per attempt / per run): 7x7 window "
              f"{cb[11] / att:.0f} / {cb[11] / max(cb[8], 1):.0f}, bitboard {cb[12] / att:.0f} / "
              f"{cb[12] / max(cb[9], 1):.0f}, list search {cb[13] / att:.0f} / "
              f"{cb[13] / max(cb[10], 1):.0f}")
    if cb[16] + cb[17] + cb[18]:
        bbs = max(int(cb[9]), 1)
        print(f"64-row bitboard (two-class path): {cb[16] / bbs:.1f} levels on 32 columns, "
              f"{cb[17] / bbs:.1f} on 64 per run; 128-wide stage: {cb[18] / att:.4f} runs per "
              f"attempt, {cb[19] / max(cb[18], 1):.0f} clk per run ({cb[19] / att:.0f} per attempt)")
