"""Per-work-unit wall times of one grid-kernel launch (diagnostic stamps build).

Each unit (a quad of four chains x a slice of the launch's steps) records s_memrealtime
(100 MHz) when it starts and when its state is written back.  Prints the launch span,
the spread of unit start times (dispatch) and the distribution of unit durations: with
fewer quads than resident waves the launch lasts as long as its slowest unit.

    python scripts/unit_times.py [chains] [warm launches] [config]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["FLIPWALK_LIB"] = os.path.join(ROOT, "flipcomplexityempirical_amd", "libflipwalk_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from flipcomplexityempirical_amd import _lib  # noqa: E402
from flipcomplexityempirical_amd.chain import Chains, DeviceGraph, population_bounds  # noqa: E402
from flipcomplexityempirical_amd.workloads import workload  # noqa: E402

nch = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = workload(sys.argv[3] if len(sys.argv) > 3 else "c3")
L = _lib.load()
L.fw_debug_unit_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
dg = DeviceGraph(w.graph)
ch = Chains(dg, nch, w.k, w.init, proposal=w.proposal,
            pop_bounds=population_bounds(w.graph.total_pop, w.k, w.percent), base=w.bases(0, nch))
for _ in range(warm):
    ch.run(1000)
ch.run(1000)
nq = (nch + 3) // 4
slices = int(os.environ.get("FLIPWALK_SLICES", "0")) or None
buf = np.zeros(3 * 65536, np.uint64)
assert L.fw_debug_unit_times(buf.ctypes.data_as(ctypes.c_void_p), 65536) == 0
t = buf[:2 * 65536].reshape(-1, 2).astype(np.int64)
hw = buf[2 * 65536:]
used = t[:, 1] > 0
t = t[used]
hw = hw[used]
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0   # microseconds
dur = en - st
print(f"chains {nch}: units {len(t)} (quads {nq}), kernel {ch.last_kernel_ms():.3f} ms by HIP events")
print(f"launch span {en.max():.1f} us; unit starts: p50 {np.percentile(st, 50):.1f} "
      f"p99 {np.percentile(st, 99):.1f} max {st.max():.1f} us")
print("unit durations (us): mean %.1f  p10 %.1f  p50 %.1f  p90 %.1f  p99 %.1f  max %.1f" % (
    dur.mean(), *np.percentile(dur, [10, 50, 90, 99]), dur.max()))
print("unit ends (us):      p10 %.1f  p50 %.1f  p90 %.1f  p99 %.1f  max %.1f" % (
    *np.percentile(en, [10, 50, 90, 99]), en.max()))
st_ch = ch.stats()
att = st_ch["attempts"].astype(np.int64)
if len(t) == nq:
    qa = att[:nq * 4].reshape(nq, 4).max(1)
    print("corr(unit duration, max attempts of the quad so far) = %.3f" % np.corrcoef(dur, qa[used[:nq]])[0, 1])

# where units ran: HW_ID bits [3:0] wave slot, [5:4] SIMD, [11:8] CU, [12] SA, [15:13] SE;
# XCC_ID in the high word.  Group unit durations by how many units shared their SIMD.
simd = ((hw >> 32) & 0xF) << 12 | ((hw >> 13) & 7) << 9 | ((hw >> 12) & 1) << 8 | ((hw >> 8) & 0xF) << 4 | ((hw >> 4) & 3)
cu = simd >> 2
_, sinv, scnt = np.unique(simd, return_inverse=True, return_counts=True)
_, cinv, ccnt = np.unique(cu, return_inverse=True, return_counts=True)
print(f"SIMDs used {len(scnt)}, CUs used {len(ccnt)}; units per SIMD: " +
      ", ".join(f"{v}:{c}" for v, c in zip(*np.unique(scnt, return_counts=True))))
print("units per CU: " + ", ".join(f"{v}:{c}" for v, c in zip(*np.unique(ccnt, return_counts=True))))
per = scnt[sinv]
for v in np.unique(per):
    m = per == v
    print(f"  units on a SIMD with {v}: n={m.sum():5d} duration mean {dur[m].mean():.1f} p90 {np.percentile(dur[m], 90):.1f} max {dur[m].max():.1f}")
perc = ccnt[cinv]
for v in np.unique(perc):
    m = perc == v
    print(f"  units on a CU with {v}: n={m.sum():5d} duration mean {dur[m].mean():.1f} max {dur[m].max():.1f}")

# VALU issue is arbitrated by priority, then wave age (MI355X_MICROARCH.md): among the
# units that shared a SIMD and started within the first 50 us, compare durations by
# start order on that SIMD
early = st < 50.0
order = np.zeros(len(st), np.int64)
for sid in np.unique(simd[early]):
    idx = np.where((simd == sid) & early)[0]
    order[idx[np.argsort(st[idx], kind="stable")]] = np.arange(len(idx))
for o in range(int(order[early].max()) + 1 if early.any() else 0):
    m = early & (order == o)
    if m.sum():
        print(f"  start order {o} on its SIMD: n={m.sum():5d} duration mean {dur[m].mean():.1f} "
              f"p10 {np.percentile(dur[m], 10):.1f} p90 {np.percentile(dur[m], 90):.1f}")
slot = (hw & 0xF).astype(np.int64)
for s_ in np.unique(slot[early]):
    m = early & (slot == s_)
    print(f"  wave slot {s_}: n={m.sum():5d} duration mean {dur[m].mean():.1f}")

# per XCD (XCC_ID, the high word): a slower die shows as a shifted duration distribution
xcc = ((hw >> 32) & 0xF).astype(np.int64)
for x_ in np.unique(xcc):
    m = xcc == x_
    print(f"  XCD {x_}: n={m.sum():5d} duration mean {dur[m].mean():.1f} p10 {np.percentile(dur[m], 10):.1f} "
          f"p90 {np.percentile(dur[m], 90):.1f} max {dur[m].max():.1f}")
# per quad: the quad's own chains (attempts this launch) vs its duration
if len(t) == nq:
    se = ((hw >> 13) & 7).astype(np.int64)
    for s_ in np.unique(se):
        m = se == s_
        print(f"  SE {s_}: n={m.sum():5d} duration mean {dur[m].mean():.1f}")
