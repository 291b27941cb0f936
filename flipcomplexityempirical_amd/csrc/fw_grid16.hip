// fw_grid16.hip — the row-major-grid chain kernel: four chains per wavefront, 1-4
// wavefronts per workgroup.
//
// The chain loop is latency-bound (one dependent LDS round trip or DPP chain per
// phase, no phase dominant), so throughput follows the number of chains resident per
// CU, which LDS sets.  Each 16-lane DPP row of a wavefront owns one chain, so every
// instruction of the common path serves four chains: Philox runs on the VALU,
// per-chain scalars live in row-uniform VGPRs, prefix scans are 4-step row_shr DPP
// scans, a lane's value is broadcast to its row by a masked row scan + row_newbcast,
// and row-level votes are bit fields of one 64-bit ballot.
//
// Per chain, LDS holds only the packed labels (2 bits/node when k <= 4, else 4) and a
// u16 proposal-weight sum per 64-node group (C3, 100x100 k=4: 2,832 B).  The exact
// contiguity search (needed by <1% of proposals) runs wave-cooperatively on one chain
// at a time and marks visited nodes in a 4-bit scratch array shared by the
// workgroup's waves (held under an LDS lock), together with one shared visit list.
// Its level-synchronous race is the one of fw_device.h / the oracle, so verdicts and
// search counters match bit for bit.
//
// Semantics: oracle/flipchain_oracle.c (chain loop, proposals, contiguity, accept,
// observables), reference grid_chain_sec11.py:117-179,340-402.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>

#include "fw_device.h"

#ifdef FW_STAMPS
// Diagnostic build only (libflipwalk_stamps.so): per-phase s_memtime shares.
__device__ unsigned long long g_stamps[16];
// per work unit: s_memrealtime (100 MHz) at its start and at its write-back (units < 2^16)
// and where it ran: HW_ID (wave slot, SIMD, CU, SA, SE) | XCC_ID << 32
__device__ unsigned long long g_unit_t[2 * 65536];
__device__ unsigned long long g_unit_hw[65536];
#define UNIT_TIME(u, e)                                                         \
  do {                                                                          \
    uint64_t t_;                                                                \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    if (__lane_id() == 0 && (u) < 65536) {                                      \
      g_unit_t[2 * (u) + (e)] = t_;                                             \
      if ((e) == 0)                                                             \
        g_unit_hw[u] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) | \
                       ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32); \
    }                                                                           \
  } while (0)
#define STAMP_DECL uint64_t st_acc[16] = {}; uint64_t st_t0 = 0;
#define STAMP(i)                                              \
  do {                                                        \
    __builtin_amdgcn_sched_barrier(0);                        \
    uint64_t st_t1;                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t1)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                        \
    if (i >= 0) st_acc[(i) < 0 ? 0 : (i)] += st_t1 - st_t0;   \
    st_t0 = st_t1;                                            \
  } while (0)
#define STAMP_FLUSH                                           \
  if (__lane_id() == 0)                                       \
    for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_stamps[i_], (unsigned long long)st_acc[i_]);
#define STAMP_COUNT(i, v) st_acc[i] += (uint64_t)(v)
#else
#define STAMP_COUNT(i, v)
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#define UNIT_TIME(u, e)
#endif

#include <cstddef>

// the write-back stores the stats record as 8-byte pairs in declaration order
static_assert(sizeof(fw_chain_stats) == 136, "fw_chain_stats layout");
static_assert(offsetof(fw_chain_stats, yields) == 88 && offsetof(fw_chain_stats, sum_invb) == 112 &&
                  offsetof(fw_chain_stats, cut) == 120 && offsetof(fw_chain_stats, npairs) == 128,
              "fw_chain_stats layout");

#define HIST_ADD(ptr, v) atomicAdd(ptr, v)

// Pickers of the instantiations compiled in their own translation units (the Makefile
// schedules each differently): fw_grid16_lean.hip the small-grid lean kernels,
// fw_grid16_w2.hip the W2 ones.  The stamps build compiles everything here.
void* fw_grid16_pick_lean(int lb, int mode, int G);
void* fw_grid16_pick_w2(int mode, int G);

namespace {

constexpr int ROW = 16;
constexpr int MAX_NW = 4;          // waves per workgroup
constexpr uint32_t SCR_BLOCK = 15;  // scratch code of v during a search
constexpr int LDS_GUARD = 16;       // bytes in front of the first chain slot

// v's neighbourhood as one lane sees it (labels < 16 here, so 32-bit label sets)
struct Hood16 {
  int x;          // node id, -1 if absent
  uint32_t lx;    // label of x (NOLAB if absent)
  uint32_t bits;  // OR of 1<<label over x's neighbours other than v
  uint32_t cnt;   // number of x's neighbours other than v with label != lx
  bool has_v;     // v is a neighbour of x
  int deg;        // degree of x
};

// x / W for 0 <= x < 2^15 with a full-rate 24-bit multiply (host-verified magic)
struct GDiv {
  uint32_t m, s;
  __device__ __forceinline__ int operator()(int x) const {
    return (int)(__umul24((uint32_t)x, m) >> s);
  }
};
// r * W (+ c): full-rate 24-bit multiply (grid coordinates < 2^14; out-of-grid values
// are computed but never used)
__device__ __forceinline__ int mulW(int r, int W) { return (int)__umul24((uint32_t)r, (uint32_t)W); }

__device__ __forceinline__ uint32_t rowbits(uint64_t bal, int row) {
  return (uint32_t)(bal >> (row * ROW)) & 0xFFFFu;
}
// inclusive prefix sum within each 16-lane row
__device__ __forceinline__ uint32_t row_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
  return x;
}
// lane 15 of each row broadcast to the row (row_newbcast:15)
__device__ __forceinline__ uint32_t row_last(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x15F, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t row_sum(uint32_t x) { return row_last(row_scan(x)); }
// lane 0 of each row broadcast to the row (row_newbcast:0)
__device__ __forceinline__ uint32_t row_first(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x150, 0xF, 0xF, false);
}
// lane q takes lane q+1 of its row (row_shl:1; lane 15 gets 0)
__device__ __forceinline__ uint32_t row_shl1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, false);
}
// value held by row-lane L (row-uniform L in 0..15; anything else gives 0)
__device__ __forceinline__ uint32_t row_pick(uint32_t x, int L, int q) {
  // one LDS-crossbar permute instead of a four-step DPP row sum
  const int src = ((__lane_id() - q) + L) << 2;
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)x);
}

// Labels of the six consecutive nodes x-1 .. x+4 of a packed LB-bit label array, LB
// bits each (field 0 = x-1, fields 1..4 = x..x+3, field 5 = x+4).  Two aligned dword
// reads; the label region is padded so the second read stays inside the slot.
template <int LB>
__device__ __forceinline__ uint32_t lab_window(const LDS uint8_t* lab, int x) {
  const int bit = (x - 1) * LB;  // x - 1 may be -1: field 0 is then garbage, masked by callers
  const int wi = bit >> 5;       // arithmetic shift: -1 -> -1
  const LDS uint32_t* w = reinterpret_cast<const LDS uint32_t*>(lab);
  // wi >= -1: w[-1] is the word before the slot (the previous slot's tail, or the 16-B
  // guard in front of slot 0), masked below; one base address -> one ds_read2_b32
  const uint32_t lo0 = w[wi];
  const uint32_t lo = wi >= 0 ? lo0 : 0u;
  const uint32_t hi = w[wi + 1];
  const uint64_t both = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(both >> (uint32_t)(bit - wi * 32)) & ((1u << (6 * LB)) - 1u);
}

// Proposal weights (and cut degrees) of the four nodes x0..x0+3 (x0 a multiple of 4)
// of a row-major W x H grid, packed one per byte.  A window may wrap into the next grid
// row when W is not a multiple of 4, so neighbour windows are read whenever ANY of the
// four nodes has that neighbour; per-node row/column checks mask the rest.
template <int LB, int MODE>
__device__ __forceinline__ void weights4(const LDS uint8_t* lab, int x0, int W, int H, int n,
                                         GDiv gd, uint32_t& w4, uint32_t& cd4) {
  constexpr uint32_t M = (1u << LB) - 1u;
  w4 = 0;
  cd4 = 0;
  if (x0 >= n) return;
  const uint32_t own = lab_window<LB>(lab, x0);
  const uint32_t up = x0 + 3 - W >= 0 ? lab_window<LB>(lab, x0 - W) : 0u;
  const uint32_t dn = x0 + W < n ? lab_window<LB>(lab, x0 + W) : 0u;
  const int r0 = gd(x0);
  const int c0 = x0 - mulW(r0, W);
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    int ct = c0 + tt, rt = r0;
    if (ct >= W) {
      ct -= W;
      rt += 1;
    }
    const uint32_t lx = (own >> (LB * (tt + 1))) & M;
    const uint32_t ll = (own >> (LB * tt)) & M;
    const uint32_t lr = (own >> (LB * (tt + 2))) & M;
    const uint32_t lu = (up >> (LB * (tt + 1))) & M, ld = (dn >> (LB * (tt + 1))) & M;
    uint32_t bits = 0, cd = 0;
    if (rt > 0) { bits |= 1u << lu; cd += lu != lx; }
    if (ct > 0) { bits |= 1u << ll; cd += ll != lx; }
    if (ct < W - 1) { bits |= 1u << lr; cd += lr != lx; }
    if (rt < H - 1) { bits |= 1u << ld; cd += ld != lx; }
    uint32_t w = MODE == FW_PROPOSE_CUTEDGE ? cd : (uint32_t)__popc(bits & ~(1u << lx));
    if (x0 + tt >= n) w = cd = 0;
    w4 |= w << (8 * tt);
    cd4 |= cd << (8 * tt);
  }
}

__device__ __forceinline__ uint32_t bsum4(uint32_t v) {
  return (v & 0xFFu) + ((v >> 8) & 0xFFu) + ((v >> 16) & 0xFFu) + (v >> 24);
}

// ---- SWAR form for 2-bit labels (k <= 4): the four nodes of a lane are the four bytes
// of a dword.  A label becomes a one-hot byte (1 << label) with one v_perm_b32, so a
// node's neighbour label set is an OR of bytes and its weight a per-byte popcount.
__device__ __forceinline__ uint32_t spread4(uint32_t u) {  // fields 0..3 of u (2 bits) -> bytes
  const uint32_t t = ((u << 12) | u) & 0x000F000Fu;
  return ((t << 6) | t) & 0x03030303u;
}
__device__ __forceinline__ uint32_t onehot4(uint32_t s) {  // bytes 0..3 -> 1 << byte
  return __builtin_amdgcn_perm(0u, 0x08040201u, s);
}
__device__ __forceinline__ uint32_t low_bytes(int t) {  // 0xFF in bytes 0..t-1
  // branch-free: clamp, then a select (no exec-mask branch in the level-2 walk)
  const uint32_t tc = (uint32_t)min(max(t, 0), 4);
  return tc == 4u ? 0xFFFFFFFFu : (1u << (8u * tc)) - 1u;
}
// per byte: 0x80 where the one-hot bytes a and b differ (different labels)
__device__ __forceinline__ uint32_t ne_bytes(uint32_t a, uint32_t b) {
  return ~((a & b) + 0x7F7F7F7Fu) & 0x80808080u;
}
__device__ __forceinline__ uint32_t byte_popc(uint32_t f) {  // per-byte popcount (bytes < 16)
  const uint32_t t = f - ((f >> 1) & 0x55555555u);
  return (t & 0x33333333u) + ((t >> 2) & 0x33333333u);
}

template <int MODE, bool NEED_CD, bool BATCH = true>
__device__ __forceinline__ void weights4_swar(const LDS uint8_t* lab, int x0, int W, int H, int n,
                                              GDiv gd, uint32_t& w4, uint32_t& cd4) {
  w4 = 0;
  cd4 = 0;
  // branch-free: every read is issued at a valid position and its result masked (mN is
  // all-zero for a group tail past n)
  const int xs = x0 < n ? x0 : 0;
  const bool hasU = xs + 3 - W >= 0, hasD = xs + W < n;
  // the three windows' dword pairs (lab_window: fields x-1 .. x+4), all loaded before any
  // is used -- one LDS round trip; at the register limit the scheduler otherwise waits for
  // each pair before issuing the next -- with the edge masks computed while they land
  const LDS uint32_t* lw32 = reinterpret_cast<const LDS uint32_t*>(lab);
  const int xw[3] = {xs, hasU ? xs - W : xs, hasD ? xs + W : xs};
  uint32_t wlo[3], whi[3];
  int wbit[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    wbit[t] = (xw[t] - 1) * 2;
    const int wi = wbit[t] >> 5;  // arithmetic: -1 for x = 0 (the guard word, masked)
    wlo[t] = lw32[wi];
    whi[t] = lw32[wi + 1];
  }
  // which of the four nodes have each neighbour (W >= 4: at most one row wrap, at tw)
  const int r0 = gd(x0);
  const int c0 = x0 - mulW(r0, W);
  const int tw = W - c0;  // first byte on the next grid row (>= 4: none); >= 1
  // byte masks from 64-bit shifts of constants (a shift by 32 empties the low dword): the
  // bytes on the next grid row, the column-0 bytes (byte tw, or byte 0 when c0 == 0) and the
  // column-(W-1) byte (byte tw - 1 when tw <= 4).  Bytes past n (row H and beyond) are
  // cleared by mN, so row H - 1 may clear its next-row bytes too.  Equal to the per-byte
  // clamp/select form after the & mN on every grid W >= 4, H <= 40, all groups (host check).
  const uint32_t t8 = (uint32_t)min(tw, 4) << 3;
  const uint32_t nxt = (uint32_t)(~0ull << t8);
  const uint32_t mN = low_bytes(n - x0);
  const uint32_t mU = r0 > 0 ? 0xFFFFFFFFu : nxt;
  const uint32_t mD = r0 < H - 2 ? 0xFFFFFFFFu : (r0 == H - 2 ? ~nxt : 0u);
  const uint32_t mL = ~((uint32_t)(0xFFull << t8) | (c0 == 0 ? 0xFFu : 0u));
  const uint32_t mR = ~(uint32_t)(0xFFull << (((uint32_t)min(tw, 5) << 3) - 8u));
  if constexpr (BATCH) __builtin_amdgcn_sched_barrier(0);  // not needed under the W2 budget
  uint32_t win[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int wi = wbit[t] >> 5;
    const uint64_t both = ((uint64_t)whi[t] << 32) | (wi >= 0 ? wlo[t] : 0u);
    win[t] = (uint32_t)(both >> (uint32_t)(wbit[t] - wi * 32)) & 0xFFFu;
  }
  const uint32_t own = win[0];
  const uint32_t up = hasU ? win[1] : 0u, dn = hasD ? win[2] : 0u;
  const uint32_t o_lo = onehot4(spread4(own)), o_hi = onehot4(spread4(own >> 8));
  const uint32_t L = o_lo;                                     // x-1
  const uint32_t O = __builtin_amdgcn_alignbyte(o_hi, o_lo, 1);  // x
  const uint32_t R = __builtin_amdgcn_alignbyte(o_hi, o_lo, 2);  // x+1
  const uint32_t U = onehot4(spread4(up >> 2)), Dn = onehot4(spread4(dn >> 2));
  if constexpr (MODE != FW_PROPOSE_CUTEDGE) {
    const uint32_t bits = (U & mU) | (L & mL) | (R & mR) | (Dn & mD);
    w4 = byte_popc(bits & ~O & mN);
  }
  if constexpr (NEED_CD || MODE == FW_PROPOSE_CUTEDGE) {
    const uint32_t ne = (ne_bytes(U, O) & mU) >> 7, nl = (ne_bytes(L, O) & mL) >> 7,
                   nr = (ne_bytes(R, O) & mR) >> 7, nd = (ne_bytes(Dn, O) & mD) >> 7;
    cd4 = (ne + nl + nr + nd) & mN;
    if constexpr (MODE == FW_PROPOSE_CUTEDGE) w4 = cd4;
  }
}

// weights (and, when NEED_CD, cut degrees) of nodes x0..x0+3, one per byte
template <int LB, int MODE, bool NEED_CD, bool BATCH = true>
__device__ __forceinline__ void weights4x(const LDS uint8_t* lab, int x0, int W, int H, int n,
                                          GDiv gd, uint32_t& w4, uint32_t& cd4) {
  if constexpr (LB == 2)
    weights4_swar<MODE, NEED_CD, BATCH>(lab, x0, W, H, n, gd, w4, cd4);
  else
    weights4<LB, MODE>(lab, x0, W, H, n, gd, w4, cd4);
}

// bytes of w (each < 64) summed
__device__ __forceinline__ uint32_t bsum4m(uint32_t v) { return (v * 0x01010101u) >> 24; }


// window_verdict (fw_device.h, = the oracle's orc_window_verdict) with the four source
// flood fills run side by side in row-lanes 0..3 instead of one after another.  Fills
// of sources in one window component are equal and other fills disjoint, so the
// sequential verdict is order-free: 1 if some fill holds every source, else 0 if some
// fill touches no border, else -1 (undecided).  Row-uniform result.
// Layout: window row r (0..6, v's row 3) in byte r, column c (0..6, v's column 3) at bit c;
// bit 7 of every byte is a zero guard column, so a dilation needs no column masks (a shift
// into the guard is removed by & A): 4 shifts, 2 ORs of three and one AND per 32-bit half.
__device__ __forceinline__ int window_verdict8(uint64_t A, int q, int row, bool need, uint32_t& nflood) {
#ifdef FW_STAMPS
#define FLOOD_COUNT ++nflood
#else
#define FLOOD_COUNT
#endif
  constexpr uint64_t BORDER = 0x7Full | (0x7Full << 48) | 0x0001010101010101ull | 0x0040404040404040ull;
  // sources up (row 2, column 3), left (3, 2), right (3, 4), down (4, 3)
  const uint64_t src = A & ((1ull << 19) | (1ull << 26) | (1ull << 28) | (1ull << 35));
  const int sb = q == 0 ? 19 : q == 1 ? 26 : q == 2 ? 28 : 35;
  uint64_t x = (need && q < 4) ? src & (1ull << sb) : 0ull;
  if (x) {
    // two dilations per convergence test (same fixpoint, half the loop-exit tests)
    for (;;) {
      const uint64_t y = (x | (x << 1) | (x >> 1) | (x << 8) | (x >> 8)) & A;
      x = (y | (y << 1) | (y >> 1) | (y << 8) | (y >> 8)) & A;
      FLOOD_COUNT;
      if (x == y) break;
    }
  }
  const uint32_t full = rowbits(ballot(x != 0ull && (x & src) == src), row);
  const uint32_t closed = rowbits(ballot(x != 0ull && (x & BORDER) == 0ull), row);
  return full ? 1 : (closed ? 0 : -1);
}

// grid_race_bb (fw_device.h) run by every row at once on its own chain, in a 16-row x
// 32-column window: row-lane q holds grid row vr - 8 + q, bit b column vc - 16 + b.  The
// same level-synchronous race on bitboards, with row-level DPP shifts and row ballots, so
// the four chains of a wave search side by side instead of one after another (C5's
// fractal low-base chains need an exact search on a quarter of their steps).  Rows with
// need == false return -1 untouched; a row returns 1 / 0 (connected / disconnected, with
// its dequeued cells and their degrees in nodes / degs, row-uniform) or -1 when a
// frontier about to be processed reaches a window-edge cell with an on-grid neighbour
// outside (nothing counted: the caller continues with the 64x32 wave form).  Whatever the
// window, the processed levels are the list search's, so the verdicts and counters are
// bit-identical to the oracle's.
__device__ __forceinline__ uint32_t from_prev_row_lane(uint32_t x) {  // row_shr:1, 0 at lane 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_next_row_lane(uint32_t x) {  // row_shl:1, 0 at lane 15
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dilate_row(uint32_t x) {
  return x | (x << 1) | (x >> 1) | from_prev_row_lane(x) | from_next_row_lane(x);
}

template <int LB>
__device__ int grid_race_bb_row(const LDS uint8_t* lab, int n, int W, int H, int q, int row,
                                bool need, int vr, int vc, uint32_t a, uint32_t am4, uint32_t lk,
                                uint32_t& nodes, uint32_t& degs) {
  const int r = vr - 8 + q, c0 = vc - 16;
  const bool rin = (r >= 0) & (r < H);
  uint32_t A = eq_bits32<LB>(lab, n, (rin ? r : vr) * W + c0, a);
  const int lo_cut = c0 < 0 ? -c0 : 0;  // bits of columns < 0
  const int hi_n = W - c0;              // bits >= hi_n: columns >= W (hi_n >= 17)
  uint32_t cm = ~0u << lo_cut;
  if (hi_n < 32) cm &= (1u << hi_n) - 1u;
  A &= rin ? cm : 0u;
  if (q == 8) A &= ~(1u << 16);  // v
  uint32_t E = ((q == 0) & (r > 0)) | ((q == 15) & (r < H - 1)) ? ~0u : 0u;
  if (c0 > 0) E |= 1u;
  if (c0 + 31 < W - 1) E |= 1u << 31;
  E &= A;
  uint32_t F[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {  // sources up (7, 16), left (8, 15), right (8, 17), down (9, 16)
    const int sl = d == 0 ? 7 : (d == 3 ? 9 : 8), sb = d == 1 ? 15 : (d == 2 ? 17 : 16);
    F[d] = (q == sl && ((am4 >> d) & 1u)) ? (1u << sb) : 0u;
  }
  uint32_t M = 0x8421u;  // class of direction d: 4-bit member mask at bits 4d (row-uniform)
  auto unite = [&](int i, int j) {
    const uint32_t m = ((M >> (4 * i)) | (M >> (4 * j))) & 15u;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      M = ((m >> d) & 1u) ? (M & ~(15u << (4 * d))) | (m << (4 * d)) : M;
  };
  if (lk & 1u) unite(0, 2);  // N-E
  if (lk & 2u) unite(2, 3);  // E-S
  if (lk & 4u) unite(3, 1);  // S-W
  if (lk & 8u) unite(1, 0);  // W-N
  auto n_classes = [&]() {
    int nc = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      nc += (int)(((am4 >> d) & 1u) && (__ffs((M >> (4 * d)) & 15u) - 1) == d);
    return nc;
  };
  uint32_t V = F[0] | F[1] | F[2] | F[3];
  int verdict = need ? -2 : -1;  // -2: still searching
  uint32_t P = 0;                // processed cells
  while (ballot(verdict == -2)) {
    const bool run = verdict == -2;
    const uint32_t lvl = F[0] | F[1] | F[2] | F[3];
    if (run && n_classes() == 1) {
      verdict = 1;
      P = V & ~lvl;
    }
    const bool esc = rowbits(ballot((lvl & E) != 0u), row) != 0u;
    if (verdict == -2 && esc) verdict = -3;  // escaped: caller falls back
    const bool go = verdict == -2;
    uint32_t D[4], nw = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      D[d] = ((am4 >> d) & 1u) ? dilate_row(F[d]) & A : 0u;
      nw |= D[d];
    }
    nw &= ~V;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = i + 1; j < 4; ++j) {
        const bool cand = go && ((am4 >> i) & 1u) && ((am4 >> j) & 1u) && !((M >> (4 * i + j)) & 1u);
        if (rowbits(ballot(cand && (D[i] & (F[j] | (D[j] & nw))) != 0u), row)) unite(i, j);
      }
    uint32_t reach = 0;  // directions with a new cell
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t fd = D[d] & nw;
      F[d] = go ? fd : F[d];
      reach |= rowbits(ballot(fd != 0u), row) ? (1u << d) : 0u;
    }
    if (go) {
      P = V;
      if (n_classes() == 1) {
        verdict = 1;
      } else {
        bool closed = false;
#pragma unroll
        for (int d = 0; d < 4; ++d)
          closed |= ((am4 >> d) & 1u) && (reach & (M >> (4 * d)) & 15u) == 0u;
        if (closed)
          verdict = 0;
        else
          V |= nw;
      }
    }
  }
  if (verdict < 0) return -1;
  // counters over the processed cells: degree = on-grid 4-neighbours
  const uint32_t pc = (uint32_t)__popc(P);
  uint32_t dg = pc * (uint32_t)((r > 0) + (r < H - 1) + 2);
  if (c0 <= 0) dg -= (P >> (-c0)) & 1u;          // column 0
  if (hi_n <= 32) dg -= (P >> (hi_n - 1)) & 1u;  // column W - 1
  nodes = row_sum(pc);
  degs = row_sum(dg);
  return verdict;
}

// value of lane L (any lane of the wave; every lane must execute it)
__device__ __forceinline__ uint32_t lane_read(uint32_t x, int L) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(L << 2, (int)x);
}
// speculative attempts (R rows per chain): the sum of x over the R rows of this lane's group
// (row-lane q of each), every lane of the group getting it
template <int R>
__device__ __forceinline__ uint32_t grp_sum(uint32_t x, int gb, int q) {
  uint32_t t = 0;
#pragma unroll
  for (int s = 0; s < R; ++s) t += lane_read(x, gb + s * ROW + q);
  return t;
}
template <int R>
__device__ __forceinline__ uint64_t grp_sum64(uint64_t x, int gb, int q) {
  uint64_t t = 0;
#pragma unroll
  for (int s = 0; s < R; ++s)
    t += (uint64_t)lane_read((uint32_t)x, gb + s * ROW + q) |
         ((uint64_t)lane_read((uint32_t)(x >> 32), gb + s * ROW + q) << 32);
  return t;
}

// 4-bit scratch field x := 0 (atomic on the shared word)
__device__ __forceinline__ void scr_clear(LDS uint8_t* scr, int x) {
  __atomic_fetch_and(PK<4>::word(scr, x), ~(15u << PK<4>::shift(x)), __ATOMIC_RELAXED);
}

// Exact single_flip_contiguous verdict on a grid: "(district a) minus v is connected".
// The level-synchronous race search of fw_device.h (Ctx::race_search) and of the
// oracle (contiguous_after), with visited marks in the shared 4-bit scratch (0 =
// unvisited, 1+o = reached from source o, SCR_BLOCK = v) instead of in the labels.
// Wave-cooperative: all 64 lanes call it for one chain; the caller holds the lock.
template <int LB>
__device__ bool grid_race(const LDS uint8_t* lab, LDS uint8_t* scr, LDS uint32_t* list,
                          GLB uint32_t* spill, int qcap, int W, int H, GDiv gd, int lane,
                          int v, uint32_t a, int m, int src, uint64_t cls, uint64_t& bfs_nodes,
                          uint64_t& bfs_deg) {
  using P = PK<LB>;
  using S = PK<4>;
  auto list_get = [&](int i) -> uint32_t {
    const uint32_t in_lds = list[i < qcap ? i : qcap - 1];
    uint32_t in_hbm = 0;
    if (i >= qcap) in_hbm = spill[i - qcap];
    return i < qcap ? in_lds : in_hbm;
  };
  auto list_put = [&](int i, uint32_t x) {
    if (i < qcap) list[i] = x;
    if (i >= qcap) spill[i - qcap] = x;
  };
  if (lane == 0) S::axor(scr, v, SCR_BLOCK);
  if (lane < m) {
    S::axor(scr, src, 1u + (uint32_t)lane);
    list_put(lane, (uint32_t)src);
  }
  lds_order();
  int nl = m, lb = 0, le = m;
  uint32_t my_deg = 0;
  int verdict = -1;
  for (;;) {
    uint64_t rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
    if (__popcll(rep) == 1) {
      verdict = 1;
      break;
    }
    uint64_t pushed_src = 0;
    for (int base = lb; base < le; base += WAVE) {
      const int idx = base + lane;
      const bool act = idx < le;
      const int x = act ? (int)list_get(idx) : 0;
      const uint32_t o = act ? S::get(scr, x) - 1u : 0u;
      const int xr = gd(x);
      const int xc = x - mulW(xr, W);
      if (act) my_deg += (uint32_t)((xr > 0) + (xc > 0) + (xc < W - 1) + (xr < H - 1));
      bfs_nodes += (uint64_t)__popcll(ballot(act));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int y = -1;
        if (act) {
          if (j == 0 && xr > 0) y = x - W;
          if (j == 1 && xc > 0) y = x - 1;
          if (j == 2 && xc < W - 1) y = x + 1;
          if (j == 3 && xr < H - 1) y = x + W;
        }
        bool push = false, req = false;
        uint32_t other = 0;
        if (y >= 0 && P::get(lab, y) == a) {
          const uint32_t got = S::claim(scr, y, 0u, 1u + o);
          if (got == 0u) {
            push = true;
          } else if (got - 1u < (uint32_t)m) {  // v (SCR_BLOCK) is never a class
            req = true;
            other = got - 1u;
          }
        }
        const uint64_t pm = ballot(push);
        if (push) list_put(nl + (int)mbcnt(pm), (uint32_t)y);
        nl += __popcll(pm);
        if (pm) {
          for (int si = 0; si < m; ++si)
            pushed_src |= ballot(push && o == (uint32_t)si) ? (1ull << si) : 0ull;
        }
        uint64_t rm = ballot(req && o != other);
        while (rm) {  // merges, serial over requesting lanes
          const int Lr = __ffsll((unsigned long long)rm) - 1;
          rm &= rm - 1;
          const int o1 = rdl((int32_t)o, Lr), o2 = rdl((int32_t)other, Lr);
          const uint64_t m1 = rdl64(cls, o1), m2 = rdl64(cls, o2);
          if (m1 != m2) {
            const uint64_t nm = m1 | m2;
            if (lane < m && ((nm >> lane) & 1ull)) cls = nm;
          }
        }
      }
      if (nl > qcap) __threadfence_block();  // spilled entries are read next level
    }
    lds_order();
    lb = le;
    le = nl;
    rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
    if (__popcll(rep) == 1) {
      verdict = 1;
      break;
    }
    // a class with no pushes this level is closed: disconnected
    const bool closed = lane < m && ((rep >> lane) & 1ull) && ((cls & pushed_src) == 0ull);
    if (ballot(closed)) {
      verdict = 0;
      break;
    }
  }
  bfs_deg += wave_sum(my_deg);
  for (int base = 0; base < nl; base += WAVE) {  // clear the visited marks
    const int idx = base + lane;
    if (idx < nl) scr_clear(scr, (int)list_get(idx));
  }
  if (lane == 0) scr_clear(scr, v);
  lds_order();
  return verdict == 1;
}

// FULL = false: the lean instantiation for the common configuration (cut_accept, no
// spatial maps), which then costs no registers for the optional features.
// BIG = true: grids of more than 256 weight groups (n > 16,384, up to 65,536 nodes: C5's
// 200x200): selection gets a third level — u16 sums of supergroups of 16 groups (1,024
// nodes) are scanned first (PER per lane), then the 16 group sums of the chosen supergroup
// (one per lane), then the 64 nodes of the group — and labels take 3 bits when k <= 8,
// so that two waves (eight 40,000-node chains) fit one CU's LDS.
//
// R (speculative attempts, lean small-grid instantiations only): R rows of a wavefront
// work on ONE chain, 4/R chains per wave.  Row s of a chain's group evaluates proposal
// attempt t + s on the same state; the group then consumes attempts in order up to and
// including the first one that changes the state (valid and accepted), so attempts after
// it are discarded and drawn again from the new state.  The state changes only on an
// accepted flip, so every consumed evaluation is the one the sequential chain makes and
// trajectories, counters and sums stay bit-identical.  It raises the attempts per chain
// per wave iteration (C3: 1.56 at R = 2, 2.05 at R = 4) where too few chains are left to
// fill the GPU: an 8,192-chain shard leaves a third of the wave slots empty at R = 1.
template <int LB, int MODE, int PER, bool FULL, bool BIG, int R, bool W2 = false>
__device__ __forceinline__ void grid16_body(const FwRunParams& p) {
  static_assert(PER % 2 == 0, "group sums are read as u16 pairs");
  static_assert(R == 1 || R == 2 || R == 4, "rows per chain");
  static_assert(R == 1 || (!FULL && !BIG), "speculation: lean small-grid kernels only");
  constexpr int CPW = 4 / R;  // chains per wavefront
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ int32_t s_lock;
  using P = PK<LB>;
  const int lane = __lane_id(), row = lane >> 4, q = lane & 15;
  const int sx = row & (R - 1);     // speculation index of this row within its chain's group
  const int grp = row / R;          // the chain of this row within the wave
  const int gb = grp * R * ROW;     // first lane of the group
  const bool owner = sx == 0;       // the row that keeps the chain's observations
  const int wv = (int)(threadIdx.x >> 6);
  // grid shape and bounds live in VGPRs: the hot loop uses them only in vector ops, and
  // the scalar file is the scarce one (SGPR spills cost v_readlane round trips)
  const int W = (int)in_vgpr((uint32_t)p.g.gw), H = (int)in_vgpr((uint32_t)p.g.gh);
  const int n = (int)in_vgpr((uint32_t)p.g.n);
  const int D = (int)in_vgpr((uint32_t)p.g.maxdeg), G = (int)in_vgpr((uint32_t)p.G);
  const int k = (int)in_vgpr((uint32_t)p.k);
  LDS uint8_t* const sm = (LDS uint8_t*)smem;
  // this row's chain slot (after a 16-B guard: lab_window may read the word before a slot)
  LDS uint8_t* const lab = sm + LDS_GUARD + (wv * CPW + grp) * p.slot_stride;
  LDS uint32_t* const gsum = reinterpret_cast<LDS uint32_t*>(lab + p.off_gsum);  // u16 pairs
  // BIG: supergroup sums (u16 pairs, the level-1 array); otherwise level 1 reads gsum
  LDS uint32_t* const ssum = reinterpret_cast<LDS uint32_t*>(lab + p.off_ssum);
  LDS uint32_t* const lvl1 = BIG ? ssum : gsum;
  LDS uint8_t* const scr = sm + p.off_scr;                                        // shared
  LDS uint32_t* const list = reinterpret_cast<LDS uint32_t*>(sm + p.off_list16);  // shared
  GLB uint32_t* const spill = (GLB uint32_t*)(p.spill + (size_t)blockIdx.x * (size_t)n);
  const uint32_t key0 = (uint32_t)p.seed, key1 = (uint32_t)(p.seed >> 32);
  const int GW = (G + 1) >> 1;  // u16-pair words of group sums
  const int SG = (G + 15) >> 4;  // BIG: supergroups of 16 groups
  const bool maps_on = FULL && p.m_acc != nullptr;
  // population bounds as int32 (the host routes graphs with total population >= 2^31 to
  // the one-chain-per-wave kernel); clamped so comparisons keep their meaning
  const int32_t pop_lo = (int32_t)in_vgpr((uint32_t)(int32_t)max(p.pop_lo, (int64_t)INT32_MIN));
  const int32_t pop_hi = (int32_t)in_vgpr((uint32_t)(int32_t)min(p.pop_hi, (int64_t)INT32_MAX));
  const GDiv gd{in_vgpr(p.g.gm24), in_vgpr(p.g.gs24)};
  const int32_t rule = FULL ? p.accept : FW_ACCEPT_CUT;
  int my_dr, my_dc;
  role_off(q <= 8 ? q : 0, my_dr, my_dc);
  // 2-bit labels: row-lanes 9..12 also take the cells two steps from v (UU, LL, RR, DD),
  // so the whole radius-2 diamond is read with one LDS round trip (one cell per lane)
  // and each 4-neighbour's label set comes from per-label row ballots.  nb_lanes: the
  // lanes holding the neighbours of this lane's cell other than v.
  if (LB == 2 && q >= 9 && q <= 12) {
    my_dr = q == 9 ? -2 : (q == 12 ? 2 : 0);
    my_dc = q == 10 ? -2 : (q == 11 ? 2 : 0);
  }
  const uint32_t nb_lanes = q == 0   ? 0x1Eu
                            : q == 1 ? (1u << 9) | (1u << 8) | (1u << 5)
                            : q == 2 ? (1u << 10) | (1u << 8) | (1u << 7)
                            : q == 3 ? (1u << 11) | (1u << 5) | (1u << 6)
                            : q == 4 ? (1u << 12) | (1u << 6) | (1u << 7)
                                     : 0u;
  auto divmod = [&](int x, int& r, int& c) {
    r = gd(x);
    c = x - mulW(r, W);
  };
  STAMP_DECL

  // the search scratch starts all-zero; every search clears what it marked
  {
    LDS uint32_t* s32 = reinterpret_cast<LDS uint32_t*>(scr);
    for (int i = (int)threadIdx.x; i < p.scr_bytes / 4; i += (int)blockDim.x) s32[i] = 0u;
    if (threadIdx.x == 0) s_lock = 0;
  }
  __syncthreads();

  // Work units: quad (four chains, one per row) x slice of the launch's steps, handed out
  // slice-major (unit u = slice u / nq of quad u % nq; p.slices = 1: whole quads).  With
  // more quads than resident waves the host picks the slice count that makes the units a
  // whole number of residency rounds (65,536 chains: 16,384 quads x 3 = 16 rounds of 3,072
  // waves), so the launch does not end on a partly filled round.  A slice starts once its
  // quad's previous slice is written back (seg_done, agent-scope release / acquire: the
  // previous slice ran a round or more earlier, so the wait is normally already over); the
  // trajectory equals separate launches of the slices' step counts.
  const int nq = (p.n_chains + CPW - 1) / CPW;
  for (;;) {
    int cb = 0;
    if (lane == 0) cb = atomicAdd(p.next_chain, 1);
    const int u = rdl(cb, 0);
    if (u >= nq * p.slices) break;
    const int seg = u / nq;
    const int quad = u - seg * nq;
    const uint32_t ustep = (uint32_t)(p.steps * (seg + 1) / p.slices - p.steps * seg / p.slices);
    if (seg > 0) {
      // a wave-uniform loop (readfirstlane of the flag): a lane-0-only loop or store lets
      // the compiler restructure the unit loop around a divergent exit, running the next
      // unit without lane 0
      for (;;) {
        const int done =
            rfl(__hip_atomic_load(p.seg_done + quad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (done >= seg) break;
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    UNIT_TIME(u, 0);
    const int cbase = quad * CPW;
    const int c = cbase + grp;
    const bool has = c < p.n_chains;
    const int cc = has ? c : cbase;  // a valid index for loads of absent rows
    const uint64_t gid = (uint64_t)(p.chain_id0 + c);
    const bool cached = p.gcache_ok != 0 || seg > 0;  // derived-state cache (FwRunParams)

    // ---- load state (each row loads its own chain).  OPQ: the record addresses, here and
    // at the write-back, from an opaque lane id; hoisted to the kernel entry, their 64-bit
    // lane offsets were what the register budget spilled in the speculative and cut-edge
    // instantiations (12-28 B of scratch per lane).  Not in the pairs kernels, which do not
    // spill and lose 0.4% (C3) to the recomputation.
    constexpr bool OPQ = R > 1 || MODE == FW_PROPOSE_CUTEDGE;
    int ql = q;
    if constexpr (OPQ) asm volatile("" : "+v"(ql));
    {
      const u32x4* src = reinterpret_cast<const u32x4*>(p.labels + (size_t)cc * p.lab_stride);
      LDS u32x4* dst = reinterpret_cast<LDS u32x4*>(lab);
      // with a valid derived-state cache the slot's group sums come along (see lab_copy16)
      const int nv = cached ? p.lab_copy16 : p.lab_bytes / 16;
      for (int i = sx * ROW + ql; i < nv; i += R * ROW) dst[i] = src[i];
    }
    int32_t pops = ql < k ? (int32_t)p.pops[(size_t)cc * k + ql] : 0;  // total pop < 2^31
    double thr_l = FULL && ql < 2 * D + 1 ? p.thr[(size_t)cc * p.thr_stride + ql] : 0.0;
    uint64_t thr53_l = ql < 2 * D + 1 ? p.thr53[(size_t)cc * p.thr_stride + ql] : 0ull;
    fw_chain_stats* stp = p.stats + cc;
    const uint64_t acc0 = FULL && p.sched ? stp->accepts : 0ull;
    // scheduled bounds: the row of the next proposal's step_num (accepted flips + 1)
    auto sched_row = [&](uint64_t nacc) {
      const int64_t t = (int64_t)(acc0 + nacc) + 1 - p.sched_t0;
      const int64_t r = t < 0 ? 0 : (t >= p.sched_rows ? p.sched_rows - 1 : t);
      if (q < 2 * D + 1) {
        thr_l = p.sched[r * (2 * D + 1) + q];
        thr53_l = p.sched53[r * (2 * D + 1) + q];
      }
    };
    if (FULL && p.sched) sched_row(0);
    // attempts and yields of this launch in 32 bits: attempts = att0 + n_att, and every
    // counted step is one yield (plus the initial state's on a chain's first launch).
    // The counters that grow with attempts (n_att, n_popf, n_conf, n_sdeg) are folded
    // into the 64-bit totals at a Philox refill once n_sdeg (the fastest: >= 2 per
    // attempt) reaches p.fold_at (2^31; tests lower it), so no launch length wraps them; the host caps the counted
    // steps of one launch (fw_chains_run_async), which bounds the rest.
    uint64_t att0 = stp->attempts;
    const bool first = has && !stp->stuck && stp->yields == 0 && att0 == 0;
    uint32_t n_att = 0;
    const uint64_t yields0 = stp->yields;
    int32_t stuck = has ? stp->stuck : 1;
    int64_t sum_cut = stp->sum_cut, sum_bnodes = stp->sum_bnodes;
    double sum_invb = stp->sum_invb;
    // sampled geometric waits (FULL only): the running sum and the current state's draw
    const bool waits_on = FULL && p.wsamp != nullptr;
    double wsum = waits_on ? p.wsamp[2 * (size_t)cc] : 0.0;
    double wcur = waits_on ? p.wsamp[2 * (size_t)cc + 1] : 0.0;
    uint32_t n_steps = 0, n_acc = 0, n_popf = 0, n_conf = 0, n_sdeg = 0, n_adeg = 0, n_bchg = 0;
    uint32_t retries = 0;
    uint64_t n_bfs = 0, n_bfsn = 0, n_bfsd = 0;
    uint32_t bpos_w = ROW * R;  // R > 1: next unconsumed attempt of the group's Philox batch
    Pend pend = maps_on ? pend_load(p, cc) : Pend{-1, 0, 0u};
    // boundary_node-flagged nodes of district q (FW_ACCEPT_BOUNDARY), lane q
    int32_t bcnt = rule == FW_ACCEPT_BOUNDARY && ql < k ? p.bcnt[(size_t)cc * k + ql] : 0;
    lds_order();

    // ---- derive group sums, cut / boundary / proposal-set counts (per row), unless the
    // derived-state cache holds them (group sums loaded with the labels, counts in stats)
    int32_t cut, bnodes, npairs;
    {
      uint32_t cut2 = 0, bn = 0, np = 0;
      for (int t2 = 0; t2 < (cached ? 0 : GW); ++t2) {
        uint32_t tot[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t w4, cd4;
          weights4x<LB, MODE, true>(lab, (2 * t2 + h) * 64 + q * 4, W, H, n, gd, w4, cd4);
          const uint32_t ws = bsum4m(w4);
          cut2 += bsum4m(cd4);
          bn += ((cd4 & 0xFFu) != 0) + ((cd4 & 0xFF00u) != 0) + ((cd4 & 0xFF0000u) != 0) +
                ((cd4 & 0xFF000000u) != 0);
          np += ws;
          tot[h] = row_sum(ws);
        }
        if (q == 0 && has) gsum[t2] = tot[0] | (tot[1] << 16);
      }
      if constexpr (BIG) {
        // group sums zero-padded to whole supergroups (level 2 reads 16 per supergroup)
        for (int t2 = GW + q; t2 < SG * 8; t2 += ROW)
          if (has) gsum[t2] = 0u;
        lds_order();
        // supergroup sums, two per word, zero past SG: level 1 reads every word unmasked
        for (int w2 = q; w2 < 8 * PER; w2 += ROW) {
          uint32_t s2[2] = {0u, 0u};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int sg = 2 * w2 + h;
            if (sg < SG)
              for (int i = 0; i < 8; ++i) {
                const uint32_t g2 = gsum[sg * 8 + i];
                s2[h] += (g2 & 0xFFFFu) + (g2 >> 16);
              }
          }
          if (has) ssum[w2] = s2[0] | (s2[1] << 16);
        }
      } else {
        // zero padding up to 16 lanes x PER/2 words: level 1 reads every word unmasked
        for (int t2 = GW + q; t2 < 8 * PER; t2 += ROW)
          if (has) gsum[t2] = 0u;
      }
      if (cached) {
        cut = stp->cut;
        bnodes = stp->bnodes;
        npairs = stp->npairs;
      } else {
        cut = (int32_t)(row_sum(cut2) / 2);
        bnodes = (int32_t)row_sum(bn);
        npairs = (int32_t)row_sum(np);
      }
    }
    lds_order();
    double invb = p.g.invb[bnodes];  // 1/|B| from the graph's table, no fp64 divide

    // district-shape observable (FULL only): the pair of the first two cut ring edges in
    // ring order, per row, counted per yield in runs flushed when it changes (a flip of a
    // ring node) and at the end of the launch
    const int RN = FULL ? p.ring_n : 0;
    auto ring_pair = [&]() -> int32_t {  // row-uniform; called by whole rows
      int f = -1, sc = -1;
      for (int b0 = 0; b0 < RN; b0 += ROW) {
        const int r = b0 + q;
        const int ri = r < RN ? r : 0;
        uint32_t m = rowbits(ballot(r < RN && P::get(lab, p.ring_u[ri]) != P::get(lab, p.ring_w[ri])),
                             row);
        if (m && f < 0) {
          f = b0 + __ffs(m) - 1;
          m &= m - 1;
        }
        if (m && sc < 0) sc = b0 + __ffs(m) - 1;
      }
      return sc >= 0 ? f * RN + sc : RN * RN;
    };
    int32_t rpair = RN && has ? ring_pair() : 0;
    uint32_t rrun = 0;

    // histogram windows: row-lane q counts values base+q and base+16+q
    uint32_t hc0 = 0, hc1 = 0, hb0 = 0, hb1 = 0;
    int32_t base_c = max(0, cut - 16), base_b = max(0, bnodes - 16);
    auto observe = [&](bool on) {
      if (!on) return;
      if (FULL) rrun += 1;
      if (waits_on) wsum += wcur;
      sum_cut += cut;
      sum_bnodes += bnodes;
      sum_invb += invb;
      int ic = cut - base_c;
      if (ic < 0 || ic >= 2 * ROW) {
        if (hc0) HIST_ADD(p.hist_cut + base_c + q, (unsigned long long)hc0);
        if (hc1) HIST_ADD(p.hist_cut + base_c + ROW + q, (unsigned long long)hc1);
        hc0 = hc1 = 0;
        base_c = max(0, cut - ROW);
        ic = cut - base_c;
      }
      hc0 += ic == q;
      hc1 += ic == q + ROW;
      int ib = bnodes - base_b;
      if (ib < 0 || ib >= 2 * ROW) {
        if (hb0) HIST_ADD(p.hist_b + base_b + q, (unsigned long long)hb0);
        if (hb1) HIST_ADD(p.hist_b + base_b + ROW + q, (unsigned long long)hb1);
        hb0 = hb1 = 0;
        base_b = max(0, bnodes - ROW);
        ib = bnodes - base_b;
      }
      hb0 += ib == q;
      hb1 += ib == q + ROW;
    };
    if (waits_on && first) wcur = wait_draw(p.seed, FW_WAIT_T0, gid, p.wlp[bnodes]);
    observe(first && owner);

    // Philox batches: lane q of a row holds the draw of its chain's attempt (base + q).
    // Active rows consume one attempt per loop iteration in lockstep: each iteration
    // broadcasts lane 0 of the row (row_newbcast:0) and shifts the batch down one lane
    // (row_shl:1), all DPP; a row that stops stays stopped for this launch.
    U4 pb = {0u, 0u, 0u, 0u};
    int bpos = ROW;

    const bool unit_pop = !FULL || p.g.pop == nullptr;  // node populations: FULL only
    // Wave priority by progress.  A SIMD issues VALU to the higher-priority wave, then the
    // older one: at equal priority the younger waves of a SIMD get the leftover slots and
    // finish their units ~25% later (8,192 chains, 2 waves per SIMD: 2.38 vs 3.01 ms,
    // scripts/unit_times.py), and with no more units to take the launch waits for them.
    // Priority 3 - (level mod 4), the level counting 2^-prio_shift of the unit's steps done
    // by row 0 (launch_prio_shift: 8ths or quarters), hands the issue slots to the wave one
    // level behind (except across a wrap), which keeps a SIMD's waves close to the end.
    const uint32_t psh = (uint32_t)p.prio_shift;
    const uint32_t pstep = ustep >= (2u << psh) ? ustep >> psh : 2u;
    uint32_t pnext = pstep, plev = 0;
    // one unit per wave slot (psh == 3): the older wave of a SIMD (even slot) wins priority
    // ties, so it starts one level on; equal progress then favours the younger wave
    if (psh == 3u && (__builtin_amdgcn_s_getreg((3 << 11) | 4) & 1u) == 0u) plev = 1;
    if (plev == 0) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(2);
    for (;;) {
      STAMP(-1);
      // ---- who proposes this round
      if (!stuck && (retries >= (uint32_t)p.max_retries || npairs == 0)) stuck = 1;
      const bool act = has && !stuck && n_steps < ustep;
      if (ballot(act) == 0ull) break;
      if (rfl(n_steps) >= pnext) {
        pnext += pstep;
        plev = (plev + 1u) & 3u;
        if (plev == 0) __builtin_amdgcn_s_setprio(3);
        else if (plev == 1) __builtin_amdgcn_s_setprio(2);
        else if (plev == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }

      U4 x;
      if constexpr (R == 1) {
        if (bpos == ROW) {
          if (n_sdeg >= p.fold_at) {  // rare: fold (see att0); one row at a time
            if (q == 0 && has) {
              stp->pop_fail += n_popf;
              stp->contig_fail += n_conf;
              stp->sum_deg += n_sdeg;
            }
            att0 += n_att;
            n_att = n_popf = n_conf = n_sdeg = 0;
          }
          const uint64_t t = att0 + (uint64_t)(n_att + (uint32_t)q);
          pb = philox((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid, (uint32_t)(gid >> 32),
                      in_vgpr(key0), in_vgpr(key1));
          bpos = 0;
        }
        // lane 0 of the row holds this attempt's draw; shift the batch for the next one
        x = U4{row_first(pb.x0), row_first(pb.x1), row_first(pb.x2), row_first(pb.x3)};
        pb = U4{row_shl1(pb.x0), row_shl1(pb.x1), row_shl1(pb.x2), row_shl1(pb.x3)};
        ++bpos;
        n_att += act ? 1u : 0u;
      } else {
        // the group's R rows hold 16 R consecutive attempts (row s: base + 16 s + q); row s
        // takes attempt bpos_w + s; refilled from the next unconsumed attempt when fewer
        // than R are left
        if (bpos_w > (uint32_t)(ROW * R - R)) {
          if (4u * n_att >= p.fold_at) {  // rare (grids: degree <= 4): fold, group-uniform
            const uint32_t f0 = grp_sum<R>(n_popf, gb, q), f1 = grp_sum<R>(n_conf, gb, q);
            const uint32_t f2 = grp_sum<R>(n_sdeg, gb, q);
            if (q == 0 && owner && has) {
              stp->pop_fail += f0;
              stp->contig_fail += f1;
              stp->sum_deg += f2;
            }
            att0 += n_att;
            n_att = n_popf = n_conf = n_sdeg = 0;
          }
          const uint64_t t = att0 + (uint64_t)(n_att + (uint32_t)(sx * ROW + q));
          pb = philox((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid, (uint32_t)(gid >> 32),
                      in_vgpr(key0), in_vgpr(key1));
          bpos_w = 0;
        }
        const int srcl = gb + (int)bpos_w + sx;
        x = U4{lane_read(pb.x0, srcl), lane_read(pb.x1, srcl), lane_read(pb.x2, srcl),
               lane_read(pb.x3, srcl)};
      }
      const uint32_t r = scale64(x.x0, x.x1, (uint32_t)(npairs > 0 ? npairs : 1));

      STAMP(0);  // draw
      // ---- select, level 1: group sums (PER per lane, read as PER/2 u16 pairs)
      uint32_t w2[PER / 2];
      uint32_t s = 0;
#pragma unroll
      for (int t = 0; t < PER / 2; ++t) {
        w2[t] = lvl1[q * (PER / 2) + t];  // words past GW (SG) are zero padding
        s += (w2[t] & 0xFFFFu) + (w2[t] >> 16);
      }
      // packed u16 prefixes of the lane's groups, pair t = (c_{2t+1}, c_{2t+2}) with c_j the
      // sum of its first j groups (< 2^15 on the chosen lane: <= 16 groups of <= 64 x 4, or
      // BIG's <= 4 supergroups of <= 16 x 192); independent of r, so they fill the scan's
      // DPP wait states
      uint32_t pp[PER / 2];
      {
        uint32_t base = 0;
#pragma unroll
        for (int t = 0; t < PER / 2; ++t) {
          pp[t] = __umul24(base, 0x10001u) + (w2[t] + (w2[t] << 16));
          base = pp[t] >> 16;
        }
      }
      const uint32_t incl = row_scan(s);
      const uint32_t rb1 = rowbits(ballot(incl > r), row);
      const int Lw = __ffs(rb1) - 1;
      // the group holding rank rl among this lane's PER (only lane Lw's, where 0 <= rl < s,
      // is used): e_j = rl - c_j in u16 arithmetic wraps past 2^15 exactly when c_j > rl, so
      // the groups before it are the prefixes that do not wrap and the remaining rank is
      // min(rl, the smallest e_j) -- packed u16 ops, no compare / carry chain
      const uint32_t rl = r - (incl - s);
      typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
      const u16x2 rl2 = __builtin_bit_cast(u16x2, __umul24(rl & 0xFFFFu, 0x10001u));
      u16x2 mn = {0xFFFFu, 0xFFFFu}, wraps = {0u, 0u};
#pragma unroll
      for (int t = 0; t < PER / 2; ++t) {
        const u16x2 e = rl2 - __builtin_bit_cast(u16x2, pp[t]);
        mn = __builtin_elementwise_min(mn, e);
        wraps += e >> (uint16_t)15;
      }
      const uint32_t rem = min(rl, (uint32_t)min(mn.x, mn.y));
      const int tfu = PER - (int)wraps.x - (int)wraps.y;
      const int tf = min(tfu, PER - 1);
      // pack (group, remaining rank) into one row broadcast
      const uint32_t pk1 = row_pick(((uint32_t)(q * PER + tf) << 16) | (rem & 0xFFFFu), Lw, q);
      int gi;
      uint32_t r1;
      uint32_t rbg = 1u;
      if constexpr (BIG) {
        // level 1.5: the 16 group sums of supergroup sgi, one per row-lane
        const int sgi = min((int)(pk1 >> 16), SG - 1);
        const uint32_t r1s = pk1 & 0xFFFFu;
        const uint32_t g2 = gsum[sgi * 8 + (q >> 1)];
        const uint32_t gv = (q & 1) ? (g2 >> 16) : (g2 & 0xFFFFu);
        const uint32_t incg = row_scan(gv);
        rbg = rowbits(ballot(incg > r1s), row);
        const int Lg = __ffs(rbg) - 1;
        const uint32_t pkg =
            row_pick(((uint32_t)(sgi * 16 + q) << 16) | ((r1s - (incg - gv)) & 0xFFFFu), Lg, q);
        gi = min((int)(pkg >> 16), G - 1);
        r1 = pkg & 0xFFFFu;
      } else {
        gi = min((int)(pk1 >> 16), G - 1);
        r1 = pk1 & 0xFFFFu;
      }

      STAMP(1);  // level 1
      // ---- select, level 2: weights of the group's 64 nodes, 4 per lane
      const int x0 = gi * 64 + q * 4;
      uint32_t w4, cd4;  // four 8-bit weights
      weights4x<LB, MODE, false, !W2>(lab, x0, W, H, n, gd, w4, cd4);
      // byte t: weights of nodes 0..t (<= 16); two shift-adds, not a quarter-rate multiply
      const uint32_t pref1 = w4 + (w4 << 8);
      const uint32_t pref = pref1 + (pref1 << 16);
      const uint32_t ws = pref >> 24;
      const uint32_t incl2 = row_scan(ws);
      const uint32_t rb2 = rowbits(ballot(incl2 > r1), row);
      const int L2 = __ffs(rb2) - 1;
      const uint32_t r2 = min(r1 - (incl2 - ws), 127u);  // < ws on the chosen lane
      // first byte with prefix > r2 (SWAR compare; no borrow across bytes as r2 < 128)
      const uint32_t gt = ((pref | 0x80808080u) - __builtin_amdgcn_perm(0u, r2 + 1u, 0u)) & 0x80808080u;
      const int t2 = gt ? (__ffs(gt) - 1) >> 3 : 3;
      const uint32_t bef2 = t2 ? (pref >> (8 * t2 - 8)) & 0xFFu : 0u;
      const uint32_t pk2 = row_pick(((uint32_t)(q * 4 + t2) << 16) | ((r2 - bef2) & 0xFFFFu), L2, q);
      const int v = min(gi * 64 + (int)(pk2 >> 16), n - 1);
      const uint32_t j = pk2 & 0xFFFFu;
      // inconsistent sums: flag, stop (R > 1: if the attempt is consumed, in the merge)
      if (R == 1 && act && (rb1 == 0 || rb2 == 0 || rbg == 0)) stuck = 2;
      const bool go = act && rb1 != 0 && rb2 != 0 && rbg != 0;

      STAMP(2);  // level 2
      // ---- v's neighbourhood: row-lane roles 0 v, 1 up, 2 left, 3 right, 4 down,
      //      5 NE, 6 SE, 7 SW, 8 NW; lanes 0..4 also read their node's neighbours
      int vr, vc;
      divmod(v, vr, vc);
      const int dv = (vr > 0) + (vc > 0) + (vc < W - 1) + (vr < H - 1);
      Hood16 h;
      h.x = -1;
      h.lx = NOLAB;
      h.bits = 0;
      h.cnt = 0;
      h.has_v = false;
      h.deg = 0;
      if constexpr (LB == 2) {
        // one unconditional read per lane (cells off the grid read v and are masked)
        const int xr = vr + my_dr, xc = vc + my_dc;
        const bool inb = (q <= 12) & ((uint32_t)xr < (uint32_t)H) & ((uint32_t)xc < (uint32_t)W);
        const int xx = mulW(xr, W) + xc;
        const uint32_t l0 = P::get(lab, inb ? xx : v);
        h.x = inb ? xx : -1;
        h.lx = inb ? l0 : NOLAB;
        const uint32_t m0 = rowbits(ballot(h.lx == 0u), row) & nb_lanes;
        const uint32_t m1 = rowbits(ballot(h.lx == 1u), row) & nb_lanes;
        const uint32_t m2 = rowbits(ballot(h.lx == 2u), row) & nb_lanes;
        const uint32_t m3 = rowbits(ballot(h.lx == 3u), row) & nb_lanes;
        h.bits = (m0 ? 1u : 0u) | (m1 ? 2u : 0u) | (m2 ? 4u : 0u) | (m3 ? 8u : 0u);
        if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
          const uint32_t same = h.lx == 0u ? m0 : h.lx == 1u ? m1 : h.lx == 2u ? m2 : m3;
          h.cnt = (uint32_t)__popc(m0 | m1 | m2 | m3) - (uint32_t)__popc(same);
          h.deg = q == 0 ? (int)h.cnt + (int)__popc(same) : 0;
        }
        h.has_v = q >= 1 && q <= 4 && inb;
        if (!(inb && q <= 4)) {
          h.bits = 0;
          h.cnt = 0;
        }
      } else {
        const int xr = vr + my_dr, xc = vc + my_dc;
        if (q <= 8 && xr >= 0 && xr < H && xc >= 0 && xc < W) {
          h.x = xr * W + xc;
          h.lx = P::get(lab, h.x);
          if (q <= 4) {
            h.deg = (xr > 0) + (xc > 0) + (xc < W - 1) + (xr < H - 1);
            const int vslot = 4 - q;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              int y = -1;
              if (jj == 0 && xr > 0) y = h.x - W;
              if (jj == 1 && xc > 0) y = h.x - 1;
              if (jj == 2 && xc < W - 1) y = h.x + 1;
              if (jj == 3 && xr < H - 1) y = h.x + W;
              if (y < 0) continue;
              if (q > 0 && jj == vslot) {
                h.has_v = true;
                continue;
              }
              const uint32_t ly = P::get(lab, y);
              h.bits |= 1u << ly;
              h.cnt += ly != h.lx;
            }
          }
        }
      }
      const uint32_t a = row_first(h.lx);  // v's label (row-lane 0)
      const bool isnb = q >= 1 && q <= 4 && h.x >= 0;
      uint32_t d;
      if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
        const uint32_t cm = rowbits(ballot(isnb && h.lx != a), row) >> 1;  // bits: up,left,right,down
        uint32_t mm = cm;
        for (uint32_t t = 0; t < j && t < 4; ++t) mm &= mm - 1;
        const int Lc = __ffs(mm);  // row-lane 1..4
        d = row_pick(h.lx, Lc, q);
      } else {
        // distinct foreign labels among the 4 neighbours, then the j-th smallest
        uint32_t mask;
        if constexpr (LB == 2) {
          mask = row_first(h.bits) & ~(1u << a);  // row-lane 0 holds v's neighbour label set
        } else {
          uint32_t fb = (isnb && h.lx != a) ? (1u << h.lx) : 0u;
          fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x111, 0xF, 0xF, true);  // row_shr:1
          fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x112, 0xF, 0xF, true);  // row_shr:2
          fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x114, 0xF, 0xF, true);  // row_shr:4
          mask = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x154, 0xF, 0xF, false);  // row_newbcast:4
        }
        uint32_t mm = mask;
        if constexpr (LB == 2) {  // k <= 4: at most 3 foreign labels, j <= 2 (no loop)
          const uint32_t m1 = mm & (mm - 1u), m2 = m1 & (m1 - 1u);
          mm = j == 0u ? mm : (j == 1u ? m1 : m2);
        } else {
          for (uint32_t t = 0; t < j && t < 15; ++t) mm &= mm - 1;
        }
        d = (uint32_t)(__ffs(mm) - 1);
      }
      const uint32_t amb = rowbits(ballot(isnb && h.lx == a), row) >> 1;
      const int m = __popc(amb);
      const int nbd = __popc(rowbits(ballot(isnb && h.lx == d), row) >> 1);
      const int dcut = m - nbd;

      // ---- population bound (lane q holds district q)
      const int32_t pv = unit_pop ? 1 : (int32_t)p.g.pop[v];
      const bool bad = (((uint32_t)q == a) & (pops - pv < pop_lo)) |
                       (((uint32_t)q == d) & (pops + pv > pop_hi));
      const bool pop_ok = rowbits(ballot(bad), row) == 0u;

      STAMP(3);  // gather, target, Δcut, population
      // ---- weights of v's neighbourhood before / after the flip (commit and |B'|)
      uint32_t wo = 0, wn = 0;
      const bool mine = (q <= 4) & (h.x >= 0);
      // branch-free (selects, no exec-mask if/else between v's lane and its neighbours')
      if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
        const uint32_t wo_v = (uint32_t)(h.deg - m), wn_v = (uint32_t)(h.deg - nbd);
        const uint32_t wo_u = h.cnt + (uint32_t)(h.has_v & (a != h.lx));
        const uint32_t wn_u = h.cnt + (uint32_t)(h.has_v & (d != h.lx));
        wo = q == 0 ? wo_v : wo_u;
        wn = q == 0 ? wn_v : wn_u;
      } else {
        // v: its neighbour label set minus the old / new label; a neighbour u: its set
        // (plus v's old / new label) minus u's own label
        const uint32_t hv = h.has_v ? 0xFFFFFFFFu : 0u;
        const uint32_t ka = q == 0 ? ~(1u << a) : ~(1u << h.lx);
        const uint32_t kd = q == 0 ? ~(1u << d) : ~(1u << h.lx);
        wo = (uint32_t)__popc((h.bits | ((1u << a) & hv)) & ka);
        wn = (uint32_t)__popc((h.bits | ((1u << d) & hv)) & kd);
      }
      wo = mine ? wo : 0u;
      wn = mine ? wn : 0u;
      // boundary changes if this flip is made (used only when it is accepted, which implies
      // valid): 1/|B'| is read now, before the contiguity stages, so its L2 latency hides
      // behind them
      const uint64_t b_plus = ballot(go && mine && wo == 0 && wn > 0);
      const uint64_t b_minus = ballot(go && mine && wo > 0 && wn == 0);
      const int plus = __popc(rowbits(b_plus, row)), minus = __popc(rowbits(b_minus, row));
      const double invb_new = p.g.invb[bnodes + plus - minus];
      // R > 1: the Metropolis verdict is known before contiguity; an exact search is skipped
      // when an earlier attempt of the same chain is known to change the state
      bool wacc = false;
      if constexpr (R > 1) {
        const bool acc_l = (((uint64_t)(x.x2 >> 5) << 26) | (uint64_t)(x.x3 >> 6)) < thr53_l;
        wacc = ((rowbits(ballot(acc_l), row) >> (dcut + D)) & 1u) != 0u;
      }
      // this attempt's exact search: runs, dequeued cells, their degrees (R > 1: counted
      // only if the attempt is consumed; R = 1: straight into the unit's counters)
      uint32_t it_bfs = 0;
      uint64_t it_bfsn = 0, it_bfsd = 0;
      auto count_search = [&](uint64_t bn_, uint64_t bd_) {
        if constexpr (R == 1) {
          n_bfs += 1;
          n_bfsn += bn_;
          n_bfsd += bd_;
        } else {
          it_bfs = 1;
          it_bfsn = bn_;
          it_bfsd = bd_;
        }
      };
      // ---- contiguity: 8-cell ring test, 7x7 window, exact race search when undecided
      const uint32_t rbits8 = rowbits(ballot(q >= 1 && q <= 8 && h.lx == a), row) >> 1;
      const int pN = rbits8 & 1, pW = (rbits8 >> 1) & 1, pE = (rbits8 >> 2) & 1, pS = (rbits8 >> 3) & 1;
      const int NE = (rbits8 >> 4) & 1, SE = (rbits8 >> 5) & 1, SW = (rbits8 >> 6) & 1,
                NW = (rbits8 >> 7) & 1;
      const int lNE = pN & pE & NE, lES = pE & pS & SE, lSW = pS & pW & SW, lWN = pW & pN & NW;
      // bitwise, not short-circuit: no exec-mask branches
      bool contig = (m == 1) | ((m >= 2) & (m - (lNE + lES + lSW + lWN) <= 1));
      bool need = go & pop_ok & (m >= 2) & !contig;
      if (ballot(need)) {  // 7x7 window flood fill (window_verdict8's layout)
        // read t: row-lane q takes window row 2t + q / 8, column q % 8 (column 7: the guard,
        // never a cell), so row ballot t is bits 16t .. 16t + 15 of A
        uint64_t A = 0;
        bool inw[4];
        uint32_t raw[4], lw[4];
        int xw[4];
        const int wcol = q & 7;
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // branch-free: all four reads issued, then masked
          const int wrow = 2 * t + (q >> 3);
          const int rr = vr + wrow - 3, cw = vc + wcol - 3;
          inw[t] = (wcol < 7) & (wrow < 7) & ((uint32_t)rr < (uint32_t)H) & ((uint32_t)cw < (uint32_t)W);
          xw[t] = inw[t] ? mulW(rr, W) + cw : v;
          raw[t] = lab[xw[t] >> 2];  // P::get's byte (2-bit labels) or nibble pair (4-bit)
          if constexpr (LB != 2) raw[t] = P::get(lab, xw[t]);
        }
        // the four loads stay together (one LDS round trip): at the register limit the
        // scheduler otherwise put each load's wait before the next load
        if constexpr (!W2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t) lw[t] = LB == 2 ? (raw[t] >> ((xw[t] & 3) << 1)) & 3u : raw[t];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          A |= (uint64_t)rowbits(ballot(inw[t] & (lw[t] == a)), row) << (ROW * t);
        A &= ~(1ull << 27);  // v (row 3, column 3)
        uint32_t nflood = 0;
        const int wvd = window_verdict8(A, q, row, need, nflood);
        STAMP_COUNT(12, 1);
        STAMP_COUNT(13, __builtin_amdgcn_readfirstlane(__reduce_max_sync(~0ull, nflood)));
        if (wvd >= 0) {
          contig = wvd == 1;
          need = false;
        }
      }
      STAMP(7);  // ring + 7x7 window
      // large grids (C5: an exact search on a quarter of the steps): every row's search at
      // once in a 16x32 window first; small grids search rarely (C3: 1%) and keep their
      // registers for occupancy
      if (BIG && !p.no_bb && !p.no_rowbb && ballot(need)) {
        uint32_t bn16 = 0, bd16 = 0;
        const int vb = grid_race_bb_row<LB>(lab, n, W, H, q, row, need, vr, vc, a, amb,
                                            (uint32_t)(lNE | (lES << 1) | (lSW << 2) | (lWN << 3)),
                                            bn16, bd16);
        if (need && vb >= 0) {
          contig = vb == 1;
          need = false;
          count_search(bn16, bd16);
        }
      }
      uint64_t rows_need = ballot(q == 0 && need);
      bool locked = false;
      while (rows_need) {  // wave-cooperative exact search, one chain slot at a time
        const int L0 = __ffsll((unsigned long long)rows_need) - 1;
        rows_need &= rows_need - 1;
        const int rr = L0 >> 4;
        if constexpr (R > 1) {
          if (rr % R) {  // an earlier attempt of this chain changes the state: discarded
            const uint64_t sure = ballot(q == 0 && go && pop_ok && contig && wacc);
            const uint32_t before = (uint32_t)((1u << (rr % R)) - 1u) << (rr - rr % R);
            uint32_t rows_sure = 0;
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) rows_sure |= ((sure >> (16 * r4)) & 1u) << r4;
            if (rows_sure & before) continue;
          }
        }
        const uint32_t aa = rdl(a, L0);
        const uint32_t am4 = rdl(amb, L0);
        const uint32_t lk = rdl((uint32_t)(lNE | (lES << 1) | (lSW << 2) | (lWN << 3)), L0);
        uint64_t bn = 0, bd = 0;
        int verdict = -1;
        if (!p.no_bb)  // bitboard form first; the list search past its window
          verdict = grid_race_bb<LB>(sm + LDS_GUARD + (wv * CPW + rr / R) * p.slot_stride, n, W, H,
                                    lane, rdl(vr, L0), rdl(vc, L0), aa, am4, lk, bn, bd);
        if (verdict >= 0) {
          if (row == rr) {
            contig = verdict == 1;
            count_search(bn, bd);
          }
          continue;
        }
        if (!locked) {
          // the scratch and visit list are shared by the workgroup's waves
          if (lane == 0) {
            int expect = 0;
            while (!__hip_atomic_compare_exchange_strong(&s_lock, &expect, 1, __ATOMIC_ACQUIRE,
                                                         __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP)) {
              expect = 0;
              __builtin_amdgcn_s_sleep(1);
            }
          }
          lds_order();
          locked = true;
        }
        const int vv = rdl(v, L0);
        const int mr = __popc(am4);
        // sources in CSR order (up, left, right, down) into lanes 0..m-1
        int srcn = -1;
        uint32_t mm = am4;
        for (int i = 0; i < mr; ++i) {
          const int bit = __ffs(mm) - 1;
          mm &= mm - 1;
          const int val = rdl(h.x, L0 + 1 + bit);
          if (lane == i) srcn = val;
        }
        uint64_t cls = lane < mr ? (1ull << lane) : 0ull;
        auto sx = [&](int b) { return __popc(am4 & ((1u << b) - 1u)); };
        auto merge = [&](int s1, int s2) {
          const uint64_t nm = rdl64(cls, s1) | rdl64(cls, s2);
          if (lane < mr && ((nm >> lane) & 1ull)) cls = nm;
        };
        if (lk & 1) merge(sx(0), sx(2));  // N-E
        if (lk & 2) merge(sx(2), sx(3));  // E-S
        if (lk & 4) merge(sx(3), sx(1));  // S-W
        if (lk & 8) merge(sx(1), sx(0));  // W-N
        const bool ok = grid_race<LB>(sm + LDS_GUARD + (wv * CPW + rr / R) * p.slot_stride, scr, list, spill,
                                      p.qcap16, W, H, gd, lane, vv, aa, mr, srcn, cls, bn,
                                      bd);
        if (row == rr) {
          contig = ok;
          count_search(bn, bd);
        }
      }
      if (locked && lane == 0)
        __hip_atomic_store(&s_lock, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);

      STAMP(4);  // exact searches
      // ---- outcome
      const bool valid = go && pop_ok && contig;
      if constexpr (R > 1) {
        // the group consumes its attempts in order up to the first state change (valid and
        // accepted), the step limit or the retry limit; group-uniform, from row ballots
        const bool accepted = valid && wacc;
        const uint64_t b_go = ballot(q == 0 && go), b_val = ballot(q == 0 && valid);
        const uint64_t b_acc = ballot(q == 0 && accepted);
        uint32_t cons = 0, kold = 0, ns = n_steps, rt = retries;
        int fpos = -1;
        bool stop = !act;
#pragma unroll
        for (int s2 = 0; s2 < R; ++s2) {
          const int L = gb + s2 * ROW;
          const bool g2 = (b_go >> L) & 1ull, v2 = (b_val >> L) & 1ull, a2 = (b_acc >> L) & 1ull;
          if (!stop && !g2) {  // inconsistent sums: flag, stop
            stuck = 2;
            stop = true;
          }
          if (!stop) {
            cons = (uint32_t)s2 + 1u;
            if (v2) {
              ns += 1u;
              rt = 0u;
              if (a2) {
                fpos = s2;
                stop = true;
              } else {
                kold += 1u;
              }
              if (ns >= ustep) stop = true;
            } else {
              rt += 1u;
              if (rt >= (uint32_t)p.max_retries) stop = true;
            }
          }
        }
        if (sx < (int)cons) {  // this row's attempt was consumed: its counters
          n_sdeg += (uint32_t)dv;
          if (!pop_ok) n_popf += 1;
          else if (!contig) n_conf += 1;
          n_bfs += it_bfs;
          n_bfsn += it_bfsn;
          n_bfsd += it_bfsd;
        }
        n_steps = ns;
        retries = rt;
        n_att += cons;
        bpos_w += cons;
        const bool commit_me = sx == fpos;
        if (commit_me) {
          n_acc += 1;
          n_adeg += (uint32_t)dv;
          n_bchg += (uint32_t)(plus + minus);
          if (q == 0) P::axor(lab, v, a ^ d);
          if (mine && wn != wo) lds_add(gsum + (h.x >> 7), (wn - wo) << (16 * ((h.x >> 6) & 1)));
        }
        lds_order();
        uint32_t dl = commit_me && mine ? wn - wo : 0u;
        dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x111, 0xF, 0xF, true);
        dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x112, 0xF, 0xF, true);
        dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x114, 0xF, 0xF, true);
        const int dnp = (int)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x154, 0xF, 0xF, false);
        // the committing row's deltas, read by every row of its group (all lanes execute)
        const int fsrc = gb + (fpos < 0 ? 0 : fpos) * ROW + q;
        const uint32_t pk = (uint32_t)(dcut + 8) | ((uint32_t)plus << 4) | ((uint32_t)minus << 8) |
                            (a << 12) | (d << 16) | ((uint32_t)(dnp + 64) << 20);
        const uint32_t pkf = lane_read(pk, fsrc);
        const uint64_t ib = (uint64_t)__double_as_longlong(invb_new);
        const uint32_t ibl = lane_read((uint32_t)ib, fsrc), ibh = lane_read((uint32_t)(ib >> 32), fsrc);
        // yields: the old state once per consumed valid attempt before the change, then the
        // new state (the owner row keeps the chain's sums and histogram windows)
        for (uint32_t i = 0; i < kold; ++i) observe(owner);
        if (fpos >= 0) {
          npairs += (int)((pkf >> 20) & 127u) - 64;
          cut += (int)(pkf & 15u) - 8;
          bnodes += (int)((pkf >> 4) & 15u) - (int)((pkf >> 8) & 15u);
          invb = __longlong_as_double((long long)(((uint64_t)ibh << 32) | ibl));
          if ((uint32_t)q == ((pkf >> 12) & 15u)) pops -= 1;  // lean kernel: unit populations
          if ((uint32_t)q == ((pkf >> 16) & 15u)) pops += 1;
          observe(owner);
        }
        STAMP(5);
        continue;
      }
      if (go) {
        n_sdeg += (uint32_t)dv;
        if (!pop_ok) n_popf += 1;
        else if (!contig) n_conf += 1;
        retries = valid ? 0u : retries + 1u;
      }
      // ---- accept rule (lane dcut+D holds the tabulated bound; include/flipwalk.h)
      bool accepted;
      if (rule == FW_ACCEPT_BOUNDARY) {  // uniform_accept + boundary_condition
        const int32_t fv = p.flags[v] ? 1 : 0;
        const int32_t cnt = bcnt - ((uint32_t)q == a ? fv : 0) + ((uint32_t)q == d ? fv : 0);
        accepted = valid && __popc(rowbits(ballot(q < k && cnt > 0), row)) >= 2;
      } else {
        // cut_accept (grid_chain_sec11.py:171-179), or with the |B'|/|B| factor of
        // annealing_cut_accept_backwards (:81-110)
        bool acc_l;
        if (rule == FW_ACCEPT_BRATIO) {
          const double bound = thr_l * ((double)(bnodes + plus - minus) / (double)bnodes);
          acc_l = u53(x.x2, x.x3) < bound;
        } else {  // integer form of u53(x2, x3) < thr_l (exact)
          acc_l = (((uint64_t)(x.x2 >> 5) << 26) | (uint64_t)(x.x3 >> 6)) < thr53_l;
        }
        accepted = valid & (((rowbits(ballot(acc_l), row) >> (dcut + D)) & 1u) != 0u);
      }
      STAMP(8);  // outcome, accept rule
      if (FULL && p.trace != nullptr && valid && q == 0)
        p.trace[(size_t)c * p.steps + n_steps] = accepted ? v * 64 + (int)d : -1;
      n_steps += valid ? 1u : 0u;
      if (maps_on && accepted) {  // spatial observables: fire-and-forget atomics
        // index of the new state's yield (n_steps already counts this step)
        const int64_t t = (int64_t)(yields0 + (n_steps - 1u) + (first ? 1u : 0u));
        if (q >= 1 && q <= 4 && h.x >= 0 && (h.lx == a || h.lx == d)) {
          const int e = q == 1   ? grid_eid_down(vr - 1, vc, W, H)
                        : q == 2 ? grid_eid_right(vr, vc - 1, W, H)
                        : q == 3 ? grid_eid_right(vr, vc, W, H)
                                 : grid_eid_down(vr, vc, W, H);
          map_edge(p, c, e, h.lx == a, t);
        }
        if (q == 0) map_run_end(p, c, pend, t);
        pend = Pend{v, (int32_t)d, (uint32_t)t};
      }

      // ---- commit (accepting rows)
      if (accepted) {
        if (q == 0) P::axor(lab, v, a ^ d);
        // u16 group sum inside its u32 pair: a wrapping 32-bit add of the shifted
        // delta changes only that half (both halves stay in [0, 65535])
        if (mine && wn != wo) {
          lds_add(gsum + (h.x >> 7), (wn - wo) << (16 * ((h.x >> 6) & 1)));
          if (BIG) lds_add(ssum + (h.x >> 11), (wn - wo) << (16 * ((h.x >> 10) & 1)));
        }
      }
      lds_order();
      // lanes 0..4 hold the changes: a 3-step row_shr scan leaves their sum on lane 4
      uint32_t dl = accepted && mine ? wn - wo : 0u;
      dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x111, 0xF, 0xF, true);
      dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x112, 0xF, 0xF, true);
      dl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x114, 0xF, 0xF, true);
      const int dnp = (int)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x154, 0xF, 0xF, false);  // row_newbcast:4
      if (FULL && RN && accepted && p.ring_node[v]) {  // only a ring node's flip moves the pair
        const int32_t np2 = ring_pair();
        if (np2 != rpair) {
          if (q == 0 && rrun) atomicAdd(p.hist_ring + rpair, (unsigned long long)rrun);
          rrun = 0;
          rpair = np2;
        }
      }
      STAMP(9);  // commit
      // 1/|B'| by a select every lane executes: the table load completes here, before the
      // observation's histogram flush atomics, and its register is free for the next
      // iteration (consumed inside the exec-masked branch, a later reuse of that register
      // waited on vmcnt(0) -- for the flush atomics issued after it as well)
      // (the empty asm reads the loaded value in every lane, so its wait cannot sink into
      // the accepted-rows branch)
      asm volatile("" ::"v"(invb_new));
      invb = accepted ? invb_new : invb;
      if (accepted) {
        n_acc += 1;
        if (FULL && p.sched) sched_row(n_acc);
        n_adeg += (uint32_t)dv;
        npairs += dnp;
        cut += dcut;
        bnodes += plus - minus;
        n_bchg += (uint32_t)(plus + minus);
        if ((uint32_t)q == a) pops -= pv;
        if ((uint32_t)q == d) pops += pv;
        if (rule == FW_ACCEPT_BOUNDARY && p.flags[v]) {
          if ((uint32_t)q == a) bcnt -= 1;
          if ((uint32_t)q == d) bcnt += 1;
        }
        // the new state's wait draw (its proposal was attempt att0 + n_att - 1)
        if (waits_on) wcur = wait_draw(p.seed, att0 + (uint64_t)(n_att - 1u), gid, p.wlp[bnodes]);
      }
      observe(valid);
      STAMP(5);  // counters, observe
    }

    STAMP(6);  // loop exit
    if constexpr (R > 1) {  // the row-local counters of the group, summed into every row
      n_popf = grp_sum<R>(n_popf, gb, q);
      n_conf = grp_sum<R>(n_conf, gb, q);
      n_sdeg = grp_sum<R>(n_sdeg, gb, q);
      n_acc = grp_sum<R>(n_acc, gb, q);
      n_adeg = grp_sum<R>(n_adeg, gb, q);
      n_bchg = grp_sum<R>(n_bchg, gb, q);
      n_bfs = grp_sum64<R>(n_bfs, gb, q);
      n_bfsn = grp_sum64<R>(n_bfsn, gb, q);
      n_bfsd = grp_sum64<R>(n_bfsd, gb, q);
    }
    // ---- write back (R > 1: the owner row)
    if (has && owner) {
      if (hc0) HIST_ADD(p.hist_cut + base_c + q, (unsigned long long)hc0);
      if (hc1) HIST_ADD(p.hist_cut + base_c + ROW + q, (unsigned long long)hc1);
      if (hb0) HIST_ADD(p.hist_b + base_b + q, (unsigned long long)hb0);
      if (hb1) HIST_ADD(p.hist_b + base_b + ROW + q, (unsigned long long)hb1);
      if (FULL && RN && q == 0 && rrun) atomicAdd(p.hist_ring + rpair, (unsigned long long)rrun);
      int qw = q;  // OPQ: see the state load
      if constexpr (OPQ) asm volatile("" : "+v"(qw));
      u32x4* dst = reinterpret_cast<u32x4*>(p.labels + (size_t)c * p.lab_stride);
      const LDS u32x4* src = reinterpret_cast<const LDS u32x4*>(lab);
      for (int i = qw; i < p.lab_copy16; i += ROW) dst[i] = src[i];  // labels + group sums
      if (qw < k) p.pops[(size_t)c * k + qw] = (int64_t)pops;
      if (qw < k && rule == FW_ACCEPT_BOUNDARY) p.bcnt[(size_t)c * k + qw] = bcnt;
      if (q == 0 && maps_on) pend_store(p, c, pend);
      if (q == 0 && waits_on) {
        p.wsamp[2 * (size_t)c] = wsum;
        p.wsamp[2 * (size_t)c + 1] = wcur;
      }
      // the 136-byte stats record as 16-byte read-modify-writes by row-lanes 0..8 (every
      // lane of a row holds the row-uniform values): 9 requests instead of 19 4- and 8-byte
      // ones (no measurable change in time or PMC WRITE_SIZE: profiles/r02/c3)
      if (q <= 8) {
        // the record address from an opaque lane id in every instantiation: hoisted, its
        // 64-bit lane offset was the one value the C3 kernel's 3-wave budget spilled
        int qr = qw;
        if constexpr (!OPQ) asm volatile("" : "+v"(qr));
        uint64_t* rec = reinterpret_cast<uint64_t*>(stp) + 2 * qr;
        const uint64_t o0 = rec[0];
        const uint64_t o1 = qr < 8 ? rec[1] : 0ull;
        const uint64_t yinc = (uint64_t)n_steps + (first ? 1u : 0u);
        uint64_t w0, w1;
        switch (q) {
          case 0: w0 = att0 + n_att; w1 = o1 + n_steps; break;
          case 1: w0 = o0 + n_acc; w1 = o1 + n_popf; break;
          case 2: w0 = o0 + n_conf; w1 = o1 + n_bfs; break;
          case 3: w0 = o0 + n_bfsn; w1 = o1 + n_bfsd; break;
          case 4: w0 = o0 + n_sdeg; w1 = o1 + n_adeg; break;
          case 5: w0 = o0 + n_bchg; w1 = o1 + yinc; break;
          case 6: w0 = (uint64_t)sum_cut; w1 = (uint64_t)sum_bnodes; break;
          case 7:
            w0 = (uint64_t)__double_as_longlong(sum_invb);
            w1 = (uint64_t)(uint32_t)cut | ((uint64_t)(uint32_t)bnodes << 32);
            break;
          default: w0 = (uint64_t)(uint32_t)npairs | ((uint64_t)(uint32_t)stuck << 32); w1 = 0;
        }
        if (qr < 8) {
          typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u64x2*>(rec) = u64x2{w0, w1};
        } else {
          rec[0] = w0;
        }
      }
    }
    lds_order();
    UNIT_TIME(u, 1);
    if (seg + 1 < p.slices) {  // hand the quad to its next slice (every lane, one word)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(p.seg_done + quad, seg + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  STAMP_FLUSH
}

// Register budgets.  The kernel holds 48 chains per CU at 3 waves per SIMD, which LDS and
// 168 VGPRs allow together; its search paths want a few more registers, so the default
// instantiation is held to 3 waves per SIMD (a few VGPRs spilled, outside the hot path:
// C3 +0.8%, +2% at 15,000-35,000 steps, profiles/r06/ab/ab_*_v6.jsonl) and a second lean
// one (W2) keeps every register, at 2 waves per SIMD, for launches with no more than 2
// waves of work per SIMD (the 8-GPU job's 8,192-chain shards: +4.6%).
template <int LB, int MODE, int PER, bool FULL, bool BIG>
__global__ __launch_bounds__(64 * MAX_NW) __attribute__((amdgpu_waves_per_eu(3))) void fw_grid16_kernel(FwRunParams p) {
  static_assert(!FULL, "FULL instantiations: fw_grid16_full_kernel");
  grid16_body<LB, MODE, PER, FULL, BIG, 1>(p);
}
// FULL (optional features on): the compiler's own register budget, as in round 5 (held to 3
// waves per SIMD it spilled 130-190 B per lane)
template <int LB, int MODE, int PER, bool FULL, bool BIG>
__global__ __launch_bounds__(64 * MAX_NW) void fw_grid16_full_kernel(FwRunParams p) {
  grid16_body<LB, MODE, PER, true, BIG, 1>(p);
}
template <int LB, int MODE, int PER>
__global__ __launch_bounds__(64 * MAX_NW) void fw_grid16_w2_kernel(FwRunParams p) {
  grid16_body<LB, MODE, PER, false, false, 1, true>(p);
}

// speculative attempts: R rows per chain.  A 3-waves-per-SIMD register budget (168 VGPRs:
// 2-4 spilled, against ~60 under the 4-wave budget of round 3): C2 (4,096 chains, R = 4)
// 1.256 -> 1.316 x 10^9, the 8,192-chain C3 shard R = 2 equal to R = 1
// (profiles/r04/spec_wpe3/)
#ifndef FW_SPEC_WPE
#define FW_SPEC_WPE 3
#endif
template <int LB, int MODE, int PER, int R>
__global__ __launch_bounds__(64 * MAX_NW) __attribute__((amdgpu_waves_per_eu(FW_SPEC_WPE))) void
fw_grid16_spec_kernel(FwRunParams p) {
  grid16_body<LB, MODE, PER, false, false, R>(p);
}

// group sums per lane (PER) for G groups; BIG: supergroup sums per lane for G groups
int per16(int G) { return G <= 16 * 2 ? 2 : G <= 16 * 4 ? 4 : G <= 16 * 10 ? 10 : 16; }
int per16_big(int G) { return (G + 15) / 16 <= 32 ? 2 : 4; }
bool is_big(int G) { return G > 16 * 16; }

template <int LB, int MODE, int PER, bool FULL, bool BIG>
void* k16() {
  if constexpr (FULL)
    return reinterpret_cast<void*>(&fw_grid16_full_kernel<LB, MODE, PER, true, BIG>);
  else
    return reinterpret_cast<void*>(&fw_grid16_kernel<LB, MODE, PER, false, BIG>);
}

// the small-grid lean instantiations (fw_grid16_lean.hip; the stamps build: here)
template <int LB, int MODE>
void* pick16_small_lean(int G) {
  switch (per16(G)) {
    case 2: return k16<LB, MODE, 2, false, false>();
    case 4: return k16<LB, MODE, 4, false, false>();
    case 10: return k16<LB, MODE, 10, false, false>();
    default: return k16<LB, MODE, 16, false, false>();
  }
}

template <int LB, int MODE, bool FULL>
void* pick16(int G) {
  if (is_big(G)) {
    if constexpr (LB == 4) {
      return nullptr;  // large grids take 2- or 3-bit labels
    } else {
      return per16_big(G) == 2
                 ? k16<LB, MODE, 2, FULL, true>()
                 : k16<LB, MODE, 4, FULL, true>();
    }
  }
  if constexpr (LB == 3) {
    return nullptr;  // small grids keep 2- or 4-bit labels
  } else if constexpr (FULL) {
    switch (per16(G)) {
      case 2: return k16<LB, MODE, 2, true, false>();
      case 4: return k16<LB, MODE, 4, true, false>();
      case 10: return k16<LB, MODE, 10, true, false>();
      default: return k16<LB, MODE, 16, true, false>();
    }
  } else {
#if defined(FW_STAMPS)
    return pick16_small_lean<LB, MODE>(G);
#else
    return fw_grid16_pick_lean(LB, MODE, G);  // fw_grid16_lean.hip
#endif
  }
}

template <int MODE>
void* pick16_w2(int G) {
  if (is_big(G)) return nullptr;
  switch (per16(G)) {
    case 2: return reinterpret_cast<void*>(&fw_grid16_w2_kernel<2, MODE, 2>);
    case 4: return reinterpret_cast<void*>(&fw_grid16_w2_kernel<2, MODE, 4>);
    case 10: return reinterpret_cast<void*>(&fw_grid16_w2_kernel<2, MODE, 10>);
    default: return reinterpret_cast<void*>(&fw_grid16_w2_kernel<2, MODE, 16>);
  }
}

template <int LB, int MODE, int R>
void* pick16_spec(int G) {
  if (is_big(G) || LB == 3) return nullptr;
  switch (per16(G)) {
    case 2: return reinterpret_cast<void*>(&fw_grid16_spec_kernel<LB, MODE, 2, R>);
    case 4: return reinterpret_cast<void*>(&fw_grid16_spec_kernel<LB, MODE, 4, R>);
    case 10: return reinterpret_cast<void*>(&fw_grid16_spec_kernel<LB, MODE, 10, R>);
    default: return reinterpret_cast<void*>(&fw_grid16_spec_kernel<LB, MODE, 16, R>);
  }
}

template <int R>
void* pick16_spec_mode(const FwRunParams& p) {
  const bool cut = p.mode == FW_PROPOSE_CUTEDGE;
  if (p.lb == 2)
    return cut ? pick16_spec<2, FW_PROPOSE_CUTEDGE, R>(p.G) : pick16_spec<2, FW_PROPOSE_PAIRS, R>(p.G);
  if (p.lb == 4)
    return cut ? pick16_spec<4, FW_PROPOSE_CUTEDGE, R>(p.G) : pick16_spec<4, FW_PROPOSE_PAIRS, R>(p.G);
  return nullptr;
}

template <bool FULL>
void* pick16_mode(const FwRunParams& p) {
  const bool cut = p.mode == FW_PROPOSE_CUTEDGE;
  if (p.lb == 2)
    return cut ? pick16<2, FW_PROPOSE_CUTEDGE, FULL>(p.G) : pick16<2, FW_PROPOSE_PAIRS, FULL>(p.G);
  if (p.lb == 3)
    return cut ? pick16<3, FW_PROPOSE_CUTEDGE, FULL>(p.G) : pick16<3, FW_PROPOSE_PAIRS, FULL>(p.G);
  return cut ? pick16<4, FW_PROPOSE_CUTEDGE, FULL>(p.G) : pick16<4, FW_PROPOSE_PAIRS, FULL>(p.G);
}

int round16i(int x) { return (x + 15) / 16 * 16; }

}  // namespace

// fw_grid16_w2.hip and fw_grid16_lean.hip include this file with FW_G16_W2_TU /
// FW_G16_LEAN_TU and compile only their pickers' instantiations
#if defined(FW_G16_W2_TU) || defined(FW_STAMPS)
void* fw_grid16_pick_w2(int mode, int G) {
  return mode == FW_PROPOSE_CUTEDGE ? pick16_w2<FW_PROPOSE_CUTEDGE>(G) : pick16_w2<FW_PROPOSE_PAIRS>(G);
}
#endif
#if defined(FW_G16_LEAN_TU) || defined(FW_STAMPS)
void* fw_grid16_pick_lean(int lb, int mode, int G) {
  const bool cut = mode == FW_PROPOSE_CUTEDGE;
  if (is_big(G)) return nullptr;  // fw_grid16.hip's large-grid plan
  if (lb == 2) return cut ? pick16_small_lean<2, FW_PROPOSE_CUTEDGE>(G) : pick16_small_lean<2, FW_PROPOSE_PAIRS>(G);
  if (lb == 4) return cut ? pick16_small_lean<4, FW_PROPOSE_CUTEDGE>(G) : pick16_small_lean<4, FW_PROPOSE_PAIRS>(G);
  return nullptr;
}
#endif
#if !defined(FW_G16_W2_TU) && !defined(FW_G16_LEAN_TU)

#ifdef FW_STAMPS
extern "C" int fw_debug_unit_times(unsigned long long* out, int n) {
  if (n > 65536) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_unit_t), sizeof(unsigned long long) * 2 * n) !=
      hipSuccess)
    return -1;
  return hipMemcpyFromSymbol(out + 2 * n, HIP_SYMBOL(g_unit_hw), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : -1;
}
extern "C" int fw_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// Largest k the large-grid plan takes.  With k <= 4 (2-bit labels, 12 chains per CU) it
// runs 200x200 chains 2.6x faster than the one-chain-per-wave kernel; with 5 <= k <= 8
// (3-bit labels) only 8 chains fit a CU in two waves, and C5's search-heavy low-base
// chains ran 10% slower than on the one-chain-per-wave kernel (profiles/r02/ab_big.jsonl),
// so those stay there unless FLIPWALK_BIG_K8=1.
int big_max_k() {
  const char* e = getenv("FLIPWALK_BIG_K8");
  return e && e[0] == '1' ? 8 : 4;
}

bool fw_grid16_candidate(int gw, int maxdeg, int G, int k, int64_t total_pop) {
  // gw >= 4: four consecutive nodes span at most one row wrap (weights4_swar masks);
  // populations are held as int32; large grids (> 256 groups, <= 1,024) need k <= 8
  return gw >= 4 && maxdeg == 4 && total_pop < (1ll << 31) - 1 &&
         ((G <= 16 * 16 && k <= 15) || (G <= 64 * 16 && k <= big_max_k()));
}

int fw_grid16_lb(int G, int k) { return k <= 4 ? 2 : (is_big(G) ? 3 : 4); }

static bool grid16_full(const FwRunParams& p) {
  return p.m_acc != nullptr || p.accept != FW_ACCEPT_CUT || p.sched != nullptr || p.ring_n > 0 ||
         p.trace != nullptr || p.g.pop != nullptr || p.wsamp != nullptr;
}

int fw_grid16_launch_rows(const FwRunParams& p) { return grid16_full(p) ? 1 : p.spec; }

// waves per workgroup of a launch: the plan holds nw * 4 / spec chain slots per workgroup,
// which the R = 1 kernels (FULL features on) fill with nw / spec waves of four chains
int fw_grid16_launch_nw(const FwRunParams& p) { return p.nw * fw_grid16_launch_rows(p) / p.spec; }

// the W2 instantiation (2-bit labels, small grids, lean, R = 1)
static void* grid16_fn_w2(const FwRunParams& p) {
  if (p.lb != 2) return nullptr;
  return fw_grid16_pick_w2(p.mode, p.G);
}

static void* grid16_fn_r(const FwRunParams& p, bool full, int R) {
  if (full) return pick16_mode<true>(p);
  if (R == 1 && p.w2) {
    void* f = grid16_fn_w2(p);
    if (f) return f;
  }
  if (R == 2) return pick16_spec_mode<2>(p);
  if (R == 4) return pick16_spec_mode<4>(p);
  return pick16_mode<false>(p);
}

void* fw_grid16_fn(const FwRunParams& p) {
  return grid16_fn_r(p, grid16_full(p), fw_grid16_launch_rows(p));
}

// LDS plan of the grid kernel: per chain slot [labels | u16 group sums], slot stride
// 16 B mod 128 B so the four rows of a wave start on different banks; then the shared
// 4-bit search scratch and visit list.  Picks the rows per chain R (speculative attempts,
// grid16_body) and the waves per workgroup (1..4) that maximise a throughput model: chains
// in flight (resident waves x 4/R, at most the chains there are) x the attempts a chain
// consumes per wave iteration, E(R) = 1 + q + ... + q^(R-1) with q = 0.56 the probability
// that an attempt leaves the state unchanged (C3), x the measured per-row speed of the R > 1
// kernels.  Ties: R = 1, then fewer waves.  FLIPWALK_SPEC=1/2/4 forces R.
int fw_grid16_plan(FwRunParams& p, int device, int* grid) {
  p.w2 = 0;  // chosen below, once the plan's rows and waves are known
  // slot: labels | u16 group sums (16 x PER per row; BIG: padded to whole supergroups) |
  // BIG: u16 supergroup sums (16 x PER)
  const bool big = is_big(p.G);
  const int gbytes = big ? round16i((p.G + 15) / 16 * 16 * 2) : 4 * 8 * per16(p.G);
  const int sbytes = big ? 4 * 8 * per16_big(p.G) : 0;
  const int slot = round16i(p.lab_bytes) + gbytes + sbytes;
  int stride = slot;
  while (stride % 128 != 16) stride += 16;
  p.slot_stride = stride;
  p.off_gsum = round16i(p.lab_bytes);
  p.off_ssum = p.off_gsum + gbytes;
  p.scr_bytes = round16i((p.g.n + 1) / 2 + 8);
  if (p.qcap16 <= 0) p.qcap16 = 384;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const char* es = getenv("FLIPWALK_SPEC");
  const int force = es && es[0] ? atoi(es) : 0;
  const char* en = getenv("FLIPWALK_GRID16_NW");  // force the waves per workgroup
  const int force_nw = en && en[0] ? atoi(en) : 0;
  const bool full = grid16_full(p);
  const bool spec_ok = !big && (p.lb == 2 || p.lb == 4) && !full;
  double best_score = -1.0;
  int best_nw = 0, best_r = 1, best_blocks = 0, best_lds = 0;
  for (int R = 1; R <= 4; R *= 2) {
    if (R > 1 && !spec_ok) break;
    if (force && force != R) continue;
    void* fn = grid16_fn_r(p, full, R);
    if (!fn) return -1;
    const int cpw = 4 / R;
    // waves per workgroup for this R: the most resident waves per CU (ties: fewer).  With
    // fewer waves of work than resident slots (the 8-GPU job's 8,192-chain shards) the
    // busiest SIMD sets the launch time: the workgroups are dealt evenly over the CUs and a
    // CU's waves over its four SIMDs, so the pick is the fewest waves on the busiest SIMD
    // (3-wave workgroups put 683 of them on 256 CUs: 3, 2, 2, 2 waves; 4-wave ones 2 each).
    const long long wunits = (p.n_chains + cpw - 1) / cpw;
    const int cus = prop.multiProcessorCount;
    auto busiest_simd = [&](int nw, int per_cu) -> long long {
      const long long wgs = (wunits + nw - 1) / nw;
      if (wgs > (long long)per_cu * cus) return -1;  // more work than slots: rounds
      return ((wgs + cus - 1) / cus * nw + 3) / 4;
    };
    int r_nw = 0, r_blocks = 0, r_lds = 0;
    long long r_busy = -1;
    for (int nw = R; nw <= MAX_NW; ++nw) {
      if (nw % R) continue;  // the R = 1 kernels must fill the same slots (fw_grid16_launch_nw)
      if (force_nw && nw != force_nw) continue;
      const int lds = LDS_GUARD + cpw * nw * stride + p.scr_bytes + 4 * p.qcap16;
      if (lds > 160 * 1024 - 256) break;
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * nw, (size_t)lds) !=
          hipSuccess)
        return -1;
      const long long busy = per_cu > 0 ? busiest_simd(nw, per_cu) : -1;
      bool take;
      if (r_nw == 0)
        take = per_cu > 0;
      else if (busy >= 0 && r_busy >= 0)  // both hold all the work: the less loaded SIMD
        take = busy < r_busy || (busy == r_busy && per_cu * nw > r_blocks * r_nw);
      else if (busy >= 0 || r_busy >= 0)  // only one holds all the work
        take = busy >= 0;
      else
        take = per_cu * nw > r_blocks * r_nw;
      if (take) {
        r_nw = nw;
        r_blocks = per_cu;
        r_lds = lds;
        r_busy = busy;
      }
    }
    if (r_nw == 0) continue;
    const double e_r = R == 1 ? 1.0 : (R == 2 ? 1.56 : 1.0 + 0.56 + 0.56 * 0.56 + 0.56 * 0.56 * 0.56);
    // per-row speed of the speculative kernels relative to R = 1 (the merge, a few spilled
    // VGPRs), calibrated on the measured lines: C2 (4,096 chains) R = 4 ~ +10% over R = 1
    // and +1.5% over R = 2, the 8,192-chain C3 shard R = 2 equal to R = 1 and R = 4 -28%
    // (profiles/r03/e/ab_spec.jsonl, profiles/r04/spec_wpe3/)
    const double eff = R == 1 ? 1.0 : (R == 2 ? 0.6 : 0.72);
    const double waves = (double)r_blocks * r_nw * prop.multiProcessorCount;
    const double units = (double)((p.n_chains + cpw - 1) / cpw);
    const double score = std::min(units, waves) * cpw * e_r * eff;
    if (score > best_score * (1.0 + 1e-9)) {
      best_score = score;
      best_nw = r_nw;
      best_r = R;
      best_blocks = r_blocks;
      best_lds = r_lds;
    }
  }
  if (best_nw == 0) return -1;
  // W2: with no more than 2 waves of work per SIMD the lean R = 1 kernel runs under the
  // 2-waves-per-SIMD register budget (no spills; FLIPWALK_W2=0 / 1 forbids / forces it)
  p.w2 = 0;
  {
    const char* ew = getenv("FLIPWALK_W2");
    const int want = ew && ew[0] ? atoi(ew) : -1;
    void* fw2 = (best_r == 1 && !full && want != 0) ? grid16_fn_w2(p) : nullptr;
    const long long quads = (p.n_chains + 3) / 4;
    const int cus = prop.multiProcessorCount;
    if (fw2 && (want == 1 || quads <= 2ll * 4 * cus)) {
      int w_nw = 0, w_blocks = 0, w_lds = 0;
      long long w_busy = -1;
      for (int nw = 1; nw <= MAX_NW; ++nw) {
        if (force_nw && nw != force_nw) continue;
        const int lds = LDS_GUARD + 4 * nw * stride + p.scr_bytes + 4 * p.qcap16;
        if (lds > 160 * 1024 - 256) break;
        if (hipFuncSetAttribute(fw2, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
          return -1;
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fw2, 64 * nw, (size_t)lds) !=
                hipSuccess || per_cu <= 0)
          continue;
        const long long wgs = (quads + nw - 1) / nw;
        const long long busy = wgs > (long long)per_cu * cus ? -1 : ((wgs + cus - 1) / cus * nw + 3) / 4;
        if (busy < 0) continue;  // W2 must hold all the work in one round
        if (w_nw == 0 || busy < w_busy) {
          w_nw = nw;
          w_blocks = per_cu;
          w_lds = lds;
          w_busy = busy;
        }
      }
      if (w_nw) {
        p.w2 = 1;
        best_nw = w_nw;
        best_blocks = w_blocks;
        best_lds = w_lds;
      }
    }
  }
  p.spec = best_r;
  p.nw = best_nw;
  const int cpw = 4 / best_r;
  p.off_scr = LDS_GUARD + cpw * best_nw * stride;
  p.off_list16 = p.off_scr + p.scr_bytes;
  p.lds16 = best_lds;
  // both the lean kernel of the plan (W2 or not) and the FULL one (features switched on later)
  for (int f = 0; f < 2; ++f) {
    void* fn = grid16_fn_r(p, f == 1, f == 1 ? 1 : best_r);
    if (fn && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, best_lds) != hipSuccess)
      return -1;
  }
  const char* verbose = getenv("FLIPWALK_VERBOSE");
  if (verbose && verbose[0] == '1')
    fprintf(stderr, "flipwalk: grid kernel %s%s, %d-bit labels, %d row(s) per chain, LDS %d B per "
            "workgroup of %d waves, %d workgroups (%d chains) per CU\n",
            is_big(p.G) ? "large-grid plan" : "small-grid plan", p.w2 ? " (W2 register budget)" : "",
            p.lb, best_r, best_lds, best_nw, best_blocks, best_blocks * best_nw * cpw);
  const long long per_wg = (long long)cpw * best_nw;
  long long gsz = (long long)best_blocks * prop.multiProcessorCount;
  const long long need = (p.n_chains + per_wg - 1) / per_wg;
  if (gsz > need) gsz = need;
  *grid = (int)(gsz < 1 ? 1 : gsz);
  return 0;
}

int fw_grid16_launch(const FwRunParams& p, int grid, void* stream) {
  void* args[] = {const_cast<FwRunParams*>(&p)};
  void* fn = fw_grid16_fn(p);  // the lean or the FULL instantiation (same LDS plan)
  if (!fn) return (int)hipErrorInvalidDeviceFunction;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds16);
  if (e != hipSuccess) return (int)e;
  return (int)hipLaunchKernel(fn, dim3(grid), dim3(64 * fw_grid16_launch_nw(p)), args,
                              (size_t)p.lds16, (hipStream_t)stream);
}
#endif  // !FW_G16_W2_TU && !FW_G16_LEAN_TU
