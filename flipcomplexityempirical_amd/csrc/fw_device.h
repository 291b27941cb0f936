// fw_device.h — device-side building blocks shared by the gfx950 chain kernels
// (fw_kernels.hip: one chain per wavefront; fw_grid16.hip: four chains per
// wavefront on row-major grids): wave utilities (DPP scans, ballots, readlane),
// Philox4x32-10, packed LDS labels, the neighbourhood gather and the exact
// level-synchronous race search for single_flip_contiguous.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "fw_internal.h"
#include "fw_math.h"

// Explicit address spaces: every chain-state access must be a DS (LDS) or global
// instruction.  Generic pointers let the compiler emit FLAT accesses, which are not
// ordered against DS atomics of the same wave.
#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // 16-byte copies (no class ops)

namespace {

constexpr int WAVE = 64;

// ---------------------------------------------------------------- wave utilities
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int32_t rfl(int32_t x) {
  return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rdl(uint32_t x, int l) {
  return __builtin_amdgcn_readlane(x, l);
}
__device__ __forceinline__ int32_t rdl(int32_t x, int l) {
  return (int32_t)__builtin_amdgcn_readlane((uint32_t)x, l);
}
// Launders a wave-uniform value into a VGPR (keeps it out of the scarce SGPRs; the
// volatile asm is not hoisted, so per-use copies are not turned back into SGPR constants)
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}
__device__ __forceinline__ uint64_t in_vgpr64(uint64_t x) {
  return ((uint64_t)in_vgpr((uint32_t)(x >> 32)) << 32) | in_vgpr((uint32_t)x);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t x, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double rdl_f64(double x, int l) {
  return __longlong_as_double((long long)rdl64((uint64_t)__double_as_longlong(x), l));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Inclusive wave-wide prefix sum with DPP (row_shr within 16-lane rows, then the
// row_bcast:15 / row_bcast:31 carries across rows).  No LDS traffic.
__device__ __forceinline__ uint32_t scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}
// wave-wide sum, returned uniform
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) { return rdl(scan_incl(x), 63); }
// wave-wide OR / max of 32-bit values with the DPP pattern of scan_incl (no LDS round
// trips; wave_or64's ds_bpermute steps each wait on the LDS pipe), returned uniform
__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return rdl(x, 63);
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
  return rdl(x, 63);
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x |= __shfl_xor(x, d, WAVE);
  return x;
}
// index of the (j+1)-th set bit of m (m has more than j set bits)
__device__ __forceinline__ int nth_bit(uint64_t m, uint32_t j) {
  for (uint32_t t = 0; t < j; ++t) m &= m - 1;
  return __ffsll((unsigned long long)m) - 1;
}

// Compiler-only ordering point.  LDS instructions of one wave execute in program
// order, so a single-wave workgroup needs no s_waitcnt to see its own LDS writes.
__device__ __forceinline__ void lds_order() { __asm__ __volatile__("" ::: "memory"); }

// ---------------------------------------------------------------- Philox4x32-10
struct U4 {
  uint32_t x0, x1, x2, x3;
};
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}
// floor(((x1<<32)|x0) * P / 2^64)
__device__ __forceinline__ uint32_t scale64(uint32_t x0, uint32_t x1, uint32_t P) {
  uint64_t lo = (uint64_t)x0 * P;
  uint64_t hi = (uint64_t)x1 * P + (lo >> 32);
  return (uint32_t)(hi >> 32);
}
__device__ __forceinline__ double u53(uint32_t x2, uint32_t x3) {
  return ((double)(x2 >> 5) * 67108864.0 + (double)(x3 >> 6)) * (1.0 / 9007199254740992.0);
}

// The sampled geometric wait of the state created by proposal attempt t of chain gid
// (FW_WAIT_T0: the initial state), given lp = log1p(-|B|/(N^k - 1)) of that state: the
// Philox block (t, hi(t) | 2^31, gid) of key seed, u = CPython random() of words (x0, x1),
// wait = floor(log1p(-u) / lp) — the oracle's wait_draw (oracle/flipchain_oracle.c).
__device__ __forceinline__ double wait_draw(uint64_t seed, uint64_t t, uint64_t gid, double lp) {
  const U4 y = philox((uint32_t)t, (uint32_t)(t >> 32) | 0x80000000u, (uint32_t)gid,
                      (uint32_t)(gid >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  const double lu = fw_log1p(-u53(y.x0, y.x1));
  return lu == 0.0 ? 0.0 : floor(lu / lp);
}

// ---------------------------------------------------------------- packed labels
template <int LB>
struct PK {
  static constexpr uint32_t MASK = (1u << LB) - 1u;
  __device__ static __forceinline__ uint32_t get(const LDS uint8_t* b, int x) {
    if constexpr (LB == 8) {
      return b[x];
    } else if constexpr (LB == 4) {
      return (uint32_t)(b[x >> 1] >> ((x & 1) << 2)) & 15u;
    } else {
      static_assert(LB == 2, "labels are 2, 4 or 8 bits");
      return (uint32_t)(b[x >> 2] >> ((x & 3) << 1)) & 3u;
    }
  }
  __device__ static __forceinline__ LDS uint32_t* word(LDS uint8_t* b, int x) {
    return reinterpret_cast<LDS uint32_t*>(b) + ((x * LB) >> 5);
  }
  __device__ static __forceinline__ int shift(int x) { return (x * LB) & 31; }
  // field ^= d, safe against concurrent updates of other fields of the word
  __device__ static __forceinline__ void axor(LDS uint8_t* b, int x, uint32_t d) {
    __atomic_fetch_xor(word(b, x), d << shift(x), __ATOMIC_RELAXED);
  }
  // claim field x: a -> code, if it still holds a; returns the value found (a on success)
  __device__ static __forceinline__ uint32_t claim(LDS uint8_t* b, int x, uint32_t a,
                                                   uint32_t code) {
    LDS uint32_t* w = word(b, x);
    const int sh = shift(x);
    uint32_t old = *w;
    for (;;) {
      const uint32_t cur = (old >> sh) & MASK;
      if (cur != a) return cur;
      const uint32_t nw = old ^ ((a ^ code) << sh);
      if (__atomic_compare_exchange_n(w, &old, nw, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
        return a;  // on failure `old` now holds the current word
    }
  }
};

// 3-bit labels (k <= 8 on the grid kernel's large-grid plan): node x in bits [3x, 3x+3) of
// a little-endian dword stream, so a field may straddle two dwords.  Reads take the dword
// pair (one ds_read2_b32; the label region is padded past its last field); an update xors
// each dword the field touches (two atomics for a straddling field).
template <>
struct PK<3> {
  static constexpr uint32_t MASK = 7u;
  __device__ static __forceinline__ uint32_t get(const LDS uint8_t* b, int x) {
    const LDS uint32_t* w = reinterpret_cast<const LDS uint32_t*>(b);
    const int bit = 3 * x, wi = bit >> 5;
    const uint64_t both = ((uint64_t)w[wi + 1] << 32) | w[wi];
    return (uint32_t)(both >> (bit & 31)) & 7u;
  }
  __device__ static __forceinline__ void axor(LDS uint8_t* b, int x, uint32_t d) {
    LDS uint32_t* w = reinterpret_cast<LDS uint32_t*>(b);
    const int bit = 3 * x, wi = bit >> 5, sh = bit & 31;
    __atomic_fetch_xor(w + wi, d << sh, __ATOMIC_RELAXED);
    if (sh > 29) __atomic_fetch_xor(w + wi + 1, d >> (32 - sh), __ATOMIC_RELAXED);
  }
};

// 5-bit labels (the chain kernel on general graphs with 16 <= k <= 31, e.g. C4's k = 18;
// the list search keeps its marks in HBM): the same dword-pair reads and straddle updates.
template <>
struct PK<5> {
  static constexpr uint32_t MASK = 31u;
  __device__ static __forceinline__ uint32_t get(const LDS uint8_t* b, int x) {
    const LDS uint32_t* w = reinterpret_cast<const LDS uint32_t*>(b);
    const int bit = 5 * x, wi = bit >> 5;
    const uint64_t both = ((uint64_t)w[wi + 1] << 32) | w[wi];
    return (uint32_t)(both >> (bit & 31)) & 31u;
  }
  __device__ static __forceinline__ void axor(LDS uint8_t* b, int x, uint32_t d) {
    LDS uint32_t* w = reinterpret_cast<LDS uint32_t*>(b);
    const int bit = 5 * x, wi = bit >> 5, sh = bit & 31;
    __atomic_fetch_xor(w + wi, d << sh, __ATOMIC_RELAXED);
    if (sh > 27) __atomic_fetch_xor(w + wi + 1, d >> (32 - sh), __ATOMIC_RELAXED);
  }
};

__device__ __forceinline__ void lds_add(LDS uint32_t* p, uint32_t v) {
  __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}

constexpr uint32_t NOLAB = 0xFFFFu;  // label of an absent cell (never a district or code)

// Second-level local contiguity test on the 7x7 window centred at v (bit i*7+j, v = bit
// 24, A = a-labelled in-grid window cells except v).  1: every a-neighbour of v lies in
// one window component (connected); 0: some source's window component touches no border
// cell, i.e. it is a closed component of (district minus v) missing a source
// (disconnected); -1: undecided.  Identical to orc_window_verdict (the oracle).
__device__ __forceinline__ int window_verdict(uint64_t A) {
  const uint64_t C0 = 0x0040810204081ull, C6 = C0 << 6;
  const uint64_t BORDER = C0 | C6 | 0x7Full | (0x7Full << 42);
  const uint64_t src = A & ((1ull << 17) | (1ull << 23) | (1ull << 25) | (1ull << 31));
  uint64_t covered = 0;
  int verdict = -1;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int sb = s == 0 ? 17 : s == 1 ? 23 : s == 2 ? 25 : 31;
    const uint64_t b = 1ull << sb;
    if (verdict >= 0 || !(src & b) || (covered & b)) continue;
    uint64_t x = b;
    for (;;) {
      const uint64_t y = (x | ((x << 1) & ~C0) | ((x >> 1) & ~C6) | (x >> 7) | (x << 7)) & A;
      if (y == x) break;
      x = y;
    }
    if ((x & src) == src)
      verdict = 1;
    else if (!(x & BORDER))
      verdict = 0;
    covered |= x;
  }
  return verdict;
}
// window_verdict with the four source flood fills run side by side in lanes 0..3 (VALU,
// two dilations per convergence test) instead of one after another on the scalar unit.
// Fills of sources in one window component are equal and the others disjoint, so the
// sequential verdict is order-free: 1 if some fill holds every source, else 0 if some
// fill touches no border, else -1.  Wave-uniform result.
__device__ __forceinline__ int window_verdict_lanes(uint64_t A, int lane) {
  const uint64_t C0 = 0x0040810204081ull, C6 = C0 << 6;
  const uint64_t BORDER = C0 | C6 | 0x7Full | (0x7Full << 42);
  const uint64_t src = A & ((1ull << 17) | (1ull << 23) | (1ull << 25) | (1ull << 31));
  const int sb = lane == 0 ? 17 : lane == 1 ? 23 : lane == 2 ? 25 : 31;
  uint64_t x = lane < 4 ? src & (1ull << sb) : 0ull;
  for (;;) {
    const uint64_t y = (x | ((x << 1) & ~C0) | ((x >> 1) & ~C6) | (x >> 7) | (x << 7)) & A;
    const uint64_t z = (y | ((y << 1) & ~C0) | ((y >> 1) & ~C6) | (y >> 7) | (y << 7)) & A;
    const bool moving = z != y;
    x = z;
    if (!ballot(moving)) break;
  }
  if (ballot(x != 0ull && (x & src) == src)) return 1;
  return ballot(x != 0ull && (x & BORDER) == 0ull) ? 0 : -1;
}

// window cell c in [0,48) (v skipped) -> bit position and (di, dj) offsets from v
__device__ __forceinline__ int window_pos(int c) { return c < 24 ? c : c + 1; }

// ---------------------------------------------------------------- spatial observables
// Canonical id of a grid edge (node (r,c) to its right / lower neighbour): the position
// of the pair in CSR row order of the row-major W x H grid (include/flipwalk.h).
__device__ __forceinline__ int grid_eid_right(int r, int c, int W, int H) {
  return r * (2 * W - 1) + c * (1 + (r < H - 1 ? 1 : 0));
}
__device__ __forceinline__ int grid_eid_down(int r, int c, int W, int H) {
  return grid_eid_right(r, c, W, H) + (c < W - 1 ? 1 : 0);
}

// The pending run of the current state's creating flip (f < 0: the initial state).
struct Pend {
  int32_t f, lab;
  uint32_t t0;  // yield index at which the state was first yielded
};

__device__ __forceinline__ Pend pend_load(const FwRunParams& p, int c) {
  if (p.m_acc == nullptr) return Pend{-1, 0, 0u};
  const int32_t* pe = p.m_pend + 4 * (size_t)c;
  return Pend{pe[0], pe[1], (uint32_t)pe[2]};
}
__device__ __forceinline__ void pend_store(const FwRunParams& p, int c, const Pend& pd) {
  int32_t* pe = p.m_pend + 4 * (size_t)c;
  pe[0] = pd.f;
  pe[1] = pd.lab;
  pe[2] = (int32_t)pd.t0;
}
// Edge e of chain c changes status at yield t (the new state's index):
// cut_times = acc + [cut now] * yields, so becoming cut subtracts t, uncut adds t.
__device__ __forceinline__ void map_edge(const FwRunParams& p, int c, int e, bool becomes_cut,
                                         int64_t t) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p.m_acc + (size_t)c * p.g.nedges + e),
            (unsigned long long)(becomes_cut ? -t : t));
}
// The run of pd.f (yields pd.t0 .. t-1) ends: the reference's per-yield updates
// part_sum[f] -= L*(t_i - last_flipped); last_flipped = t_i; num_flips += 1, summed.
__device__ __forceinline__ void map_run_end(const FwRunParams& p, int c, const Pend& pd,
                                            int64_t t) {
  if (pd.f < 0) return;
  const size_t o = (size_t)c * p.g.n + pd.f;
  atomicAdd(p.m_nf + o, (uint32_t)(t - (int64_t)pd.t0));
  const uint32_t old = atomicExch(p.m_lf + o, (uint32_t)(t - 1));
  atomicAdd(reinterpret_cast<unsigned long long*>(p.m_ps + o),
            (unsigned long long)(-p.m_labval[pd.lab] * ((t - 1) - (int64_t)old)));
}

// ---------------------------------------------------------------- chain context
// Grid lane roles for v's neighbourhood: 0 v, 1 up, 2 left, 3 right, 4 down
// (= CSR order of v's neighbours), 5 NE, 6 SE, 7 SW, 8 NW.
__device__ __forceinline__ void role_off(int l, int& dr, int& dc) {
  dr = 0;
  dc = 0;
  switch (l) {
    case 1: dr = -1; break;
    case 2: dc = -1; break;
    case 3: dc = 1; break;
    case 4: dr = 1; break;
    case 5: dr = -1; dc = 1; break;
    case 6: dr = 1; dc = 1; break;
    case 7: dr = 1; dc = -1; break;
    case 8: dr = -1; dc = -1; break;
    default: break;
  }
}

// What one lane learns about its node x of v's neighbourhood.
// MT: the label-set mask, 32 bits wherever labels are below 32 (every width but 8 bits)
template <typename MT>
struct HoodT {
  int x;          // node id, -1 if absent
  uint32_t lx;    // label of x (NOLAB if absent)
  MT bits;        // OR of 1<<label over x's neighbours other than v
  uint32_t cnt;   // number of x's neighbours other than v with label != lx
  bool has_v;     // v is a neighbour of x
  int deg;        // degree of x
};
__device__ __forceinline__ uint32_t popcnt(uint32_t x) { return (uint32_t)__popc(x); }
__device__ __forceinline__ uint32_t popcnt(uint64_t x) { return (uint32_t)__popcll(x); }

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// the value of the previous / next lane (wave_shr:1 / wave_shl:1 DPP; 0 at the wave's ends)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, true);
}
// cells of X and their 4-neighbours (lane = grid row, bit = column)
__device__ __forceinline__ uint32_t dilate32(uint32_t x) {
  return x | (x << 1) | (x >> 1) | from_prev_lane(x) | from_next_lane(x);
}

// 32 bits "label == a" of the 32 nodes x0 .. x0+31 of a packed LB-bit label array of n
// nodes.  Words before the array (x0 < 0) or past it are read at clamped positions: they
// hold only nodes < 0 or >= n, which the caller masks.
template <int LB>
__device__ __forceinline__ uint32_t eq_bits32(const LDS uint8_t* lab, int n, int x0, uint32_t a) {
  const LDS uint32_t* w = reinterpret_cast<const LDS uint32_t*>(lab);
  const int bit = x0 * LB;
  const int wi = bit >> 5;  // arithmetic
  const uint32_t sh = (uint32_t)bit & 31u;
  const int wlast = (n * LB - 1) >> 5;
  uint32_t wd[LB + 1];
#pragma unroll
  for (int j = 0; j <= LB; ++j) wd[j] = w[min(max(wi + j, 0), wlast)];
  if constexpr (LB == 3) {
    // realign the 96 bits of the 32 fields to bit 0; XOR with a repeated every 3 bits, so
    // a field equals a iff its 3 bits are 0; OR each field's bits onto its lowest (funnel
    // shifts carry the two fields that straddle words); then the fields' low bits, at
    // stride 3 in each word (phases 0, 1, 2), are compacted as a 3-D Morton decode does
    const uint32_t r0 = __builtin_amdgcn_alignbit(wd[1], wd[0], sh);
    const uint32_t r1 = __builtin_amdgcn_alignbit(wd[2], wd[1], sh);
    const uint32_t r2 = __builtin_amdgcn_alignbit(wd[3], wd[2], sh);
    const uint32_t pa = a * 0x49249249u;
    const uint32_t y0 = r0 ^ pa, y1 = r1 ^ ((pa << 1) | (a >> 2)), y2 = r2 ^ ((pa << 2) | (a >> 1));
    const uint32_t z0 = y0 | __builtin_amdgcn_alignbit(y1, y0, 1) | __builtin_amdgcn_alignbit(y1, y0, 2);
    const uint32_t z1 = y1 | __builtin_amdgcn_alignbit(y2, y1, 1) | __builtin_amdgcn_alignbit(y2, y1, 2);
    const uint32_t z2 = y2 | (y2 >> 1) | (y2 >> 2);
    auto compact3 = [](uint32_t x) {  // bits 0, 3, ..., 30 -> 0 .. 10
      x &= 0x49249249u;
      x = (x ^ (x >> 2)) & 0xC30C30C3u;
      x = (x ^ (x >> 4)) & 0x0F00F00Fu;
      x = (x ^ (x >> 8)) & 0xFF0000FFu;
      return (x ^ (x >> 16)) & 0x000007FFu;
    };
    return compact3(~z0) | (compact3(~z1 >> 1) << 11) | ((compact3(~z2 >> 2) & 0x3FFu) << 22);
  }
  uint32_t out = 0;
#pragma unroll
  for (int j = 0; j < (LB == 3 ? 0 : LB); ++j) {  // 32 / LB labels per aligned dword
    const uint32_t x = __builtin_amdgcn_alignbit(wd[j + 1], wd[j], sh);
    uint32_t e;
    if constexpr (LB == 2) {
      const uint32_t y = x ^ (a * 0x55555555u);
      e = ~(y | (y >> 1)) & 0x55555555u;
      e = (e | (e >> 1)) & 0x33333333u;
      e = (e | (e >> 2)) & 0x0F0F0F0Fu;
      e = (e | (e >> 4)) & 0x00FF00FFu;
      e = (e | (e >> 8)) & 0x0000FFFFu;
    } else if constexpr (LB == 4) {
      const uint32_t y = x ^ (a * 0x11111111u);
      e = ~(y | (y >> 1) | (y >> 2) | (y >> 3)) & 0x11111111u;
      e = (e | (e >> 3)) & 0x03030303u;
      e = (e | (e >> 6)) & 0x000F000Fu;
      e = (e | (e >> 12)) & 0x000000FFu;
    } else {
      static_assert(LB == 8 || LB == 3, "labels are 2, 3, 4 or 8 bits");
      const uint32_t y = x ^ (a * 0x01010101u);
      e = (~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u) >> 7;
      e = (e | (e >> 7)) & 0x00030003u;
      e = (e | (e >> 14)) & 0x0000000Fu;
    }
    out |= e << (j * (32 / LB));
  }
  return out;
}

// The exact race search of single_flip_contiguous (fw_device.h Ctx::race_search, the
// oracle's contiguous_after) on bitboards, for row-major grids: a 64-row x 32-column
// window around v, lane i = grid row vr - 32 + i, bit b = column vc - 16 + b, one u32 of
// a-labelled cells (v excluded) per lane.  Level by level it holds the sets the list
// search builds: per source direction d (0 up, 1 left, 2 right, 3 down) the frontier
// cells reached from d, and the cells new at the next level.  Two classes merge when a
// frontier cell of one is adjacent to a frontier cell or to a new cell of the other:
// exactly the merges the list search makes, whatever its claim order.  The stopping rules
// are the list search's, so the verdict and the counters (cells of the processed levels,
// their degrees) equal its own.  No scratch, no lock, one VGPR per set.  am4: source
// directions; lk: ring links pre-merged (bit 0 N-E, 1 E-S, 2 S-W, 3 W-N).  Returns -1
// (nothing counted) when a frontier about to be processed holds a window-edge cell whose
// outward neighbour is on the grid: the caller then runs the list search.
template <int LB>
__device__ int grid_race_bb(const LDS uint8_t* lab, int n, int W, int H, int lane, int vr,
                            int vc, uint32_t a, uint32_t am4, uint32_t lk, uint64_t& bfs_nodes,
                            uint64_t& bfs_deg) {
  const int r = vr - 32 + lane, c0 = vc - 16;
  const bool rin = (r >= 0) & (r < H);
  uint32_t A = eq_bits32<LB>(lab, n, (rin ? r : vr) * W + c0, a);
  const int lo_cut = c0 < 0 ? -c0 : 0;  // bits of columns < 0
  const int hi_n = W - c0;              // bits >= hi_n: columns >= W (hi_n >= 17)
  uint32_t cm = ~0u << lo_cut;
  if (hi_n < 32) cm &= (1u << hi_n) - 1u;
  A &= rin ? cm : 0u;
  if (lane == 32) A &= ~(1u << 16);  // v
  // window-edge cells with an on-grid neighbour outside the window
  uint32_t E = ((lane == 0) & (r > 0)) | ((lane == 63) & (r < H - 1)) ? ~0u : 0u;
  if (c0 > 0) E |= 1u;
  if (c0 + 31 < W - 1) E |= 1u << 31;
  E &= A;
  // frontier per direction; sources up (31, 16), left (32, 15), right (32, 17), down (33, 16)
  uint32_t F[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int sl = d == 0 ? 31 : (d == 3 ? 33 : 32), sb = d == 1 ? 15 : (d == 2 ? 17 : 16);
    F[d] = (lane == sl && ((am4 >> d) & 1u)) ? (1u << sb) : 0u;
  }
  // class of direction d: 4-bit member mask at bits 4d (uniform)
  uint32_t M = 0x8421u;
  auto unite = [&](int i, int j) {
    const uint32_t m = ((M >> (4 * i)) | (M >> (4 * j))) & 15u;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if ((m >> d) & 1u) M = (M & ~(15u << (4 * d))) | (m << (4 * d));
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
  int verdict = -1;
  uint32_t P;  // processed cells
  if (n_classes() == 2) {
    // two classes after the ring links (most searches): one frontier per class, the union
    // of its directions' frontiers -- dilation and the merge test distribute over unions,
    // and a class is closed when every direction of it is -- one merge test and two reach
    // ballots per level; the general loop's levels, stopping rules and counters
    // (grid_race_bb2's two-class path on this 32-column window)
    uint32_t fa = 0u, fb = 0u;
    int ra = -1;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!((am4 >> d) & 1u)) continue;
      const int rep = __ffs((M >> (4 * d)) & 15u) - 1;
      if (ra < 0) ra = rep;
      if (rep == ra)
        fa |= F[d];
      else
        fb |= F[d];
    }
    for (;;) {
      if (ballot(((fa | fb) & E) != 0u)) return -1;
      const uint32_t da = dilate32(fa) & A, db = dilate32(fb) & A;
      const uint32_t nw = (da | db) & ~V;
      const bool met = ballot((da & (fb | (db & nw))) != 0u) != 0ull;
      fa = da & nw;
      fb = db & nw;
      // met: connected; a class with no new cell: closed, disconnected.  Either way the
      // processed cells are the visited ones before this level's new cells.
      if (met || !ballot(fa != 0u) || !ballot(fb != 0u)) {
        verdict = met ? 1 : 0;
        break;
      }
      V |= nw;
    }
    P = V;
  } else
  for (;;) {
    const uint32_t lvl = F[0] | F[1] | F[2] | F[3];
    if (n_classes() == 1) {
      verdict = 1;
      P = V & ~lvl;
      break;
    }
    if (ballot((lvl & E) != 0u)) return -1;
    uint32_t D[4], nw = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      D[d] = ((am4 >> d) & 1u) ? dilate32(F[d]) & A : 0u;
      nw |= D[d];
    }
    nw &= ~V;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = i + 1; j < 4; ++j) {
        if (!((am4 >> i) & 1u) || !((am4 >> j) & 1u) || ((M >> (4 * i + j)) & 1u)) continue;
        if (ballot((D[i] & (F[j] | (D[j] & nw))) != 0u)) unite(i, j);
      }
    uint32_t reach = 0;  // directions with a new cell
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      F[d] = D[d] & nw;
      reach |= ballot(F[d] != 0u) ? (1u << d) : 0u;
    }
    P = V;
    if (n_classes() == 1) {
      verdict = 1;
      break;
    }
    // a class none of whose directions reached a new cell is closed: disconnected
    bool closed = false;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      closed |= ((am4 >> d) & 1u) && (reach & (M >> (4 * d)) & 15u) == 0u;
    if (closed) {
      verdict = 0;
      break;
    }
    V |= nw;
  }
  // counters over the processed cells: degree = on-grid 4-neighbours
  const uint32_t pc = (uint32_t)__popc(P);
  uint32_t dg = pc * (uint32_t)((r > 0) + (r < H - 1) + 2);
  if (c0 <= 0) dg -= (P >> (-c0)) & 1u;          // column 0
  if (hi_n <= 32) dg -= (P >> (hi_n - 1)) & 1u;  // column W - 1
  bfs_nodes += wave_sum(pc);
  bfs_deg += wave_sum(dg);
  return verdict;
}

// Where grid_race_bb2's two-class race stopped when its frontier reached the window edge:
// per lane (grid row vr - 32 + lane, columns vc - 32 ...) each class's current frontier
// (level L) and previous one (level L - 1), the count and degree sum of the cells already
// processed (levels < L), and the direction that represents each class.  The list search
// continues the race from here instead of from the sources (race_search_b3).  Only levels
// L - 1 and L need marks: the race is a breadth-first search of (district a) minus v, so a
// neighbour of a level-L cell lies at level L - 1, L or L + 1, and the cells of levels
// < L - 1 are never met again.
struct BBSeed {
  uint32_t qa0, qa1, qb0, qb1, fa0, fa1, fb0, fb1;
  uint32_t pc, pdeg;  // processed cells of this lane's row, their degree sum
  int ra, rb;  // representative directions (0 up, 1 left, 2 right, 3 down)
  bool ok;
};

// grid_race_bb on a 64-row x 64-column window: lane i = grid row vr - 32 + i, bit b of
// dword w = column vc - 32 + 32 w + b, two VGPRs per set.  The same sets, levels, merges,
// stopping rules and counters; a window-edge frontier returns -1 as there.  Used by the
// one-chain-per-wave kernel on large grids (C5), whose steady-state searches leave the
// 32-column window in a quarter of the runs and the 64-column one in 5% (200x200, k=8,
// base 0.1 after 30,000 steps: scripts/search_stats.c).
template <int LB>
__device__ int grid_race_bb2(const LDS uint8_t* lab, int n, int W, int H, int lane, int vr,
                             int vc, uint32_t a, uint32_t am4, uint32_t lk, uint64_t& bfs_nodes,
                             uint64_t& bfs_deg, BBSeed& sd, uint32_t& lv_mid,
                             uint32_t& lv_64) {
  sd.ok = false;
  const int r = vr - 32 + lane, c0 = vc - 32;
  const bool rin = (r >= 0) & (r < H);
  const int rowb = (rin ? r : vr) * W + c0;
  // bits of columns cb .. cb + 31 inside [0, W)
  auto colmask = [W](int cb) -> uint32_t {
    uint32_t mk = cb <= -32 ? 0u : (cb < 0 ? ~0u << (-cb) : ~0u);
    const int hi = W - cb;
    if (hi < 32) mk &= hi <= 0 ? 0u : (1u << hi) - 1u;
    return mk;
  };
  uint32_t A0 = eq_bits32<LB>(lab, n, rowb, a), A1 = eq_bits32<LB>(lab, n, rowb + 32, a);
  A0 &= rin ? colmask(c0) : 0u;
  A1 &= rin ? colmask(c0 + 32) : 0u;
  if (lane == 32) A1 &= ~1u;  // v
  // window-edge cells with an on-grid neighbour outside the window
  const uint32_t er = ((lane == 0) & (r > 0)) | ((lane == 63) & (r < H - 1)) ? ~0u : 0u;
  uint32_t E0 = er, E1 = er;
  if (c0 > 0) E0 |= 1u;
  if (c0 + 63 < W - 1) E1 |= 1u << 31;
  E0 &= A0;
  E1 &= A1;
  // frontier per direction; sources up (31, 32), left (32, 31), right (32, 33), down (33, 32)
  auto src_bits = [lane](int d, uint32_t& b0, uint32_t& b1) {
    const int sl = d == 0 ? 31 : (d == 3 ? 33 : 32);
    const bool on = lane == sl;
    b0 = on && d == 1 ? 0x80000000u : 0u;
    b1 = on && d != 1 ? (d == 2 ? 2u : 1u) : 0u;
  };
  uint32_t M = 0x8421u;  // class of direction d: 4-bit member mask at bits 4d (uniform)
  auto unite = [&](int i, int j) {
    const uint32_t m = ((M >> (4 * i)) | (M >> (4 * j))) & 15u;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if ((m >> d) & 1u) M = (M & ~(15u << (4 * d))) | (m << (4 * d));
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
  if (n_classes() == 2) {
    // two classes after the ring links (91% of C5's exact searches at steady state): one
    // frontier per class (the union of its directions' frontiers: dilation and the merge
    // test distribute over unions, and a class is closed when every direction of it is),
    // one merge test per level; the general loop's levels, stopping rules and counters
    uint32_t Fa0 = 0u, Fa1 = 0u, Fb0 = 0u, Fb1 = 0u;
    int ra = -1, rb = -1;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (!((am4 >> d) & 1u)) continue;
      uint32_t b0, b1;
      src_bits(d, b0, b1);
      const int rep = __ffs((M >> (4 * d)) & 15u) - 1;
      if (ra < 0) ra = rep;
      if (rep == ra) {
        Fa0 |= b0;
        Fa1 |= b1;
      } else {
        rb = rep;
        Fb0 |= b0;
        Fb1 |= b1;
      }
    }
    uint32_t Qa0 = 0u, Qa1 = 0u, Qb0 = 0u, Qb1 = 0u;  // the previous level, per class
    uint32_t V0 = Fa0 | Fb0, V1 = Fa1 | Fb1;
    int vd = -1;
    {
      // The race starts on the window's middle 32 columns (vc - 16 .. vc + 15, one VGPR per
      // set: half the work per level) and moves to the 64 columns with its state when a
      // frontier reaches that strip's edge.  The levels are the same: a frontier clear of
      // the strip's edge dilates inside it.
      auto mid = [](uint32_t x0, uint32_t x1) { return (x0 >> 16) | (x1 << 16); };
      const uint32_t am = mid(A0, A1);
      uint32_t em = er;
      if (c0 + 16 > 0) em |= 1u;
      if (c0 + 47 < W - 1) em |= 1u << 31;
      em &= am;
      uint32_t fa = mid(Fa0, Fa1), fb = mid(Fb0, Fb1), qa = 0u, qb = 0u, vv = fa | fb;
      for (;;) {
        if (ballot(((fa | fb) & em) != 0u)) break;  // on to the 64 columns
        ++lv_mid;
        const uint32_t da = (fa | (fa << 1) | (fa >> 1) | from_prev_lane(fa) | from_next_lane(fa)) & am;
        const uint32_t db = (fb | (fb << 1) | (fb >> 1) | from_prev_lane(fb) | from_next_lane(fb)) & am;
        const uint32_t nw = (da | db) & ~vv;
        const bool met = ballot((da & (fb | (db & nw))) != 0u) != 0ull;
        qa = fa;
        qb = fb;
        fa = da & nw;
        fb = db & nw;
        vv |= nw;
        const bool closed = !ballot(fa != 0u) || !ballot(fb != 0u);
        if (met || closed) {
          vd = met ? 1 : 0;
          vv &= ~nw;
          break;
        }
      }
      Qa0 = qa << 16;
      Qa1 = qa >> 16;
      Qb0 = qb << 16;
      Qb1 = qb >> 16;
      Fa0 = fa << 16;
      Fa1 = fa >> 16;
      Fb0 = fb << 16;
      Fb1 = fb >> 16;
      V0 = vv << 16;
      V1 = vv >> 16;
    }
    if (vd < 0) for (;;) {
      if (ballot((((Fa0 | Fb0) & E0) | ((Fa1 | Fb1) & E1)) != 0u)) {
        // processed cells (levels < L) and their degrees, counted as the list search counts
        // its dequeued nodes
        const uint32_t P0 = V0 & ~(Fa0 | Fb0), P1 = V1 & ~(Fa1 | Fb1);
        const uint32_t pc = (uint32_t)(__popc(P0) + __popc(P1));
        uint32_t dg = pc * (uint32_t)((r > 0) + (r < H - 1) + 2);
        auto pbit = [&](int pos) { return pos < 32 ? (P0 >> pos) & 1u : (P1 >> (pos - 32)) & 1u; };
        if (c0 <= 0) dg -= pbit(-c0);
        if (W - c0 <= 64) dg -= pbit(W - c0 - 1);
        sd = BBSeed{Qa0, Qa1, Qb0, Qb1, Fa0, Fa1, Fb0, Fb1, pc, dg, ra, rb, true};
        return -1;
      }
      ++lv_64;
      const uint32_t Da0 = (Fa0 | (Fa0 << 1) | (Fa0 >> 1) | (Fa1 << 31) | from_prev_lane(Fa0) | from_next_lane(Fa0)) & A0;
      const uint32_t Da1 = (Fa1 | (Fa1 << 1) | (Fa1 >> 1) | (Fa0 >> 31) | from_prev_lane(Fa1) | from_next_lane(Fa1)) & A1;
      const uint32_t Db0 = (Fb0 | (Fb0 << 1) | (Fb0 >> 1) | (Fb1 << 31) | from_prev_lane(Fb0) | from_next_lane(Fb0)) & A0;
      const uint32_t Db1 = (Fb1 | (Fb1 << 1) | (Fb1 >> 1) | (Fb0 >> 31) | from_prev_lane(Fb1) | from_next_lane(Fb1)) & A1;
      const uint32_t nw0 = (Da0 | Db0) & ~V0, nw1 = (Da1 | Db1) & ~V1;
      const bool met = ballot(((Da0 & (Fb0 | (Db0 & nw0))) | (Da1 & (Fb1 | (Db1 & nw1)))) != 0u) != 0ull;
      // the state advances unconditionally and the loop has one exit (no per-exit copies
      // of the loop-carried sets)
      Qa0 = Fa0;
      Qa1 = Fa1;
      Qb0 = Fb0;
      Qb1 = Fb1;
      Fa0 = Da0 & nw0;
      Fa1 = Da1 & nw1;
      Fb0 = Db0 & nw0;
      Fb1 = Db1 & nw1;
      V0 |= nw0;
      V1 |= nw1;
      const bool closed = !ballot((Fa0 | Fa1) != 0u) || !ballot((Fb0 | Fb1) != 0u);
      if (met || closed) {
        // met: the two classes met, connected; closed: a class reached no new cell,
        // disconnected.  Either way the cells processed are the visited ones before this
        // level's new cells.
        vd = met ? 1 : 0;
        V0 &= ~nw0;
        V1 &= ~nw1;
        break;
      }
    }
    const uint32_t pc = (uint32_t)(__popc(V0) + __popc(V1));
    uint32_t dg = pc * (uint32_t)((r > 0) + (r < H - 1) + 2);
    auto vbit = [&](int pos) { return pos < 32 ? (V0 >> pos) & 1u : (V1 >> (pos - 32)) & 1u; };
    if (c0 <= 0) dg -= vbit(-c0);
    if (W - c0 <= 64) dg -= vbit(W - c0 - 1);
    bfs_nodes += wave_sum(pc);
    bfs_deg += wave_sum(dg);
    return vd;
  }
  uint32_t F0[4], F1[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    src_bits(d, F0[d], F1[d]);
    if (!((am4 >> d) & 1u)) F0[d] = F1[d] = 0u;
  }
  uint32_t V0 = F0[0] | F0[1] | F0[2] | F0[3], V1 = F1[0] | F1[1] | F1[2] | F1[3];
  int verdict = -1;
  uint32_t P0, P1;  // processed cells
  for (;;) {
    const uint32_t l0 = F0[0] | F0[1] | F0[2] | F0[3], l1 = F1[0] | F1[1] | F1[2] | F1[3];
    if (n_classes() == 1) {
      verdict = 1;
      P0 = V0 & ~l0;
      P1 = V1 & ~l1;
      break;
    }
    if (ballot(((l0 & E0) | (l1 & E1)) != 0u)) return -1;
    uint32_t D0[4], D1[4], nw0 = 0, nw1 = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if ((am4 >> d) & 1u) {
        const uint32_t x0 = F0[d], x1 = F1[d];
        D0[d] = (x0 | (x0 << 1) | (x0 >> 1) | (x1 << 31) | from_prev_lane(x0) | from_next_lane(x0)) & A0;
        D1[d] = (x1 | (x1 << 1) | (x1 >> 1) | (x0 >> 31) | from_prev_lane(x1) | from_next_lane(x1)) & A1;
      } else {
        D0[d] = D1[d] = 0u;
      }
      nw0 |= D0[d];
      nw1 |= D1[d];
    }
    nw0 &= ~V0;
    nw1 &= ~V1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = i + 1; j < 4; ++j) {
        if (!((am4 >> i) & 1u) || !((am4 >> j) & 1u) || ((M >> (4 * i + j)) & 1u)) continue;
        if (ballot(((D0[i] & (F0[j] | (D0[j] & nw0))) | (D1[i] & (F1[j] | (D1[j] & nw1)))) != 0u))
          unite(i, j);
      }
    uint32_t reach = 0;  // directions with a new cell
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      F0[d] = D0[d] & nw0;
      F1[d] = D1[d] & nw1;
      reach |= ballot((F0[d] | F1[d]) != 0u) ? (1u << d) : 0u;
    }
    P0 = V0;
    P1 = V1;
    if (n_classes() == 1) {
      verdict = 1;
      break;
    }
    bool closed = false;  // a class none of whose directions reached a new cell
#pragma unroll
    for (int d = 0; d < 4; ++d)
      closed |= ((am4 >> d) & 1u) && (reach & (M >> (4 * d)) & 15u) == 0u;
    if (closed) {
      verdict = 0;
      break;
    }
    V0 |= nw0;
    V1 |= nw1;
  }
  // counters over the processed cells: degree = on-grid 4-neighbours
  const uint32_t pc = (uint32_t)(__popc(P0) + __popc(P1));
  uint32_t dg = pc * (uint32_t)((r > 0) + (r < H - 1) + 2);
  auto bit = [&](int pos) { return pos < 32 ? (P0 >> pos) & 1u : (P1 >> (pos - 32)) & 1u; };
  if (c0 <= 0) dg -= bit(-c0);                // column 0 (window position -c0 <= 32)
  if (W - c0 <= 64) dg -= bit(W - c0 - 1);    // column W - 1 (position >= 32)
  bfs_nodes += wave_sum(pc);
  bfs_deg += wave_sum(dg);
  return verdict;
}

// Level-1 group sums of the one-chain-per-wave kernel: lane l owns groups l*PER .. l*PER +
// PER-1 (PER even), stored as u16 pairs in dwords l*SD .. l*SD + PER/2 - 1, so a select
// reads them with PER/2 dword loads.  The lane stride SD (PER/2, padded to the next odd
// number) keeps those loads conflict-free: 32 distinct banks per 32-lane group (stride 8
// put the 32 lanes of a ds_read_b32 group on 4 banks).
__host__ __device__ constexpr int gsum_stride_dw(int per) {
  return (per / 2) % 2 ? per / 2 : per / 2 + 1;
}
template <int PER>
__device__ __forceinline__ int gsum_slot(int g) {
  return (g / PER) * (2 * gsum_stride_dw(PER)) + (g % PER);
}

// E16: a general graph of max degree <= 16 whose adjacency rows are read from the padded
// 16-wide table (four 16-byte loads in flight together) instead of walking CSR entries.
template <int LB, bool GRID, bool E16 = false>
struct Ctx {
  using P = PK<LB>;
  using MaskT = typename std::conditional<LB == 8, uint64_t, uint32_t>::type;
  using Hood = HoodT<MaskT>;
  FwGraphDev g;
  LDS uint8_t* lab;
  LDS uint16_t* gsum;  // u16 group sums (<= 64 nodes x weight <= 63), gsum_slot layout
  LDS uint32_t* wts;   // select<.., WB>: 2-bit per-node weights (node x at bits 2x), saturated at 3
  LDS uint32_t* list;  // LDS part of the search list
  GLB uint32_t* spill; // HBM part (this workgroup's slice)
  GLB uint32_t* gscr;  // race_search_gscr: this workgroup's 32-bit visit mark per node in
                       // HBM (all zero between searches; 5-bit labels cannot hold the codes)
  int32_t qcap, k;
  int32_t scap;  // race_search_b3: next-level entries staged over the group sums (<= 128)
  int lane;
  bool bb;  // grids: exact searches try the bitboard form first
  uint64_t nbadj_pre = 0;  // gather_ids: lane l's entry of v's row of nbadj
  int my_dr, my_dc;
#ifdef FW_STAMPS
  uint32_t n_win = 0, n_bbs = 0, n_list = 0;  // contiguity checks by the path that decided
  uint64_t c_win = 0, c_bbs = 0, c_list = 0;  // s_memtime cycles spent in each path
  uint64_t n_bbl = 0;                          // bitboard levels run (decided or escaped)
  uint64_t n_lvl = 0, c_clear = 0;  // race_search_b3: levels, restore cycles
  uint64_t n_mapt = 0, n_seed = 0;  // rounds of map tests; searches seeded by the bitboard
  uint64_t n_lv_mid = 0, n_lv_64 = 0;  // grid_race_bb2 levels on 32 / 64 columns
  uint64_t n_bb4 = 0, c_bb4 = 0;       // race_bb4 runs and their cycles
  __device__ static __forceinline__ uint64_t now() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
  }
#define CTX_T0 const uint64_t t_c0_ = now(); uint64_t t_c1_ = t_c0_;
#define CTX_LAP(field) do { const uint64_t t_ = now(); field += t_ - t_c1_; t_c1_ = t_; } while (0)
#else
#define CTX_T0
#define CTX_LAP(field)
#endif

  __device__ void init_roles() {
    lane = lane_id();
    role_off(lane <= 8 ? lane : 0, my_dr, my_dc);
  }
  __device__ __forceinline__ void divmod(int x, int& r, int& c) const {
    r = (int)(((uint64_t)(uint32_t)x * g.gmagic) >> 42);
    c = x - r * g.gw;
  }
  __device__ __forceinline__ uint32_t L(int x) const { return P::get(lab, x); }
  // LDS part and HBM part are read by separately typed loads: a select between the two
  // pointers would compile to a FLAT load, unordered against the list's DS writes.
  __device__ __forceinline__ uint32_t list_get(int i) const {
    const uint32_t in_lds = list[i < qcap ? i : qcap - 1];
    uint32_t in_hbm = 0;
    if (i >= qcap) in_hbm = spill[i - qcap];
    return i < qcap ? in_lds : in_hbm;
  }
  __device__ __forceinline__ void list_put(int i, uint32_t x) {
    if (i < qcap) list[i] = x;
    if (i >= qcap) spill[i - qcap] = x;
  }
  // j-th neighbour of x (grid: j = 0 up, 1 left, 2 right, 3 down); -1 if absent
  __device__ __forceinline__ int nbr(int x, int j, int xr, int xc) const {
    if constexpr (GRID) {
      switch (j) {
        case 0: return xr > 0 ? x - g.gw : -1;
        case 1: return xc > 0 ? x - 1 : -1;
        case 2: return xc < g.gw - 1 ? x + 1 : -1;
        default: return xr < g.gh - 1 ? x + g.gw : -1;
      }
    } else {
      int e = g.rowptr[x] + j;
      return e < g.rowptr[x + 1] ? g.col[e] : -1;
    }
  }
  // x's neighbours (CSR order, -1 padding) from the padded table
  __device__ __forceinline__ void row16(int x, int (&r)[16]) const {
    const i32x4* p4 = reinterpret_cast<const i32x4*>(g.ell + (size_t)x * 16);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const i32x4 q = p4[t];
      r[4 * t] = q.x;
      r[4 * t + 1] = q.y;
      r[4 * t + 2] = q.z;
      r[4 * t + 3] = q.w;
    }
  }
  __device__ __forceinline__ int degree(int x, int xr, int xc) const {
    if constexpr (GRID) {
      return (xr > 0) + (xc > 0) + (xc < g.gw - 1) + (xr < g.gh - 1);
    } else {
      return g.rowptr[x + 1] - g.rowptr[x];
    }
  }

  // E16: proposal weight and cut degree of x from its padded row, walking md entries
  // (wave-uniform, >= x's degree: the rest of a row is -1 padding)
  template <int MODE>
  __device__ __forceinline__ void weight_row(int x, int md, uint32_t& w, uint32_t& cd) const {
    int r[16];
    row16(x, r);
    const uint32_t lx = L(x);
    MaskT bits = 0;
    cd = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j >= md) break;  // uniform
      const int y = r[j];
      const uint32_t ly = L(y >= 0 ? y : x);
      bits |= y >= 0 ? MaskT(1) << ly : MaskT(0);
      cd += (y >= 0 && ly != lx) ? 1u : 0u;
    }
    w = (MODE == FW_PROPOSE_CUTEDGE) ? cd : popcnt(bits & ~(MaskT(1) << lx));
  }

  // Proposal weight and cut degree of x under the current labels.
  template <int MODE>
  __device__ __forceinline__ void weight_now(int x, uint32_t& w, uint32_t& cd) const {
    if constexpr (E16) {
      weight_row<MODE>(x, g.maxdeg, w, cd);
      return;
    }
    int xr = 0, xc = 0;
    if constexpr (GRID) divmod(x, xr, xc);
    const uint32_t lx = L(x);
    MaskT bits = 0;
    cd = 0;
    if constexpr (GRID) {
      // branch-free: the four reads issued together at clamped positions, then masked
      const bool hu = xr > 0, hl = xc > 0, hr = xc < g.gw - 1, hd = xr < g.gh - 1;
      const uint32_t lu = L(hu ? x - g.gw : x), ll = L(hl ? x - 1 : x);
      const uint32_t lr = L(hr ? x + 1 : x), ld = L(hd ? x + g.gw : x);
      const MaskT one = 1;
      bits = (hu ? one << lu : 0) | (hl ? one << ll : 0) | (hr ? one << lr : 0) |
             (hd ? one << ld : 0);
      cd = (uint32_t)(hu & (lu != lx)) + (uint32_t)(hl & (ll != lx)) + (uint32_t)(hr & (lr != lx)) +
           (uint32_t)(hd & (ld != lx));
      w = (MODE == FW_PROPOSE_CUTEDGE) ? cd : popcnt(bits & ~(one << lx));
      return;
    }
    const int dx = g.rowptr[x + 1] - g.rowptr[x];
    for (int j = 0; j < dx; ++j) {
      const int y = nbr(x, j, xr, xc);
      if (y < 0) continue;
      const uint32_t ly = L(y);
      bits |= MaskT(1) << ly;
      cd += ly != lx;
    }
    w = (MODE == FW_PROPOSE_CUTEDGE) ? cd : popcnt(bits & ~(MaskT(1) << lx));
  }

  // Weights of v's neighbourhood before and after v: a -> d (lane roles above).
  template <int MODE>
  __device__ __forceinline__ void weights_old_new(const Hood& h, uint32_t a, uint32_t d, int m,
                                                  int nb, uint32_t& wo, uint32_t& wn) const {
    if (h.x < 0) {
      wo = wn = 0;
      return;
    }
    if (lane == 0) {  // x == v: its label changes
      if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
        wo = (uint32_t)(h.deg - m);
        wn = (uint32_t)(h.deg - nb);
      } else {
        wo = popcnt(h.bits & ~(MaskT(1) << a));
        wn = popcnt(h.bits & ~(MaskT(1) << d));
      }
      return;
    }
    if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
      wo = h.cnt + (h.has_v && a != h.lx);
      wn = h.cnt + (h.has_v && d != h.lx);
    } else {
      const MaskT keep = ~(MaskT(1) << h.lx);
      wo = popcnt((h.bits | (h.has_v ? MaskT(1) << a : MaskT(0))) & keep);
      wn = popcnt((h.bits | (h.has_v ? MaskT(1) << d : MaskT(0))) & keep);
    }
  }

  // E16: v's neighbours (lanes 1..dv) and their labels, from v's padded row only
  __device__ __forceinline__ Hood gather_ids(int v, int& dv) {
    Hood h;
    h.x = -1;
    h.lx = NOLAB;
    h.bits = 0;
    h.cnt = 0;
    h.has_v = false;
    h.deg = 0;
    const int xn = (lane >= 1 && lane <= 16) ? g.ell[(size_t)v * 16 + lane - 1] : -1;
    // the local contiguity test's adjacency among v's neighbours, issued with v's row
    // (C4 +3.5%, profiles/r04/c4_nbpre)
    nbadj_pre = (lane >= 1 && lane <= 16) ? g.nbadj[(size_t)v * 16 + lane - 1] : 0ull;
    dv = __popcll(ballot(xn >= 0));
    if (lane > dv) return h;
    h.x = lane == 0 ? v : xn;
    h.lx = L(h.x);
    return h;
  }

  // One LDS round trip: every lane with a role reads its node and (lanes 0..dv) the
  // node's neighbours.
  __device__ __forceinline__ Hood gather(int v, int& dv) const {
    Hood h;
    h.x = -1;
    h.lx = NOLAB;
    h.bits = 0;
    h.cnt = 0;
    h.has_v = false;
    h.deg = 0;
    if constexpr (GRID) {
      int vr, vc;
      divmod(v, vr, vc);
      dv = degree(v, vr, vc);
      const int xr = vr + my_dr, xc = vc + my_dc;
      const bool ok = lane <= 8 && xr >= 0 && xr < g.gh && xc >= 0 && xc < g.gw;
      // branch-free: every lane reads its cell and the cell's four neighbours at clamped
      // positions (one LDS round trip), and the roles mask the results
      const int xx = ok ? xr * g.gw + xc : v;
      const uint32_t lxx = L(xx);
      const bool hu = ok & (xr > 0), hl = ok & (xc > 0), hr = ok & (xc < g.gw - 1),
                 hd = ok & (xr < g.gh - 1);
      const uint32_t lu = L(hu ? xx - g.gw : xx), ll = L(hl ? xx - 1 : xx);
      const uint32_t lr = L(hr ? xx + 1 : xx), ld = L(hd ? xx + g.gw : xx);
      if (!ok) return h;
      h.x = xx;
      h.lx = lxx;
      if (lane <= 4) {
        h.deg = (int)hu + (int)hl + (int)hr + (int)hd;
        // v's slot among the neighbour's neighbours: up's down, left's right, ...
        const bool vu = lane == 4, vl = lane == 3, vrr = lane == 2, vd = lane == 1;
        h.has_v = lane > 0;
        const bool uu = hu & !vu, ul = hl & !vl, ur = hr & !vrr, ud = hd & !vd;
        const MaskT one = 1;
        h.bits = (uu ? one << lu : 0) | (ul ? one << ll : 0) | (ur ? one << lr : 0) |
                 (ud ? one << ld : 0);
        h.cnt = (uint32_t)(uu & (lu != lxx)) + (uint32_t)(ul & (ll != lxx)) +
                (uint32_t)(ur & (lr != lxx)) + (uint32_t)(ud & (ld != lxx));
      }
    } else if constexpr (E16) {
      // lanes 1..16 read v's padded row: its neighbours (a prefix) and so its degree; the
      // rows below are walked up to the largest degree among v and its neighbours
      const int md = rfl(g.dbound[v]);
      const int xn = (lane >= 1 && lane <= 16) ? g.ell[(size_t)v * 16 + lane - 1] : -1;
      dv = __popcll(ballot(xn >= 0));
      if (lane > dv) return h;
      h.x = lane == 0 ? v : xn;
      h.lx = L(h.x);
      int r[16];
      row16(h.x, r);
      int deg = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j >= md) break;  // uniform
        const int y = r[j];
        const bool ok = y >= 0 && y != v;
        const uint32_t ly = L(ok ? y : h.x);
        deg += y >= 0 ? 1 : 0;
        h.has_v = h.has_v || y == v;
        h.bits |= ok ? MaskT(1) << ly : MaskT(0);
        h.cnt += (ok && ly != h.lx) ? 1u : 0u;
      }
      h.deg = deg;
      return h;
    } else {
      const int e0 = g.rowptr[v];
      dv = g.rowptr[v + 1] - e0;
      if (lane > dv) return h;
      h.x = lane == 0 ? v : g.col[e0 + lane - 1];
      h.lx = L(h.x);
      const int f0 = g.rowptr[h.x], f1 = g.rowptr[h.x + 1];
      h.deg = f1 - f0;
      for (int e = f0; e < f1; ++e) {
        const int y = g.col[e];
        if (y == v) {
          h.has_v = true;
          continue;
        }
        const uint32_t ly = L(y);
        h.bits |= MaskT(1) << ly;
        h.cnt += ly != h.lx;
      }
    }
    return h;
  }

  // -------------------------------------------------------------- select
  // rank r in [0, P) -> node v and in-node index j (canonical (node, ·) order).
  // PER = group sums held per lane (compile-time bound, >= ceil(G/64)).
  template <int MODE, int PER, bool WB = false>
  __device__ __forceinline__ void select(uint32_t r, int G, int& v, uint32_t& j) const {
    static_assert(PER % 2 == 0, "group sums are read as u16 pairs");
    constexpr int SD = gsum_stride_dw(PER);
    uint32_t gs[PER];
    uint32_t s = 0;
    const int g0 = lane * PER;
    const int dw_last = gsum_slot<PER>(G - 1) >> 1;
    const LDS uint32_t* g32 = reinterpret_cast<const LDS uint32_t*>(gsum);
#pragma unroll
    for (int t = 0; t < PER / 2; ++t) {  // unconditional (clamped) u16-pair reads, masked values
      const uint32_t w = g32[min(lane * SD + t, dw_last)];
      gs[2 * t] = g0 + 2 * t < G ? (w & 0xFFFFu) : 0u;
      gs[2 * t + 1] = g0 + 2 * t + 1 < G ? (w >> 16) : 0u;
      s += gs[2 * t] + gs[2 * t + 1];
    }
    const uint32_t incl = scan_incl(s);
    const uint64_t m = ballot(incl > r);
    if (m == 0) {  // inconsistent weights: report instead of reading out of range
      v = -1;
      return;
    }
    // lane-local walk over this lane's groups (only the owning lane's result is used)
    const uint32_t rl = r - (incl - s);
    uint32_t c = 0, before = 0;
    int tf = PER;
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const uint32_t c2 = c + gs[t];
      if (tf == PER && rl < c2) {
        tf = t;
        before = c;
      }
      c = c2;
    }
    const int Lw = __ffsll((unsigned long long)m) - 1;
    const int gi = rdl(tf < PER ? g0 + tf : G, Lw);
    const uint32_t r1 = rdl(rl - before, Lw);
    if (gi >= G) {
      v = -1;
      return;
    }
    const int x = gi * 64 + lane;
    uint32_t wx = 0, cd;
    if constexpr (E16 && WB) {
      // the group's weights from LDS; a saturated one (>= 3: four districts around a node,
      // a few groups in a hundred at C4) from its padded row
      wx = x < g.n ? (wts[x >> 4] >> ((x & 15) << 1)) & 3u : 0u;
      if (ballot(wx == 3u)) {
        const int md = rfl(g.dbound[g.n + gi]);
        if (wx == 3u) weight_row<MODE>(x, md, wx, cd);
      }
    } else if constexpr (E16) {
      // the group's rows are walked up to its largest degree (C4: 9.7 on average, not 14)
      const int md = rfl(g.dbound[g.n + gi]);
      if (x < g.n) weight_row<MODE>(x, md, wx, cd);
    } else {
      if (x < g.n) weight_now<MODE>(x, wx, cd);
    }
    const uint32_t incl2 = scan_incl(wx);
    const uint64_t m2 = ballot(incl2 > r1);
    if (m2 == 0) {
      v = -1;
      return;
    }
    const int L2 = __ffsll((unsigned long long)m2) - 1;
    v = gi * 64 + L2;
    j = r1 - rdl(incl2 - wx, L2);
  }

  // -------------------------------------------------------------- contiguity
  // -- visit marks in HBM (LB == 5 only: 3-bit labels run on grids, race_search_b3): one 32-bit word per node in
  // this workgroup's slice of gscr, 0 = unvisited, 1 + source index, ~0 = v.  A claim is
  // ONE compare-and-swap that returns the mark it found (the class of an already visited
  // node): no separate load and no retry loop, as 4-bit marks sharing a word needed
  // (Hilbert-numbered neighbours share words, so their claims collided).  Agent-scope
  // atomics: they execute in the L2, and the marks are read back within the same search.
  __device__ __forceinline__ void gm_set(int x, uint32_t code) const {
    __hip_atomic_store(gscr + x, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ uint32_t gm_claim(int x, uint32_t code) const {
    uint32_t old = 0u;
    __hip_atomic_compare_exchange_strong(gscr + x, &old, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return old;  // 0: claimed (the CAS stored code); else the mark found
  }

  // The race search with the visit marks in gscr instead of in the labels (5-bit labels
  // cannot hold the codes): the same levels, pushes, merges and counters as race_search
  // (and as the grid kernel's grid_race).  A level's nodes are processed four at a time,
  // sixteen lanes per node, lane j of a node's group taking its padded row's entry j: one
  // round of dependent memory trips (row entry, label, claim) serves every neighbour of four
  // nodes, where a lane per node walked its row entry by entry, two L2 round trips per entry
  // (C4: ~50,000 cycles per run, the kernel's largest cost).  The order in which a level's
  // claims are made changes no level, verdict or counter (the merges they produce do not
  // depend on it: grid_race_bb).  A list entry carries its node's source index (node |
  // index << 28), so the node's mark is never read back.
  __device__ bool race_search_gscr(int v, uint32_t a, int m, int src, uint64_t cls,
                                   uint64_t& bfs_nodes, uint64_t& bfs_deg) {
    // one 16-lane group per node: a CSR row past 16 entries would lose neighbours 16 and up,
    // so only padded rows (E16: max degree <= 16) and grids (slots 0..3) may use it; node
    // ids live in bits 0..27 of a list entry (fw_chains_create: n <= 65,536, G <= 1,024)
    static_assert(E16 || GRID, "race_search_gscr: padded 16-wide rows or grids only");
    constexpr uint32_t XM = (1u << 28) - 1u;
    if (lane == 0) gm_set(v, ~0u);  // v: never a class (any m, up to the row's 16 sources)
    if (lane < m) {
      gm_set(src, 1u + (uint32_t)lane);
      list_put(lane, (uint32_t)src | ((uint32_t)lane << 28));
    }
    __threadfence_block();
    int nl = m, lb = 0, le = m;
    uint32_t my_deg = 0;
    int verdict = -1;
    const int j = lane & 15;
    for (;;) {
      uint64_t rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
      if (__popcll(rep) == 1) {
        verdict = 1;
        break;
      }
      uint64_t pushed_src = 0;
      for (int base = lb; base < le; base += WAVE) {
        const int nb = min(WAVE, le - base);
        bfs_nodes += (uint64_t)nb;
        // the node's entry (its group's 16 lanes read the same word), then its row entry j;
        // the next four nodes' are fetched while this step's claims are made
        auto fetch = [&](int f0, uint32_t& e, int& y) {
          const int f = f0 + (lane >> 4);
          const bool fa = f < nb;
          e = fa ? list_get(base + f) : 0u;
          const int x = (int)(e & XM);
          if constexpr (E16) {
            y = fa ? g.ell[(size_t)x * 16 + j] : -1;
          } else {
            int xr = 0, xc = 0;
            if constexpr (GRID) divmod(x, xr, xc);
            // CSR rows of degree <= 16 (one group per node); grids: slots 0..3
            y = fa && (!GRID || j < 4) ? nbr(x, j, xr, xc) : -1;
          }
        };
        uint32_t e_n;
        int y_n;
        fetch(0, e_n, y_n);
        for (int f0 = 0; f0 < nb; f0 += 4) {
          const uint32_t e = e_n;
          const int y = y_n;
          if (f0 + 4 < nb) fetch(f0 + 4, e_n, y_n);
          const uint32_t o = e >> 28;
          my_deg += y >= 0 ? 1u : 0u;
          bool push = false, req = false;
          uint32_t other = 0;
          if (y >= 0 && L(y) == a) {
            const uint32_t got = gm_claim(y, 1u + o);
            if (got == 0u) {
              push = true;
            } else if (got - 1u < (uint32_t)m) {  // v (~0) is never a class
              req = true;
              other = got - 1u;
            }
          }
          const uint64_t pm = ballot(push);
          if (push) list_put(nl + (int)mbcnt(pm), (uint32_t)y | (o << 28));
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
        __threadfence_block();  // marks and spilled entries are read next level
      }
      lds_order();
      lb = le;
      le = nl;
      rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
      if (__popcll(rep) == 1) {
        verdict = 1;
        break;
      }
      const bool closed = lane < m && ((rep >> lane) & 1ull) && ((cls & pushed_src) == 0ull);
      if (ballot(closed)) {
        verdict = 0;
        break;
      }
    }
    bfs_deg += wave_sum(my_deg);
    for (int base = 0; base < nl; base += WAVE) {  // clear the visit marks
      const int idx = base + lane;
      if (idx < nl) gm_set((int)(list_get(idx) & XM), 0u);
    }
    if (lane == 0) gm_set(v, 0u);
    __threadfence_block();
    return verdict == 1;
  }

  // race_search_b3's start when a bitboard stage hands its race over: the class codes, the
  // stage's displaced group-sum words, the head of the visit list (n1 entries of level L - 1,
  // then the n2 of level L, marked and staged), the processed cells (per-lane partial
  // counts) and the two classes' representative sources
  struct B3Run {
    uint32_t codes, ambig, sv0, sv1, pc, pdeg;
    int n1, n2, ra, rb;
    bool ok;
  };

  // race_search_b3's class codes: the unused labels k..7 first, then borrowed district
  // labels (ambiguous: bit o), preferring those absent from a sample of 256 cells around v
  // (a 16 x 16 lattice of step 4): a code met by a frontier is then rarely a real district
  // cell, so merge tests stay rare.  3-bit code of class o at bits 3o.
  __device__ void b3_codes(int v, uint32_t a, int m, uint32_t& codes, uint32_t& ambig) const {
    codes = 0;
    ambig = 0;
    int vr, vc;
    divmod(v, vr, vc);
    uint32_t seen = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cell = lane + WAVE * t;  // 0..255
      const int rr = vr + 4 * (cell >> 4) - 30, cc = vc + 4 * (cell & 15) - 30;
      if (rr >= 0 && rr < g.gh && cc >= 0 && cc < g.gw) seen |= 1u << L(rr * g.gw + cc);
    }
    seen = wave_or32(seen);
    int o = 0;
    for (uint32_t c = (uint32_t)k; c < 8u && o < m; ++c, ++o) codes |= c << (3 * o);
    for (int pass = 0; pass < 2; ++pass)  // absent labels first, then present ones
      for (uint32_t t = 1; t < 8u && o < m; ++t) {
        const uint32_t c = (a + t) & 7u;
        if (c >= (uint32_t)k || ((seen >> c) & 1u) != (uint32_t)pass) continue;
        codes |= c << (3 * o);
        ambig |= 1u << o;
        ++o;
      }
  }

  // The two-class race continued on a 128 x 128 window when grid_race_bb2's left its 64 x 64
  // one (C5's steady state: 19% of the exact searches at base 0.1 after 10^5 steps leave the
  // 64 x 64 window, 3% the 128 x 128 one; scripts/search_stats.c).  Lane j holds grid rows
  // vr - 64 + 2j (p = 0) and vr - 63 + 2j (p = 1), dword d of a row the columns vc - 64 + 32d
  // ...; four dwords per row, eight VGPRs per set.  The race is breadth-first, so the cells
  // a level meets lie in the previous level Q, the frontier F or the next level: the visited
  // set is never needed, only Q (the sets are A, Fa, Fb, Q).  The levels, merges, stopping
  // rules and counters are grid_race_bb2's.  When a frontier about to be processed holds a
  // window-edge cell whose outward neighbour is on the grid it returns -1, having written
  // the list search's start (B3Run): level L (the frontier) and the cells of level L - 1
  // next to it take their class's code and head the visit list.  The rest of level L - 1
  // is never met again: its neighbours lie at levels L - 2 .. L, and level L is F.
  template <int ND>
  __device__ int race_bb4(int v, int vr, int vc, uint32_t a, int m, const BBSeed& s2,
                          uint64_t& bfs_nodes, uint64_t& bfs_deg, B3Run& rs) {
    const int W = g.gw, H = g.gh;
    constexpr int WC = 32 * ND;  // window columns
    const int R0 = vr - 64, C0 = vc - WC / 2;
    const int re = R0 + 2 * lane;
    // a-labelled cells of dword d of row p (v excluded)
    auto district = [&](int p, int d) -> uint32_t {
      const int r = re + p, cb = C0 + 32 * d;
      if (r < 0 || r >= H) return 0u;
      uint32_t mk = cb <= -32 ? 0u : (cb < 0 ? ~0u << (-cb) : ~0u);
      const int hi = W - cb;
      if (hi < 32) mk &= hi <= 0 ? 0u : (1u << hi) - 1u;
      uint32_t x = eq_bits32<LB>(lab, g.n, r * W + cb, a) & mk;
      if (lane == 32 && p == 0 && d == (WC / 2) / 32) x &= ~(1u << ((WC / 2) % 32));  // v
      return x;
    };
    // bb2's 64 x 64 state: its lane i (row vr - 32 + i) is row 32 + i here, i.e. lane
    // 16 + i / 2, p = i & 1; its 64 columns start at window column WC / 2 - 32
    const bool tin = lane >= 16 && lane < 48;
    const int se = tin ? 2 * (lane - 16) : 0;
    auto xfer = [&](uint32_t x, int p) -> uint32_t {
      const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((se + p) << 2, (int)x);
      return tin ? y : 0u;
    };
    // a 64-column row (x1:x0) placed at window column WC / 2 - 32, as dword d
    auto place = [](uint32_t x0, uint32_t x1, int d) -> uint32_t {
      if constexpr (ND == 4) {
        return d == 1 ? x0 : d == 2 ? x1 : 0u;
      } else {
        static_assert(ND == 3, "race_bb4: 96- or 128-column windows");
        return d == 0 ? x0 << 16 : d == 1 ? (x0 >> 16) | (x1 << 16) : x1 >> 16;
      }
    };
    // U: the district's cells not yet reached (bb2's last two levels removed; its older
    // levels stay in U but are never met again), F: the frontier of each class
    uint32_t U[2][ND], Fa[2][ND], Fb[2][ND];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t fa0 = xfer(s2.fa0, p), fa1 = xfer(s2.fa1, p);
      const uint32_t fb0 = xfer(s2.fb0, p), fb1 = xfer(s2.fb1, p);
      const uint32_t q0 = xfer(s2.qa0 | s2.qb0, p), q1 = xfer(s2.qa1 | s2.qb1, p);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        Fa[p][d] = place(fa0, fa1, d);
        Fb[p][d] = place(fb0, fb1, d);
        U[p][d] = district(p, d) & ~(place(q0, q1, d) | Fa[p][d] | Fb[p][d]);
      }
    }
    uint32_t pc = s2.pc, pdeg = s2.pdeg;  // processed cells (bb2's, then this window's)
    // on-grid degree of a cell: per row, minus one in grid columns 0 and W - 1
    const uint32_t fdeg0 = (uint32_t)((re > 0) + (re < H - 1) + 2);
    const uint32_t fdeg1 = (uint32_t)((re + 1 > 0) + (re + 1 < H - 1) + 2);
    const int w0 = -C0, w1 = W - 1 - C0;  // window positions of grid columns 0 and W - 1
    // bit `pos` (wave-uniform) of a row held as ND dwords.  The dword is picked by masks,
    // not by a select over an array: LLVM turned that select into an indexed load of a
    // stack copy of the array (a scratch store and load per call, C5's only non-spill
    // scratch traffic)
    auto wbit = [](const uint32_t (&f)[ND], int pos) -> uint32_t {
      const int sel = pos >> 5;
      uint32_t dd = 0u;
#pragma unroll
      for (int d = 0; d < ND; ++d) dd |= f[d] & (0u - (uint32_t)(sel == d));
      return (dd >> (pos & 31)) & 1u;
    };
    // The processed cells are counted once, after the loop: they are the frontier handed
    // over plus the cells reached since, less the current frontier, i.e. per row
    // |F0| + |U0| - |U| - |F| (F0, U0 disjoint; U only shrinks), and a grid-edge column's
    // cell is processed when it was in F0 | U0 and is in neither U nor F now.
    uint32_t cnt[2], ebits = 0u;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t f[ND];
      cnt[p] = 0u;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        f[d] = Fa[p][d] | Fb[p][d] | U[p][d];
        cnt[p] += (uint32_t)__popc(f[d]);
      }
      if (w0 >= 0 && w0 < WC) ebits |= wbit(f, w0) << (2 * p);
      if (w1 >= 0 && w1 < WC) ebits |= wbit(f, w1) << (2 * p + 1);
    }
    // window-edge cells with an on-grid neighbour outside the window
    const bool e_top = lane == 0 && R0 > 0, e_bot = lane == 63 && R0 + 127 < H - 1;
    const bool e_left = C0 > 0, e_right = C0 + WC - 1 < W - 1;
    int vd = -1;
    for (;;) {
      bool edge = false;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint32_t any = 0u;
#pragma unroll
        for (int d = 0; d < ND; ++d) any |= Fa[p][d] | Fb[p][d];
        edge |= (e_left && ((Fa[p][0] | Fb[p][0]) & 1u)) || (e_right && ((Fa[p][ND - 1] | Fb[p][ND - 1]) >> 31));
        if (p == 0 ? e_top : e_bot) edge |= any != 0u;
      }
      if (ballot(edge)) break;
      // dilations, the new cells and the merge test, one column of dwords at a time (both
      // rows), updating the sets in place: the old values a later dword needs (its left
      // neighbour's carry) are held in pa / pb, and the other lanes' rows are read by DPP
      // before this dword of theirs is updated (one instruction stream).  bb2's merge test
      // D_a & (F_b | (D_b & new)) is (dil F_a & F_b) | (dil F_a & dil F_b & U) here
      bool met = false;
      bool any_a = false, any_b = false;
      uint32_t pa0 = 0u, pa1 = 0u, pb0 = 0u, pb1 = 0u;  // old F of dword d - 1, rows 0 / 1
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const uint32_t a0 = Fa[0][d], a1 = Fa[1][d], b0 = Fb[0][d], b1 = Fb[1][d];
        const uint32_t na0 = d < ND - 1 ? Fa[0][d + 1] : 0u, na1 = d < ND - 1 ? Fa[1][d + 1] : 0u;
        const uint32_t nb0 = d < ND - 1 ? Fb[0][d + 1] : 0u, nb1 = d < ND - 1 ? Fb[1][d + 1] : 0u;
        const uint32_t ra0 = a0 | (a0 << 1) | (a0 >> 1) | (pa0 >> 31) | (na0 << 31) | from_prev_lane(a1) | a1;
        const uint32_t ra1 = a1 | (a1 << 1) | (a1 >> 1) | (pa1 >> 31) | (na1 << 31) | a0 | from_next_lane(a0);
        const uint32_t rb0 = b0 | (b0 << 1) | (b0 >> 1) | (pb0 >> 31) | (nb0 << 31) | from_prev_lane(b1) | b1;
        const uint32_t rb1 = b1 | (b1 << 1) | (b1 >> 1) | (pb1 >> 31) | (nb1 << 31) | b0 | from_next_lane(b0);
        const uint32_t da0 = ra0 & U[0][d], da1 = ra1 & U[1][d];
        const uint32_t db0 = rb0 & U[0][d], db1 = rb1 & U[1][d];
        met |= ((ra0 & b0) | (ra1 & b1) | (da0 & db0) | (da1 & db1)) != 0u;
        Fa[0][d] = da0;
        Fa[1][d] = da1;
        Fb[0][d] = db0;
        Fb[1][d] = db1;
        U[0][d] &= ~(da0 | db0);
        U[1][d] &= ~(da1 | db1);
        any_a |= (da0 | da1) != 0u;
        any_b |= (db0 | db1) != 0u;
        pa0 = a0;
        pa1 = a1;
        pb0 = b0;
        pb1 = b1;
      }
      vd = ballot(met) ? 1 : (!ballot(any_a) || !ballot(any_b)) ? 0 : -1;
      if (vd >= 0) break;  // the two classes met: connected; a class closed: disconnected
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t f[ND];
      uint32_t c = cnt[p];
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        f[d] = Fa[p][d] | Fb[p][d] | U[p][d];
        c -= (uint32_t)__popc(f[d]);
      }
      uint32_t dg = c * (p == 0 ? fdeg0 : fdeg1);
      if (w0 >= 0 && w0 < WC) dg -= ((ebits >> (2 * p)) & 1u) & (wbit(f, w0) ^ 1u);
      if (w1 >= 0 && w1 < WC) dg -= ((ebits >> (2 * p + 1)) & 1u) & (wbit(f, w1) ^ 1u);
      pc += c;
      pdeg += dg;
    }
    if (vd >= 0) {
      bfs_nodes += wave_sum(pc);
      bfs_deg += wave_sum(pdeg);
      return vd;
    }
    // left the window: hand the race to the list search
    b3_codes(v, a, m, rs.codes, rs.ambig);
    LDS uint32_t* const stage = reinterpret_cast<LDS uint32_t*>(gsum);
    rs.sv0 = lane < scap ? stage[lane] : 0u;
    rs.sv1 = lane + WAVE < scap ? stage[lane + WAVE] : 0u;
    lds_order();
    // level L - 1 cells next to each class's frontier: reached district cells (not in U, not
    // in F) adjacent to it (a level L - 1 cell adjacent to both classes would have merged
    // them); U is turned into those reached cells
    uint32_t c1 = 0, c2 = 0;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        U[p][d] = district(p, d) & ~(U[p][d] | Fa[p][d] | Fb[p][d]);
        c2 += (uint32_t)(__popc(Fa[p][d]) + __popc(Fb[p][d]));
      }
    auto adj = [&](const uint32_t (&X)[2][ND], int p, int d) -> uint32_t {
      const uint32_t x = X[p][d], pv = d > 0 ? X[p][d - 1] : 0u, nx = d < ND - 1 ? X[p][d + 1] : 0u;
      uint32_t h = x | (x << 1) | (x >> 1) | (pv >> 31) | (nx << 31);
      h |= p == 0 ? (from_prev_lane(X[1][d]) | X[1][d]) : (X[0][d] | from_next_lane(X[0][d]));
      return h;
    };
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int d = 0; d < ND; ++d)
        c1 += (uint32_t)(__popc(U[p][d] & adj(Fa, p, d)) + __popc(U[p][d] & adj(Fb, p, d)));
    const uint32_t i1 = scan_incl(c1), i2 = scan_incl(c2);
    const int n1 = (int)rdl(i1, 63), n2 = (int)rdl(i2, 63);
    const uint32_t ca = (rs.codes >> (3 * s2.ra)) & 7u, cb = (rs.codes >> (3 * s2.rb)) & 7u;
    // one class's cells of one dword of one of this lane's rows, from list index idx on
    auto emit = [&](uint32_t bits, int row, int col, uint32_t o, uint32_t code, int& idx,
                    bool staged) {
      while (bits) {
        const int t = __ffs(bits) - 1;
        bits &= bits - 1;
        const int x = row * W + col + t;
        const uint32_t e = (uint32_t)x | (o << 16);
        spill[idx] = e;
        if (staged && idx - n1 < scap) stage[idx - n1] = e;
        P::axor(lab, x, a ^ code);
        ++idx;
      }
    };
    int idx = (int)(i1 - c1);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        emit(U[p][d] & adj(Fa, p, d), re + p, C0 + 32 * d, (uint32_t)s2.ra, ca, idx, false);
        emit(U[p][d] & adj(Fb, p, d), re + p, C0 + 32 * d, (uint32_t)s2.rb, cb, idx, false);
      }
    idx = n1 + (int)(i2 - c2);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        emit(Fa[p][d], re + p, C0 + 32 * d, (uint32_t)s2.ra, ca, idx, true);
        emit(Fb[p][d], re + p, C0 + 32 * d, (uint32_t)s2.rb, cb, idx, true);
      }
    rs.pc = pc;
    rs.pdeg = pdeg;
    rs.n1 = n1;
    rs.n2 = n2;
    rs.ra = s2.ra;
    rs.rb = s2.rb;
    rs.ok = true;
    return -1;
  }

  // The race search of 3-bit-label grids (C5's 200x200 chains) with its visit marks in the
  // labels themselves: the levels, pushes, merges and counters of race_search_gscr and of
  // the oracle's contiguous_after, with LDS round trips where an HBM-marked search pays
  // memory-side atomics (global atomics execute past the XCD's L2).  A claimed node's label
  // a becomes its class's code (b3_codes).  A borrowed code is ambiguous (a cell of that
  // district, or a visited one): when a frontier node of one class meets the code of
  // another, unmerged class (the merge test), the node is looked up among the entries of
  // the current level and of the next level so far.  That is complete: the race is
  // breadth-first, so a visited neighbour of a level-L node lies at level L - 1, L or L + 1,
  // and one of another class at level L - 1 would already have merged the two classes.
  // Within a level the four neighbour directions run one after another, so a node claimed
  // in an earlier direction reads as claimed (LDS ops of one wave execute in program order)
  // and no node is pushed twice: on a grid two frontier nodes reach the same node in one
  // direction only if they are the same node.  A list entry carries its class (node |
  // class << 16).  The next level is staged in LDS over the chain's group sums (not read
  // while the search runs; up to scap entries, the displaced words held in two VGPRs);
  // every entry also goes to the HBM visit list (coalesced 4-byte stores), from which a
  // larger level is read and the labels are restored at the end.  With rs.ok (race_bb4's
  // two-class race left its 128 x 128 window) the race continues from the head of the
  // list race_bb4 wrote instead of from the sources.
  __device__ bool race_search_b3(int v, uint32_t a, int m, int src, uint64_t cls, int scap,
                                 const B3Run& rs, uint64_t& bfs_nodes, uint64_t& bfs_deg) {
    LDS uint32_t* const stage = reinterpret_cast<LDS uint32_t*>(gsum);
    uint32_t codes, ambig;
    if (rs.ok) {
      codes = rs.codes;
      ambig = rs.ambig;
    } else {
      b3_codes(v, a, m, codes, ambig);
    }
    // code -> class + 1 (0: not a class code), 8 entries of 3 bits
    uint32_t cls_of = 0;
    for (int o = 0; o < m; ++o) cls_of |= (uint32_t)(o + 1) << (3 * ((codes >> (3 * o)) & 7u));
    // classes as 4-bit member masks of the sources (uniform), from the pre-merged cls
    uint32_t M = 0;
    for (int i = 0; i < m; ++i) M |= ((uint32_t)rdl64(cls, i) & 15u) << (4 * i);
    auto unite = [&](int i, int j) {
      const uint32_t mm = ((M >> (4 * i)) | (M >> (4 * j))) & 15u;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        if ((mm >> d) & 1u) M = (M & ~(15u << (4 * d))) | (mm << (4 * d));
    };
    auto n_classes = [&]() {
      int nc = 0;
      for (int i = 0; i < m; ++i) nc += (__ffs((M >> (4 * i)) & 15u) - 1) == i;
      return nc;
    };
    uint32_t sv0, sv1;
    if (rs.ok) {
      sv0 = rs.sv0;
      sv1 = rs.sv1;
    } else {
      sv0 = lane < scap ? stage[lane] : 0u;
      sv1 = lane + WAVE < scap ? stage[lane + WAVE] : 0u;
    }
    lds_order();
    int lb = 0, le = m;
    uint32_t my_deg = 0;
    uint64_t nodes = 0;
    // the merge test of an ambiguous code: is y (held by the lanes of `want`) an entry of the
    // current level [lb, le) (in q0 / q1 when the level is staged) or of the next level so
    // far [le, le + nn) (its first scap entries in the stage)?  Rare (a code absent from the
    // sample met far from v), so the lanes are served one at a time.
    auto listed = [&](uint64_t want, int y, int cnt, bool staged, uint32_t q0, uint32_t q1,
                      int nn) -> bool {
      const int ns = nn < scap ? nn : scap;
      const uint32_t s0 = lane < ns ? stage[lane] : 0u;
      const uint32_t s1 = lane + WAVE < ns ? stage[lane + WAVE] : 0u;
      const bool hbm = !staged || nn > scap;
      const int h0 = staged ? le + scap : lb, h1 = le + nn;  // entries read from the HBM list
      if (hbm) __threadfence_block();  // this level's spilled entries are read back
      bool hit = false;
      while (want) {
        const int Lr = __ffsll((unsigned long long)want) - 1;
        want &= want - 1;
        const uint32_t yy = (uint32_t)rdl((int32_t)y, Lr);
        bool f = (lane < ns && (s0 & 0xFFFFu) == yy) || (lane + WAVE < ns && (s1 & 0xFFFFu) == yy);
        if (staged)
          f = f || (lane < cnt && (q0 & 0xFFFFu) == yy) || (lane + WAVE < cnt && (q1 & 0xFFFFu) == yy);
        if (hbm) {
          for (int b = h0; b < h1; b += WAVE) {
            const int i = b + lane;
            uint32_t e = 0u;
            if (i < h1) e = spill[i];
            f = f || (i < h1 && (e & 0xFFFFu) == yy);
          }
        }
        if (ballot(f)) hit = hit || lane == Lr;
      }
      return hit;
    };
    if (rs.ok) {
#ifdef FW_STAMPS
      n_seed += 1;
#endif
      // the bitboards' counters over their processed cells
      my_deg += rs.pdeg;
      nodes += (uint64_t)wave_sum(rs.pc);
      lb = rs.n1;
      le = rs.n1 + rs.n2;
      if (rs.n2 > scap) __threadfence_block();  // the level is read from the HBM list
    } else if (lane < m) {
      const uint32_t e = (uint32_t)src | ((uint32_t)lane << 16);
      P::axor(lab, src, a ^ ((codes >> (3 * lane)) & 7u));
      spill[lane] = e;
      stage[lane] = e;
    }
    lds_order();
    int verdict = -1;
    if (rs.ok) {
      // the seeded race has two classes: one code test per neighbour, a merge ends it
      const uint32_t oa = (uint32_t)rs.ra;
      const uint32_t ca = (codes >> (3 * rs.ra)) & 7u, cb = (codes >> (3 * rs.rb)) & 7u;
      const bool ma = (ambig >> rs.ra) & 1u, mb = (ambig >> rs.rb) & 1u;
      for (;;) {
        const int cnt = le - lb;
        const bool staged = cnt <= scap;
        uint32_t q0 = 0u, q1 = 0u;
        if (staged) {
          if (lane < cnt) q0 = stage[lane];
          if (lane + WAVE < cnt) q1 = stage[lane + WAVE];
        }
        lds_order();
        bool merged = false, pa = false, pb = false;
        int nn = 0;
        for (int cb0 = 0; cb0 < cnt; cb0 += WAVE) {
          const int idx = cb0 + lane;
          const bool act = idx < cnt;
          uint32_t e = 0u;
          if (staged)
            e = cb0 == 0 ? q0 : q1;
          else if (act)
            e = spill[lb + idx];
          const int x = (int)(e & 0xFFFFu);
          const uint32_t o = e >> 16;
          const bool isa = o == oa;
          const uint32_t co = isa ? ca : cb, cother = isa ? cb : ca;
          const bool amb_other = isa ? mb : ma;
          int xr = 0, xc = 0;
          divmod(x, xr, xc);
          if (act) my_deg += (uint32_t)degree(x, xr, xc);
          nodes += (uint64_t)__popcll(ballot(act));
          bool pushed = false, met = false;
          uint32_t chk = 0;
          int ys[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int y = act ? nbr(x, j, xr, xc) : -1;
            ys[j] = y;
            const bool ok = y >= 0 && y != v;
            const uint32_t ly = L(ok ? y : x);
            const bool push = ok && ly == a;
            if (push) P::axor(lab, y, a ^ co);
            const uint64_t pm = ballot(push);
            if (pm) {
              if (push) {
                const int slot = nn + (int)mbcnt(pm);
                const uint32_t ent = (uint32_t)y | (o << 16);
                spill[le + slot] = ent;
                if (slot < scap) stage[slot] = ent;
              }
              nn += __popcll(pm);
            }
            pushed |= push;
            const bool oth = ok && ly == cother;  // the other class, or (ambiguous) a district
            met |= oth && !amb_other;
            if (oth && amb_other) chk |= 1u << j;
          }
          merged |= ballot(met) != 0ull;
          if (!merged && ballot(chk != 0u)) {  // merge tests of ambiguous codes
#ifdef FW_STAMPS
            n_mapt += 1;
#endif
            lds_order();
            bool hit = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint64_t want = ballot((chk >> j) & 1u);
              if (want) hit |= listed(want, ys[j], cnt, staged, q0, q1, nn);
            }
            merged |= ballot(hit) != 0ull;
          }
          pa |= ballot(pushed && isa) != 0ull;
          pb |= ballot(pushed && !isa) != 0ull;
        }
#ifdef FW_STAMPS
        n_lvl += 1;
#endif
        lb = le;
        le += nn;
        if (nn > scap) __threadfence_block();  // the next level is read from the HBM list
        lds_order();
        if (merged) {  // one class: connected
          verdict = 1;
          break;
        }
        if (!pa || !pb) {  // a class pushed nothing: closed, disconnected
          verdict = 0;
          break;
        }
      }
    }
    for (; verdict < 0;) {
      if (n_classes() == 1) {
        verdict = 1;
        break;
      }
      const int cnt = le - lb;
      const bool staged = cnt <= scap;
      uint32_t q0 = 0u, q1 = 0u;
      if (staged) {
        if (lane < cnt) q0 = stage[lane];
        if (lane + WAVE < cnt) q1 = stage[lane + WAVE];
      }
      lds_order();
      uint32_t pushed_src = 0;
      int nn = 0;
      for (int cb = 0; cb < cnt; cb += WAVE) {
        const int idx = cb + lane;
        const bool act = idx < cnt;
        uint32_t e = 0u;
        if (staged)
          e = cb == 0 ? q0 : q1;
        else if (act)
          e = spill[lb + idx];
        const int x = (int)(e & 0xFFFFu);
        const uint32_t o = e >> 16;
        const uint32_t co = (codes >> (3 * o)) & 7u;
        int xr = 0, xc = 0;
        divmod(x, xr, xc);
        if (act) my_deg += (uint32_t)degree(x, xr, xc);
        nodes += (uint64_t)__popcll(ballot(act));
        bool pushed = false;
        uint32_t chk = 0;   // ambiguous merge tests: bit j
        uint32_t chk_o = 0; // their classes, 3 bits per j
        int ys[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int y = act ? nbr(x, j, xr, xc) : -1;
          ys[j] = y;
          const bool ok = y >= 0 && y != v;
          const uint32_t ly = L(ok ? y : x);
          const bool push = ok && ly == a;
          if (push) P::axor(lab, y, a ^ co);
          const uint64_t pm = ballot(push);
          if (pm) {
            if (push) {
              const int slot = nn + (int)mbcnt(pm);
              const uint32_t ent = (uint32_t)y | (o << 16);
              spill[le + slot] = ent;
              if (slot < scap) stage[slot] = ent;
            }
            nn += __popcll(pm);
          }
          pushed |= push;
          // a class code of another class not yet merged with this one: a merge if the
          // node is a visited one (certain for unused-label codes, a list lookup otherwise)
          const uint32_t c1 = ok && !push ? (cls_of >> (3 * ly)) & 7u : 0u;
          const bool other = c1 != 0u && ((M >> (4 * o + (c1 - 1u))) & 1u) == 0u;
          const bool sure = other && !((ambig >> (c1 - 1u)) & 1u);
          if (other && !sure) {
            chk |= 1u << j;
            chk_o |= (c1 - 1u) << (3 * j);
          }
          uint64_t rm = ballot(sure);
          while (rm) {  // merges, serial over requesting lanes
            const int Lr = __ffsll((unsigned long long)rm) - 1;
            rm &= rm - 1;
            unite(rdl((int32_t)o, Lr), rdl((int32_t)(c1 - 1u), Lr));
          }
        }
        if (ballot(chk != 0u)) {  // the merge tests of this chunk, after its claims
#ifdef FW_STAMPS
          n_mapt += 1;
#endif
          lds_order();
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint64_t want = ballot((chk >> j) & 1u);
            if (!want) continue;
            const bool hit = listed(want, ys[j], cnt, staged, q0, q1, nn);
            uint64_t rm = ballot(hit);
            while (rm) {
              const int Lr = __ffsll((unsigned long long)rm) - 1;
              rm &= rm - 1;
              unite(rdl((int32_t)o, Lr), rdl((int32_t)((chk_o >> (3 * j)) & 7u), Lr));
            }
          }
        }
        for (int si = 0; si < m; ++si)
          pushed_src |= ballot(pushed && o == (uint32_t)si) ? (1u << si) : 0u;
      }
#ifdef FW_STAMPS
      n_lvl += 1;
#endif
      lb = le;
      le += nn;
      if (nn > scap) __threadfence_block();  // the next level is read from the HBM list
      lds_order();
      if (n_classes() == 1) {
        verdict = 1;
        break;
      }
      // a class none of whose sources pushed this level is closed: disconnected
      bool closed = false;
      for (int i = 0; i < m; ++i)
        closed |= (__ffs((M >> (4 * i)) & 15u) - 1) == i && ((M >> (4 * i)) & pushed_src & 15u) == 0u;
      if (closed) {
        verdict = 0;
        break;
      }
    }
    bfs_nodes += nodes;
    bfs_deg += wave_sum(my_deg);
#ifdef FW_STAMPS
    const uint64_t t_cl = now();
#endif
    __threadfence_block();  // the visit list is read back
    for (int base = 0; base < le; base += WAVE) {  // restore the labels
      const int idx = base + lane;
      if (idx < le) {
        const uint32_t e = spill[idx];
        const int x = (int)(e & 0xFFFFu);
        const uint32_t o = e >> 16;
        P::axor(lab, x, a ^ ((codes >> (3 * o)) & 7u));
      }
    }
    if (lane < scap) stage[lane] = sv0;
    if (lane + WAVE < scap) stage[lane + WAVE] = sv1;
    lds_order();
#ifdef FW_STAMPS
    c_clear += now() - t_cl;
#endif
    return verdict == 1;
  }

  // Exact verdict on "(district a) minus v is connected and non-empty", by a
  // level-synchronous race search from the m a-labelled neighbours of v (the
  // sources, in CSR order); cls holds, in lanes 0..m-1, the pre-merged class masks.
  // src: lane i < m holds source i's node id.  Wave-cooperative: every lane calls it.
  __device__ bool race_search(int v, uint32_t a, int m, int src, uint64_t cls, uint64_t& bfs_nodes,
                              uint64_t& bfs_deg) {
    const uint32_t BLOCK = P::MASK;
    if (lane == 0) P::axor(lab, v, a ^ BLOCK);
    if (lane < m) {
      P::axor(lab, src, a ^ ((uint32_t)k + (uint32_t)lane));
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
        const uint32_t o = act ? L(x) - (uint32_t)k : 0u;
        int xr = 0, xc = 0;
        int dmax = 0;
        int r16[16];
        if constexpr (E16) {
          if (act) {
            row16(x, r16);
#pragma unroll
            for (int j = 0; j < 16; ++j) dmax += r16[j] >= 0 ? 1 : 0;
            my_deg += (uint32_t)dmax;
          }
        } else if (act) {
          if constexpr (GRID) divmod(x, xr, xc);
          dmax = GRID ? 4 : g.rowptr[x + 1] - g.rowptr[x];
          my_deg += (uint32_t)degree(x, xr, xc);
        }
        bfs_nodes += (uint64_t)__popcll(ballot(act));
        int jmax = 4;
        if constexpr (!GRID) {
          jmax = (int)wave_max32((uint32_t)dmax);
        }
        for (int j = 0; j < (E16 ? 16 : 64); ++j) {  // r16[j]: uniform j (v_movrels)
          if (j >= jmax) break;  // uniform
          int y;
          if constexpr (E16)
            y = (act && j < dmax) ? r16[j] : -1;
          else
            y = (act && j < dmax) ? nbr(x, j, xr, xc) : -1;
          bool push = false, req = false;
          uint32_t other = 0;
          if (y >= 0) {
            const uint32_t ly = L(y);
            if (ly == a) {
              const uint32_t got = P::claim(lab, y, a, (uint32_t)k + o);
              if (got == a) {
                push = true;
              } else if (got >= (uint32_t)k && got < (uint32_t)k + (uint32_t)m) {
                req = true;
                other = got - (uint32_t)k;
              }
            } else if (ly >= (uint32_t)k && ly < (uint32_t)k + (uint32_t)m) {
              req = true;
              other = ly - (uint32_t)k;
            }
          }
          const uint64_t pm = ballot(push);
          if (push) list_put(nl + (int)mbcnt(pm), (uint32_t)y);
          nl += __popcll(pm);
          if (pm) {  // sources whose search pushed this level (m <= 64 ballots, usually 2-4)
            for (int si = 0; si < m; ++si) pushed_src |= ballot(push && o == (uint32_t)si) ? (1ull << si) : 0ull;
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
    for (int base = 0; base < nl; base += WAVE) {  // restore visited nodes and v to a
      const int idx = base + lane;
      if (idx < nl) {
        const int x = (int)list_get(idx);
        P::axor(lab, x, L(x) ^ a);
      }
    }
    if (lane == 0) P::axor(lab, v, BLOCK ^ a);
    lds_order();
    return verdict == 1;
  }

  // Contiguity of the proposal given the neighbourhood gathered for it (PRE: gather_ids
  // fetched v's row of the neighbour adjacency).
  template <bool PRE = false>
  __device__ __forceinline__ bool contiguous(int v, uint32_t a, int m, const Hood& h,
                                             uint64_t am, uint64_t& bfs_runs, uint64_t& bfs_nodes,
                                             uint64_t& bfs_deg) {
    if (m == 0) return false;
    if (m == 1) return true;
    CTX_T0
    uint64_t cls = lane < m ? (1ull << lane) : 0ull;
    B3Run rs;
    rs.ok = false;
    // source index (rank in am) of the source held by lane ln
    auto sx = [&](int ln) { return __popcll(am & ((1ull << ln) - 1ull)); };
    auto merge = [&](int s1, int s2) {
      const uint64_t nm = rdl64(cls, s1) | rdl64(cls, s2);
      if (lane < m && ((nm >> lane) & 1ull)) cls = nm;
    };
    if constexpr (!GRID) {
      // sources joined by a direct edge form one local component (the same links as the
      // oracle's contiguous_after): one component is connected; otherwise pre-merge
      // nbadj has the padded [n][16] layout whenever the padded table exists
      const size_t e0 = (E16 || g.ell) ? (size_t)v * 16 : (size_t)g.rowptr[v];
      const uint64_t adjl = ((am >> lane) & 1ull) ? ((PRE ? nbadj_pre : g.nbadj[e0 + lane - 1]) << 1) & am : 0ull;
      // components of the sources' adjacency, one ballot per closure step: the relation
      // is symmetric, so a source joins when its own row meets the component
      uint64_t rest = am;
      for (bool first = true; rest; first = false) {
        uint64_t comp = rest & (~rest + 1ull);  // the lowest source left
        for (;;) {
          const uint64_t nxt = comp | ballot((adjl & comp) != 0ull);
          if (nxt == comp) break;
          comp = nxt;
        }
        if (first && comp == am) return true;
        rest &= ~comp;
        const int L0 = __ffsll((unsigned long long)comp) - 1;
        for (uint64_t t = comp & (comp - 1ull); t; t &= t - 1ull)
          merge(sx(L0), sx(__ffsll((unsigned long long)t) - 1));
      }
      CTX_LAP(c_win);  // stamps: the local test's cycles of the searches it did not decide
    }
    if constexpr (GRID) {
      const uint64_t rb = ballot(lane >= 1 && lane <= 8 && h.lx == a) >> 1;
      const int pN = rb & 1, pW = (rb >> 1) & 1, pE = (rb >> 2) & 1, pS = (rb >> 3) & 1;
      const int NE = (rb >> 4) & 1, SE = (rb >> 5) & 1, SW = (rb >> 6) & 1, NW = (rb >> 7) & 1;
      const int lNE = pN & pE & NE, lES = pE & pS & SE, lSW = pS & pW & SW, lWN = pW & pN & NW;
      if (m - (lNE + lES + lSW + lWN) <= 1) return true;
      {  // 7x7 window: lanes 0..47 read one cell each
        int vr, vc;
        divmod(v, vr, vc);
        const int pos = window_pos(lane < 48 ? lane : 0);
        const int rr = vr - 3 + pos / 7, cc = vc - 3 + pos % 7;
        const bool in = lane < 48 && rr >= 0 && rr < g.gh && cc >= 0 && cc < g.gw &&
                        L(rr * g.gw + cc) == a;
        const uint64_t b48 = ballot(in) & ((1ull << 48) - 1ull);
        const uint64_t A = (b48 & ((1ull << 24) - 1ull)) | ((b48 >> 24) << 25);
        const int wv = window_verdict_lanes(A, lane);
#ifdef FW_STAMPS
        n_win += 1;
#endif
        CTX_LAP(c_win);
        if (wv >= 0) return wv == 1;
      }
      if (bb) {  // bitboard search first; the list search past its window
        int vr, vc;
        divmod(v, vr, vc);
        // 3-bit labels (large grids, C5): the 64-column window, whose two-class race hands
        // its state to the list search when it leaves the window
        const uint32_t am4 = (uint32_t)(am >> 1) & 15u;
        const uint32_t lk = (uint32_t)(lNE | (lES << 1) | (lSW << 2) | (lWN << 3));
        int wv;
        if constexpr (LB == 3) {
          BBSeed s2;
          uint32_t lv_mid = 0, lv_64 = 0;
          wv = grid_race_bb2<LB>(lab, g.n, g.gw, g.gh, lane, vr, vc, a, am4, lk, bfs_nodes,
                                 bfs_deg, s2, lv_mid, lv_64);
#ifdef FW_STAMPS
          n_lv_mid += lv_mid;
          n_lv_64 += lv_64;
#endif
          CTX_LAP(c_bbs);
          if (s2.ok) {  // the classes' source indices (CSR order of v's neighbours)
            s2.ra = sx(s2.ra + 1);
            s2.rb = sx(s2.rb + 1);
            wv = race_bb4<4>(v, vr, vc, a, m, s2, bfs_nodes, bfs_deg, rs);
#ifdef FW_STAMPS
            n_bb4 += 1;
#endif
            CTX_LAP(c_bb4);
          }
        } else {
          wv = grid_race_bb<LB>(lab, g.n, g.gw, g.gh, lane, vr, vc, a, am4, lk, bfs_nodes,
                                bfs_deg);
        }
#ifdef FW_STAMPS
        n_bbs += 1;
#endif
        CTX_LAP(c_bbs);
        if (wv >= 0) {
          bfs_runs += 1;
          return wv == 1;
        }
      }
      // pre-merge the ring links
      if (lNE) merge(sx(1), sx(3));
      if (lES) merge(sx(3), sx(4));
      if (lSW) merge(sx(4), sx(2));
      if (lWN) merge(sx(2), sx(1));
    }
    bfs_runs += 1;
#ifdef FW_STAMPS
    n_list += 1;
#endif
    // sources (a-labelled neighbours, CSR order) compacted into lanes 0..m-1
    int src = -1;
    uint64_t mm = am;
    for (int i = 0; i < m; ++i) {
      const int Ls = __ffsll((unsigned long long)mm) - 1;
      mm &= mm - 1;
      const int val = rdl(h.x, Ls);
      if (lane == i) src = val;
    }
    bool verdict;
    if constexpr (LB == 3 && GRID)
      verdict = race_search_b3(v, a, m, src, cls, scap, rs, bfs_nodes, bfs_deg);
    else if constexpr (LB == 5)
      verdict = race_search_gscr(v, a, m, src, cls, bfs_nodes, bfs_deg);
    else
      verdict = race_search(v, a, m, src, cls, bfs_nodes, bfs_deg);
    CTX_LAP(c_list);
    return verdict;
  }
};

}  // namespace
