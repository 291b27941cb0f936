// fw_kernels.hip — gfx950 kernels of the batched single-node flip walk.
//
// One 64-lane wavefront owns one chain at a time; a persistent grid of single-wave
// workgroups pulls chains from an atomic counter.  The chain's state lives in LDS
// for the whole launch:
//   lab   packed LB-bit district labels (LB = 4: 0.5 B/node; LB = 8: 1 B/node).  The
//         contiguity search marks visited nodes in place with codes k..k+deg-1.
//   gsum  u32 proposal-weight sum per 64-node group (rank/select level 1)
//   list  the contiguity search's visit list (spills to HBM past qcap entries)
// Per-node proposal weights (#distinct foreign labels, or cut degree) are recomputed
// from labels where needed instead of being stored, which halves LDS per chain and
// doubles the chains resident per CU.  District populations and the Metropolis table
// are held one entry per lane.  HBM holds only the packed labels, a 144-byte stats
// record and k populations per chain, read and written once per launch.
//
// Per counted step (MarkovChain.__next__ [ext]; grid_chain_sec11.py:340-342,366):
//   Philox draw (scalar unit) -> rank r -> level 1: DPP scan of the group sums ->
//   level 2: weights of the 64 nodes of the group recomputed + DPP scan -> v, j ->
//   one LDS round trip for v's neighbourhood (grid: v, its 4 neighbours with their
//   own neighbours, 4 diagonals; CSR: v and its neighbours' rows) -> target, Δcut,
//   population bound, ring test / exact race search -> retry if invalid ->
//   Metropolis on the pre-tabulated base**(-Δcut) -> commit -> per-yield observables.
// The semantics are stated once, in oracle/flipchain_oracle.c; this file must match it
// bit for bit (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include "fw_internal.h"

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

// ---------------------------------------------------------------- packed labels
template <int LB>
struct PK {
  static constexpr uint32_t MASK = (1u << LB) - 1u;
  __device__ static __forceinline__ uint32_t get(const uint8_t* b, int x) {
    if constexpr (LB == 8) {
      return b[x];
    } else {
      return (uint32_t)(b[x >> 1] >> ((x & 1) << 2)) & 15u;
    }
  }
  __device__ static __forceinline__ uint32_t* word(uint8_t* b, int x) {
    return reinterpret_cast<uint32_t*>(b) + ((x * LB) >> 5);
  }
  __device__ static __forceinline__ int shift(int x) { return (x * LB) & 31; }
  // field ^= d, safe against concurrent updates of other fields of the word
  __device__ static __forceinline__ void axor(uint8_t* b, int x, uint32_t d) {
    atomicXor(word(b, x), d << shift(x));
  }
  // claim field x: a -> code, if it still holds a; returns the value found (a on success)
  __device__ static __forceinline__ uint32_t claim(uint8_t* b, int x, uint32_t a, uint32_t code) {
    uint32_t* w = word(b, x);
    const int sh = shift(x);
    uint32_t old = *reinterpret_cast<volatile uint32_t*>(w);
    for (;;) {
      uint32_t cur = (old >> sh) & MASK;
      if (cur != a) return cur;
      uint32_t nw = old ^ ((a ^ code) << sh);
      uint32_t prev = atomicCAS(w, old, nw);
      if (prev == old) return a;
      old = prev;
    }
  }
};

constexpr uint32_t NOLAB = 0xFFFFu;  // label of an absent cell (never a district or code)

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
struct Hood {
  int x;          // node id, -1 if absent
  uint32_t lx;    // label of x (NOLAB if absent)
  uint64_t bits;  // OR of 1<<label over x's neighbours other than v
  uint32_t cnt;   // number of x's neighbours other than v with label != lx
  bool has_v;     // v is a neighbour of x
  int deg;        // degree of x
};

template <int LB, bool GRID>
struct Ctx {
  using P = PK<LB>;
  FwGraphDev g;
  uint8_t* lab;
  uint32_t* gsum;
  uint32_t* list;   // LDS part of the search list
  uint32_t* spill;  // HBM part (this workgroup's slice)
  int32_t qcap, k;
  int lane;
  int my_dr, my_dc;

  __device__ void init_roles() {
    lane = lane_id();
    role_off(lane <= 8 ? lane : 0, my_dr, my_dc);
  }
  __device__ __forceinline__ void divmod(int x, int& r, int& c) const {
    r = (int)(((uint64_t)(uint32_t)x * g.gmagic) >> 42);
    c = x - r * g.gw;
  }
  __device__ __forceinline__ uint32_t L(int x) const { return P::get(lab, x); }
  __device__ __forceinline__ uint32_t list_get(int i) const {
    return i < qcap ? list[i] : spill[i - qcap];
  }
  __device__ __forceinline__ void list_put(int i, uint32_t x) {
    if (i < qcap)
      list[i] = x;
    else
      spill[i - qcap] = x;
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
  __device__ __forceinline__ int degree(int x, int xr, int xc) const {
    if constexpr (GRID) {
      return (xr > 0) + (xc > 0) + (xc < g.gw - 1) + (xr < g.gh - 1);
    } else {
      return g.rowptr[x + 1] - g.rowptr[x];
    }
  }

  // Proposal weight and cut degree of x under the current labels.
  template <int MODE>
  __device__ __forceinline__ void weight_now(int x, uint32_t& w, uint32_t& cd) const {
    int xr = 0, xc = 0;
    if constexpr (GRID) divmod(x, xr, xc);
    const uint32_t lx = L(x);
    const int dx = GRID ? 4 : g.rowptr[x + 1] - g.rowptr[x];
    uint64_t bits = 0;
    cd = 0;
    for (int j = 0; j < dx; ++j) {
      const int y = nbr(x, j, xr, xc);
      if (y < 0) continue;
      const uint32_t ly = L(y);
      bits |= 1ull << ly;
      cd += ly != lx;
    }
    w = (MODE == FW_PROPOSE_CUTEDGE) ? cd : (uint32_t)__popcll(bits & ~(1ull << lx));
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
        wo = (uint32_t)__popcll(h.bits & ~(1ull << a));
        wn = (uint32_t)__popcll(h.bits & ~(1ull << d));
      }
      return;
    }
    if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
      wo = h.cnt + (h.has_v && a != h.lx);
      wn = h.cnt + (h.has_v && d != h.lx);
    } else {
      const uint64_t keep = ~(1ull << h.lx);
      wo = (uint32_t)__popcll((h.bits | (h.has_v ? 1ull << a : 0ull)) & keep);
      wn = (uint32_t)__popcll((h.bits | (h.has_v ? 1ull << d : 0ull)) & keep);
    }
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
      if (!ok) return h;
      h.x = xr * g.gw + xc;
      h.lx = L(h.x);
      if (lane <= 4) {
        h.deg = degree(h.x, xr, xc);
        const int vslot = 4 - lane;  // up's down, left's right, right's left, down's up
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int y = nbr(h.x, j, xr, xc);
          if (y < 0) continue;
          if (lane > 0 && j == vslot) {
            h.has_v = true;
            continue;
          }
          const uint32_t ly = L(y);
          h.bits |= 1ull << ly;
          h.cnt += ly != h.lx;
        }
      }
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
        h.bits |= 1ull << ly;
        h.cnt += ly != h.lx;
      }
    }
    return h;
  }

  // -------------------------------------------------------------- select
  // rank r in [0, P) -> node v and in-node index j (canonical (node, ·) order).
  // PER = group sums held per lane (compile-time bound, >= ceil(G/64)).
  template <int MODE, int PER>
  __device__ __forceinline__ void select(uint32_t r, int G, int& v, uint32_t& j) const {
    uint32_t gs[PER];
    uint32_t s = 0;
    const int g0 = lane * PER;
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      gs[t] = (g0 + t < G) ? gsum[g0 + t] : 0u;
      s += gs[t];
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
    if (x < g.n) weight_now<MODE>(x, wx, cd);
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
  // Exact verdict on "(district a) minus v is connected and non-empty", by a
  // level-synchronous race search from the m a-labelled neighbours of v (the
  // sources, in CSR order); cls holds, in lanes 0..m-1, the pre-merged class masks.
  __device__ bool race_search(int v, uint32_t a, int m, int src_node, bool is_src, uint32_t src_idx,
                              uint64_t cls, uint64_t& bfs_nodes, uint64_t& bfs_deg) {
    const uint32_t BLOCK = P::MASK;
    if (lane == 0) P::axor(lab, v, a ^ BLOCK);
    if (is_src) P::axor(lab, src_node, a ^ ((uint32_t)k + src_idx));
    const uint64_t sm = ballot(is_src);
    if (is_src) list_put((int)mbcnt(sm), (uint32_t)src_node);
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
        if (act) {
          if constexpr (GRID) divmod(x, xr, xc);
          dmax = GRID ? 4 : g.rowptr[x + 1] - g.rowptr[x];
          my_deg += (uint32_t)degree(x, xr, xc);
        }
        bfs_nodes += (uint64_t)__popcll(ballot(act));
        int jmax = 4;
        if constexpr (!GRID) {
          uint32_t dm = (uint32_t)dmax;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) dm = max(dm, (uint32_t)__shfl_xor(dm, d, WAVE));
          jmax = (int)rfl(dm);
        }
        for (int j = 0; j < jmax; ++j) {
          const int y = (act && j < dmax) ? nbr(x, j, xr, xc) : -1;
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

  // Contiguity of the proposal given the neighbourhood gathered for it.
  __device__ __forceinline__ bool contiguous(int v, uint32_t a, int m, const Hood& h,
                                             uint64_t am, uint64_t& bfs_runs, uint64_t& bfs_nodes,
                                             uint64_t& bfs_deg) {
    if (m == 0) return false;
    if (m == 1) return true;
    uint64_t cls = lane < m ? (1ull << lane) : 0ull;
    // sources: lanes whose node is an a-labelled neighbour; index = rank among them
    const bool is_src = ((am >> lane) & 1ull) != 0ull;
    const uint32_t sidx = mbcnt(am);
    if constexpr (GRID) {
      const uint64_t rb = ballot(lane >= 1 && lane <= 8 && h.lx == a) >> 1;
      const int pN = rb & 1, pW = (rb >> 1) & 1, pE = (rb >> 2) & 1, pS = (rb >> 3) & 1;
      const int NE = (rb >> 4) & 1, SE = (rb >> 5) & 1, SW = (rb >> 6) & 1, NW = (rb >> 7) & 1;
      const int lNE = pN & pE & NE, lES = pE & pS & SE, lSW = pS & pW & SW, lWN = pW & pN & NW;
      if (m - (lNE + lES + lSW + lWN) <= 1) return true;
      // pre-merge the ring links; source index of lane l = rank of l among am's bits
      auto sx = [&](int ln) { return __popcll(am & ((1ull << ln) - 1ull)); };
      auto merge = [&](int s1, int s2) {
        const uint64_t nm = rdl64(cls, s1) | rdl64(cls, s2);
        if (lane < m && ((nm >> lane) & 1ull)) cls = nm;
      };
      if (lNE) merge(sx(1), sx(3));
      if (lES) merge(sx(3), sx(4));
      if (lSW) merge(sx(4), sx(2));
      if (lWN) merge(sx(2), sx(1));
    }
    bfs_runs += 1;
    return race_search(v, a, m, h.x, is_src, sidx, cls, bfs_nodes, bfs_deg);
  }
};

// ---------------------------------------------------------------- the chain kernel
template <int LB, bool GRID, int MODE, int PER>
__global__ __launch_bounds__(64) void fw_run_kernel(FwRunParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID> C;
  C.g = p.g;
  C.lab = smem;
  C.gsum = reinterpret_cast<uint32_t*>(smem + p.off_gsum);
  C.list = reinterpret_cast<uint32_t*>(smem + p.off_list);
  C.spill = p.spill + (size_t)blockIdx.x * (size_t)p.g.n;
  C.qcap = p.qcap;
  C.k = p.k;
  C.init_roles();
  const int lane = C.lane;
  const int n = p.g.n;
  const int D = p.g.maxdeg;
  const int G = p.G;
  const int k = p.k;
  const uint32_t key0 = (uint32_t)p.seed, key1 = (uint32_t)(p.seed >> 32);
  __shared__ int32_t s_chain;

  for (;;) {
    if (lane == 0) s_chain = atomicAdd(p.next_chain, 1);
    __syncthreads();
    const int c = rfl(s_chain);
    if (c >= p.n_chains) break;
    const uint64_t gid = (uint64_t)(p.chain_id0 + c);

    // ---- load state
    {
      const uint4* src = reinterpret_cast<const uint4*>(p.labels + (size_t)c * p.lab_stride);
      uint4* dst = reinterpret_cast<uint4*>(C.lab);
      for (int i = lane; i < p.lab_bytes / 16; i += WAVE) dst[i] = src[i];
    }
    int64_t pops = lane < k ? p.pops[(size_t)c * k + lane] : 0;  // lane d holds district d
    const double thr_l = lane < 2 * D + 1 ? p.thr[(size_t)c * p.thr_stride + lane] : 0.0;
    fw_chain_stats* stp = p.stats + c;
    uint64_t attempts = rfl64(stp->attempts);
    const uint64_t yields0 = rfl64(stp->yields);
    int32_t stuck = rfl(stp->stuck);
    int64_t sum_cut = (int64_t)rfl64((uint64_t)stp->sum_cut);
    int64_t sum_bnodes = (int64_t)rfl64((uint64_t)stp->sum_bnodes);
    double sum_invb = stp->sum_invb;  // running total: keeps the oracle's summation order
    // per-launch counters (added to the 64-bit totals at the end)
    uint32_t n_steps = 0, n_acc = 0, n_popf = 0, n_conf = 0;
    uint32_t n_sdeg = 0, n_adeg = 0, n_bchg = 0, n_yield = 0;
    uint64_t n_bfs = 0, n_bfsn = 0, n_bfsd = 0;
    __syncthreads();

    // ---- derive group sums, cut count, boundary count, proposal-set size
    int32_t cut, bnodes, npairs;
    {
      uint32_t cut2 = 0, bn = 0, np = 0;
      for (int t = 0; t < G; ++t) {
        const int x = t * 64 + lane;
        uint32_t w = 0, cd = 0;
        if (x < n) C.template weight_now<MODE>(x, w, cd);
        const uint32_t gsum_t = wave_sum(w);
        if (lane == 0) C.gsum[t] = gsum_t;
        cut2 += cd;
        bn += cd > 0;
        np += w;
      }
      cut = (int32_t)(wave_sum(cut2) / 2);
      bnodes = (int32_t)wave_sum(bn);
      npairs = (int32_t)wave_sum(np);
    }
    lds_order();
    double invb = 1.0 / (double)bnodes;

    // histogram windows: lane i counts value base+i
    uint32_t hc = 0, hb = 0;
    int32_t base_c = max(0, cut - 32), base_b = max(0, bnodes - 32);
    auto observe = [&]() {
      n_yield += 1;
      sum_cut += cut;
      sum_bnodes += bnodes;
      sum_invb += invb;
      int ic = cut - base_c;
      if (ic < 0 || ic >= WAVE) {
        if (hc) atomicAdd(p.hist_cut + base_c + lane, (unsigned long long)hc);
        hc = 0;
        base_c = max(0, cut - 32);
        ic = cut - base_c;
      }
      hc += (lane == ic);
      int ib = bnodes - base_b;
      if (ib < 0 || ib >= WAVE) {
        if (hb) atomicAdd(p.hist_b + base_b + lane, (unsigned long long)hb);
        hb = 0;
        base_b = max(0, bnodes - 32);
        ib = bnodes - base_b;
      }
      hb += (lane == ib);
    };
    if (yields0 == 0 && attempts == 0) observe();

    const bool unit_pop = p.g.pop == nullptr;
    for (int64_t s = 0; s < p.steps && !stuck; ++s) {
      int32_t retries = 0;
      int v = 0, dcut = 0, m = 0, nbd = 0, dv = 0;
      uint32_t a = 0, d = 0;
      int64_t pv = 1;
      U4 x;
      Hood h;
      bool valid = false;
      for (;;) {
        if (retries >= p.max_retries || npairs == 0) {
          stuck = 1;
          break;
        }
        x = philox((uint32_t)attempts, (uint32_t)(attempts >> 32), (uint32_t)gid,
                   (uint32_t)(gid >> 32), key0, key1);
        attempts += 1;
        const uint32_t r = scale64(x.x0, x.x1, (uint32_t)npairs);
        uint32_t j = 0;
        C.template select<MODE, PER>(r, G, v, j);
        v = rfl(v);
        if (v < 0) {  // internal inconsistency: stop this chain, flag it
          stuck = 2;
          break;
        }
        j = rfl(j);
        // ---- v's neighbourhood (one LDS round trip)
        h = C.gather(v, dv);
        dv = rfl(dv);
        a = rfl(rdl(h.lx, 0));
        n_sdeg += (uint32_t)dv;
        const bool isnb = GRID ? (lane >= 1 && lane <= 4 && h.x >= 0) : (lane >= 1 && lane <= dv);
        if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
          const uint64_t cm = ballot(isnb && h.lx != a);
          d = rfl(rdl(h.lx, nth_bit(cm, j)));
        } else {
          uint64_t mask = 0;
          if constexpr (GRID) {
#pragma unroll
            for (int l = 1; l <= 4; ++l) {
              const uint32_t ll = rdl(h.lx, l);
              mask |= (ll != a && ll != NOLAB) ? (1ull << ll) : 0ull;
            }
          } else {
            mask = rfl64(wave_or64((isnb && h.lx != a) ? (1ull << h.lx) : 0ull));
          }
          d = (uint32_t)nth_bit(mask, j);
        }
        const uint64_t am = ballot(isnb && h.lx == a);
        m = __popcll(am);
        nbd = __popcll(ballot(isnb && h.lx == d));
        dcut = m - nbd;
        // ---- population bound (Bounds over the two changed districts)
        pv = unit_pop ? 1 : p.g.pop[v];
        const int64_t pa = (int64_t)rdl64((uint64_t)pops, (int)a);
        const int64_t pb = (int64_t)rdl64((uint64_t)pops, (int)d);
        if (pa - pv < p.pop_lo || pb + pv > p.pop_hi) {
          n_popf += 1;
          ++retries;
          continue;
        }
        // ---- contiguity (single_flip_contiguous)
        if (!C.contiguous(v, a, m, h, am, n_bfs, n_bfsn, n_bfsd)) {
          n_conf += 1;
          ++retries;
          continue;
        }
        valid = true;
        break;
      }
      if (!valid) break;
      n_steps += 1;
      // ---- Metropolis (cut_accept, grid_chain_sec11.py:171-179)
      const bool accepted = u53(x.x2, x.x3) < rdl_f64(thr_l, dcut + D);
      if (p.trace && lane == 0) p.trace[(size_t)c * p.steps + s] = accepted ? v * 64 + (int)d : -1;
      if (accepted) {
        n_acc += 1;
        n_adeg += (uint32_t)dv;
        uint32_t wo, wn;
        C.template weights_old_new<MODE>(h, a, d, m, nbd, wo, wn);
        const bool mine = GRID ? lane <= 4 : lane <= dv;
        if (lane == 0) PK<LB>::axor(C.lab, v, a ^ d);
        if (mine && h.x >= 0 && wn != wo) atomicAdd(C.gsum + (h.x >> 6), wn - wo);
        lds_order();
        const int plus = __popcll(ballot(mine && wo == 0 && wn > 0));
        const int minus = __popcll(ballot(mine && wo > 0 && wn == 0));
        npairs += (int32_t)wave_sum(mine ? wn - wo : 0u);
        cut += dcut;
        bnodes += plus - minus;
        n_bchg += (uint32_t)(plus + minus);
        if (plus | minus) invb = 1.0 / (double)bnodes;
        if (lane == (int)a) pops -= pv;
        if (lane == (int)d) pops += pv;
      }
      observe();
    }

    // ---- write back
    if (hc) atomicAdd(p.hist_cut + base_c + lane, (unsigned long long)hc);
    if (hb) atomicAdd(p.hist_b + base_b + lane, (unsigned long long)hb);
    {
      uint4* dst = reinterpret_cast<uint4*>(p.labels + (size_t)c * p.lab_stride);
      const uint4* src = reinterpret_cast<const uint4*>(C.lab);
      for (int i = lane; i < p.lab_bytes / 16; i += WAVE) dst[i] = src[i];
      if (lane < k) p.pops[(size_t)c * k + lane] = pops;
    }
    if (lane == 0) {
      stp->attempts = attempts;
      stp->steps += n_steps;
      stp->accepts += n_acc;
      stp->pop_fail += n_popf;
      stp->contig_fail += n_conf;
      stp->bfs_runs += n_bfs;
      stp->bfs_nodes += n_bfsn;
      stp->bfs_deg += n_bfsd;
      stp->sum_deg += n_sdeg;
      stp->acc_deg += n_adeg;
      stp->n_bchg += n_bchg;
      stp->yields += n_yield;
      stp->sum_cut = sum_cut;
      stp->sum_bnodes = sum_bnodes;
      stp->sum_invb = sum_invb;
      stp->cut = cut;
      stp->bnodes = bnodes;
      stp->npairs = npairs;
      stp->stuck = stuck;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- per-flip evaluation
template <int LB, bool GRID>
__global__ __launch_bounds__(64) void fw_eval_kernel(FwEvalParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID> C;
  C.g = p.g;
  C.lab = smem;
  C.gsum = nullptr;
  C.list = reinterpret_cast<uint32_t*>(smem + p.off_list);
  C.spill = p.spill + (size_t)blockIdx.x * (size_t)p.g.n;
  C.qcap = p.qcap;
  C.k = p.k;
  C.init_roles();
  const int lane = C.lane;
  for (int i = blockIdx.x; i < p.m; i += gridDim.x) {
    {
      const uint4* src = reinterpret_cast<const uint4*>(p.labels);
      uint4* dst = reinterpret_cast<uint4*>(C.lab);
      for (int t = lane; t < p.lab_bytes / 16; t += WAVE) dst[t] = src[t];
    }
    __syncthreads();
    const int v = p.v[i];
    const uint32_t b = (uint32_t)p.target[i];
    int dv = 0;
    const Hood h = C.gather(v, dv);
    const uint32_t a = rfl(rdl(h.lx, 0));
    const bool isnb = GRID ? (lane >= 1 && lane <= 4 && h.x >= 0) : (lane >= 1 && lane <= dv);
    const uint64_t am = ballot(isnb && h.lx == a);
    const int m = __popcll(am);
    const int nb = __popcll(ballot(isnb && h.lx == b));
    const int64_t pv = p.g.pop ? p.g.pop[v] : 1;
    const bool pok = !(p.pops[a] - pv < p.pop_lo || p.pops[b] + pv > p.pop_hi);
    uint64_t d0 = 0, d1 = 0, d2 = 0;
    const bool ok = C.contiguous(v, a, m, h, am, d0, d1, d2);
    // boundary membership (cut degree > 0) of v and its neighbours before/after
    uint32_t wo, wn;
    C.template weights_old_new<FW_PROPOSE_CUTEDGE>(h, a, b, m, nb, wo, wn);
    const bool mine = GRID ? lane <= 4 : lane <= dv;
    const int db = __popcll(ballot(mine && wn > 0)) - __popcll(ballot(mine && wo > 0));
    if (lane == 0) {
      p.dcut[i] = m - nb;
      p.contig[i] = ok ? 1 : 0;
      p.pop_ok[i] = pok ? 1 : 0;
      p.dboundary[i] = db;
    }
    __syncthreads();
  }
}

template <int LB, bool GRID, int MODE>
void* pick_per(int G) {
  if (G <= 64 * 2) return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 2>);
  if (G <= 64 * 4) return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 4>);
  if (G <= 64 * 8) return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 8>);
  return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 16>);
}

void* pick_run(int lb, bool grid, int mode, int G) {
  const bool cut = mode == FW_PROPOSE_CUTEDGE;
  if (lb == 4) {
    if (grid) return cut ? pick_per<4, true, 2>(G) : pick_per<4, true, 1>(G);
    return cut ? pick_per<4, false, 2>(G) : pick_per<4, false, 1>(G);
  }
  if (grid) return cut ? pick_per<8, true, 2>(G) : pick_per<8, true, 1>(G);
  return cut ? pick_per<8, false, 2>(G) : pick_per<8, false, 1>(G);
}

}  // namespace

int fw_run_grid_size(const FwRunParams& p, int lb, int device, int* grid) {
  if (p.G > 64 * 16) return -2;
  void* fn = pick_run(lb, p.g.gw > 0, p.mode, p.G);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  if (e != hipSuccess) return -1;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, (size_t)p.lds_bytes);
  if (e != hipSuccess || per_cu <= 0) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  long long gsz = (long long)per_cu * prop.multiProcessorCount;
  if (gsz > p.n_chains) gsz = p.n_chains;
  *grid = (int)(gsz < 1 ? 1 : gsz);
  return 0;
}

int fw_launch_run(const FwRunParams& p, int lb, int grid, void* stream) {
  void* fn = pick_run(lb, p.g.gw > 0, p.mode, p.G);
  void* args[] = {const_cast<FwRunParams*>(&p)};
  hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(64), args, (size_t)p.lds_bytes,
                                 (hipStream_t)stream);
  return e == hipSuccess ? 0 : -1;
}

int fw_launch_eval(const FwEvalParams& p, int lb, int grid, void* stream) {
  void* fn;
  if (lb == 4)
    fn = p.g.gw > 0 ? reinterpret_cast<void*>(&fw_eval_kernel<4, true>)
                    : reinterpret_cast<void*>(&fw_eval_kernel<4, false>);
  else
    fn = p.g.gw > 0 ? reinterpret_cast<void*>(&fw_eval_kernel<8, true>)
                    : reinterpret_cast<void*>(&fw_eval_kernel<8, false>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes) !=
      hipSuccess)
    return -1;
  void* args[] = {const_cast<FwEvalParams*>(&p)};
  hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(64), args, (size_t)p.lds_bytes,
                                 (hipStream_t)stream);
  return e == hipSuccess ? 0 : -1;
}
