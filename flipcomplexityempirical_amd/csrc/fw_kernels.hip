// fw_kernels.hip — gfx950 kernels of the batched single-node flip walk.
//
// One 64-lane wavefront owns one chain at a time.  The chain's whole state lives
// in LDS for the duration of a launch:
//   lab   packed LB-bit district labels           (LB = 4: 0.5 B/node, LB = 8: 1 B/node)
//   wgt   packed LB-bit proposal weight per node  (#distinct foreign labels, or cut degree)
//   gsum  u32 weight sum per 64-node group        (two-level rank/select)
//   pops  int64 district populations
//   list  the contiguity search's visit list (spills to HBM past qcap entries)
// HBM holds only the packed labels, a 144-byte stats record and k populations per
// chain, read once and written once per launch.  The CSR (general graphs) is shared
// by every chain and stays L2-resident; row-major grids use implicit neighbours.
//
// Per counted step (MarkovChain.__next__ [ext]; grid_chain_sec11.py:340-342,366):
//   Philox draw -> rank/select over the proposal set (two wave scans) -> neighbour
//   gather -> population bound -> contiguity (grid: 8-cell ring test; otherwise or
//   when inconclusive: exact level-synchronous race search from v's old-district
//   neighbours) -> retry if invalid -> Metropolis on the pre-tabulated base**(-Δcut)
//   -> commit (labels, weights, group sums, pops, counters) -> per-yield observables.
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

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    uint32_t y = __shfl_up(x, d, WAVE);
    if (l >= d) x += y;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, WAVE);
  return x;
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

// LDS-visibility point for the single-wave workgroup (also a compiler barrier).
__device__ __forceinline__ void wave_sync() { __syncthreads(); }

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

// ---------------------------------------------------------------- packed fields
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

__device__ __forceinline__ uint32_t nibble_sum(uint32_t v) {
  uint32_t s = (v & 0x0F0F0F0Fu) + ((v >> 4) & 0x0F0F0F0Fu);
  return (s * 0x01010101u) >> 24;
}
__device__ __forceinline__ uint32_t byte_sum(uint32_t v) {
  uint32_t s = (v & 0x00FF00FFu) + ((v >> 8) & 0x00FF00FFu);
  return (s & 0xFFFFu) + (s >> 16);
}

// ---------------------------------------------------------------- chain context
// Lane roles for the grid path (lane < 8): ring cell of v, in the order
//   0 up, 1 left, 2 right, 3 down   (= CSR order: ascending node id)
//   4 NE, 5 SE, 6 SW, 7 NW          (diagonals between N-E, E-S, S-W, W-N)
__device__ __forceinline__ void ring_dir(int l, int& dr, int& dc) {
  dr = 0;
  dc = 0;
  switch (l) {
    case 0: dr = -1; break;
    case 1: dc = -1; break;
    case 2: dc = 1; break;
    case 3: dr = 1; break;
    case 4: dr = -1; dc = 1; break;
    case 5: dr = 1; dc = 1; break;
    case 6: dr = 1; dc = -1; break;
    case 7: dr = -1; dc = -1; break;
    default: break;
  }
}

template <int LB, bool GRID>
struct Ctx {
  using P = PK<LB>;
  FwGraphDev g;
  uint8_t* lab;
  uint8_t* wgt;
  uint32_t* gsum;
  int64_t* pops;
  uint32_t* list;   // LDS part of the search list
  uint32_t* spill;  // HBM part (this workgroup's slice)
  int32_t qcap, k;
  int lane;
  int my_dr, my_dc;  // ring direction of this lane (grid)
  int cm_dr, cm_dc;  // commit role: lane 0 = v, lanes 1..4 = up/left/right/down

  __device__ void init_roles() {
    lane = lane_id();
    ring_dir(lane < 8 ? lane : 8, my_dr, my_dc);
    ring_dir(lane >= 1 && lane <= 4 ? lane - 1 : 8, cm_dr, cm_dc);
  }

  __device__ __forceinline__ void divmod(int x, int& r, int& c) const {
    r = x / g.gw;
    c = x - r * g.gw;
  }
  __device__ __forceinline__ int deg(int x) const {
    if constexpr (GRID) {
      int r, c;
      divmod(x, r, c);
      return (r > 0) + (c > 0) + (c < g.gw - 1) + (r < g.gh - 1);
    } else {
      return g.rowptr[x + 1] - g.rowptr[x];
    }
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

  // proposal weight and cut degree of node x under the current labels
  template <int MODE>
  __device__ __forceinline__ void node_weight(int x, uint32_t& w, uint32_t& cd) const {
    const uint32_t lx = L(x);
    uint64_t bits = 0;
    cd = 0;
    int xr = 0, xc = 0;
    int dmax;
    if constexpr (GRID) {
      divmod(x, xr, xc);
      dmax = 4;
    } else {
      dmax = g.rowptr[x + 1] - g.rowptr[x];
    }
    for (int j = 0; j < dmax; ++j) {
      int y = nbr(x, j, xr, xc);
      if (y < 0) continue;
      uint32_t ly = L(y);
      if (ly != lx) {
        ++cd;
        bits |= 1ull << ly;
      }
    }
    w = (MODE == FW_PROPOSE_CUTEDGE) ? cd : (uint32_t)__popcll(bits);
  }

  // -------------------------------------------------------------- derive
  // Rebuild weights, group sums and the cut / boundary / pair counts from labels.
  template <int MODE>
  __device__ void derive(int32_t& cut, int32_t& bnodes, int32_t& npairs, int G) {
    const int wbytes = G * 64 * LB / 8;
    for (int i = lane * 4; i < wbytes; i += WAVE * 4) *reinterpret_cast<uint32_t*>(wgt + i) = 0u;
    wave_sync();
    uint64_t cut2 = 0, bn = 0, np = 0;
    constexpr int PER = (LB == 4) ? 2 : 1;
    for (int x0 = lane * PER; x0 < g.n; x0 += WAVE * PER) {
      uint32_t packed = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        int x = x0 + q;
        if (x < g.n) {
          uint32_t w, cd;
          node_weight<MODE>(x, w, cd);
          cut2 += cd;
          bn += w > 0;
          np += w;
          packed |= w << (q * LB);
        }
      }
      wgt[x0 * LB / 8] = (uint8_t)packed;
    }
    wave_sync();
    for (int gi = lane; gi < G; gi += WAVE) {
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(wgt + gi * 64 * LB / 8);
      uint32_t s = 0;
#pragma unroll
      for (int t = 0; t < 2 * LB; ++t) s += (LB == 4) ? nibble_sum(wp[t]) : byte_sum(wp[t]);
      gsum[gi] = s;
    }
    wave_sync();
    cut = (int32_t)rfl((uint32_t)(wave_sum64(cut2) / 2));
    bnodes = (int32_t)rfl((uint32_t)wave_sum64(bn));
    npairs = (int32_t)rfl((uint32_t)wave_sum64(np));
  }

  // -------------------------------------------------------------- select
  // rank r in [0, P) -> node v and in-node index j (canonical (node, ·) order)
  __device__ __forceinline__ void select(uint32_t r, int G, int& v, uint32_t& j) const {
    const int per = (G + WAVE - 1) / WAVE;
    uint32_t s = 0;
    const int g0 = lane * per;
    for (int t = 0; t < per; ++t)
      if (g0 + t < G) s += gsum[g0 + t];
    uint32_t incl = wave_incl_scan(s);
    uint64_t m = ballot(incl > r);
    if (m == 0) {  // inconsistent weights: report instead of reading out of range
      v = -1;
      j = 0;
      return;
    }
    int Lw = __ffsll((unsigned long long)m) - 1;
    uint32_t r1 = r - rdl(incl - s, Lw);
    int gi = rfl(Lw * per);
    const int gend = min(G, gi + per);
    for (; gi < gend; ++gi) {  // uniform walk over <= per groups
      uint32_t gs = rfl(gsum[gi]);
      if (r1 < gs) break;
      r1 -= gs;
    }
    if (gi >= gend) {
      v = -1;
      j = 0;
      return;
    }
    const int x = gi * 64 + lane;
    uint32_t wx = x < g.n ? P::get(wgt, x) : 0u;
    uint32_t incl2 = wave_incl_scan(wx);
    uint64_t m2 = ballot(incl2 > r1);
    if (m2 == 0) {
      v = -1;
      j = 0;
      return;
    }
    int L2 = __ffsll((unsigned long long)m2) - 1;
    v = gi * 64 + L2;
    j = r1 - rdl(incl2 - wx, L2);
  }

  // -------------------------------------------------------------- contiguity
  // Exact: is (district a) \ {v} connected and non-empty?  nl_io counts search stats.
  // srcmask: bit i = lane i holds an a-labelled neighbour (the sources, in CSR order),
  // src_node: this lane's neighbour id; cls: pre-merged class mask (lanes < m).
  __device__ bool race_search(int v, uint32_t a, int m, int src_node, bool is_src, uint32_t src_idx,
                              uint64_t cls, uint64_t& bfs_nodes, uint64_t& bfs_deg) {
    const uint32_t BLOCK = P::MASK;
    // mark v blocked and the sources with their codes k + i
    if (lane == 0) P::axor(lab, v, a ^ BLOCK);
    if (is_src) P::axor(lab, src_node, a ^ ((uint32_t)k + src_idx));
    uint64_t sm = ballot(is_src);
    if (is_src) list_put((int)mbcnt(sm), (uint32_t)src_node);
    wave_sync();
    int nl = m, lb = 0, le = m;
    uint64_t my_deg = 0;
    int verdict = -1;
    for (;;) {
      // classes: representatives are lanes i < m whose mask's lowest bit is i
      uint64_t rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
      if (__popcll(rep) == 1) {
        verdict = 1;
        break;
      }
      uint64_t pushed_src = 0;
      for (int base = lb; base < le; base += WAVE) {
        const int idx = base + lane;
        const bool act = idx < le;
        int x = act ? (int)list_get(idx) : 0;
        uint32_t o = act ? L(x) - (uint32_t)k : 0u;
        int xr = 0, xc = 0;
        int dmax;
        if constexpr (GRID) {
          if (act) divmod(x, xr, xc);
          dmax = 4;
        } else {
          dmax = act ? g.rowptr[x + 1] - g.rowptr[x] : 0;
        }
        if (act) my_deg += (uint64_t)deg(x);
        bfs_nodes += (uint64_t)__popcll(ballot(act));
        int jmax = 4;
        if constexpr (!GRID) {
          // uniform bound: max degree over the active lanes
          uint32_t dm = act ? (uint32_t)dmax : 0u;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) dm = max(dm, (uint32_t)__shfl_xor(dm, d, WAVE));
          jmax = (int)rfl(dm);
        }
        for (int j = 0; j < jmax; ++j) {
          int y = (act && j < dmax) ? nbr(x, j, xr, xc) : -1;
          bool push = false, req = false;
          uint32_t other = 0;
          if (y >= 0) {
            uint32_t ly = L(y);
            if (ly == a) {
              uint32_t got = P::claim(lab, y, a, (uint32_t)k + o);
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
          uint64_t pm = ballot(push);
          if (push) list_put(nl + (int)mbcnt(pm), (uint32_t)y);
          nl += __popcll(pm);
          // sources whose search pushed something this level
          uint64_t pb = push ? (1ull << o) : 0ull;
          pushed_src |= wave_or64(pb);
          // merges (serial over requesting lanes)
          uint64_t rm = ballot(req && o != other);
          while (rm) {
            int Lr = __ffsll((unsigned long long)rm) - 1;
            rm &= rm - 1;
            int o1 = rdl((int32_t)o, Lr), o2 = rdl((int32_t)other, Lr);
            uint64_t m1 = rdl64(cls, o1), m2 = rdl64(cls, o2);
            if (m1 != m2) {
              uint64_t nm = m1 | m2;
              if (lane < m && ((nm >> lane) & 1ull)) cls = nm;
            }
          }
        }
        if (nl > qcap) __threadfence_block();
      }
      wave_sync();
      lb = le;
      le = nl;
      rep = ballot(lane < m && (__ffsll((unsigned long long)cls) - 1) == lane);
      if (__popcll(rep) == 1) {
        verdict = 1;
        break;
      }
      // a class with no pushes this level is closed: disconnected
      bool closed = lane < m && ((rep >> lane) & 1ull) && ((cls & pushed_src) == 0ull);
      if (ballot(closed)) {
        verdict = 0;
        break;
      }
    }
    bfs_deg += wave_sum64(my_deg);
    // restore: visited nodes back to a, v back to a
    for (int base = 0; base < nl; base += WAVE) {
      const int idx = base + lane;
      if (idx < nl) {
        int x = (int)list_get(idx);
        P::axor(lab, x, L(x) ^ a);
      }
    }
    if (lane == 0) P::axor(lab, v, BLOCK ^ a);
    wave_sync();
    return verdict == 1;
  }
};

// ---------------------------------------------------------------- the chain kernel
template <int LB, bool GRID, int MODE>
__global__ __launch_bounds__(64) void fw_run_kernel(FwRunParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID> C;
  C.g = p.g;
  C.lab = smem;
  C.wgt = smem + p.off_w;
  C.gsum = reinterpret_cast<uint32_t*>(smem + p.off_gsum);
  C.pops = reinterpret_cast<int64_t*>(smem + p.off_pops);
  C.list = reinterpret_cast<uint32_t*>(smem + p.off_list);
  C.spill = p.spill + (size_t)blockIdx.x * (size_t)p.g.n;
  C.qcap = p.qcap;
  C.k = p.k;
  C.init_roles();
  const int lane = C.lane;
  const int D = p.g.maxdeg;
  const int G = p.G;
  const int k = p.k;
  const uint32_t key0 = (uint32_t)p.seed, key1 = (uint32_t)(p.seed >> 32);
  __shared__ int32_t s_chain;

  for (;;) {
    if (lane == 0) s_chain = atomicAdd(p.next_chain, 1);
    wave_sync();
    const int c = rfl(s_chain);
    wave_sync();
    if (c >= p.n_chains) break;
    const uint64_t gid = (uint64_t)(p.chain_id0 + c);

    // ---- load state
    {
      const uint4* src = reinterpret_cast<const uint4*>(p.labels + (size_t)c * p.lab_stride);
      uint4* dst = reinterpret_cast<uint4*>(C.lab);
      for (int i = lane; i < p.lab_bytes / 16; i += WAVE) dst[i] = src[i];
      for (int i = lane; i < k; i += WAVE) C.pops[i] = p.pops[(size_t)c * k + i];
    }
    fw_chain_stats* stp = p.stats + c;
    uint64_t attempts = stp->attempts, steps_done = stp->steps, accepts = stp->accepts;
    uint64_t pop_fail = stp->pop_fail, contig_fail = stp->contig_fail, bfs_runs = stp->bfs_runs;
    uint64_t bfs_nodes = stp->bfs_nodes, bfs_deg = stp->bfs_deg, sum_deg = stp->sum_deg;
    uint64_t acc_deg = stp->acc_deg, n_bchg = stp->n_bchg, yields = stp->yields;
    int64_t sum_cut = stp->sum_cut, sum_bnodes = stp->sum_bnodes;
    double sum_invb = stp->sum_invb;
    int32_t stuck = stp->stuck;
    const double thr_l =
        lane < 2 * D + 1 ? p.thr[(size_t)c * p.thr_stride + lane] : 0.0;  // lane-held table
    wave_sync();
    int32_t cut, bnodes, npairs;
    C.template derive<MODE>(cut, bnodes, npairs, G);
    double invb = 1.0 / (double)bnodes;

    // histogram windows: lane i counts value base+i
    uint32_t hc = 0, hb = 0;
    int32_t base_c = max(0, cut - 32), base_b = max(0, bnodes - 32);
    auto observe = [&]() {
      yields += 1;
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
    if (yields == 0 && attempts == 0) observe();

    const bool unit_pop = p.g.pop == nullptr;
    for (int64_t s = 0; s < p.steps && !stuck; ++s) {
      int32_t retries = 0;
      int v = 0, dcut = 0;
      uint32_t a = 0, d = 0;
      int64_t pv = 1;
      U4 x;
      bool valid = false;
      for (;;) {
        if (retries >= p.max_retries || npairs == 0) {
          stuck = 1;
          break;
        }
        x = philox((uint32_t)attempts, (uint32_t)(attempts >> 32), (uint32_t)gid,
                   (uint32_t)(gid >> 32), key0, key1);
        attempts += 1;
        uint32_t r = scale64(x.x0, x.x1, (uint32_t)npairs);
        uint32_t j;
        C.select(r, G, v, j);
        v = rfl(v);
        j = rfl(j);
        if (v < 0) {  // internal inconsistency: stop this chain, flag it
          stuck = 2;
          break;
        }
        a = rfl(C.L(v));
        // ---- gather v's ring (grid) / neighbours (CSR)
        int cell = -1;
        int dv;
        bool isn;
        if constexpr (GRID) {
          int vr, vc;
          C.divmod(v, vr, vc);
          int nr = vr + C.my_dr, nc = vc + C.my_dc;
          bool ok = lane < 8 && nr >= 0 && nr < p.g.gh && nc >= 0 && nc < p.g.gw;
          cell = ok ? nr * p.g.gw + nc : -1;
          isn = lane < 4 && ok;
          dv = (vr > 0) + (vc > 0) + (vc < p.g.gw - 1) + (vr < p.g.gh - 1);
        } else {
          const int e0 = p.g.rowptr[v];
          dv = rfl(p.g.rowptr[v + 1] - e0);
          isn = lane < dv;
          cell = isn ? p.g.col[e0 + lane] : -1;
        }
        const uint32_t l = cell >= 0 ? C.L(cell) : 0xFFFFu;
        sum_deg += (uint64_t)dv;
        if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
          uint64_t cm = ballot(isn && l != a);
          int Lc = nth_bit(cm, j);
          d = rfl(rdl(l, Lc));
        } else {
          uint64_t fb = (isn && l != a) ? (1ull << l) : 0ull;
          uint64_t mask;
          if constexpr (GRID) {
            mask = rdl64(fb, 0) | rdl64(fb, 1) | rdl64(fb, 2) | rdl64(fb, 3);
          } else {
            mask = wave_or64(fb);
            mask = ((uint64_t)rfl((uint32_t)(mask >> 32)) << 32) | rfl((uint32_t)mask);
          }
          d = (uint32_t)nth_bit(mask, j);
        }
        const uint64_t am = ballot(isn && l == a);
        const int m = __popcll(am);
        dcut = m - __popcll(ballot(isn && l == d));
        // ---- population bound (Bounds over the two changed districts)
        pv = unit_pop ? 1 : p.g.pop[v];
        const int64_t pa = C.pops[a], pb = C.pops[d];
        if (pa - pv < p.pop_lo || pb + pv > p.pop_hi) {
          pop_fail += 1;
          ++retries;
          continue;
        }
        // ---- contiguity (single_flip_contiguous)
        bool ok;
        if (m == 0) {
          ok = false;
        } else if (m == 1) {
          ok = true;
        } else {
          const bool is_src = isn && l == a;
          const uint32_t sidx = mbcnt(am);
          uint64_t cls = lane < m ? (1ull << lane) : 0ull;
          bool need = true;
          if constexpr (GRID) {
            const uint64_t rm = ballot(lane < 8 && l == a);
            const int pN = rm & 1, pW = (rm >> 1) & 1, pE = (rm >> 2) & 1, pS = (rm >> 3) & 1;
            const int NE = (rm >> 4) & 1, SE = (rm >> 5) & 1, SW = (rm >> 6) & 1, NW = (rm >> 7) & 1;
            const int lNE = pN & pE & NE, lES = pE & pS & SE, lSW = pS & pW & SW, lWN = pW & pN & NW;
            int comps = m - (lNE + lES + lSW + lWN);
            if (comps <= 1) {
              need = false;
            } else {
              // pre-merge the ring links; source index = rank among lanes 0..3
              auto sx = [&](int ln) { return __popcll(am & ((1ull << ln) - 1ull)); };
              auto merge = [&](int s1, int s2) {
                uint64_t m1 = rdl64(cls, s1), m2 = rdl64(cls, s2);
                uint64_t nm = m1 | m2;
                if (lane < m && ((nm >> lane) & 1ull)) cls = nm;
              };
              if (lNE) merge(sx(0), sx(2));
              if (lES) merge(sx(2), sx(3));
              if (lSW) merge(sx(3), sx(1));
              if (lWN) merge(sx(1), sx(0));
            }
          }
          if (need) {
            bfs_runs += 1;
            ok = C.race_search(v, a, m, cell, is_src, sidx, cls, bfs_nodes, bfs_deg);
          } else {
            ok = true;
          }
        }
        if (!ok) {
          contig_fail += 1;
          ++retries;
          continue;
        }
        valid = true;
        break;
      }
      if (!valid) break;
      steps_done += 1;
      // ---- Metropolis (cut_accept, grid_chain_sec11.py:171-179)
      const double bound = rdl_f64(thr_l, dcut + D);
      const bool accepted = u53(x.x2, x.x3) < bound;
      if (p.trace && lane == 0) p.trace[(size_t)c * p.steps + s] = accepted ? v * 64 + (int)d : -1;
      if (accepted) {
        accepts += 1;
        // ---- commit
        if (lane == 0) {
          PK<LB>::axor(C.lab, v, a ^ d);
          C.pops[a] -= pv;
          C.pops[d] += pv;
        }
        wave_sync();
        cut += dcut;
        int xn = -1;
        if constexpr (GRID) {
          int vr, vc;
          C.divmod(v, vr, vc);
          int nr = vr + C.cm_dr, nc = vc + C.cm_dc;
          bool okc = lane <= 4 && nr >= 0 && nr < p.g.gh && nc >= 0 && nc < p.g.gw;
          xn = okc ? nr * p.g.gw + nc : -1;
          acc_deg += (uint64_t)((vr > 0) + (vc > 0) + (vc < p.g.gw - 1) + (vr < p.g.gh - 1));
        } else {
          const int e0 = p.g.rowptr[v];
          const int dv = rfl(p.g.rowptr[v + 1] - e0);
          xn = lane == 0 ? v : (lane <= dv ? p.g.col[e0 + lane - 1] : -1);
          acc_deg += (uint64_t)dv;
        }
        uint32_t wo = 0, wn = 0;
        if (xn >= 0) {
          uint32_t cd;
          C.template node_weight<MODE>(xn, wn, cd);
          wo = PK<LB>::get(C.wgt, xn);
        }
        wave_sync();
        if (xn >= 0 && wn != wo) {
          PK<LB>::axor(C.wgt, xn, wo ^ wn);
          atomicAdd(C.gsum + (xn >> 6), wn - wo);
        }
        const int plus = __popcll(ballot(xn >= 0 && wo == 0 && wn > 0));
        const int minus = __popcll(ballot(xn >= 0 && wo > 0 && wn == 0));
        bnodes += plus - minus;
        n_bchg += (uint64_t)(plus + minus);
        npairs += (int32_t)rfl((uint32_t)wave_sum64((uint64_t)(int64_t)((int32_t)wn - (int32_t)wo)));
        if (plus | minus) invb = 1.0 / (double)bnodes;
        wave_sync();
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
      for (int i = lane; i < k; i += WAVE) p.pops[(size_t)c * k + i] = C.pops[i];
    }
    if (lane == 0) {
      stp->attempts = attempts;
      stp->steps = steps_done;
      stp->accepts = accepts;
      stp->pop_fail = pop_fail;
      stp->contig_fail = contig_fail;
      stp->bfs_runs = bfs_runs;
      stp->bfs_nodes = bfs_nodes;
      stp->bfs_deg = bfs_deg;
      stp->sum_deg = sum_deg;
      stp->acc_deg = acc_deg;
      stp->n_bchg = n_bchg;
      stp->yields = yields;
      stp->sum_cut = sum_cut;
      stp->sum_bnodes = sum_bnodes;
      stp->sum_invb = sum_invb;
      stp->cut = cut;
      stp->bnodes = bnodes;
      stp->npairs = npairs;
      stp->stuck = stuck;
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------- per-flip evaluation
template <int LB, bool GRID>
__global__ __launch_bounds__(64) void fw_eval_kernel(FwEvalParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID> C;
  C.g = p.g;
  C.lab = smem;
  C.wgt = nullptr;
  C.gsum = nullptr;
  C.pops = nullptr;
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
    wave_sync();
    const int v = p.v[i];
    const uint32_t b = (uint32_t)p.target[i];
    const uint32_t a = rfl(C.L(v));
    int cell = -1;
    bool isn;
    if constexpr (GRID) {
      int vr, vc;
      C.divmod(v, vr, vc);
      int nr = vr + C.my_dr, nc = vc + C.my_dc;
      bool ok = lane < 8 && nr >= 0 && nr < p.g.gh && nc >= 0 && nc < p.g.gw;
      cell = ok ? nr * p.g.gw + nc : -1;
      isn = lane < 4 && ok;
    } else {
      const int e0 = p.g.rowptr[v];
      const int dv = p.g.rowptr[v + 1] - e0;
      isn = lane < dv;
      cell = isn ? p.g.col[e0 + lane] : -1;
    }
    const uint32_t l = cell >= 0 ? C.L(cell) : 0xFFFFu;
    const uint64_t am = ballot(isn && l == a);
    const int m = __popcll(am);
    const int dcut = m - __popcll(ballot(isn && l == b));
    const int64_t pv = p.g.pop ? p.g.pop[v] : 1;
    const bool pok = !(p.pops[a] - pv < p.pop_lo || p.pops[b] + pv > p.pop_hi);
    bool ok;
    uint64_t dummy0 = 0, dummy1 = 0;
    if (m == 0) {
      ok = false;
    } else if (m == 1) {
      ok = true;
    } else {
      const bool is_src = isn && l == a;
      const uint32_t sidx = mbcnt(am);
      uint64_t cls = lane < m ? (1ull << lane) : 0ull;
      ok = C.race_search(v, a, m, cell, is_src, sidx, cls, dummy0, dummy1);
    }
    // boundary membership of v and its neighbours before/after the flip
    int xn = -1;
    if constexpr (GRID) {
      int vr, vc;
      C.divmod(v, vr, vc);
      int nr = vr + C.cm_dr, nc = vc + C.cm_dc;
      bool okc = lane <= 4 && nr >= 0 && nr < p.g.gh && nc >= 0 && nc < p.g.gw;
      xn = okc ? nr * p.g.gw + nc : -1;
    } else {
      const int e0 = p.g.rowptr[v];
      const int dv = p.g.rowptr[v + 1] - e0;
      xn = lane == 0 ? v : (lane <= dv ? p.g.col[e0 + lane - 1] : -1);
    }
    uint32_t w0 = 0, w1 = 0, cd;
    if (xn >= 0) C.template node_weight<FW_PROPOSE_CUTEDGE>(xn, w0, cd);
    wave_sync();
    if (lane == 0) PK<LB>::axor(C.lab, v, a ^ b);
    wave_sync();
    if (xn >= 0) C.template node_weight<FW_PROPOSE_CUTEDGE>(xn, w1, cd);
    const int db = __popcll(ballot(xn >= 0 && w1 > 0)) - __popcll(ballot(xn >= 0 && w0 > 0));
    wave_sync();
    if (lane == 0) {
      p.dcut[i] = dcut;
      p.contig[i] = ok ? 1 : 0;
      p.pop_ok[i] = pok ? 1 : 0;
      p.dboundary[i] = db;
    }
    wave_sync();
  }
}

template <int LB, bool GRID, int MODE>
void* run_kernel_ptr() {
  return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE>);
}

void* pick_run(int lb, bool grid, int mode) {
  const bool cut = mode == FW_PROPOSE_CUTEDGE;
  if (lb == 4) {
    if (grid) return cut ? run_kernel_ptr<4, true, 2>() : run_kernel_ptr<4, true, 1>();
    return cut ? run_kernel_ptr<4, false, 2>() : run_kernel_ptr<4, false, 1>();
  }
  if (grid) return cut ? run_kernel_ptr<8, true, 2>() : run_kernel_ptr<8, true, 1>();
  return cut ? run_kernel_ptr<8, false, 2>() : run_kernel_ptr<8, false, 1>();
}

}  // namespace

int fw_run_grid_size(const FwRunParams& p, int lb, int device, int* grid) {
  void* fn = pick_run(lb, p.g.gw > 0, p.mode);
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
  void* fn = pick_run(lb, p.g.gw > 0, p.mode);
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
