// fw_grid16.hip — the row-major-grid chain kernel, four chains per wavefront.
//
// The one-chain-per-wave kernel (fw_kernels.hip) is bound by the CU's scalar unit:
// per proposal it issues ~340 scalar instructions (Philox on the SALU plus the exec-
// mask bookkeeping of lane-role branches) for one chain.  Here each 16-lane DPP row
// of a wavefront owns one chain, so every instruction of the common path serves four
// chains: Philox runs on the VALU, per-chain scalars live in row-uniform VGPRs,
// prefix scans are 4-step row_shr DPP scans, a lane's value is broadcast to its row
// by a masked row scan + row_newbcast, and row-level votes are bit fields of one
// 64-bit ballot.  The exact contiguity search (needed by a few percent of proposals)
// runs wave-cooperatively on one chain slot at a time with the shared race search of
// fw_device.h, so its result is the same bit for bit as in the other kernel.
//
// LDS: four chain slots (labels | group sums), slot stride padded so the four rows
// start on different banks, then one search list shared by the four chains.
// Semantics: oracle/flipchain_oracle.c.
#include <hip/hip_runtime.h>

#include "fw_device.h"

#ifdef FW_STAMPS
// Diagnostic build only (libflipwalk_stamps.so): per-phase s_memtime shares.
__device__ unsigned long long g_stamps[8];
#define STAMP_DECL uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t st_t0 = 0;
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
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_stamps[i_], (unsigned long long)st_acc[i_]);
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#endif

namespace {

constexpr int ROW = 16;

// v's neighbourhood as one lane sees it (labels < 16 here, so 32-bit label sets)
struct Hood16 {
  int x;          // node id, -1 if absent
  uint32_t lx;    // label of x (NOLAB if absent)
  uint32_t bits;  // OR of 1<<label over x's neighbours other than v
  uint32_t cnt;   // number of x's neighbours other than v with label != lx
  bool has_v;     // v is a neighbour of x
  int deg;        // degree of x
};

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
// value held by row-lane L (row-uniform L in 0..15; anything else gives 0)
__device__ __forceinline__ uint32_t row_pick(uint32_t x, int L, int q) {
  return row_sum(q == L ? x : 0u);
}

// Four consecutive nibbles x..x+3 of a packed 4-bit label array (16 bits), plus the
// nibbles at x-1 and x+4 (returned in bits 16..19 and 20..23).  Two aligned dword
// reads; the label region is padded so the second read stays inside the slot.
__device__ __forceinline__ uint32_t nib_window(const LDS uint8_t* lab, int x) {
  const int xm = x - 1;  // may be -1: then the low nibble is garbage and masked by callers
  const int bit = xm * 4;
  const int wi = bit >> 5;  // dword holding nibble xm (arithmetic shift: -1 -> -1)
  const LDS uint32_t* w = reinterpret_cast<const LDS uint32_t*>(lab);
  const uint32_t lo = wi >= 0 ? w[wi] : 0u;
  const uint32_t hi = w[wi + 1];
  const uint64_t both = ((uint64_t)hi << 32) | lo;
  const uint32_t sh = (uint32_t)(bit - wi * 32);
  const uint32_t six = (uint32_t)(both >> sh) & 0xFFFFFFu;  // nibbles xm .. xm+5
  // reorder: own 4 nibbles in bits 0..15, x-1 in 16..19, x+4 in 20..23
  return ((six >> 4) & 0xFFFFu) | ((six & 0xFu) << 16) | (((six >> 20) & 0xFu) << 20);
}

// Proposal weights (and cut degrees) of the four nodes x0..x0+3 (x0 a multiple of 4)
// of a row-major W x H grid, packed one per byte.  A window may wrap into the next grid
// row when W is not a multiple of 4, so neighbour windows are read whenever ANY of the
// four nodes has that neighbour; per-node row/column checks mask the rest.
template <int MODE>
__device__ __forceinline__ void weights4(const LDS uint8_t* lab, int x0, int W, int H, int n,
                                         uint64_t gmagic, uint32_t& w4, uint32_t& cd4) {
  w4 = 0;
  cd4 = 0;
  if (x0 >= n) return;
  const uint32_t own = nib_window(lab, x0);
  const uint32_t up = x0 + 3 - W >= 0 ? nib_window(lab, x0 - W) : 0u;
  const uint32_t dn = x0 + W < n ? nib_window(lab, x0 + W) : 0u;
  const int r0 = (int)(((uint64_t)(uint32_t)x0 * gmagic) >> 42);
  const int c0 = x0 - r0 * W;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    int ct = c0 + tt, rt = r0;
    if (ct >= W) {
      ct -= W;
      rt += 1;
    }
    const uint32_t lx = (own >> (4 * tt)) & 15u;
    const uint32_t ll = tt == 0 ? (own >> 16) & 15u : (own >> (4 * tt - 4)) & 15u;
    const uint32_t lr = tt == 3 ? (own >> 20) & 15u : (own >> (4 * tt + 4)) & 15u;
    const uint32_t lu = (up >> (4 * tt)) & 15u, ld = (dn >> (4 * tt)) & 15u;
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

template <int MODE, int PER>
__global__ __launch_bounds__(64) void fw_grid16_kernel(FwRunParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int lane = __lane_id(), row = lane >> 4, q = lane & 15;
  const int W = p.g.gw, H = p.g.gh, n = p.g.n, D = p.g.maxdeg, G = p.G, k = p.k;
  LDS uint8_t* const sm = (LDS uint8_t*)smem;
  LDS uint8_t* const lab = sm + row * p.slot_stride;  // this row's chain slot
  LDS uint32_t* const gsum = reinterpret_cast<LDS uint32_t*>(lab + p.off_gsum);
  const uint32_t key0 = (uint32_t)p.seed, key1 = (uint32_t)(p.seed >> 32);
  using P = PK<4>;
  int my_dr, my_dc;
  role_off(q <= 8 ? q : 0, my_dr, my_dc);
  auto divmod = [&](int x, int& r, int& c) {
    r = (int)(((uint64_t)(uint32_t)x * p.g.gmagic) >> 42);
    c = x - r * W;
  };
  __shared__ int32_t s_base;
  STAMP_DECL

  for (;;) {
    if (lane == 0) s_base = atomicAdd(p.next_chain, 4);
    __syncthreads();
    const int cbase = rfl(s_base);
    if (cbase >= p.n_chains) break;
    const int c = cbase + row;
    const bool has = c < p.n_chains;
    const int cc = has ? c : cbase;  // a valid index for loads of absent rows
    const uint64_t gid = (uint64_t)(p.chain_id0 + c);

    // ---- load state (each row loads its own chain)
    {
      const u32x4* src = reinterpret_cast<const u32x4*>(p.labels + (size_t)cc * p.lab_stride);
      LDS u32x4* dst = reinterpret_cast<LDS u32x4*>(lab);
      for (int i = q; i < p.lab_bytes / 16; i += ROW) dst[i] = src[i];
    }
    int64_t pops = q < k ? p.pops[(size_t)cc * k + q] : 0;
    const double thr_l = q < 2 * D + 1 ? p.thr[(size_t)cc * p.thr_stride + q] : 0.0;
    fw_chain_stats* stp = p.stats + cc;
    uint64_t attempts = stp->attempts;
    const uint64_t yields0 = stp->yields;
    int32_t stuck = has ? stp->stuck : 1;
    int64_t sum_cut = stp->sum_cut, sum_bnodes = stp->sum_bnodes;
    double sum_invb = stp->sum_invb;
    uint32_t n_steps = 0, n_acc = 0, n_popf = 0, n_conf = 0, n_sdeg = 0, n_adeg = 0, n_bchg = 0;
    uint32_t n_yield = 0, retries = 0;
    uint64_t n_bfs = 0, n_bfsn = 0, n_bfsd = 0;
    __syncthreads();

    // ---- derive group sums, cut / boundary / proposal-set counts (per row)
    int32_t cut, bnodes, npairs;
    {
      uint32_t cut2 = 0, bn = 0, np = 0;
      for (int t = 0; t < G; ++t) {
        uint32_t w4, cd4;
        weights4<MODE>(lab, t * 64 + q * 4, W, H, n, p.g.gmagic, w4, cd4);
        const uint32_t ws = bsum4(w4);
        cut2 += bsum4(cd4);
        bn += ((cd4 & 0xFFu) != 0) + ((cd4 & 0xFF00u) != 0) + ((cd4 & 0xFF0000u) != 0) +
              ((cd4 & 0xFF000000u) != 0);
        np += ws;
        const uint32_t tot = row_sum(ws);
        if (q == 0 && has) gsum[t] = tot;
      }
      cut = (int32_t)(row_sum(cut2) / 2);
      bnodes = (int32_t)row_sum(bn);
      npairs = (int32_t)row_sum(np);
    }
    lds_order();
    double invb = 1.0 / (double)(bnodes > 0 ? bnodes : 1);

    // histogram windows: row-lane q counts values base+q and base+16+q
    uint32_t hc0 = 0, hc1 = 0, hb0 = 0, hb1 = 0;
    int32_t base_c = max(0, cut - 16), base_b = max(0, bnodes - 16);
    auto observe = [&](bool on) {
      if (!on) return;
      n_yield += 1;
      sum_cut += cut;
      sum_bnodes += bnodes;
      sum_invb += invb;
      int ic = cut - base_c;
      if (ic < 0 || ic >= 2 * ROW) {
        if (hc0) atomicAdd(p.hist_cut + base_c + q, (unsigned long long)hc0);
        if (hc1) atomicAdd(p.hist_cut + base_c + ROW + q, (unsigned long long)hc1);
        hc0 = hc1 = 0;
        base_c = max(0, cut - ROW);
        ic = cut - base_c;
      }
      hc0 += ic == q;
      hc1 += ic == q + ROW;
      int ib = bnodes - base_b;
      if (ib < 0 || ib >= 2 * ROW) {
        if (hb0) atomicAdd(p.hist_b + base_b + q, (unsigned long long)hb0);
        if (hb1) atomicAdd(p.hist_b + base_b + ROW + q, (unsigned long long)hb1);
        hb0 = hb1 = 0;
        base_b = max(0, bnodes - ROW);
        ib = bnodes - base_b;
      }
      hb0 += ib == q;
      hb1 += ib == q + ROW;
    };
    observe(has && !stuck && yields0 == 0 && attempts == 0);

    // Philox batches: lane q of a row holds the draw of its chain's attempt (base + q).
    // Active rows consume one attempt per loop iteration in lockstep, so every row reads
    // lane `bpos` of its own row; a row that stops stays stopped for this launch.
    U4 pb = {0u, 0u, 0u, 0u};
    int bpos = ROW;

    const bool unit_pop = p.g.pop == nullptr;
    for (;;) {
      STAMP(-1);
      // ---- who proposes this round
      if (!stuck && (retries >= (uint32_t)p.max_retries || npairs == 0)) stuck = 1;
      const bool act = has && !stuck && (int64_t)n_steps < p.steps;
      if (ballot(act) == 0ull) break;

      if (bpos == ROW) {
        const uint64_t t = attempts + (uint64_t)q;
        pb = philox((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid, (uint32_t)(gid >> 32), key0,
                    key1);
        bpos = 0;
      }
      const int src = (row * ROW + bpos) * 4;  // ds_bpermute byte address of the source lane
      const U4 x = {(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pb.x0),
                    (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pb.x1),
                    (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pb.x2),
                    (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pb.x3)};
      ++bpos;
      attempts += act ? 1u : 0u;
      const uint32_t r = scale64(x.x0, x.x1, (uint32_t)(npairs > 0 ? npairs : 1));

      STAMP(0);  // draw
      // ---- select, level 1: group sums (PER per lane)
      uint32_t gs[PER];
      uint32_t s = 0;
#pragma unroll
      for (int t = 0; t < PER; ++t) {
        const int gi = q * PER + t;
        gs[t] = gi < G ? gsum[gi] : 0u;
        s += gs[t];
      }
      const uint32_t incl = row_scan(s);
      const uint32_t rb1 = rowbits(ballot(incl > r), row);
      const int Lw = __ffs(rb1) - 1;
      uint32_t rl = r - (incl - s), c1 = 0, before = 0;
      int tf = PER - 1;
      bool found = false;
#pragma unroll
      for (int t = 0; t < PER; ++t) {
        const uint32_t c2 = c1 + gs[t];
        if (!found && rl < c2) {
          tf = t;
          before = c1;
          found = true;
        }
        c1 = c2;
      }
      // pack (group, remaining rank) into one row broadcast
      const uint32_t pk1 = row_pick(((uint32_t)(q * PER + tf) << 16) | ((rl - before) & 0xFFFFu), Lw, q);
      const int gi = min((int)(pk1 >> 16), G - 1);
      const uint32_t r1 = pk1 & 0xFFFFu;

      STAMP(1);  // level 1
      // ---- select, level 2: weights of the group's 64 nodes, 4 per lane
      const int x0 = gi * 64 + q * 4;
      uint32_t w4, cd4;  // four 8-bit weights
      weights4<MODE>(lab, x0, W, H, n, p.g.gmagic, w4, cd4);
      const uint32_t ws = bsum4(w4);
      const uint32_t incl2 = row_scan(ws);
      const uint32_t rb2 = rowbits(ballot(incl2 > r1), row);
      const int L2 = __ffs(rb2) - 1;
      uint32_t r2 = r1 - (incl2 - ws), c3 = 0, bef2 = 0;
      int t2 = 3;
      bool f2 = false;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const uint32_t c4 = c3 + ((w4 >> (8 * tt)) & 0xFFu);
        if (!f2 && r2 < c4) {
          t2 = tt;
          bef2 = c3;
          f2 = true;
        }
        c3 = c4;
      }
      const uint32_t pk2 = row_pick(((uint32_t)(q * 4 + t2) << 16) | ((r2 - bef2) & 0xFFFFu), L2, q);
      const int v = min(gi * 64 + (int)(pk2 >> 16), n - 1);
      const uint32_t j = pk2 & 0xFFFFu;
      if (act && (rb1 == 0 || rb2 == 0)) stuck = 2;  // inconsistent state: flag, stop chain
      const bool go = act && rb1 != 0 && rb2 != 0;

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
      {
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
      const uint32_t a = row_pick(h.lx, 0, q);
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
        uint32_t fb = (isnb && h.lx != a) ? (1u << h.lx) : 0u;
        fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x111, 0xF, 0xF, true);  // row_shr:1
        fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x112, 0xF, 0xF, true);  // row_shr:2
        fb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x114, 0xF, 0xF, true);  // row_shr:4
        const uint32_t mask = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fb, 0x154, 0xF, 0xF, false);  // row_newbcast:4
        uint32_t mm = mask;
        for (uint32_t t = 0; t < j && t < 15; ++t) mm &= mm - 1;
        d = (uint32_t)(__ffs(mm) - 1);
      }
      const uint32_t amb = rowbits(ballot(isnb && h.lx == a), row) >> 1;
      const int m = __popc(amb);
      const int nbd = __popc(rowbits(ballot(isnb && h.lx == d), row) >> 1);
      const int dcut = m - nbd;

      // ---- population bound (lane q holds district q)
      const int64_t pv = unit_pop ? 1 : p.g.pop[v];
      const bool bad = ((uint32_t)q == a && pops - pv < p.pop_lo) ||
                       ((uint32_t)q == d && pops + pv > p.pop_hi);
      const bool pop_ok = rowbits(ballot(bad), row) == 0u;

      STAMP(3);  // gather, target, Δcut, population
      // ---- contiguity: 8-cell ring test, exact race search when inconclusive
      const uint32_t rbits8 = rowbits(ballot(q >= 1 && q <= 8 && h.lx == a), row) >> 1;
      const int pN = rbits8 & 1, pW = (rbits8 >> 1) & 1, pE = (rbits8 >> 2) & 1, pS = (rbits8 >> 3) & 1;
      const int NE = (rbits8 >> 4) & 1, SE = (rbits8 >> 5) & 1, SW = (rbits8 >> 6) & 1,
                NW = (rbits8 >> 7) & 1;
      const int lNE = pN & pE & NE, lES = pE & pS & SE, lSW = pS & pW & SW, lWN = pW & pN & NW;
      bool contig = m == 1 || (m >= 2 && m - (lNE + lES + lSW + lWN) <= 1);
      bool need = go && pop_ok && m >= 2 && !contig;
      if (ballot(need)) {  // 7x7 window flood fill (3 window cells per row-lane)
        uint64_t A = 0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int pos = window_pos(q + ROW * t);
          const int rr = vr - 3 + pos / 7, cc = vc - 3 + pos % 7;
          const bool in = rr >= 0 && rr < H && cc >= 0 && cc < W && P::get(lab, rr * W + cc) == a;
          A |= (uint64_t)rowbits(ballot(in), row) << (ROW * t);
        }
        A = (A & ((1ull << 24) - 1ull)) | ((A >> 24) << 25);
        const int wv = need ? window_verdict(A) : -1;
        if (wv >= 0) {
          contig = wv == 1;
          need = false;
        }
      }
      uint64_t rows_need = ballot(q == 0 && need);
      while (rows_need) {  // wave-cooperative exact search, one chain slot at a time
        const int L0 = __ffsll((unsigned long long)rows_need) - 1;
        rows_need &= rows_need - 1;
        const int rr = L0 >> 4;
        Ctx<4, true> C;
        C.g = p.g;
        C.lab = sm + rr * p.slot_stride;
        C.gsum = nullptr;
        C.list = reinterpret_cast<LDS uint32_t*>(sm + 4 * p.slot_stride);  // shared list
        C.spill = (GLB uint32_t*)(p.spill + (size_t)blockIdx.x * (size_t)n);
        C.qcap = p.qcap;
        C.k = k;
        C.lane = lane;
        const int vv = rdl(v, L0);
        const uint32_t aa = rdl(a, L0);
        const uint32_t am4 = rdl(amb, L0);
        const int mr = __popc(am4);
        // sources in CSR order (up, left, right, down) into lanes 0..m-1
        int src = -1;
        uint32_t mm = am4;
        for (int i = 0; i < mr; ++i) {
          const int bit = __ffs(mm) - 1;
          mm &= mm - 1;
          const int val = rdl(h.x, L0 + 1 + bit);
          if (lane == i) src = val;
        }
        uint64_t cls = lane < mr ? (1ull << lane) : 0ull;
        const uint32_t lk = rdl((uint32_t)(lNE | (lES << 1) | (lSW << 2) | (lWN << 3)), L0);
        auto sx = [&](int b) { return __popc(am4 & ((1u << b) - 1u)); };
        auto merge = [&](int s1, int s2) {
          const uint64_t nm = rdl64(cls, s1) | rdl64(cls, s2);
          if (lane < mr && ((nm >> lane) & 1ull)) cls = nm;
        };
        if (lk & 1) merge(sx(0), sx(2));  // N-E
        if (lk & 2) merge(sx(2), sx(3));  // E-S
        if (lk & 4) merge(sx(3), sx(1));  // S-W
        if (lk & 8) merge(sx(1), sx(0));  // W-N
        uint64_t bn = 0, bd = 0;
        const bool ok = C.race_search(vv, aa, mr, src, cls, bn, bd);
        if (row == rr) {
          contig = ok;
          n_bfs += 1;
          n_bfsn += bn;
          n_bfsd += bd;
        }
      }

      STAMP(4);  // ring test + exact searches
      // ---- outcome
      const bool valid = go && pop_ok && contig;
      if (go) {
        n_sdeg += (uint32_t)dv;
        if (!pop_ok) n_popf += 1;
        else if (!contig) n_conf += 1;
        retries = valid ? 0u : retries + 1u;
      }
      // Metropolis (cut_accept, grid_chain_sec11.py:171-179): lane dcut+D holds the bound
      const bool acc_l = u53(x.x2, x.x3) < thr_l;
      const bool accepted = valid && ((rowbits(ballot(acc_l), row) >> (dcut + D)) & 1u);
      if (valid && p.trace && q == 0)
        p.trace[(size_t)c * p.steps + n_steps] = accepted ? v * 64 + (int)d : -1;
      n_steps += valid ? 1u : 0u;

      // ---- commit (accepting rows)
      uint32_t wo = 0, wn = 0;
      const bool mine = q <= 4 && h.x >= 0;
      if (mine) {
        if (q == 0) {
          if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
            wo = (uint32_t)(h.deg - m);
            wn = (uint32_t)(h.deg - nbd);
          } else {
            wo = (uint32_t)__popc(h.bits & ~(1u << a));
            wn = (uint32_t)__popc(h.bits & ~(1u << d));
          }
        } else if constexpr (MODE == FW_PROPOSE_CUTEDGE) {
          wo = h.cnt + (h.has_v && a != h.lx);
          wn = h.cnt + (h.has_v && d != h.lx);
        } else {
          const uint32_t keep = ~(1u << h.lx);
          wo = (uint32_t)__popc((h.bits | (h.has_v ? 1u << a : 0u)) & keep);
          wn = (uint32_t)__popc((h.bits | (h.has_v ? 1u << d : 0u)) & keep);
        }
      }
      if (accepted) {
        if (q == 0) P::axor(lab, v, a ^ d);
        if (mine && wn != wo) lds_add(gsum + (h.x >> 6), wn - wo);
      }
      lds_order();
      const uint64_t b_plus = ballot(accepted && mine && wo == 0 && wn > 0);
      const uint64_t b_minus = ballot(accepted && mine && wo > 0 && wn == 0);
      const int plus = __popc(rowbits(b_plus, row)), minus = __popc(rowbits(b_minus, row));
      const int dnp = (int)row_sum(accepted && mine ? wn - wo : 0u);
      if (accepted) {
        n_acc += 1;
        n_adeg += (uint32_t)dv;
        npairs += dnp;
        cut += dcut;
        bnodes += plus - minus;
        n_bchg += (uint32_t)(plus + minus);
        if (plus | minus) invb = 1.0 / (double)bnodes;
        if ((uint32_t)q == a) pops -= pv;
        if ((uint32_t)q == d) pops += pv;
      }
      observe(valid);
      STAMP(5);  // outcome, Metropolis, commit, observe
    }

    STAMP(6);  // loop exit
    // ---- write back
    if (has) {
      if (hc0) atomicAdd(p.hist_cut + base_c + q, (unsigned long long)hc0);
      if (hc1) atomicAdd(p.hist_cut + base_c + ROW + q, (unsigned long long)hc1);
      if (hb0) atomicAdd(p.hist_b + base_b + q, (unsigned long long)hb0);
      if (hb1) atomicAdd(p.hist_b + base_b + ROW + q, (unsigned long long)hb1);
      u32x4* dst = reinterpret_cast<u32x4*>(p.labels + (size_t)c * p.lab_stride);
      const LDS u32x4* src = reinterpret_cast<const LDS u32x4*>(lab);
      for (int i = q; i < p.lab_bytes / 16; i += ROW) dst[i] = src[i];
      if (q < k) p.pops[(size_t)c * k + q] = pops;
      if (q == 0) {
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
    }
    __syncthreads();
  }
  STAMP_FLUSH
}

template <int MODE>
void* pick16(int G) {
  if (G <= 16 * 2) return reinterpret_cast<void*>(&fw_grid16_kernel<MODE, 2>);
  if (G <= 16 * 4) return reinterpret_cast<void*>(&fw_grid16_kernel<MODE, 4>);
  if (G <= 16 * 10) return reinterpret_cast<void*>(&fw_grid16_kernel<MODE, 10>);
  return reinterpret_cast<void*>(&fw_grid16_kernel<MODE, 16>);
}

}  // namespace

#ifdef FW_STAMPS
extern "C" int fw_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

bool fw_grid16_supported(const FwRunParams& p, int lb) {
  return p.g.gw > 0 && lb == 4 && p.G <= 16 * 16 && p.k <= 15 && p.g.maxdeg == 4;
}

void* fw_grid16_fn(const FwRunParams& p) {
  return p.mode == FW_PROPOSE_CUTEDGE ? pick16<FW_PROPOSE_CUTEDGE>(p.G)
                                      : pick16<FW_PROPOSE_PAIRS>(p.G);
}
