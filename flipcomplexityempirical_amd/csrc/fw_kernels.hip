// fw_kernels.hip — gfx950 kernels of the batched single-node flip walk.
//
// One 64-lane wavefront owns one chain at a time; a persistent grid of single-wave
// workgroups pulls chains from an atomic counter.  The chain's state lives in LDS
// for the whole launch:
//   lab   packed LB-bit district labels (LB = 4: 0.5 B/node; LB = 8: 1 B/node).  The
//         contiguity search marks visited nodes in place with codes k..k+deg-1.
//   gsum  u16 proposal-weight sum per 64-node group (rank/select level 1)
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

#include <cstdio>
#include <cstdlib>

#include "fw_device.h"

#ifdef FW_STAMPS
// Diagnostic build only (libflipwalk_stamps.so): per-phase s_memtime shares of the
// one-chain-per-wave kernel (scripts/stamps.py --csr).
__device__ unsigned long long g_stamps_csr[24];
#define CSTAMP_DECL uint64_t st_acc[24] = {}; uint64_t st_t0 = 0;
#define CSTAMP(i)                                             \
  do {                                                        \
    __builtin_amdgcn_sched_barrier(0);                        \
    uint64_t st_t1;                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t1)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                        \
    if (i >= 0) st_acc[(i) < 0 ? 0 : (i)] += st_t1 - st_t0;   \
    st_t0 = st_t1;                                            \
  } while (0)
#define CSTAMP_COUNT(i, v) st_acc[i] += (uint64_t)(v)
#define CSTAMP_FLUSH                                          \
  if (__lane_id() == 0)                                       \
    for (int i_ = 0; i_ < 24; ++i_) atomicAdd(&g_stamps_csr[i_], (unsigned long long)st_acc[i_]);
#else
#define CSTAMP_DECL
#define CSTAMP(i)
#define CSTAMP_COUNT(i, v)
#define CSTAMP_FLUSH
#endif

namespace {

// ---------------------------------------------------------------- the chain kernel
// WPE: waves per SIMD the register budget targets (5 only where LDS admits 20 chains per CU)
// FULL = false: the lean instantiation for the common configuration (cut_accept, no
// spatial maps, ring observable, bound schedule or trace), as in fw_grid16_kernel
// WB: 2-bit per-node weights in LDS (padded rows, pairs proposals; FwRunParams::wb)
template <int LB, bool GRID, int MODE, int PER, bool E16, int WPE = 4, bool FULL = true, bool WB = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void fw_run_kernel(FwRunParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID, E16> C;
  C.g = p.g;
  LDS uint8_t* const sm = (LDS uint8_t*)smem;
  C.lab = sm;
  C.gsum = reinterpret_cast<LDS uint16_t*>(sm + p.off_gsum);
  C.wts = reinterpret_cast<LDS uint32_t*>(sm + p.off_w);
  C.list = reinterpret_cast<LDS uint32_t*>(sm + p.off_list);
  C.spill = (GLB uint32_t*)(p.spill + (size_t)blockIdx.x * (size_t)p.g.n);
  C.gscr = LB == 5 && p.gscr ? (GLB uint32_t*)(p.gscr + (size_t)blockIdx.x * (size_t)p.gscr_words) : nullptr;
  C.qcap = p.qcap;
  C.scap = min(128, (p.off_list - p.off_gsum) / 4);
  C.k = p.k;
  C.bb = true;
  C.bb = !p.no_bb;
  C.init_roles();
  const int lane = C.lane;
  const int n = p.g.n;
  const int D = p.g.maxdeg;
  const int G = p.G;
  const int k = p.k;
  const uint32_t key0 = (uint32_t)p.seed, key1 = (uint32_t)(p.seed >> 32);
  __shared__ int32_t s_chain;
  CSTAMP_DECL

  // Work units: chain x slice of the launch's steps, handed out slice-major (unit u =
  // slice u / n_chains of chain u % n_chains; p.slices = 1: whole chains), as in
  // fw_grid16_kernel: with more chains than resident waves the host picks the slice count
  // that ends the launch on a full residency round (C5 shard: 8,192 chains x 5 = 16 rounds
  // of 2,560 waves instead of 3.2).  A slice waits for its chain's previous one (seg_done,
  // agent-scope release / acquire); the trajectory equals separate launches of the slices.
  for (;;) {
    if (lane == 0) s_chain = atomicAdd(p.next_chain, 1);
    __syncthreads();
    const int u = rfl(s_chain);
    if (u >= p.n_chains * p.slices) break;
    const int seg = u / p.n_chains;
    const int c = u - seg * p.n_chains;
    const int64_t ustep = p.steps * (seg + 1) / p.slices - p.steps * seg / p.slices;
    if (seg > 0) {
      for (;;) {
        const int done =
            rfl(__hip_atomic_load(p.seg_done + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (done >= seg) break;
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    const uint64_t gid = (uint64_t)(p.chain_id0 + c);

    // ---- load state (with a valid derived-state cache the group sums that follow the
    // labels in the chain's record come along: FwRunParams::lab_copy16)
    const bool cached = p.gcache_ok != 0 || seg > 0;
    // the per-lane addresses of the chain's records from an opaque lane id, here and at the
    // write-back: hoisted to the kernel entry they were 64-bit pointers held across the unit
    // loop, and spilled (C4 20 B, C5 28 B of scratch per lane)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    {
      const u32x4* src = reinterpret_cast<const u32x4*>(p.labels + (size_t)c * p.lab_stride);
      LDS u32x4* dst = reinterpret_cast<LDS u32x4*>(C.lab);
      const int nv = cached ? p.lab_copy16 : p.lab_bytes / 16;
      for (int i = ln; i < nv; i += WAVE) dst[i] = src[i];
    }
    int64_t pops = ln < k ? p.pops[(size_t)c * k + ln] : 0;  // lane d holds district d
    double thr_l = ln < 2 * D + 1 ? p.thr[(size_t)c * p.thr_stride + ln] : 0.0;
    fw_chain_stats* stp = p.stats + c;
    const uint64_t acc0 = FULL && p.sched ? rfl64(stp->accepts) : 0ull;
    // scheduled bounds: the row of the next proposal's step_num (accepted flips + 1)
    auto sched_row = [&](uint64_t nacc) {
      const int64_t t = (int64_t)(acc0 + nacc) + 1 - p.sched_t0;
      const int64_t r = t < 0 ? 0 : (t >= p.sched_rows ? p.sched_rows - 1 : t);
      if (lane < 2 * D + 1) thr_l = p.sched[r * (2 * D + 1) + lane];
    };
    if (FULL && p.sched) sched_row(0);
    uint64_t attempts = rfl64(stp->attempts);
    const uint64_t yields0 = rfl64(stp->yields);
    int32_t stuck = rfl(stp->stuck);
    int64_t sum_cut = (int64_t)rfl64((uint64_t)stp->sum_cut);
    int64_t sum_bnodes = (int64_t)rfl64((uint64_t)stp->sum_bnodes);
    double sum_invb = stp->sum_invb;  // running total: keeps the oracle's summation order
    // sampled geometric waits (FULL only): the running sum and the current state's draw
    const bool waits_on = FULL && p.wsamp != nullptr;
    double wsum = waits_on ? p.wsamp[2 * (size_t)c] : 0.0;
    double wcur = waits_on ? p.wsamp[2 * (size_t)c + 1] : 0.0;
    // per-launch counters (added to the 64-bit totals at the end), held in VGPRs: the
    // chain's uniform state already fills the scalar file
    uint32_t n_steps = in_vgpr(0), n_acc = in_vgpr(0), n_popf = in_vgpr(0), n_conf = in_vgpr(0);
    uint32_t n_sdeg = in_vgpr(0), n_adeg = in_vgpr(0), n_bchg = in_vgpr(0), n_yield = in_vgpr(0);
    uint64_t n_bfs = in_vgpr64(0), n_bfsn = in_vgpr64(0), n_bfsd = in_vgpr64(0);
    Pend pend = FULL ? pend_load(p, c) : Pend{-1, 0, 0u};
    // boundary_node-flagged nodes of district `lane` (FW_ACCEPT_BOUNDARY)
    int32_t bcnt = FULL && p.accept == FW_ACCEPT_BOUNDARY && ln < k ? p.bcnt[(size_t)c * k + ln] : 0;
    __syncthreads();

    // ---- derive group sums, cut count, boundary count, proposal-set size (unless cached)
    int32_t cut, bnodes, npairs;
    if (cached) {
      cut = rfl(stp->cut);
      bnodes = rfl(stp->bnodes);
      npairs = rfl(stp->npairs);
    } else {
      uint32_t cut2 = 0, bn = 0, np = 0;
      if constexpr (WB) {
        for (int i = ln; i < (n + 15) / 16; i += WAVE) C.wts[i] = 0u;
        lds_order();
      }
      for (int t = 0; t < G; ++t) {
        const int x = t * 64 + lane;
        uint32_t w = 0, cd = 0;
        if (x < n) C.template weight_now<MODE>(x, w, cd);
        if (WB && x < n) __atomic_fetch_or(C.wts + (x >> 4), min(w, 3u) << ((x & 15) << 1), __ATOMIC_RELAXED);
        const uint32_t gsum_t = wave_sum(w);
        if (lane == 0) C.gsum[gsum_slot<PER>(t)] = (uint16_t)gsum_t;  // <= 64 x 63
        cut2 += cd;
        bn += cd > 0;
        np += w;
      }
      cut = (int32_t)(wave_sum(cut2) / 2);
      bnodes = (int32_t)wave_sum(bn);
      npairs = (int32_t)wave_sum(np);
    }
    lds_order();
    double invb = p.g.invb[bnodes];  // 1/|B| from the graph's table (|B| > 0 for k >= 2)

    // district-shape observable: the pair of the first two cut ring edges (ring order),
    // counted per yield in runs (a pair changes only when an accepted flip moves a ring
    // node), flushed to the ring histogram when it changes and at the end of the launch
    const int RN = FULL ? p.ring_n : 0;
    auto ring_pair = [&]() -> int32_t {  // wave-uniform; labels must be clean (no search marks)
      int f = -1, sc = -1;
      for (int b0 = 0; b0 < RN && sc < 0; b0 += WAVE) {
        const int r = b0 + lane;
        const int ri = r < RN ? r : 0;
        uint64_t m = ballot(r < RN && C.L(p.ring_u[ri]) != C.L(p.ring_w[ri]));
        if (m && f < 0) {
          f = b0 + __ffsll((unsigned long long)m) - 1;
          m &= m - 1;
        }
        if (m) sc = b0 + __ffsll((unsigned long long)m) - 1;
      }
      return sc >= 0 ? f * RN + sc : RN * RN;
    };
    int32_t rpair = RN ? ring_pair() : 0;
    uint32_t rrun = 0;

    // histogram windows: lane i counts value base+i
    uint32_t hc = 0, hb = 0;
    int32_t base_c = max(0, cut - 32), base_b = max(0, bnodes - 32);
    auto observe = [&]() {
      n_yield += 1;
      rrun += 1;
      if (waits_on) wsum += wcur;
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
    if (yields0 == 0 && attempts == 0) {
      if (waits_on) wcur = wait_draw(p.seed, FW_WAIT_T0, gid, p.wlp[bnodes]);
      observe();
    }
    // Philox batches on the VALU: lane l holds the draw of attempt (batch base + l); an
    // attempt reads its four words with v_readlane (no scalar round-key table to spill)
    U4 pb = {0u, 0u, 0u, 0u};
    int bpos = WAVE;

    const bool unit_pop = p.g.pop == nullptr;
  // padded rows without the optional features: the neighbours' rows only on accept
  constexpr bool LAZY = E16 && !GRID && !FULL;
    // wave priority 3 - (level mod 4), the level counting 32nds of the unit's steps: the
    // SIMD's VALU goes to the wave one level behind instead of the oldest (see
    // fw_grid16_kernel), so the waves of the last residency round finish together
    const int psh = p.prio_shift;  // launch_prio_shift (C4 / C5 / Frankengraph +0.4-0.6%)
    const int64_t pstep = ustep >= (int64_t(2) << psh) ? ustep >> psh : 2;
    int64_t pnext = pstep;
    uint32_t plev = 0;
    __builtin_amdgcn_s_setprio(3);
    for (int64_t s = 0; s < ustep && !stuck; ++s) {
      if (s >= pnext) {
        pnext += pstep;
        plev = (plev + 1u) & 3u;
        if (plev == 0) __builtin_amdgcn_s_setprio(3);
        else if (plev == 1) __builtin_amdgcn_s_setprio(2);
        else if (plev == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      int32_t retries = 0;
      int v = 0, dcut = 0, m = 0, nbd = 0, dv = 0;
      uint32_t a = 0, d = 0;
      int64_t pv = 1;
      U4 x;
      typename Ctx<LB, GRID, E16>::Hood h;
      bool valid = false;
      for (;;) {
        CSTAMP(-1);
        // 3-bit grids (C5): the lane id made opaque each attempt, so the lane-derived
        // constants are recomputed in the loop instead of hoisted to the kernel entry and
        // spilled (31 -> 6 VGPRs of scratch, C5 +2.2%; the other instantiations, which do
        // not spill, lose 0.5-3.5% to the recomputation: profiles/r05/opaque_lane/)
        if constexpr (LB == 3 && GRID) asm volatile("" : "+v"(C.lane));
        if (retries >= p.max_retries || npairs == 0) {
          stuck = 1;
          break;
        }
        if (bpos == WAVE) {
          // the per-launch counters that grow with attempts fold into the 64-bit totals
          // long before they can wrap (n_sdeg, the fastest, grows by <= 63 per attempt)
          if (n_sdeg >= p.fold_at) {
            if (lane == 0) {
              stp->pop_fail += n_popf;
              stp->contig_fail += n_conf;
              stp->sum_deg += n_sdeg;
            }
            n_popf = n_conf = n_sdeg = 0;
          }
          const uint64_t t = attempts + (uint64_t)lane;
          pb = philox((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid, (uint32_t)(gid >> 32),
                      in_vgpr(key0), in_vgpr(key1));
          bpos = 0;
        }
        x = U4{rdl(pb.x0, bpos), rdl(pb.x1, bpos), rdl(pb.x2, bpos), rdl(pb.x3, bpos)};
        ++bpos;
        attempts += 1;
        const uint32_t r = scale64(x.x0, x.x1, (uint32_t)npairs);
        uint32_t j = 0;
        CSTAMP(0);  // draw
        C.template select<MODE, PER, WB>(r, G, v, j);
        CSTAMP(1);  // select
        v = rfl(v);
        if (v < 0) {  // internal inconsistency: stop this chain, flag it
          stuck = 2;
          break;
        }
        j = rfl(j);
        // v's population, read before the neighbourhood so the table read (C4: lognormal
        // populations in HBM / L2) overlaps the LDS round trip instead of following it
        pv = unit_pop ? 1 : p.g.pop[v];
        // ---- v's neighbourhood (one LDS round trip)
        // padded rows, lean kernel: v's row and its neighbours' labels only; the neighbours'
        // own rows (their label sets, for the weights of v's neighbourhood) are read when a
        // flip is accepted (C4: 29% of attempts)
        if constexpr (LAZY)
          h = C.gather_ids(v, dv);
        else
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
            // the foreign labels among v's neighbours (DPP OR when they fit 32 bits)
            if (k <= 32)
              mask = wave_or32((isnb && h.lx != a) ? (1u << h.lx) : 0u);
            else
              mask = rfl64(wave_or64((isnb && h.lx != a) ? (1ull << h.lx) : 0ull));
          }
          d = (uint32_t)nth_bit(mask, j);
        }
        const uint64_t am = ballot(isnb && h.lx == a);
        m = __popcll(am);
        nbd = __popcll(ballot(isnb && h.lx == d));
        dcut = m - nbd;
        // ---- population bound (Bounds over the two changed districts)
        const int64_t pa = (int64_t)rdl64((uint64_t)pops, (int)a);
        const int64_t pb = (int64_t)rdl64((uint64_t)pops, (int)d);
        if (pa - pv < p.pop_lo || pb + pv > p.pop_hi) {
          n_popf += 1;
          ++retries;
          CSTAMP(2);
          continue;
        }
        // ---- contiguity (single_flip_contiguous)
        CSTAMP(2);  // gather, target, population
        const bool cg = C.template contiguous<LAZY>(v, a, m, h, am, n_bfs, n_bfsn, n_bfsd);
        CSTAMP(3);  // contiguity
        if (!cg) {
          n_conf += 1;
          ++retries;
          continue;
        }
        valid = true;
        break;
      }
      if (!valid) break;
      n_steps += 1;
      // ---- weights of v's neighbourhood before / after the flip (commit and |B'|)
      uint32_t wo, wn;
      CSTAMP(-1);
      const bool mine = GRID ? lane <= 4 : lane <= dv;
      int plus = 0, minus = 0;
      if constexpr (!LAZY) {
        C.template weights_old_new<MODE>(h, a, d, m, nbd, wo, wn);
        plus = __popcll(ballot(mine && wo == 0 && wn > 0));
        minus = __popcll(ballot(mine && wo > 0 && wn == 0));
      }
      // ---- accept rule (include/flipwalk.h FW_ACCEPT_*)
      bool accepted;
      if (FULL && p.accept == FW_ACCEPT_BOUNDARY) {  // uniform_accept + boundary_condition
        const int32_t fv = p.flags[v] ? 1 : 0;
        const int32_t cnt = bcnt - (lane == (int)a ? fv : 0) + (lane == (int)d ? fv : 0);
        accepted = __popcll(ballot(lane < k && cnt > 0)) >= 2;
      } else {  // cut_accept (grid_chain_sec11.py:171-179) [* |B'|/|B|, :81-110]
        double bound = rdl_f64(thr_l, dcut + D);
        if (FULL && p.accept == FW_ACCEPT_BRATIO)
          bound = bound * ((double)(bnodes + plus - minus) / (double)bnodes);
        accepted = u53(x.x2, x.x3) < bound;
      }
      if (FULL && p.trace && lane == 0) p.trace[(size_t)c * p.steps + s] = accepted ? v * 64 + (int)d : -1;
      if (FULL && accepted && p.m_acc != nullptr) {  // spatial observables: fire-and-forget atomics
        const int64_t t = (int64_t)(yields0 + n_yield);  // index of the new state's yield
        const bool nbl = GRID ? (lane >= 1 && lane <= 4 && h.x >= 0) : (lane >= 1 && lane <= dv);
        if (nbl && (h.lx == a || h.lx == d)) {
          int e;
          if constexpr (GRID) {
            int vr, vc;
            C.divmod(v, vr, vc);
            const int W = p.g.gw, H = p.g.gh;
            e = lane == 1   ? grid_eid_down(vr - 1, vc, W, H)
                : lane == 2 ? grid_eid_right(vr, vc - 1, W, H)
                : lane == 3 ? grid_eid_right(vr, vc, W, H)
                            : grid_eid_down(vr, vc, W, H);
          } else {
            e = p.g.eid[p.g.rowptr[v] + lane - 1];
          }
          map_edge(p, c, e, h.lx == a, t);
        }
        if (lane == 0) map_run_end(p, c, pend, t);
        pend = Pend{v, (int32_t)d, (uint32_t)t};
      }
      if (accepted) {
        if constexpr (LAZY) {
          int dv2;
          h = C.gather(v, dv2);
          C.template weights_old_new<MODE>(h, a, d, m, nbd, wo, wn);
          plus = __popcll(ballot(mine && wo == 0 && wn > 0));
          minus = __popcll(ballot(mine && wo > 0 && wn == 0));
        }
        n_acc += 1;
        if (FULL && p.sched) sched_row(n_acc);
        n_adeg += (uint32_t)dv;
        if (lane == 0) PK<LB>::axor(C.lab, v, a ^ d);
        if (mine && h.x >= 0 && wn != wo) {
          // u16 slot inside its u32 word: a wrapping 32-bit add of the shifted delta changes
          // only that half (both halves stay in [0, 65535])
          const int sl = gsum_slot<PER>(h.x >> 6);
          lds_add(reinterpret_cast<LDS uint32_t*>(C.gsum) + (sl >> 1), (wn - wo) << (16 * (sl & 1)));
          if constexpr (WB) {
            const uint32_t so = min(wo, 3u), sn = min(wn, 3u);
            if (so != sn)
              __atomic_fetch_xor(C.wts + (h.x >> 4), (so ^ sn) << ((h.x & 15) << 1), __ATOMIC_RELAXED);
          }
        }
        lds_order();
        npairs += (int32_t)wave_sum(mine ? wn - wo : 0u);
        cut += dcut;
        bnodes += plus - minus;
        n_bchg += (uint32_t)(plus + minus);
        // 1/|B| by the IEEE double division (= the host table and the oracle's 1.0/b):
        // ~150 cycles of fp64 ops instead of an exposed L2 round trip to the table
        if (plus | minus) invb = 1.0 / (double)max(bnodes, 1);
        if (lane == (int)a) pops -= pv;
        if (lane == (int)d) pops += pv;
        if (FULL && p.accept == FW_ACCEPT_BOUNDARY && p.flags[v]) {
          if (lane == (int)a) bcnt -= 1;
          if (lane == (int)d) bcnt += 1;
        }
        // the new state's wait draw (its proposal was attempt `attempts` - 1)
        if (waits_on) wcur = wait_draw(p.seed, attempts - 1, gid, p.wlp[bnodes]);
        if (RN && p.ring_node[v]) {  // only a flip of a ring node can change the pair
          const int32_t np2 = ring_pair();
          if (np2 != rpair) {
            if (lane == 0 && rrun) atomicAdd(p.hist_ring + rpair, (unsigned long long)rrun);
            rrun = 0;
            rpair = np2;
          }
        }
      }
      CSTAMP(4);  // outcome, accept, commit
      observe();
      CSTAMP(5);  // observe
    }

    // ---- write back
    if (hc) atomicAdd(p.hist_cut + base_c + lane, (unsigned long long)hc);
    if (hb) atomicAdd(p.hist_b + base_b + lane, (unsigned long long)hb);
    if (RN && lane == 0 && rrun) atomicAdd(p.hist_ring + rpair, (unsigned long long)rrun);
    {
      int lw = lane;
      asm volatile("" : "+v"(lw));
      u32x4* dst = reinterpret_cast<u32x4*>(p.labels + (size_t)c * p.lab_stride);
      const LDS u32x4* src = reinterpret_cast<const LDS u32x4*>(C.lab);
      for (int i = lw; i < p.lab_copy16; i += WAVE) dst[i] = src[i];  // labels + group sums
      if (lw < k) p.pops[(size_t)c * k + lw] = pops;
      if (FULL && lw < k && p.accept == FW_ACCEPT_BOUNDARY) p.bcnt[(size_t)c * k + lw] = bcnt;
    }
    if (FULL && lane == 0 && p.m_acc != nullptr) pend_store(p, c, pend);
    if (waits_on && lane == 0) {
      p.wsamp[2 * (size_t)c] = wsum;
      p.wsamp[2 * (size_t)c + 1] = wcur;
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
    if (seg + 1 < p.slices) {  // hand the chain to its next slice
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every lane, one word
      __hip_atomic_store(p.seg_done + c, seg + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
#ifdef FW_STAMPS
  CSTAMP_COUNT(8, C.n_win);
  CSTAMP_COUNT(9, C.n_bbs);
  CSTAMP_COUNT(10, C.n_list);
  CSTAMP_COUNT(11, C.c_win);
  CSTAMP_COUNT(12, C.c_bbs);
  CSTAMP_COUNT(13, C.c_list);
  CSTAMP_COUNT(6, C.n_lvl);
  CSTAMP_COUNT(7, C.n_seed);
  CSTAMP_COUNT(14, C.c_clear);
  CSTAMP_COUNT(15, C.n_mapt);
  CSTAMP_COUNT(16, C.n_lv_mid);
  CSTAMP_COUNT(17, C.n_lv_64);
  CSTAMP_COUNT(18, C.n_bb4);
  CSTAMP_COUNT(19, C.c_bb4);
#endif
  CSTAMP_FLUSH
}

// ---------------------------------------------------------------- per-flip evaluation
template <int LB, bool GRID>
__global__ __launch_bounds__(64) void fw_eval_kernel(FwEvalParams p) {
  extern __shared__ __align__(16) uint8_t smem[];
  Ctx<LB, GRID> C;
  C.g = p.g;
  LDS uint8_t* const sm = (LDS uint8_t*)smem;
  C.lab = sm;
  C.gsum = nullptr;
  C.list = reinterpret_cast<LDS uint32_t*>(sm + p.off_list);
  C.spill = (GLB uint32_t*)(p.spill + (size_t)blockIdx.x * (size_t)p.g.n);
  C.qcap = p.qcap;
  C.scap = 0;  // 4- and 8-bit labels only: race_search_b3 is not instantiated
  C.k = p.k;
  C.bb = true;
  C.init_roles();
  const int lane = C.lane;
  for (int i = blockIdx.x; i < p.m; i += gridDim.x) {
    {
      const u32x4* src = reinterpret_cast<const u32x4*>(p.labels);
      LDS u32x4* dst = reinterpret_cast<LDS u32x4*>(C.lab);
      for (int t = lane; t < p.lab_bytes / 16; t += WAVE) dst[t] = src[t];
    }
    __syncthreads();
    const int v = p.v[i];
    const uint32_t b = (uint32_t)p.target[i];
    int dv = 0;
    const auto h = C.gather(v, dv);
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

// ---------------------------------------------------------------- spatial-observable maps
__device__ __forceinline__ uint32_t glabel(const uint8_t* lab, int lb, int x) {
  const int bit = x * lb;  // a 3-bit field may straddle two bytes (the region is padded)
  const uint32_t v = (uint32_t)lab[bit >> 3] | ((uint32_t)lab[(bit >> 3) + 1] << 8);
  return (v >> (bit & 7)) & ((1u << lb) - 1u);
}

// part_sum := label value of the initial plan (grid_chain_sec11.py:219); pending runs none
__global__ void fw_map_init_kernel(FwRunParams p, int lb) {
  const size_t total = (size_t)p.n_chains * (size_t)p.g.n;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t c = i / (size_t)p.g.n;
    const int x = (int)(i - c * (size_t)p.g.n);
    p.m_ps[i] = p.m_labval[glabel(p.labels + c * p.lab_stride, lb, x)];
    if (x == 0) {
      p.m_pend[4 * c] = -1;
      p.m_pend[4 * c + 1] = 0;
      p.m_pend[4 * c + 2] = 0;
      p.m_pend[4 * c + 3] = 0;
    }
  }
}

// Maps current through each chain's last yield Y: open cut intervals and the pending run
// of the current state's creating flip are closed at Y - 1 (without changing the state).
__global__ void fw_map_read_kernel(FwMapRead m) {
  const int M = m.what == FW_MAP_CUT_TIMES ? m.E : m.n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
    int64_t total = 0;
    for (int cc = 0; cc < m.n_chains; ++cc) {
      const size_t c = (size_t)(m.chain0 + cc);
      const int64_t Y = (int64_t)m.stats[c].yields;
      const uint8_t* lab = m.labels + c * m.lab_stride;
      int64_t val;
      if (m.what == FW_MAP_CUT_TIMES) {
        const bool cut = glabel(lab, m.lb, m.eu[i]) != glabel(lab, m.lb, m.ew[i]);
        val = m.acc[c * m.E + i] + (cut ? Y : 0);
      } else {
        const int32_t* pe = m.pend + 4 * c;
        int64_t nf = m.nf[c * m.n + i], lf = m.lf[c * m.n + i], ps = m.ps[c * m.n + i];
        if (pe[0] == i && Y > (int64_t)(uint32_t)pe[2]) {  // pending run [t0, Y-1]
          nf += Y - (int64_t)(uint32_t)pe[2];
          ps -= m.labval[pe[1]] * ((Y - 1) - lf);
          lf = Y - 1;
        }
        if (m.what == FW_MAP_NUM_FLIPS) {
          val = nf;
        } else if (m.what == FW_MAP_LAST_FLIPPED) {
          val = lf;
        } else {
          val = ps;  // grid_chain_sec11.py:416-419
          if (m.finalize && lf == 0) val = Y * m.labval[glabel(lab, m.lb, i)];
        }
      }
      if (m.sum)
        total += val;
      else
        m.out[(size_t)cc * M + i] = val;
    }
    if (m.sum) m.out[i] = total;
  }
}

}  // namespace

#ifdef FW_STAMPS
extern "C" int fw_debug_stamps_csr(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_csr), sizeof(unsigned long long) * 24) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[24] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_csr), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// group sums per lane of the one-chain-per-wave kernel (pick_per) and the u16 LDS slots
// its padded level-1 layout (gsum_slot) takes for G groups
int fw_run_per(int G) {
  return G <= 64 * 2 ? 2 : G <= 64 * 4 ? 4 : G <= 64 * 8 ? 8 : G <= 64 * 10 ? 10 : 16;
}
int fw_run_gsum_slots(int G) {
  const int per = fw_run_per(G);
  return G <= 0 ? 0 : ((G - 1) / per) * (2 * gsum_stride_dw(per)) + (G - 1) % per + 1;
}

namespace {

template <int LB, bool GRID, int MODE, bool E16, int WPE = 4, bool FULL = true, bool WB = false>
void* pick_per(int G) {
  switch (fw_run_per(G)) {
    case 2: return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 2, E16, WPE, FULL, WB>);
    case 4: return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 4, E16, WPE, FULL, WB>);
    case 8: return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 8, E16, WPE, FULL, WB>);
    case 10: return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 10, E16, WPE, FULL, WB>);
    default: return reinterpret_cast<void*>(&fw_run_kernel<LB, GRID, MODE, 16, E16, WPE, FULL, WB>);
  }
}

// padded rows, pairs proposals (4- or 5-bit labels): with or without the LDS weights
template <int LB, int WPE, bool FULL>
void* pick_e16_pairs(int G, bool wb) {
  return wb ? pick_per<LB, false, 1, true, WPE, FULL, true>(G) : pick_per<LB, false, 1, true, WPE, FULL>(G);
}

template <bool FULL>
void* pick_run_t(int lb, bool grid, bool e16, int mode, int G, bool wpe5, bool wb) {
  const bool cut = mode == FW_PROPOSE_CUTEDGE;
  if (lb == 4) {
    // small general graphs (4-bit labels, padded rows): a 5-waves-per-SIMD register budget
    if (!grid && e16 && wpe5)
      return cut ? pick_per<4, false, 2, true, 5, FULL>(G) : pick_e16_pairs<4, 5, FULL>(G, wb);
    if (grid) return cut ? pick_per<4, true, 2, false, 4, FULL>(G) : pick_per<4, true, 1, false, 4, FULL>(G);
    if (e16) return cut ? pick_per<4, false, 2, true, 4, FULL>(G) : pick_e16_pairs<4, 4, FULL>(G, wb);
    return cut ? pick_per<4, false, 2, false, 4, FULL>(G) : pick_per<4, false, 1, false, 4, FULL>(G);
  }
  if (lb == 5)  // general graphs with padded rows, 16 <= k <= 31 (fw_chains_create)
    return !grid && e16 ? (wpe5 ? (cut ? pick_per<5, false, 2, true, 5, FULL>(G) : pick_e16_pairs<5, 5, FULL>(G, wb))
                                : (cut ? pick_per<5, false, 2, true, 4, FULL>(G) : pick_e16_pairs<5, 4, FULL>(G, wb)))
                        : nullptr;
  if (lb == 3)  // grids, k <= 8 (the large-grid LDS plan: fw_chains_create)
    return grid ? (cut ? pick_per<3, true, 2, false, 3, FULL>(G) : pick_per<3, true, 1, false, 3, FULL>(G))
                : nullptr;  // <= 3 waves per SIMD: LDS holds 9 chains per CU
  if (grid) return cut ? pick_per<8, true, 2, false, 4, FULL>(G) : pick_per<8, true, 1, false, 4, FULL>(G);
  if (e16) return cut ? pick_per<8, false, 2, true, 4, FULL>(G) : pick_per<8, false, 1, true, 4, FULL>(G);
  return cut ? pick_per<8, false, 2, false, 4, FULL>(G) : pick_per<8, false, 1, false, 4, FULL>(G);
}

// grids: implicit neighbours; general graphs: the padded 16-wide table when it exists.
// The LDS plan and residency are sized on the FULL instantiation (the optional features
// can be switched on after fw_chains_create); launches take the lean one when they are off.
void* pick_run(int lb, bool grid, bool e16, int mode, int G, bool wpe5 = false, bool full = true,
               bool wb = false) {
  return full ? pick_run_t<true>(lb, grid, e16, mode, G, wpe5, wb)
              : pick_run_t<false>(lb, grid, e16, mode, G, wpe5, wb);
}

}  // namespace

// Occupancy-sized persistent grid for the one-chain-per-wave kernel.
int fw_run_grid_size(FwRunParams& p, int lb, int device, int* grid) {
  if (p.G > 64 * 16) return -2;
  void* fn = pick_run(lb, p.g.gw > 0, p.g.ell != nullptr, p.mode, p.G, false, true, p.wb != 0);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  if (e != hipSuccess) return -1;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, (size_t)p.lds_bytes);
  if (e != hipSuccess || per_cu <= 0) return -1;
  // LDS-bound residency (C5: 23.5 KB per chain, 6 per CU): shorten the LDS visit list,
  // down to 128 entries (longer searches continue in the HBM spill area), when that keeps
  // one more chain per CU; the longest list that reaches the best residency is kept.
  // FLIPWALK_LIST_CAP pins the length (tests of the spill path).
  // With 3- or 5-bit labels the list search (a rare fallback) keeps its marks in HBM or in
  // the labels anyway, and the list may shrink to 8 entries.
  // 4- and 5-bit labels on padded rows also weigh the 5-waves-per-SIMD instantiation (the
  // Frankengraph: 16 -> 20 chains per CU, +4%), taken when it holds more chains per CU; the
  // list length is chosen together with it (C4 with its LDS weights: 17 chains per CU at
  // the 256-entry list, 19 at 8 entries).  FLIPWALK_NO_WPE5=1 keeps the 4-wave budget (A/B).
  const char* cap_env = getenv("FLIPWALK_LIST_CAP");
  const int q_min = lb == 3 || lb == 5 ? 8 : 128;
  const char* no5 = getenv("FLIPWALK_NO_WPE5");
  void* fn5 = (lb == 4 || lb == 5) && p.g.gw == 0 && p.g.ell != nullptr && !(no5 && no5[0] == '1')
                  ? pick_run(lb, false, true, p.mode, p.G, true, true, p.wb != 0)
                  : nullptr;
  auto occ = [&](void* f, int lds, int& pc) -> bool {
    pc = 0;
    return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
           hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, f, 64, (size_t)lds) == hipSuccess;
  };
  {
    const bool pinned = (cap_env && cap_env[0]) || p.qcap <= q_min;
    const int base = p.off_list;
    int best_q = p.qcap, best = 0;
    bool best5 = false;
    for (int q = p.qcap; q >= (pinned ? p.qcap : q_min); q -= 8) {
      const int lds = base + 4 * q;
      int pc4 = 0, pc5 = 0;
      if (!occ(fn, lds, pc4)) return -1;
      if (fn5 && !occ(fn5, lds, pc5)) return -1;
      if (pc4 > best) {
        best = pc4;
        best_q = q;
        best5 = false;
      }
      if (pc5 > best) {
        best = pc5;
        best_q = q;
        best5 = true;
      }
    }
    if (best <= 0) return -1;
    p.qcap = best_q;
    p.lds_bytes = base + 4 * best_q;
    p.wpe5 = best5 ? 1 : 0;
    per_cu = best;
    int dummy = 0;
    if (!occ(fn, p.lds_bytes, dummy) || (fn5 && !occ(fn5, p.lds_bytes, dummy))) return -1;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const char* verbose = getenv("FLIPWALK_VERBOSE");
  if (verbose && verbose[0] == '1')
    fprintf(stderr, "flipwalk: chain kernel LDS %d B (list %d), %d chains per CU\n", p.lds_bytes,
            p.qcap, per_cu);
  long long gsz = (long long)per_cu * prop.multiProcessorCount;
  if (gsz > p.n_chains) gsz = p.n_chains;
  *grid = (int)(gsz < 1 ? 1 : gsz);
  return 0;
}

void* fw_run_fn(const FwRunParams& p, int lb) {
  const bool full = p.m_acc != nullptr || p.accept != FW_ACCEPT_CUT || p.sched != nullptr ||
                    p.ring_n > 0 || p.trace != nullptr || p.wsamp != nullptr;
  return pick_run(lb, p.g.gw > 0, p.g.ell != nullptr, p.mode, p.G, p.wpe5 != 0, full, p.wb != 0);
}

int fw_launch_run(const FwRunParams& p, int lb, int grid, void* stream) {
  if (p.use16) return fw_grid16_launch(p, grid, stream);
  void* fn = fw_run_fn(p, lb);
  // handles of different graphs share instantiations: set this handle's LDS size
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  if (e != hipSuccess) return (int)e;
  void* args[] = {const_cast<FwRunParams*>(&p)};
  return (int)hipLaunchKernel(fn, dim3(grid), dim3(64), args, (size_t)p.lds_bytes,
                              (hipStream_t)stream);
}

// flagged nodes per district of every chain's current plan (FW_ACCEPT_BOUNDARY)
__global__ void fw_bcnt_init_kernel(FwRunParams p, int lb) {
  const size_t total = (size_t)p.n_chains * (size_t)p.g.n;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t c = i / (size_t)p.g.n;
    const int x = (int)(i - c * (size_t)p.g.n);
    if (p.flags[x]) atomicAdd(p.bcnt + c * p.k + glabel(p.labels + c * p.lab_stride, lb, x), 1);
  }
}

// Launchers return the hipError_t of the launch itself (0 = hipSuccess).
int fw_launch_bcnt_init(const FwRunParams& p, void* stream) {
  int lb = p.lb;
  void* args[] = {const_cast<FwRunParams*>(&p), &lb};
  return (int)hipLaunchKernel(reinterpret_cast<void*>(&fw_bcnt_init_kernel), dim3(2048), dim3(256),
                              args, 0, (hipStream_t)stream);
}

int fw_launch_map_init(const FwRunParams& p, void* stream) {
  int lb = p.lb;
  void* args[] = {const_cast<FwRunParams*>(&p), &lb};
  return (int)hipLaunchKernel(reinterpret_cast<void*>(&fw_map_init_kernel), dim3(2048), dim3(256),
                              args, 0, (hipStream_t)stream);
}

int fw_launch_map_read(const FwMapRead& m, void* stream) {
  const int M = m.what == FW_MAP_CUT_TIMES ? m.E : m.n;
  const int blocks = (M + 255) / 256;
  void* args[] = {const_cast<FwMapRead*>(&m)};
  return (int)hipLaunchKernel(reinterpret_cast<void*>(&fw_map_read_kernel), dim3(blocks),
                              dim3(256), args, 0, (hipStream_t)stream);
}

int fw_launch_eval(const FwEvalParams& p, int lb, int grid, void* stream) {
  void* fn;
  if (lb == 4)
    fn = p.g.gw > 0 ? reinterpret_cast<void*>(&fw_eval_kernel<4, true>)
                    : reinterpret_cast<void*>(&fw_eval_kernel<4, false>);
  else
    fn = p.g.gw > 0 ? reinterpret_cast<void*>(&fw_eval_kernel<8, true>)
                    : reinterpret_cast<void*>(&fw_eval_kernel<8, false>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  if (e != hipSuccess) return (int)e;
  void* args[] = {const_cast<FwEvalParams*>(&p)};
  return (int)hipLaunchKernel(fn, dim3(grid), dim3(64), args, (size_t)p.lds_bytes,
                              (hipStream_t)stream);
}
