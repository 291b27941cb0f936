/*
 * flipchain_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded CPU restatement of the GerryChain single-node
 * flip walk that drdeford/FlipComplexityEmpirical runs.  It is the checker
 * for the HIP product path (libflipwalk.so) and the native CPU baseline.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product never links or calls it.
 *
 * What it restates (reference = /root/reference, [ext] = GerryChain 0.2.x,
 * which is not vendored and not installed; its behaviour is restated from the
 * reference's call sites):
 *   chain loop      MarkovChain.__next__ [ext], built grid_chain_sec11.py:340-342:
 *                   invalid proposals are retried without counting; valid ones
 *                   are Metropolis-accepted or rejected and counted; the current
 *                   state is yielded once per counted step, the initial state once.
 *   proposals       slow_reversible_propose_bi     grid_chain_sec11.py:132-145
 *                   slow_reversible_propose + b_nodes grid_chain_sec11.py:117-130,151-153
 *                   propose_random_flip [ext]       imported grid_chain_sec11.py:24
 *   constraints     single_flip_contiguous [ext] (old district minus v connected and
 *                   non-empty) and within_percent_of_ideal_population [ext]
 *                   (grid_chain_sec11.py:319) as integer bounds [ceil(lo), floor(hi)]
 *   accept          cut_accept grid_chain_sec11.py:171-179: random() < base**(c_old-c_new),
 *                   with the bound pre-tabulated per Δcut by the host (same pow).
 *   updaters        cut_edges [ext], Tally [ext], b_nodes_bi :155-156
 *   observables     rce/rbn/waits grid_chain_sec11.py:367-369 (sums over yields),
 *                   histograms of |cut| and |B| over yields
 *
 * Parity status: parity of the chain law against the reference itself is
 * pinned statistically (New_plots/sec11/{a}B{b}P{p}wait.txt, tests/test_oracle_pins.py);
 * per-step verdicts are pinned against networkx ground truth on grids and the
 * Kansas dual graphs (tests/golden).  The unseeded MT19937 stream of the
 * reference cannot be replayed; the oracle uses the canonical Philox mapping
 * documented in include/flipwalk.h, so the HIP path must match it bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/flipwalk.h"

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al., SC'11), the Random123 reference constants.   */
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

static void draw(uint64_t seed, uint64_t attempt, uint64_t chain, uint32_t x[4]) {
  uint32_t ctr[4] = {(uint32_t)attempt, (uint32_t)(attempt >> 32), (uint32_t)chain,
                     (uint32_t)(chain >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(ctr, key, x);
}

/* floor(x * P / 2^64) for a 64-bit x, exactly. */
uint32_t orc_scale64(uint32_t x0, uint32_t x1, uint32_t P) {
  uint64_t lo = (uint64_t)x0 * P;
  uint64_t hi = (uint64_t)x1 * P + (lo >> 32);
  return (uint32_t)(hi >> 32);
}

/* CPython random.random() from two 32-bit words. */
double orc_u53(uint32_t x2, uint32_t x3) {
  return ((double)(x2 >> 5) * 67108864.0 + (double)(x3 >> 6)) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------- */
typedef struct {
  int32_t n, nnz, maxdeg, grid_w, grid_h;
  const int32_t* rowptr;
  const int32_t* col;
  const int64_t* pop; /* NULL = all ones */
} graph_t;

/* Sampled geometric waits (geom_wait, grid_chain_sec11.py:147-148, read per yield at :368,
 * summed and written at :410-411): int(np.random.geometric(len(b_nodes)/(N**k - 1))) - 1,
 * drawn ONCE per state object and re-used when a Metropolis rejection re-yields it (the
 * Partition caches updater values).  Restated as one inversion draw per state: the state
 * created by proposal attempt t of chain g (the initial state: t = 2^63 - 1) draws the
 * Philox block key = seed, ctr = (lo32(t), hi32(t) | 2^31, lo32(g), hi32(g)) and takes
 * u = CPython random() of its words (x0, x1); then wait = floor(log1p(-u) / lp[|B|]) with
 * lp[b] = log1p(-b/(N^k - 1)) (the geometric's number of failures, P(wait >= w) =
 * (1-p)^w).  log1p is orc_log1p below, operation for operation the kernels' fw_log1p
 * (flipcomplexityempirical_amd/csrc/fw_math.h), so the draws are bit-identical.  For
 * p below 2^-52 (k >= 5 on large graphs) the reference's int64 draw overflows; this
 * fp64 inversion does not (the value is then ~ -log(1-u)/p). */
typedef struct orc_waits {
  const double* lp; /* [n+1] log1p(-p_b), p_b = b/(N^k - 1) as the reference divides */
  double sum;       /* sum over yields of the current state's draw */
  double cur;       /* the current state's draw */
} orc_waits;

typedef struct {
  graph_t g;
  int32_t k, mode;
  int64_t pop_lo, pop_hi;
  const double* thr; /* [2*maxdeg+1] */
  uint64_t seed, chain;
  int16_t* lab;  /* [n] */
  int32_t* w;    /* [n] proposal weight per node */
  int64_t* fen;  /* Fenwick tree over w, 1-based, [n+1] */
  int64_t* pops; /* [k] */
  /* search scratch */
  int32_t* owner; /* [n], -1 unvisited */
  int32_t* list;  /* [n] */
  fw_chain_stats st;
  uint64_t* hist_cut; /* may be NULL */
  uint64_t* hist_b;   /* may be NULL */
  struct orc_maps* maps; /* may be NULL */
  const struct orc_ring* ring; /* may be NULL */
  int32_t accept_rule;   /* FW_ACCEPT_* */
  const double* sched;   /* fw_chains_set_schedule rows [sched_rows][2*maxdeg+1] or NULL */
  int32_t sched_rows;
  int64_t sched_t0;
  const uint8_t* flags;  /* [n] boundary_node flags (FW_ACCEPT_BOUNDARY), may be NULL */
  int64_t* bcnt;         /* [k] flagged nodes per district */
  orc_waits* waits;      /* sampled geometric waits, may be NULL */
} chain_t;

/* log1p for -1 < x <= 0 by the classic reduction 1 + x = 2^k m, m in [sqrt(2)/2, sqrt(2)),
 * log m = 2 atanh(f / (2 + f)) (f = m - 1) by a degree-14 odd series, plus the rounding
 * correction of 1 + x; every operation IEEE double, no fused multiply-add. */
double orc_log1p(double x) {
  if (x == 0.0) return x;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  const double u = 1.0 + x;
  uint64_t bits;
  memcpy(&bits, &u, 8);
  int k = (int)((bits >> 52) & 0x7FF) - 1023;
  uint64_t mb = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
  if (mb > 0x3FF6A09E667F3BCCull) { /* m >= sqrt(2): halve it */
    mb -= 0x0010000000000000ull;
    k += 1;
  }
  double m;
  memcpy(&m, &mb, 8);
  double c = k > 0 ? 1.0 - (u - x) : x - (u - 1.0);
  c = c / u;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

#define ORC_WAIT_T0 0x7FFFFFFFFFFFFFFFull /* attempt index of the initial state's draw */

/* the sampled wait of the state created by attempt t (|B| = b) */
static double wait_draw(const chain_t* c, uint64_t t, int32_t b) {
  uint32_t ctr[4] = {(uint32_t)t, (uint32_t)(t >> 32) | 0x80000000u, (uint32_t)c->chain,
                     (uint32_t)(c->chain >> 32)};
  uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
  uint32_t x[4];
  orc_philox4x32_10(ctr, key, x);
  const double lu = orc_log1p(-orc_u53(x[0], x[1]));
  const double lp = c->waits->lp[b];
  return lu == 0.0 ? 0.0 : floor(lu / lp);
}

/* The reference driver's spatial observables, updated once per yield exactly as
 * grid_chain_sec11.py:383-384 and :396-400 do (Frankenstein_chain.py:413-425 and
 * All_States_Chain.py:334-342 are the same code):
 *   for edge in part["cut_edges"]: cut_times[edge] += 1
 *   if part.flips is not None:     f = the node of the state's creating flip
 *       part_sum[f] -= assignment[f] * (t - last_flipped[f]); last_flipped[f] = t;
 *       num_flips[f] += 1
 * where t is the yield index (0 = initial state, whose flips is None) and a state
 * re-yielded after a Metropolis rejection keeps its creating flip.  Edges are indexed in
 * canonical order (u < w, CSR row order); assignment values come from label_value[k]. */
typedef struct orc_maps {
  int64_t* cut_times;        /* [n_edges] */
  int64_t* num_flips;        /* [n] */
  int64_t* part_sum;         /* [n], initialised by the caller to label_value[initial] */
  int64_t* last_flipped;     /* [n] */
  const int64_t* label_value; /* [k] */
  int32_t cur_f;             /* creating flip of the current state, -1: none (initial) */
  int32_t pad;
} orc_maps;

/* The district-shape observable of boundary_slope (grid_chain_sec11.py:55-78) and the
 * driver's slope/angle block (:371-394): once per yield, the pair (i, j), i < j, of the
 * first two cut ring edges in ring order, counted in hist[i*n_ring + j] (hist[n_ring^2]:
 * fewer than two).  Ring edge r joins u[r] and w[r].  A literal per-yield scan. */
typedef struct orc_ring {
  const int32_t* u;
  const int32_t* w;
  int32_t n_ring, pad;
  uint64_t* hist; /* [n_ring*n_ring + 1] */
} orc_ring;

static inline int64_t popof(const graph_t* g, int32_t v) { return g->pop ? g->pop[v] : 1; }

/* weight of node x under the proposal mode */
static int32_t weight(const chain_t* c, int32_t x) {
  const graph_t* g = &c->g;
  int16_t lx = c->lab[x];
  if (c->mode == FW_PROPOSE_CUTEDGE) {
    int32_t cnt = 0;
    for (int32_t e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) cnt += c->lab[g->col[e]] != lx;
    return cnt;
  }
  /* distinct foreign labels (k may exceed 64: use a small sorted scan) */
  int32_t cnt = 0;
  for (int32_t e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) {
    int16_t l = c->lab[g->col[e]];
    if (l == lx) continue;
    int dup = 0;
    for (int32_t f = g->rowptr[x]; f < e; ++f)
      if (c->lab[g->col[f]] == l) {
        dup = 1;
        break;
      }
    cnt += !dup;
  }
  return cnt;
}

static void fen_add(chain_t* c, int32_t i, int64_t d) {
  for (int32_t x = i + 1; x <= c->g.n; x += x & -x) c->fen[x] += d;
}

/* smallest v with prefix(v+1) > r; returns v and r - prefix(v) */
static int32_t fen_select(const chain_t* c, int64_t r, int64_t* rem) {
  int32_t pos = 0, step = 1;
  while (step * 2 <= c->g.n) step *= 2;
  for (; step; step >>= 1) {
    int32_t nx = pos + step;
    if (nx <= c->g.n && c->fen[nx] <= r) {
      pos = nx;
      r -= c->fen[nx];
    }
  }
  *rem = r;
  return pos; /* 0-based node */
}

static void derive(chain_t* c) {
  const graph_t* g = &c->g;
  memset(c->fen, 0, sizeof(int64_t) * (size_t)(g->n + 1));
  for (int32_t i = 0; i < c->k; ++i) c->pops[i] = 0;
  int64_t cut2 = 0;
  int32_t bn = 0;
  int64_t np = 0;
  for (int32_t x = 0; x < g->n; ++x) {
    c->w[x] = weight(c, x);
    fen_add(c, x, c->w[x]);
    bn += c->w[x] > 0;
    np += c->w[x];
    c->pops[c->lab[x]] += popof(g, x);
    for (int32_t e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) cut2 += c->lab[g->col[e]] != c->lab[x];
  }
  c->st.cut = (int32_t)(cut2 / 2);
  c->st.bnodes = bn;
  c->st.npairs = (int32_t)np;
  for (int32_t i = 0; i < c->k; ++i) c->bcnt[i] = 0;
  if (c->flags)
    for (int32_t x = 0; x < g->n; ++x) c->bcnt[c->lab[x]] += c->flags[x] ? 1 : 0;
}

/* |B| after flipping v -> b (b_nodes_bi of the proposed state) */
static int32_t bnodes_after(chain_t* c, int32_t v, int16_t b) {
  const graph_t* g = &c->g;
  const int16_t a = c->lab[v];
  int32_t before = 0, after = 0;
  for (int32_t e = g->rowptr[v] - 1; e < g->rowptr[v + 1]; ++e) {
    const int32_t x = e < g->rowptr[v] ? v : g->col[e];
    before += c->w[x] > 0;
  }
  c->lab[v] = b;
  for (int32_t e = g->rowptr[v] - 1; e < g->rowptr[v + 1]; ++e) {
    const int32_t x = e < g->rowptr[v] ? v : g->col[e];
    after += weight(c, x) > 0;
  }
  c->lab[v] = a;
  return c->st.bnodes + after - before;
}

/* The accept rule on a valid proposal v -> b with draw u:
 *   FW_ACCEPT_CUT      cut_accept grid_chain_sec11.py:171-179: u < base**(-dcut)
 *   FW_ACCEPT_BRATIO   annealing_cut_accept_backwards :81-110: u < base**(beta*(-dcut))
 *                      * (len(b_nodes') / len(b_nodes)), the power tabulated in thr
 *   FW_ACCEPT_BOUNDARY uniform_accept + boundary_condition :43-52,159-165: u < 1 iff the
 *                      boundary_node-flagged nodes of the proposed plan span >= 2
 *                      districts, else u < 0 */
static int accept_of(chain_t* c, int32_t v, int16_t b, int32_t dcut, double u) {
  const int32_t D = c->g.maxdeg;
  const double* thr = c->thr;
  if (c->sched) { /* step_num of the proposal (grid_chain_sec11.py:282-289) = accepts + 1 */
    const int64_t t = (int64_t)c->st.accepts + 1 - c->sched_t0;
    const int64_t r = t < 0 ? 0 : (t >= c->sched_rows ? c->sched_rows - 1 : t);
    thr = c->sched + r * (2 * D + 1);
  }
  if (c->accept_rule == FW_ACCEPT_BRATIO) {
    const double ratio = (double)bnodes_after(c, v, b) / (double)c->st.bnodes;
    return u < thr[dcut + D] * ratio;
  }
  if (c->accept_rule == FW_ACCEPT_BOUNDARY) {
    const int64_t fv = c->flags && c->flags[v] ? 1 : 0;
    const int16_t a = c->lab[v];
    int32_t parts = 0;
    for (int32_t q = 0; q < c->k; ++q) {
      const int64_t cnt = c->bcnt[q] - (q == a ? fv : 0) + (q == b ? fv : 0);
      parts += cnt > 0;
    }
    return u < (parts >= 2 ? 1.0 : 0.0);
  }
  return u < thr[dcut + D];
}

/* --- contiguity: exact verdict + the same level-synchronous race search the
 *     device runs (so the search counters match too) ------------------------ */
static int32_t uf_find(int32_t* p, int32_t x) {
  while (p[x] != x) x = p[x] = p[p[x]];
  return x;
}

/* Grid fast path: the 8-cell ring around v decides connectivity locally when
 * the a-labelled 4-neighbours lie in one ring run; returns the number of local
 * components and fills the pre-merged union-find over the sources. */
static int32_t grid_ring(const chain_t* c, int32_t v, int16_t a, const int32_t* src, int32_t m,
                         int32_t* uf) {
  const graph_t* g = &c->g;
  int32_t W = g->grid_w, H = g->grid_h;
  int32_t r = v / W, q = v % W;
#define INA(rr, qq) ((rr) >= 0 && (rr) < H && (qq) >= 0 && (qq) < W && c->lab[(rr)*W + (qq)] == a)
  /* 4-neighbours in ring order N, E, S, W and the diagonals between them */
  int32_t nb[4] = {v - W, v + 1, v + W, v - 1};
  int pres[4] = {INA(r - 1, q), INA(r, q + 1), INA(r + 1, q), INA(r, q - 1)};
  int diag[4] = {INA(r - 1, q + 1), INA(r + 1, q + 1), INA(r + 1, q - 1), INA(r - 1, q - 1)};
#undef INA
  for (int32_t i = 0; i < m; ++i) uf[i] = i;
  int32_t links = 0;
  for (int i = 0; i < 4; ++i) {
    int j = (i + 1) & 3;
    if (pres[i] && pres[j] && diag[i]) {
      ++links;
      int32_t si = -1, sj = -1;
      for (int32_t s = 0; s < m; ++s) {
        if (src[s] == nb[i]) si = s;
        if (src[s] == nb[j]) sj = s;
      }
      int32_t ri = uf_find(uf, si), rj = uf_find(uf, sj);
      if (ri != rj) uf[ri] = rj;
    }
  }
  int32_t comps = m - links;
  return comps < 1 ? 1 : comps;
}

/* Grid second-level local test on the 7x7 window centred at v (bit i*7+j, v = bit 24):
 * flood-fill the a-labelled window cells (v excluded) from each of v's a-neighbours.
 * Returns 1 if all of them lie in one window component (connected), 0 if some source's
 * component touches no window border cell (a closed component of A minus v that misses a
 * source: disconnected), -1 otherwise (undecided: the full search decides).  A pure
 * function of the window, implemented identically by the kernels (fw_device.h). */
int orc_window_verdict(uint64_t A) {
  const uint64_t C0 = 0x0040810204081ull;       /* j == 0 */
  const uint64_t C6 = C0 << 6;                  /* j == 6 */
  const uint64_t R0 = 0x7Full, R6 = 0x7Full << 42;
  const uint64_t BORDER = C0 | C6 | R0 | R6;
  const int sbit[4] = {17, 23, 25, 31};         /* up, left, right, down */
  uint64_t src = 0;
  for (int s = 0; s < 4; ++s) src |= A & (1ull << sbit[s]);
  uint64_t covered = 0;
  for (int s = 0; s < 4; ++s) {
    const uint64_t b = 1ull << sbit[s];
    if (!(src & b) || (covered & b)) continue;
    uint64_t x = b;
    for (;;) {
      const uint64_t y = (x | ((x << 1) & ~C0) | ((x >> 1) & ~C6) | (x >> 7) | (x << 7)) & A;
      if (y == x) break;
      x = y;
    }
    if ((x & src) == src) return 1;
    if (!(x & BORDER)) return 0;
    covered |= x;
  }
  return -1;
}

static uint64_t window_mask(const chain_t* c, int32_t v, int16_t a) {
  const int32_t W = c->g.grid_w, H = c->g.grid_h, r = v / W, q = v % W;
  uint64_t A = 0;
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) {
      const int32_t rr = r - 3 + i, cc = q - 3 + j;
      if ((i == 3 && j == 3) || rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
      if (c->lab[rr * W + cc] == a) A |= 1ull << (i * 7 + j);
    }
  return A;
}

static int contiguous_after(chain_t* c, int32_t v, int16_t a, int count) {
  const graph_t* g = &c->g;
  int32_t src[64];
  int32_t uf[64];
  int32_t m = 0;
  for (int32_t e = g->rowptr[v]; e < g->rowptr[v + 1]; ++e)
    if (c->lab[g->col[e]] == a) src[m++] = g->col[e];
  if (m == 0) return 0;
  if (m == 1) return 1;
  if (g->grid_w) {
    if (grid_ring(c, v, a, src, m, uf) == 1) return 1;
    const int wv = orc_window_verdict(window_mask(c, v, a));
    if (wv >= 0) return wv;
  } else {
    /* general graphs: sources joined by a direct edge are one local component; a single
     * component is connected without a search (the kernels test the same links with a
     * per-CSR-entry neighbour bitmask), otherwise the links pre-merge the search */
    for (int32_t i = 0; i < m; ++i) uf[i] = i;
    int32_t comps = m;
    for (int32_t i = 0; i < m; ++i)
      for (int32_t j = i + 1; j < m; ++j) {
        const int32_t* b = g->col + g->rowptr[src[i]];
        const int32_t* e = g->col + g->rowptr[src[i] + 1];
        int32_t lo = 0, hi = (int32_t)(e - b);
        while (lo < hi) { /* src[j] in the (ascending) row of src[i]? */
          const int32_t mid = (lo + hi) / 2;
          if (b[mid] < src[j]) lo = mid + 1; else hi = mid;
        }
        if (lo < (int32_t)(e - b) && b[lo] == src[j]) {
          const int32_t ri = uf_find(uf, i), rj = uf_find(uf, j);
          if (ri != rj) {
            uf[ri] = rj;
            --comps;
          }
        }
      }
    if (comps == 1) return 1;
  }
  if (count) c->st.bfs_runs++;
  int32_t nl = 0;
  for (int32_t i = 0; i < m; ++i) {
    c->owner[src[i]] = i;
    c->list[nl++] = src[i];
  }
  int32_t lvl_b = 0, lvl_e = nl;
  int verdict = -1;
  for (;;) {
    int32_t ncls = 0;
    for (int32_t i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
    if (ncls == 1) {
      verdict = 1;
      break;
    }
    for (int32_t li = lvl_b; li < lvl_e; ++li) {
      int32_t x = c->list[li];
      if (count) {
        c->st.bfs_nodes++;
        c->st.bfs_deg += (uint64_t)(g->rowptr[x + 1] - g->rowptr[x]);
      }
      for (int32_t e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) {
        int32_t y = g->col[e];
        if (y == v || c->lab[y] != a) continue;
        if (c->owner[y] < 0) {
          c->owner[y] = c->owner[x];
          c->list[nl++] = y;
        } else {
          int32_t rx = uf_find(uf, c->owner[x]), ry = uf_find(uf, c->owner[y]);
          if (rx != ry) uf[rx] = ry;
        }
      }
    }
    lvl_b = lvl_e;
    lvl_e = nl;
    ncls = 0;
    for (int32_t i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
    if (ncls == 1) {
      verdict = 1;
      break;
    }
    /* a class with no node in the next level is a closed component */
    uint64_t present = 0; /* m <= 64 */
    for (int32_t li = lvl_b; li < lvl_e; ++li) present |= 1ull << uf_find(uf, c->owner[c->list[li]]);
    int exhausted = 0;
    for (int32_t i = 0; i < m; ++i)
      if (uf_find(uf, i) == i && !((present >> i) & 1)) exhausted = 1;
    if (exhausted) {
      verdict = 0;
      break;
    }
  }
  for (int32_t li = 0; li < nl; ++li) c->owner[c->list[li]] = -1;
  return verdict;
}

/* Proposal target for node v with in-node index j (canonical order). */
static int16_t target_of(const chain_t* c, int32_t v, int64_t j) {
  const graph_t* g = &c->g;
  int16_t a = c->lab[v];
  if (c->mode == FW_PROPOSE_CUTEDGE) {
    for (int32_t e = g->rowptr[v]; e < g->rowptr[v + 1]; ++e) {
      int16_t l = c->lab[g->col[e]];
      if (l != a && j-- == 0) return l;
    }
    return -1;
  }
  /* j-th smallest distinct foreign label */
  int16_t prev = -1;
  for (int64_t t = 0; t <= j; ++t) {
    int16_t best = 0x7fff;
    for (int32_t e = g->rowptr[v]; e < g->rowptr[v + 1]; ++e) {
      int16_t l = c->lab[g->col[e]];
      if (l != a && l > prev && l < best) best = l;
    }
    prev = best;
  }
  return prev;
}

static void maps_yield(chain_t* c) {
  orc_maps* m = c->maps;
  const graph_t* g = &c->g;
  const int64_t t = (int64_t)c->st.yields; /* index of the state being yielded */
  int64_t e_id = 0;
  for (int32_t x = 0; x < g->n; ++x)
    for (int32_t e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) {
      const int32_t y = g->col[e];
      if (y <= x) continue;
      if (c->lab[x] != c->lab[y]) m->cut_times[e_id]++;
      ++e_id;
    }
  if (m->cur_f >= 0) {
    const int32_t f = m->cur_f;
    m->part_sum[f] -= m->label_value[c->lab[f]] * (t - m->last_flipped[f]);
    m->last_flipped[f] = t;
    m->num_flips[f] += 1;
  }
}

static void ring_yield(chain_t* c) {
  const orc_ring* R = c->ring;
  int32_t first = -1, second = -1;
  for (int32_t r = 0; r < R->n_ring && second < 0; ++r)
    if (c->lab[R->u[r]] != c->lab[R->w[r]]) {
      if (first < 0)
        first = r;
      else
        second = r;
    }
  R->hist[second >= 0 ? (int64_t)first * R->n_ring + second : (int64_t)R->n_ring * R->n_ring]++;
}

static void yield_obs(chain_t* c) {
  if (c->waits) c->waits->sum += c->waits->cur;
  if (c->maps) maps_yield(c);
  if (c->ring) ring_yield(c);
  c->st.yields++;
  c->st.sum_cut += c->st.cut;
  c->st.sum_bnodes += c->st.bnodes;
  c->st.sum_invb += 1.0 / (double)c->st.bnodes;
  if (c->hist_cut) c->hist_cut[c->st.cut]++;
  if (c->hist_b) c->hist_b[c->st.bnodes]++;
}

/* Apply flip v -> b: labels, pops, cut count, weights, boundary counters.
 * Returns the number of nodes whose boundary membership changed. */
static int32_t commit(chain_t* c, int32_t v, int16_t b, int32_t dcut) {
  const graph_t* g = &c->g;
  int16_t a = c->lab[v];
  c->lab[v] = b;
  c->pops[a] -= popof(g, v);
  c->pops[b] += popof(g, v);
  if (c->flags && c->flags[v]) {
    c->bcnt[a] -= 1;
    c->bcnt[b] += 1;
  }
  c->st.cut += dcut;
  int32_t nb = 0;
  for (int32_t e = g->rowptr[v] - 1; e < g->rowptr[v + 1]; ++e) {
    int32_t x = e < g->rowptr[v] ? v : g->col[e];
    int32_t wo = c->w[x], wn = weight(c, x);
    if (wn != wo) {
      c->w[x] = wn;
      fen_add(c, x, wn - wo);
      c->st.npairs += wn - wo;
      if ((wo > 0) != (wn > 0)) {
        c->st.bnodes += wn > 0 ? 1 : -1;
        ++nb;
      }
    }
  }
  return nb;
}

/* ------------------------------------------------------------------------- */
/* Public oracle API (ctypes).                                                */

static int setup(chain_t* c, const int32_t* rowptr, const int32_t* col, const int64_t* pop,
                 int32_t n, int32_t grid_w, int32_t k, int32_t mode, int64_t pop_lo, int64_t pop_hi,
                 const double* thr) {
  memset(c, 0, sizeof(*c));
  c->g.n = n;
  c->g.rowptr = rowptr;
  c->g.col = col;
  c->g.pop = pop;
  c->g.nnz = rowptr[n];
  c->g.maxdeg = 0;
  for (int32_t x = 0; x < n; ++x)
    if (rowptr[x + 1] - rowptr[x] > c->g.maxdeg) c->g.maxdeg = rowptr[x + 1] - rowptr[x];
  c->g.grid_w = grid_w;
  c->g.grid_h = grid_w ? n / grid_w : 0;
  c->k = k;
  c->mode = mode;
  c->pop_lo = pop_lo;
  c->pop_hi = pop_hi;
  c->thr = thr;
  c->w = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  c->fen = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
  c->pops = (int64_t*)calloc((size_t)k, sizeof(int64_t));
  c->bcnt = (int64_t*)calloc((size_t)k, sizeof(int64_t));
  c->owner = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  c->list = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  c->lab = (int16_t*)malloc(sizeof(int16_t) * (size_t)n);
  if (!c->w || !c->fen || !c->pops || !c->bcnt || !c->owner || !c->list || !c->lab) return -1;
  for (int32_t x = 0; x < n; ++x) c->owner[x] = -1;
  return 0;
}

static void teardown(chain_t* c) {
  free(c->w);
  free(c->fen);
  free(c->pops);
  free(c->bcnt);
  free(c->owner);
  free(c->list);
  free(c->lab);
}

/*
 * Run one chain for `steps` counted steps from `labels` (updated in place) and
 * `stats` (updated in place; stats->yields == 0 means "fresh chain": the
 * initial state is yielded first).  hist_cut [nedges+1] / hist_b [n+1] may be
 * NULL.  trace (may be NULL) receives per counted step: v (or -1 if the
 * Metropolis draw rejected) — used to replay trajectories in tests.
 * Returns 0, or -1 on allocation failure.
 */
int orc_run_chain_ex(const int32_t* rowptr, const int32_t* col, const int64_t* pop, int32_t n,
                     int32_t grid_w, int32_t k, int32_t mode, int64_t pop_lo, int64_t pop_hi,
                     const double* thr, uint64_t seed, uint64_t chain_id, int16_t* labels,
                     fw_chain_stats* stats, int64_t steps, int32_t max_retries,
                     uint64_t* hist_cut, uint64_t* hist_b, int32_t* trace, int64_t* pops_out,
                     orc_maps* maps, int32_t accept_rule, const uint8_t* flags,
                     const double* sched, int32_t sched_rows, int64_t sched_t0,
                     const orc_ring* ring, orc_waits* waits) {
  chain_t c;
  if (setup(&c, rowptr, col, pop, n, grid_w, k, mode, pop_lo, pop_hi, thr)) {
    teardown(&c);
    return -1;
  }
  memcpy(c.lab, labels, sizeof(int16_t) * (size_t)n);
  c.seed = seed;
  c.chain = chain_id;
  c.st = *stats;
  c.hist_cut = hist_cut;
  c.hist_b = hist_b;
  c.maps = maps;
  c.ring = ring;
  c.accept_rule = accept_rule;
  c.flags = flags;
  c.sched = sched_rows > 0 ? sched : NULL;
  c.sched_rows = sched_rows;
  c.sched_t0 = sched_t0;
  c.waits = waits;
  derive(&c);
  if (c.st.yields == 0 && c.st.attempts == 0) {
    if (waits) waits->cur = wait_draw(&c, ORC_WAIT_T0, c.st.bnodes);
    yield_obs(&c);
  }
  for (int64_t s = 0; s < steps && !c.st.stuck; ++s) {
    int32_t retries = 0;
    int32_t v = -1, dcut = 0;
    int16_t b = -1;
    uint32_t x[4];
    for (;;) {
      if (retries >= max_retries || c.st.npairs == 0) {
        c.st.stuck = 1;
        break;
      }
      draw(c.seed, c.st.attempts, c.chain, x);
      c.st.attempts++;
      int64_t j;
      uint32_t r = orc_scale64(x[0], x[1], (uint32_t)c.st.npairs);
      v = fen_select(&c, r, &j);
      int16_t a = c.lab[v];
      b = target_of(&c, v, j);
      int32_t dv = rowptr[v + 1] - rowptr[v];
      c.st.sum_deg += (uint64_t)dv;
      int32_t na = 0, nb = 0;
      for (int32_t e = rowptr[v]; e < rowptr[v + 1]; ++e) {
        na += c.lab[col[e]] == a;
        nb += c.lab[col[e]] == b;
      }
      dcut = na - nb;
      int64_t pv = popof(&c.g, v);
      if (c.pops[a] - pv < c.pop_lo || c.pops[b] + pv > c.pop_hi) {
        c.st.pop_fail++;
        ++retries;
        continue;
      }
      if (!contiguous_after(&c, v, a, 1)) {
        c.st.contig_fail++;
        ++retries;
        continue;
      }
      break;
    }
    if (c.st.stuck) break;
    c.st.steps++;
    double u = orc_u53(x[2], x[3]);
    int accepted = accept_of(&c, v, b, dcut, u);
    if (accepted) {
      c.st.accepts++;
      c.st.acc_deg += (uint64_t)(rowptr[v + 1] - rowptr[v]);
      c.st.n_bchg += (uint64_t)commit(&c, v, b, dcut);
      if (maps) maps->cur_f = v;
      if (waits) waits->cur = wait_draw(&c, c.st.attempts - 1, c.st.bnodes);
    }
    if (trace) trace[s] = accepted ? v : -1;
    yield_obs(&c);
  }
  memcpy(labels, c.lab, sizeof(int16_t) * (size_t)n);
  if (pops_out) memcpy(pops_out, c.pops, sizeof(int64_t) * (size_t)k);
  *stats = c.st;
  teardown(&c);
  return 0;
}

int orc_run_chain(const int32_t* rowptr, const int32_t* col, const int64_t* pop, int32_t n,
                  int32_t grid_w, int32_t k, int32_t mode, int64_t pop_lo, int64_t pop_hi,
                  const double* thr, uint64_t seed, uint64_t chain_id, int16_t* labels,
                  fw_chain_stats* stats, int64_t steps, int32_t max_retries, uint64_t* hist_cut,
                  uint64_t* hist_b, int32_t* trace, int64_t* pops_out) {
  return orc_run_chain_ex(rowptr, col, pop, n, grid_w, k, mode, pop_lo, pop_hi, thr, seed,
                          chain_id, labels, stats, steps, max_retries, hist_cut, hist_b, trace,
                          pops_out, NULL, FW_ACCEPT_CUT, NULL, NULL, 0, 0, NULL, NULL);
}

/* Per-flip evaluation on one state (the fw_eval_flips contract). */
int orc_eval_flips(const int32_t* rowptr, const int32_t* col, const int64_t* pop, int32_t n,
                   int32_t grid_w, int32_t k, const int16_t* labels, const int32_t* vs,
                   const int16_t* targets, int32_t m, int64_t pop_lo, int64_t pop_hi,
                   int32_t* dcut, uint8_t* contig, uint8_t* pop_ok, int32_t* dboundary) {
  chain_t c;
  if (setup(&c, rowptr, col, pop, n, grid_w, k, FW_PROPOSE_PAIRS, pop_lo, pop_hi, NULL)) {
    teardown(&c);
    return -1;
  }
  memcpy(c.lab, labels, sizeof(int16_t) * (size_t)n);
  derive(&c);
  for (int32_t i = 0; i < m; ++i) {
    int32_t v = vs[i];
    int16_t a = c.lab[v], b = targets[i];
    int32_t na = 0, nb = 0;
    for (int32_t e = rowptr[v]; e < rowptr[v + 1]; ++e) {
      na += c.lab[col[e]] == a;
      nb += c.lab[col[e]] == b;
    }
    dcut[i] = na - nb;
    int64_t pv = popof(&c.g, v);
    pop_ok[i] = !(c.pops[a] - pv < pop_lo || c.pops[b] + pv > pop_hi);
    contig[i] = (uint8_t)contiguous_after(&c, v, a, 0);
    /* boundary delta: membership of v and its neighbours before/after */
    int32_t before = 0, after = 0;
    for (int32_t e = rowptr[v] - 1; e < rowptr[v + 1]; ++e) {
      int32_t x = e < rowptr[v] ? v : col[e];
      before += weight(&c, x) > 0;
    }
    c.lab[v] = b;
    for (int32_t e = rowptr[v] - 1; e < rowptr[v + 1]; ++e) {
      int32_t x = e < rowptr[v] ? v : col[e];
      after += weight(&c, x) > 0;
    }
    c.lab[v] = a;
    dboundary[i] = after - before;
  }
  teardown(&c);
  return 0;
}

/* Whole-plan validity (MarkovChain's initial-state check): every district
 * 0..k-1 non-empty and connected, and every population inside the bounds. */
int orc_plan_valid(const int32_t* rowptr, const int32_t* col, const int64_t* pop, int32_t n,
                   int32_t k, const int16_t* labels, int64_t pop_lo, int64_t pop_hi) {
  int64_t* pops = (int64_t*)calloc((size_t)k, sizeof(int64_t));
  int32_t* seen = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  int32_t* first = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
  int ok = 1;
  for (int32_t d = 0; d < k; ++d) first[d] = -1;
  for (int32_t x = 0; x < n; ++x) {
    if (labels[x] < 0 || labels[x] >= k) {
      ok = 0;
      break;
    }
    pops[labels[x]] += pop ? pop[x] : 1;
    if (first[labels[x]] < 0) first[labels[x]] = x;
  }
  for (int32_t d = 0; ok && d < k; ++d) {
    if (first[d] < 0 || pops[d] < pop_lo || pops[d] > pop_hi) {
      ok = 0;
      break;
    }
  }
  for (int32_t d = 0; ok && d < k; ++d) {
    int32_t h = 0, t = 0;
    q[t++] = first[d];
    seen[first[d]] = 1;
    while (h < t) {
      int32_t x = q[h++];
      for (int32_t e = rowptr[x]; e < rowptr[x + 1]; ++e) {
        int32_t y = col[e];
        if (!seen[y] && labels[y] == d) {
          seen[y] = 1;
          q[t++] = y;
        }
      }
    }
    for (int32_t x = 0; x < n; ++x)
      if (labels[x] == d && !seen[x]) ok = 0;
  }
  free(pops);
  free(seen);
  free(q);
  free(first);
  return ok;
}

int32_t orc_stats_size(void) { return (int32_t)sizeof(fw_chain_stats); }
