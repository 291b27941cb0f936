/*
 * search_stats.c — DIAGNOSTIC ONLY (not product, not a test): statistics of the exact
 * contiguity searches of grid chains, to size GPU search designs.  It #includes the C
 * oracle so it can drive its chain loop and reuse its static helpers.
 *
 * For every attempt whose verdict needs the exact search (ring test and 7x7 window
 * undecided) it measures
 *   - the A-side race (the oracle's search): levels, dequeued nodes, verdict, and the
 *     extent (max |dr|, |dc| from v) of the cells it touched;
 *   - the background race: the same level-synchronous race on the complement of district
 *     a (8-connected, the off-grid outside as one node) from one cell of each gap between
 *     v's local a-components.  For a planar grid, (a minus v) is connected iff the m' gaps
 *     lie in m' different background components, so this race decides at its first merge
 *     (disconnected) or once all but one gap class are exhausted (connected).
 *
 *   gcc -O2 -o /tmp/search_stats scripts/search_stats.c -lm
 *   /tmp/search_stats W H k bw base warm_steps sample_attempts seed chain
 */
#include <stdio.h>

#include "../oracle/flipchain_oracle.c"

static int W, H;

typedef struct {
  long n;
  double levels, nodes, bglevels, bgnodes, minlevels;
  long connected, fit6432, fit6464, fit12864, fit128, fit6496, fit64128, bgwins;
  double esc_levels, esc_nodes;
  long hist[8];  /* levels of min(A, background) in bins <4, <8, <16, <32, <64, <128, <256, >= */
  long histA[8];
} acc_t;

static long g_fr_hist[6]; /* max frontier (next level) per search: <=64, <=128, <=256, <=512, <=1024, more */
static int g_fr_max;
static long g_mcls[5][5]; /* exact searches by sources m and classes after the ring links */

static int lvl_bin(int l) {
  int b = 0, t = 4;
  while (b < 7 && l >= t) { ++b; t *= 2; }
  return b;
}

/* A-side race (the oracle's contiguous_after search), with extents */
static int race_a(chain_t* c, int32_t v, int16_t a, const int32_t* src, int32_t m, int32_t* uf,
                  int* levels, long* nodes, int* maxdr, int* maxdc) {
  const graph_t* g = &c->g;
  int32_t nl = 0;
  int vr = v / W, vc = v % W;
  *maxdr = *maxdc = 0;
  for (int32_t i = 0; i < m; ++i) {
    c->owner[src[i]] = i;
    c->list[nl++] = src[i];
  }
  int32_t lb = 0, le = nl;
  int verdict = -1;
  *levels = 0;
  *nodes = 0;
  g_fr_max = 0;
  for (;;) {
    int32_t ncls = 0;
    for (int32_t i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
    if (ncls == 1) { verdict = 1; break; }
    ++*levels;
    for (int32_t li = lb; li < le; ++li) {
      int32_t x = c->list[li];
      ++*nodes;
      int dr = abs(x / W - vr), dc = abs(x % W - vc);
      if (dr > *maxdr) *maxdr = dr;
      if (dc > *maxdc) *maxdc = dc;
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
    lb = le;
    le = nl;
    if (le - lb > g_fr_max) g_fr_max = le - lb;
    ncls = 0;
    for (int32_t i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
    if (ncls == 1) { verdict = 1; break; }
    uint64_t present = 0;
    for (int32_t li = lb; li < le; ++li) present |= 1ull << uf_find(uf, c->owner[c->list[li]]);
    int ex = 0;
    for (int32_t i = 0; i < m; ++i)
      if (uf_find(uf, i) == i && !((present >> i) & 1)) ex = 1;
    if (ex) { verdict = 0; break; }
  }
  for (int32_t li = 0; li < nl; ++li) c->owner[c->list[li]] = -1;
  {
    int b = 0, t = 64;
    while (b < 5 && g_fr_max > t) { ++b; t *= 2; }
    g_fr_hist[b]++;
  }
  return verdict;
}

/* background race; node id n = the outside */
static int32_t* bown;
static int32_t* blist;
static int race_bg(chain_t* c, int32_t v, int16_t a, int* levels, long* nodes, int* mprime) {
  const int n = c->g.n;
  int vr = v / W, vc = v % W;
  /* ring in cyclic order N NE E SE S SW W NW; in-A flags */
  const int dr8[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, dc8[8] = {0, 1, 1, 1, 0, -1, -1, -1};
  int inA[8], id8[8];
  for (int i = 0; i < 8; ++i) {
    int r = vr + dr8[i], q = vc + dc8[i];
    int on = r >= 0 && r < H && q >= 0 && q < W;
    id8[i] = on ? r * W + q : n;
    inA[i] = on && c->lab[r * W + q] == a;
  }
  /* a diagonal a-cell blocks the background only next to an a 4-neighbour */
  int block[8];
  for (int i = 0; i < 8; ++i)
    block[i] = (i % 2 == 0) ? inA[i] : (inA[i] && (inA[i - 1] || inA[(i + 1) % 8]));
  /* gaps: maximal cyclic runs of non-blocking cells; sources = one cell of each */
  int start = -1;
  for (int i = 0; i < 8; ++i)
    if (block[i]) { start = i; break; }
  int32_t src[8];
  int m = 0;
  for (int t = 1; t <= 8; ++t) {
    int i = (start + t) % 8;
    if (!block[i] && block[(i + 7) % 8]) {
      /* a gap starts at i: its source is its first non-a cell (diagonal a-cells inside a
         gap are not background; a gap always holds a non-a or off-grid cell) */
      int j = i;
      while (inA[j]) j = (j + 1) % 8;
      src[m++] = id8[j];
    }
  }
  *mprime = m;
  int32_t uf[8];
  for (int i = 0; i < m; ++i) uf[i] = i;
  int32_t nl = 0;
  for (int i = 0; i < m; ++i) {
    if (bown[src[i]] >= 0) { /* two gaps through one cell (the outside): same component */
      int32_t ri = uf_find(uf, i), rj = uf_find(uf, bown[src[i]]);
      if (ri != rj) uf[ri] = rj;
      continue;
    }
    bown[src[i]] = i;
    blist[nl++] = src[i];
  }
  int verdict = -1;
  int32_t lb = 0, le = nl;
  *levels = 0;
  *nodes = 0;
  bown[v] = 99; /* v is removed: not part of the background search (sources are its ring) */
  for (;;) {
    int ncls = 0;
    for (int i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
    if (ncls < m) { verdict = 0; break; }
    ++*levels;
    uint64_t pushed = 0;
    for (int32_t li = lb; li < le; ++li) {
      int32_t x = blist[li];
      ++*nodes;
      int ox = bown[x];
      if (x == n) { /* outside: adjacent to every border cell */
        for (int32_t y = 0; y < n; ++y) {
          int r = y / W, q = y % W;
          if (!(r == 0 || r == H - 1 || q == 0 || q == W - 1)) continue;
          if (c->lab[y] == a) continue;
          if (bown[y] < 0) { bown[y] = ox; blist[nl++] = y; pushed |= 1ull << uf_find(uf, ox); }
          else if (bown[y] != 99) { int32_t rx = uf_find(uf, ox), ry = uf_find(uf, bown[y]); if (rx != ry) uf[rx] = ry; }
        }
        continue;
      }
      int xr = x / W, xq = x % W;
      for (int d = 0; d < 8; ++d) {
        int r = xr + dr8[d], q = xq + dc8[d];
        int32_t y;
        if (r < 0 || r >= H || q < 0 || q >= W) y = n;
        else {
          y = r * W + q;
          if (c->lab[y] == a || y == v) continue;
        }
        if (bown[y] < 0) { bown[y] = ox; blist[nl++] = y; pushed |= 1ull << uf_find(uf, ox); }
        else if (bown[y] != 99) { int32_t rx = uf_find(uf, ox), ry = uf_find(uf, bown[y]); if (rx != ry) uf[rx] = ry; }
      }
    }
    lb = le;
    le = nl;
    int ncls2 = 0, open = 0;
    for (int i = 0; i < m; ++i) ncls2 += uf_find(uf, i) == i;
    if (ncls2 < m) { verdict = 0; break; }
    uint64_t present = 0;
    for (int32_t li = lb; li < le; ++li) present |= 1ull << uf_find(uf, bown[blist[li]]);
    for (int i = 0; i < m; ++i)
      if (uf_find(uf, i) == i && ((present >> i) & 1)) ++open;
    if (open <= 1) { verdict = 1; break; }
  }
  for (int32_t li = 0; li < nl; ++li) bown[blist[li]] = -1;
  bown[v] = -1;
  return verdict;
}

int main(int argc, char** argv) {
  if (argc < 10) {
    fprintf(stderr, "usage: W H k bw base warm sample seed chain\n");
    return 1;
  }
  W = atoi(argv[1]);
  H = atoi(argv[2]);
  int k = atoi(argv[3]), bw = atoi(argv[4]);
  double base = atof(argv[5]);
  long warm = atol(argv[6]), sample = atol(argv[7]);
  uint64_t seed = strtoull(argv[8], 0, 10), chain = strtoull(argv[9], 0, 10);
  int n = W * H;
  int32_t* rp = malloc(sizeof(int32_t) * (n + 1));
  int32_t* col = malloc(sizeof(int32_t) * 4 * n);
  int e = 0;
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      rp[i * W + j] = e;
      if (i > 0) col[e++] = (i - 1) * W + j;
      if (j > 0) col[e++] = i * W + j - 1;
      if (j < W - 1) col[e++] = i * W + j + 1;
      if (i < H - 1) col[e++] = (i + 1) * W + j;
    }
  rp[n] = e;
  int16_t* lab = malloc(sizeof(int16_t) * n);
  int bh = k / bw; /* k = bh x bw blocks */
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) lab[i * W + j] = (int16_t)((i * bh / H) * bw + j * bw / W);
  double thr[9];
  for (int d = -4; d <= 4; ++d) thr[d + 4] = pow(base, -d);
  double ideal = (double)n / k;
  int64_t lo = (int64_t)ceil(0.95 * ideal), hi = (int64_t)floor(1.05 * ideal);
  fw_chain_stats st;
  memset(&st, 0, sizeof st);
  orc_run_chain(rp, col, NULL, n, W, k, FW_PROPOSE_PAIRS, lo, hi, thr, seed, chain, lab, &st, warm,
                1 << 20, NULL, NULL, NULL, NULL);
  fprintf(stderr, "after %ld steps: cut %d, |B| %d, attempts %llu\n", warm, st.cut, st.bnodes,
          (unsigned long long)st.attempts);
  chain_t c;
  setup(&c, rp, col, NULL, n, W, k, FW_PROPOSE_PAIRS, lo, hi, thr);
  memcpy(c.lab, lab, sizeof(int16_t) * n);
  c.seed = seed;
  c.chain = chain;
  c.st = st;
  derive(&c);
  bown = malloc(sizeof(int32_t) * (n + 1));
  blist = malloc(sizeof(int32_t) * (n + 1) * 2);
  for (int i = 0; i <= n; ++i) bown[i] = -1;
  acc_t A;
  memset(&A, 0, sizeof A);
  long att = 0, nsteps = 0;
  while (att < sample) {
    uint32_t x[4];
    draw(c.seed, c.st.attempts, c.chain, x);
    c.st.attempts++;
    ++att;
    int64_t j;
    uint32_t r = orc_scale64(x[0], x[1], (uint32_t)c.st.npairs);
    int32_t v = fen_select(&c, r, &j);
    int16_t a = c.lab[v];
    int16_t b = target_of(&c, v, j);
    int32_t na = 0, nb = 0;
    for (int32_t q = rp[v]; q < rp[v + 1]; ++q) {
      na += c.lab[col[q]] == a;
      nb += c.lab[col[q]] == b;
    }
    if (c.pops[a] - 1 < lo || c.pops[b] + 1 > hi) continue;
    /* exact search needed? (the oracle's pre-tests) */
    int32_t src[4], uf[4], m = 0;
    for (int32_t q = rp[v]; q < rp[v + 1]; ++q)
      if (c.lab[col[q]] == a) src[m++] = col[q];
    int ok;
    if (m == 0) ok = 0;
    else if (m == 1) ok = 1;
    else if (grid_ring(&c, v, a, src, m, uf) == 1) ok = 1;
    else {
      int wv = orc_window_verdict(window_mask(&c, v, a));
      if (wv >= 0) ok = wv;
      else {
        int lv, mdr, mdc, blv, mp;
        long nd, bnd;
        {
          int ncls = 0;
          for (int32_t i = 0; i < m; ++i) ncls += uf_find(uf, i) == i;
          g_mcls[m < 5 ? m : 4][ncls < 5 ? ncls : 4]++;
        }
        int va = race_a(&c, v, a, src, m, uf, &lv, &nd, &mdr, &mdc);
        int vb = race_bg(&c, v, a, &blv, &bnd, &mp);
        if (va != vb) {
          fprintf(stderr, "verdict mismatch at attempt %ld: A %d bg %d (m' %d)\n", att, va, vb, mp);
          return 2;
        }
        ok = va;
        A.n++;
        A.levels += lv;
        A.nodes += nd;
        A.bglevels += blv;
        A.bgnodes += bnd;
        A.minlevels += lv < blv ? lv : blv;
        A.bgwins += blv < lv;
        A.connected += va;
        A.fit6432 += mdr < 32 && mdc < 16;
        A.fit6464 += mdr < 32 && mdc < 32;
        A.fit128 += mdr < 64 && mdc < 64;
        A.fit12864 += mdr < 64 && mdc < 32;
        A.fit6496 += mdr < 32 && mdc < 48;
        A.fit64128 += mdr < 32 && mdc < 64;
        if (!(mdr < 32 && mdc < 16)) { A.esc_levels += lv; A.esc_nodes += nd; }
        A.hist[lvl_bin(lv < blv ? lv : blv)]++;
        A.histA[lvl_bin(lv)]++;
      }
    }
    if (!ok) continue;
    nsteps++;
    double u = orc_u53(x[2], x[3]);
    int dcut = na - nb;
    if (u < thr[dcut + 4]) commit(&c, v, b, dcut);
  }
  printf("base %.4g: %ld attempts, %ld steps, %ld exact searches (%.3f/attempt), cut %d |B| %d\n",
         base, att, nsteps, A.n, (double)A.n / att, c.st.cut, c.st.bnodes);
  if (A.n) {
    printf("  A race: levels %.1f nodes %.1f  connected %.2f  fits 64x32 %.3f 64x64 %.3f "
           "128x128 %.3f\n", A.levels / A.n, A.nodes / A.n, (double)A.connected / A.n,
           (double)A.fit6432 / A.n, (double)A.fit6464 / A.n, (double)A.fit128 / A.n);
    printf("  fits 128x64 %.3f; escapers of 64x32: levels %.1f nodes %.1f\n",
           (double)A.fit12864 / A.n, A.esc_levels / (A.n - A.fit6432 + 1e-9),
           A.esc_nodes / (A.n - A.fit6432 + 1e-9));
    printf("  bg race: levels %.1f nodes %.1f; min(A,bg) levels %.1f (bg shorter %.2f)\n",
           A.bglevels / A.n, A.bgnodes / A.n, A.minlevels / A.n, (double)A.bgwins / A.n);
    printf("  levels A     <4 <8 <16 <32 <64 <128 <256 >=:");
    for (int i = 0; i < 8; ++i) printf(" %.3f", (double)A.histA[i] / A.n);
    printf("\n  levels min   <4 <8 <16 <32 <64 <128 <256 >=:");
    for (int i = 0; i < 8; ++i) printf(" %.3f", (double)A.hist[i] / A.n);
    printf("\n  fits 64 rows x 96 cols %.3f, 64 x 128 %.3f", (double)A.fit6496 / A.n,
           (double)A.fit64128 / A.n);
    printf("\n  exact searches by (sources, classes):");
    for (int i = 2; i < 5; ++i)
      for (int j = 1; j < 5; ++j)
        if (g_mcls[i][j]) printf(" (%d,%d) %.3f", i, j, (double)g_mcls[i][j] / A.n);
    printf("\n  max frontier <=64 <=128 <=256 <=512 <=1024 more:");
    long fr_n = 0;
    for (int i = 0; i < 6; ++i) fr_n += g_fr_hist[i];
    for (int i = 0; i < 6; ++i) printf(" %.4f", (double)g_fr_hist[i] / (fr_n ? fr_n : 1));
    printf("\n");
  }
  return 0;
}
