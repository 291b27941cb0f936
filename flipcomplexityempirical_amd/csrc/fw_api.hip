// fw_api.hip — host implementation of the C-ABI in include/flipwalk.h.
//
// Owns device memory behind fw_graph / fw_chains handles, validates inputs the
// way GerryChain does (initial-state check -> FW_ESTATE, like MarkovChain's
// ValueError), packs labels into the kernels' LB-bit layout and launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fw_internal.h"
#include "fw_math.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(FW_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));             \
  } while (0)

int round16(int64_t x) { return (int)((x + 15) / 16 * 16); }

// Same rule as flipcomplexityempirical_amd.graph.detect_grid.
int detect_grid(const std::vector<int32_t>& rp, const std::vector<int32_t>& col, int n) {
  if (n < 4) return 0;
  if (rp[1] - rp[0] != 2 || col[0] != 1) return 0;
  const int w = col[1];
  if (w < 2 || n % w || n / w < 2) return 0;
  const int h = n / w;
  int e = 0;
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const int x = i * w + j;
      int nb[4], d = 0;
      if (i > 0) nb[d++] = x - w;
      if (j > 0) nb[d++] = x - 1;
      if (j < w - 1) nb[d++] = x + 1;
      if (i < h - 1) nb[d++] = x + w;
      if (rp[x] != e || rp[x + 1] - rp[x] != d) return 0;
      for (int t = 0; t < d; ++t)
        if (col[e + t] != nb[t]) return 0;
      e += d;
    }
  return w;
}

// Entries of a contiguity search's visit list held in LDS before it spills to HBM.
// FLIPWALK_LIST_CAP overrides it (tests force the spill path with a tiny cap).
int list_cap(int dflt) {
  const char* e = getenv("FLIPWALK_LIST_CAP");
  if (!e || !e[0]) return dflt;
  const int v = atoi(e);
  return v >= 1 ? v : dflt;
}

// x / gw == (x * m) >> s for every x < 2^15 with m < 2^17 (so the grid kernel divides with
// one full-rate 24-bit multiply), verified exhaustively; m = 0 if no shift works
void grid_div24(int gw, uint32_t* m_out, uint32_t* s_out) {
  *m_out = 0;
  *s_out = 0;
  for (uint32_t sh = 0; gw > 0 && sh < 32; ++sh) {
    const uint64_t m = (((uint64_t)1 << sh) + (uint64_t)gw - 1) / (uint64_t)gw;
    if (m >= ((uint64_t)1 << 17)) break;
    bool ok = m > 0;
    for (uint64_t x = 0; x < ((uint64_t)1 << 15) && ok; ++x) ok = ((x * m) >> sh) == x / (uint64_t)gw;
    if (ok) {
      *m_out = (uint32_t)m;
      *s_out = sh;
      return;
    }
  }
}

}  // namespace

struct fw_graph {
  int device = 0;
  int32_t n = 0, nnz = 0, maxdeg = 0, gw = 0, gh = 0;
  uint32_t gm24 = 0, gs24 = 0;  // grid_div24
  std::vector<int32_t> rowptr, col;
  std::vector<int64_t> pop;  // empty: unit populations
  int32_t* d_rowptr = nullptr;
  int32_t* d_col = nullptr;
  int64_t* d_pop = nullptr;
  int32_t* d_eid = nullptr;  // [nnz] canonical edge id per CSR entry
  int32_t* d_eu = nullptr;   // [E] canonical edge endpoints (u < w)
  int32_t* d_ew = nullptr;
  uint64_t* d_nbadj = nullptr;  // [nnz] (general graphs): adjacency among v's neighbours
  int32_t* d_ell = nullptr;     // [n][16] (general graphs, max degree <= 16): padded rows
  int32_t* d_dbound = nullptr;  // with d_ell: FwGraphDev::dbound
  double* d_invb = nullptr;     // [n+1] 1.0 / max(b, 1) for the Σ1/|B| observable
  int64_t popof(int x) const { return pop.empty() ? 1 : pop[x]; }
  FwGraphDev dev() const {
    FwGraphDev g;
    g.rowptr = d_rowptr;
    g.col = d_col;
    g.eid = d_eid;
    g.nbadj = d_nbadj;
    g.ell = d_ell;
    g.dbound = d_dbound;
    g.pop = d_pop;
    g.invb = d_invb;
    g.n = n;
    g.nedges = nnz / 2;
    g.maxdeg = maxdeg;
    g.gw = gw;
    g.gh = gh;
    // exact x / gw for x < 2^21 (the grid path is only taken for n < 2^21)
    g.gmagic = gw ? (((uint64_t)1 << 42) + (uint64_t)gw - 1) / (uint64_t)gw : 0;
    g.gm32 = gw ? (uint32_t)((((uint64_t)1 << 32) + (uint64_t)gw - 1) / (uint64_t)gw) : 0;
    g.gm24 = gm24;
    g.gs24 = gs24;
    return g;
  }
};

struct fw_chains {
  fw_graph* g = nullptr;
  int32_t n_chains = 0, k = 0, mode = 0, lb = 4, grid = 1, D = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  FwRunParams p{};
  uint8_t* d_labels = nullptr;
  fw_chain_stats* d_stats = nullptr;
  int64_t* d_pops = nullptr;
  double* d_thr = nullptr;
  uint64_t* d_thr53 = nullptr;
  unsigned long long* d_hist_cut = nullptr;
  unsigned long long* d_hist_b = nullptr;
  uint32_t* d_spill = nullptr;
  int32_t* d_next = nullptr;
  uint32_t* d_gscr = nullptr;  // chain kernel, 5-bit labels: search marks
  int32_t* d_segdone = nullptr;  // finished slices per work unit (launch_slices)
  uint64_t max_yields = 0;  // upper bound on any chain's yield count (maps need < 2^32)
  bool gcache_ok = false;   // the label records' group sums and the stats' cut / bnodes /
                            // npairs match the labels (FwRunParams::gcache_ok)
  bool ran = false;
  // spatial observables (fw_chains_enable_maps)
  int64_t* d_acc = nullptr;
  uint32_t* d_nf = nullptr;
  uint32_t* d_lf = nullptr;
  int64_t* d_ps = nullptr;
  int32_t* d_pend = nullptr;
  int64_t* d_labval = nullptr;
  // FW_ACCEPT_BOUNDARY
  uint8_t* d_flags = nullptr;
  int32_t* d_bcnt = nullptr;
  // fw_chains_set_schedule
  double* d_sched = nullptr;
  uint64_t* d_sched53 = nullptr;
  // fw_chains_enable_ring
  int32_t ring_n = 0;
  std::vector<int32_t> ring_u, ring_w;
  double* d_wsamp = nullptr;  // fw_chains_enable_waits: [n_chains][2] {sum, current draw}
  double* d_wlp = nullptr;    // [n+1] log1p(-p_b)
  int32_t* d_ring = nullptr;              // [2][ring_n] endpoints
  uint8_t* d_ring_node = nullptr;         // [n]
  unsigned long long* d_hist_ring = nullptr;  // [ring_n^2 + 1]
};

namespace {

// integer form of a Metropolis bound: CPython's u = M * 2^-53 with integer M < 2^53,
// so u < thr <=> M < thr * 2^53 (exact scaling) <=> M < ceil(thr * 2^53)
uint64_t thr53_of(double thr) {
  const double t = thr * 9007199254740992.0;
  return !(t > 0.0) ? 0ull : (t >= 9007199254740992.0 ? (1ull << 53) : (uint64_t)std::ceil(t));
}

// Label bits per node for a (k, maxdeg): the search marks visited nodes with codes
// k..k+deg-1 and v with the all-ones value, so k + maxdeg must stay below it.
int pick_lb(int k, int maxdeg) {
  if (k + maxdeg <= 15 && maxdeg <= 15) return 4;
  if (k + maxdeg <= 255) return 8;
  return 0;
}

// LB-bit little-endian fields: node x in bits [x*LB, x*LB + LB) of the byte stream (a
// 3-bit field may straddle two bytes; the label region is padded past its last field).
void pack_labels(const int16_t* lab, int n, int lb, uint8_t* out, int bytes) {
  std::memset(out, 0, (size_t)bytes);
  for (int x = 0; x < n; ++x) {
    const int64_t bit = (int64_t)x * lb;
    const uint32_t v = (uint32_t)(lab[x] & ((1 << lb) - 1)) << (bit & 7);
    out[bit >> 3] |= (uint8_t)v;
    if ((bit & 7) + lb > 8) out[(bit >> 3) + 1] |= (uint8_t)(v >> 8);
  }
}

void unpack_labels(const uint8_t* in, int n, int lb, int16_t* lab) {
  for (int x = 0; x < n; ++x) {
    const int64_t bit = (int64_t)x * lb;
    uint32_t v = in[bit >> 3];
    if ((bit & 7) + lb > 8) v |= (uint32_t)in[(bit >> 3) + 1] << 8;
    lab[x] = (int16_t)((v >> (bit & 7)) & ((1u << lb) - 1));
  }
}

// MarkovChain's initial-state validity: every district non-empty, connected and
// inside the population bounds.  Fills pops[k].
bool plan_valid(const fw_graph* g, const int16_t* lab, int k, int64_t lo, int64_t hi,
                int64_t* pops, std::string* why) {
  const int n = g->n;
  std::vector<int> first(k, -1);
  for (int d = 0; d < k; ++d) pops[d] = 0;
  for (int x = 0; x < n; ++x) {
    if (lab[x] < 0 || lab[x] >= k) {
      *why = "label out of range at node " + std::to_string(x);
      return false;
    }
    pops[lab[x]] += g->popof(x);
    if (first[lab[x]] < 0) first[lab[x]] = x;
  }
  std::vector<uint8_t> seen(n, 0);
  std::vector<int> q(n);
  for (int d = 0; d < k; ++d) {
    if (first[d] < 0) {
      *why = "district " + std::to_string(d) + " is empty";
      return false;
    }
    if (pops[d] < lo || pops[d] > hi) {
      *why = "district " + std::to_string(d) + " population " + std::to_string(pops[d]) +
             " outside [" + std::to_string(lo) + ", " + std::to_string(hi) + "]";
      return false;
    }
    int h = 0, t = 0;
    q[t++] = first[d];
    seen[first[d]] = 1;
    while (h < t) {
      int x = q[h++];
      for (int e = g->rowptr[x]; e < g->rowptr[x + 1]; ++e) {
        int y = g->col[e];
        if (!seen[y] && lab[y] == d) {
          seen[y] = 1;
          q[t++] = y;
        }
      }
    }
  }
  for (int x = 0; x < n; ++x)
    if (!seen[x]) {
      *why = "district " + std::to_string(lab[x]) + " is not contiguous (node " +
             std::to_string(x) + ")";
      return false;
    }
  return true;
}

size_t ring_bins(int r) { return (size_t)r * (size_t)r + 1; }

// first two cut ring edges of a plan in ring order: out = {i, j} (-1, -1 if fewer than two)
void ring_pair_of(const fw_chains* c, const int16_t* lab, int32_t* out) {
  out[0] = out[1] = -1;
  int found = 0;
  for (int r = 0; r < c->ring_n && found < 2; ++r)
    if (lab[c->ring_u[r]] != lab[c->ring_w[r]]) out[found++] = r;
  if (found < 2) out[0] = out[1] = -1;
}

}  // namespace

extern "C" {

const char* fw_last_error(void) { return g_err.c_str(); }

int32_t fw_version(void) { return 0x000700; }

int32_t fw_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int fw_graph_create(const int32_t* rowptr, const int32_t* col, const int64_t* pop, int32_t n,
                    int32_t nnz, int device, fw_graph** out) {
  if (!out || !rowptr || (nnz > 0 && !col) || n <= 0 || nnz < 0)
    return fail(FW_EINVAL, "fw_graph_create: bad arguments");
  *out = nullptr;
  if (rowptr[0] != 0 || rowptr[n] != nnz) return fail(FW_EINVAL, "rowptr[0]/rowptr[n] mismatch");
  auto g = new fw_graph();
  g->device = device;
  g->n = n;
  g->nnz = nnz;
  g->rowptr.assign(rowptr, rowptr + n + 1);
  g->col.assign(col, col + nnz);
  bool unit = true;
  if (pop) {
    for (int x = 0; x < n; ++x) unit &= pop[x] == 1;
    if (!unit) g->pop.assign(pop, pop + n);
  }
  for (int x = 0; x < n; ++x) {
    const int b = rowptr[x], e = rowptr[x + 1];
    if (e < b) {
      delete g;
      return fail(FW_EINVAL, "rowptr not monotone at %d", x);
    }
    g->maxdeg = std::max(g->maxdeg, e - b);
    for (int t = b; t < e; ++t) {
      const int y = col[t];
      if (y < 0 || y >= n || y == x || (t > b && col[t - 1] >= y)) {
        delete g;
        return fail(FW_EINVAL, "row %d: neighbours must be ascending, in range, no self loop", x);
      }
      // symmetry: x must appear in y's (sorted) row
      if (!std::binary_search(col + rowptr[y], col + rowptr[y + 1], x)) {
        delete g;
        return fail(FW_EINVAL, "adjacency not symmetric: %d->%d", x, y);
      }
    }
  }
  g->gw = n < (1 << 21) ? detect_grid(g->rowptr, g->col, n) : 0;
  g->gh = g->gw ? n / g->gw : 0;
  grid_div24(g->gw, &g->gm24, &g->gs24);
  if (hipSetDevice(device) != hipSuccess) {
    delete g;
    return fail(FW_EHIP, "hipSetDevice(%d) failed", device);
  }
  // canonical edge ids: undirected pairs (u < w) numbered in CSR row order
  std::vector<int32_t> eid(std::max(nnz, 1)), eu, ew;
  for (int x = 0; x < n; ++x)
    for (int t = rowptr[x]; t < rowptr[x + 1]; ++t) {
      const int y = col[t];
      if (y > x) {
        eid[t] = (int32_t)eu.size();
        eu.push_back(x);
        ew.push_back(y);
      } else {  // (y, x) was numbered in row y
        const int32_t* q = std::lower_bound(col + rowptr[y], col + rowptr[y + 1], x);
        eid[t] = eid[q - col];
      }
    }
  const size_t ne = std::max<size_t>(eu.size(), 1);
  // general graphs: for entry (v, i), the positions j of v's neighbours adjacent to the
  // i-th (the kernel's local contiguity test; degrees <= 63 were checked above)
  std::vector<uint64_t> nbadj;
  if (!g->gw && nnz > 0 && g->maxdeg <= 63) {
    nbadj.assign(nnz, 0);
    for (int v = 0; v < n; ++v)
      for (int i = rowptr[v]; i < rowptr[v + 1]; ++i)
        for (int j = rowptr[v]; j < rowptr[v + 1]; ++j)
          if (j != i && std::binary_search(col + rowptr[col[i]], col + rowptr[col[i] + 1], col[j]))
            nbadj[i] |= 1ull << (j - rowptr[v]);
  }
  hipError_t e1 = hipMalloc(&g->d_rowptr, sizeof(int32_t) * (n + 1));
  hipError_t e2 = hipMalloc(&g->d_col, sizeof(int32_t) * std::max(nnz, 1));
  hipError_t e3 = g->pop.empty() ? hipSuccess : hipMalloc(&g->d_pop, sizeof(int64_t) * n);
  if (e3 == hipSuccess) e3 = hipMalloc(&g->d_eid, sizeof(int32_t) * eid.size());
  if (e3 == hipSuccess) e3 = hipMalloc(&g->d_eu, sizeof(int32_t) * ne);
  if (e3 == hipSuccess) e3 = hipMalloc(&g->d_ew, sizeof(int32_t) * ne);
  std::vector<int32_t> ell, dbound;
  if (!g->gw && g->maxdeg <= 16) {
    // padded rows; the neighbour-adjacency masks move to the same [n][16] layout
    ell.assign((size_t)n * 16, -1);
    std::vector<uint64_t> nb16(nbadj.empty() ? 0 : (size_t)n * 16, 0);
    for (int x = 0; x < n; ++x)
      for (int t = rowptr[x]; t < rowptr[x + 1]; ++t) {
        ell[(size_t)x * 16 + (t - rowptr[x])] = col[t];
        if (!nbadj.empty()) nb16[(size_t)x * 16 + (t - rowptr[x])] = nbadj[t];
      }
    nbadj.swap(nb16);
    if (e3 == hipSuccess) e3 = hipMalloc(&g->d_ell, sizeof(int32_t) * ell.size());
    // loop bounds of the padded-row walks: the select's over the 64 nodes of a group, the
    // gather's over v and its neighbours (C4: 9.7 and ~10 instead of the graph's 14)
    const int ng = (n + 63) / 64;
    dbound.assign((size_t)n + ng, 0);
    for (int x = 0; x < n; ++x) {
      int md = rowptr[x + 1] - rowptr[x];
      for (int t = rowptr[x]; t < rowptr[x + 1]; ++t)
        md = std::max(md, rowptr[col[t] + 1] - rowptr[col[t]]);
      dbound[x] = md;
      dbound[(size_t)n + x / 64] = std::max(dbound[(size_t)n + x / 64], rowptr[x + 1] - rowptr[x]);
    }
    if (e3 == hipSuccess) e3 = hipMalloc(&g->d_dbound, sizeof(int32_t) * dbound.size());
  }
  if (e3 == hipSuccess && !nbadj.empty())
    e3 = hipMalloc(&g->d_nbadj, sizeof(uint64_t) * nbadj.size());
  // the kernels read 1/|B| here instead of dividing in fp64 on every accepted step
  std::vector<double> invb((size_t)n + 1);
  for (int b = 0; b <= n; ++b) invb[b] = 1.0 / (double)(b > 0 ? b : 1);
  if (e3 == hipSuccess) e3 = hipMalloc(&g->d_invb, sizeof(double) * invb.size());
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
    fw_graph_destroy(g);
    return fail(FW_EHIP, "hipMalloc failed for graph");
  }
  bool up = hipMemcpy(g->d_rowptr, rowptr, sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice) ==
            hipSuccess;
  if (nnz) up &= hipMemcpy(g->d_col, col, sizeof(int32_t) * nnz, hipMemcpyHostToDevice) == hipSuccess;
  if (g->d_pop)
    up &= hipMemcpy(g->d_pop, g->pop.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice) ==
          hipSuccess;
  up &= hipMemcpy(g->d_eid, eid.data(), sizeof(int32_t) * eid.size(), hipMemcpyHostToDevice) ==
        hipSuccess;
  if (!nbadj.empty())
    up &= hipMemcpy(g->d_nbadj, nbadj.data(), sizeof(uint64_t) * nbadj.size(),
                    hipMemcpyHostToDevice) == hipSuccess;
  up &= hipMemcpy(g->d_invb, invb.data(), sizeof(double) * invb.size(), hipMemcpyHostToDevice) ==
        hipSuccess;
  if (!ell.empty())
    up &= hipMemcpy(g->d_ell, ell.data(), sizeof(int32_t) * ell.size(), hipMemcpyHostToDevice) ==
          hipSuccess;
  if (!dbound.empty())
    up &= hipMemcpy(g->d_dbound, dbound.data(), sizeof(int32_t) * dbound.size(),
                    hipMemcpyHostToDevice) == hipSuccess;
  if (!eu.empty()) {
    up &= hipMemcpy(g->d_eu, eu.data(), sizeof(int32_t) * eu.size(), hipMemcpyHostToDevice) ==
          hipSuccess;
    up &= hipMemcpy(g->d_ew, ew.data(), sizeof(int32_t) * ew.size(), hipMemcpyHostToDevice) ==
          hipSuccess;
  }
  if (!up || hipDeviceSynchronize() != hipSuccess) {
    fw_graph_destroy(g);
    return fail(FW_EHIP, "graph upload failed");
  }
  *out = g;
  return FW_OK;
}

void fw_graph_destroy(fw_graph* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->d_rowptr) (void)hipFree(g->d_rowptr);
  if (g->d_col) (void)hipFree(g->d_col);
  if (g->d_pop) (void)hipFree(g->d_pop);
  if (g->d_eid) (void)hipFree(g->d_eid);
  if (g->d_eu) (void)hipFree(g->d_eu);
  if (g->d_ew) (void)hipFree(g->d_ew);
  if (g->d_nbadj) (void)hipFree(g->d_nbadj);
  if (g->d_ell) (void)hipFree(g->d_ell);
  if (g->d_dbound) (void)hipFree(g->d_dbound);
  if (g->d_invb) (void)hipFree(g->d_invb);
  delete g;
}

int fw_graph_info(const fw_graph* g, int64_t info[5]) {
  if (!g || !info) return fail(FW_EINVAL, "fw_graph_info: null");
  info[0] = g->n;
  info[1] = g->nnz / 2;
  info[2] = g->maxdeg;
  info[3] = g->gw;
  info[4] = g->gh;
  return FW_OK;
}

void fw_chains_destroy(fw_chains* c) {
  if (!c) return;
  (void)hipSetDevice(c->g->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_labels, c->d_stats, c->d_pops, c->d_thr, c->d_thr53, c->d_hist_cut, c->d_hist_b,
                  c->d_spill,  c->d_next,  c->d_acc,  c->d_nf,   c->d_lf,       c->d_ps,
                  c->d_pend,   c->d_labval, c->d_flags, c->d_bcnt, c->d_sched, c->d_sched53,
                  c->d_ring,   c->d_ring_node, c->d_hist_ring, c->d_gscr, c->d_segdone,
                  c->d_wsamp,  c->d_wlp};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// work units per slice: the grid kernel's chains per wave (4 / rows per chain), else chains
static long long slice_units(const fw_chains* c) {
  if (!c->p.use16) return c->n_chains;
  const int cpw = 4 / fw_grid16_launch_rows(c->p);
  return (c->n_chains + cpw - 1) / cpw;
}

int fw_chains_create(fw_graph* g, int32_t n_chains, int32_t k, const int16_t* init_labels,
                     int32_t init_per_chain, int32_t proposal_mode, int64_t pop_lo, int64_t pop_hi,
                     const double* thr, int32_t thr_per_chain, uint64_t seed, int64_t chain_id0,
                     fw_chains** out) {
  if (!out || !g || !init_labels || !thr || n_chains <= 0)
    return fail(FW_EINVAL, "fw_chains_create: bad arguments");
  *out = nullptr;
  if (k < 2 || k > FW_MAX_K) return fail(FW_EUNSUPPORTED, "k=%d outside [2, %d]", k, FW_MAX_K);
  if (proposal_mode < FW_PROPOSE_BI || proposal_mode > FW_PROPOSE_CUTEDGE)
    return fail(FW_EINVAL, "unknown proposal mode %d", proposal_mode);
  if (proposal_mode == FW_PROPOSE_BI && k != 2)
    return fail(FW_EINVAL, "slow_reversible_propose_bi needs k == 2 (got %d)", k);
  if (g->maxdeg > FW_MAX_DEG)
    return fail(FW_EUNSUPPORTED, "max degree %d > %d", g->maxdeg, FW_MAX_DEG);
  const int n = g->n, D = g->maxdeg;
  const int G = (n + 63) / 64;
  // row-major grids: the four-chains-per-wave kernel, 2-bit labels when k <= 4
  // (FLIPWALK_NO_GRID16=1 forces the one-chain-per-wave kernel, for A/B parity tests)
  const char* no16 = getenv("FLIPWALK_NO_GRID16");
  int64_t total_pop = 0;
  for (int x = 0; x < n; ++x) total_pop += g->popof(x);
  const bool use16 = fw_grid16_candidate(g->gw, D, G, k, total_pop) && g->gm24 != 0 &&
                     !(no16 && no16[0] == '1');
  int lb = use16 ? fw_grid16_lb(G, k) : pick_lb(k, g->maxdeg);
  {  // the chain kernel on a large grid (k <= 8): 3-bit labels in LDS, search marks in HBM,
     // so more chains fit a CU (C5: 7 -> 9).  FLIPWALK_CSR_LB=3 / 4 forces / forbids it.
    const char* e = getenv("FLIPWALK_CSR_LB");
    const int want = e && e[0] ? atoi(e) : 0;
    if (!use16 && g->gw > 0 && k <= 8 && lb == 4 && (want == 3 || (want == 0 && G > 256)))
      lb = 3;
    // general graphs on padded rows whose k + maxdeg needs 8-bit in-place codes: 5-bit
    // labels with the list search's marks in HBM when that fits more chains per CU — the
    // 8-bit plan is held to 16 by the 4-waves-per-SIMD register budget, the 5-bit one to 20
    // by the 5-wave budget of the lean kernel (C4, 9,000 nodes, k = 18: 16 -> 20 chains per
    // CU, 0.576 -> 0.588 x 10^9; before the lean instantiation the 5-wave budget spilled,
    // 0.495 vs 0.523, profiles/r02/ab/csr_5bit_c4.jsonl).  FLIPWALK_CSR_LB=5 / 8 forces /
    // forbids (5 also for k <= 15).
    if (!use16 && g->gw == 0 && g->d_ell != nullptr && k <= 31 && lb == 8 && want == 0) {
      const long long gs = round16((int64_t)fw_run_gsum_slots(G) * 2), lds = 160 * 1024;
      const long long wbytes = proposal_mode != FW_PROPOSE_CUTEDGE ? round16(((int64_t)n * 2 + 7) / 8) : 0;
      // the 2-bit LDS proposal weights (p.wb) need 4- or 5-bit labels: only l5 carries them
      const long long l8 = round16(((int64_t)n * 8 + 7) / 8 + 8) + gs + 4 * 128;
      const long long l5 = round16(((int64_t)n * 5 + 7) / 8 + 8) + gs + 4 * 8 + wbytes;
      if (n > 16384 || std::min(20ll, lds / l5) > std::min(16ll, lds / l8)) lb = 5;
    }
    if (!use16 && g->gw == 0 && g->d_ell != nullptr && k <= 31 && want == 5) lb = 5;
  }
  if (!lb) return fail(FW_EUNSUPPORTED, "k + maxdeg = %d too large", k + g->maxdeg);

  auto c = new fw_chains();
  c->g = g;
  c->n_chains = n_chains;
  c->k = k;
  c->mode = proposal_mode == FW_PROPOSE_BI ? FW_PROPOSE_PAIRS : proposal_mode;
  c->lb = lb;
  c->D = D;

  // ---- LDS layout
  FwRunParams& p = c->p;
  p.qcap = list_cap(256);
  p.qcap16 = list_cap(384);
  {  // FLIPWALK_FOLD_AT=x: fold the attempt-driven 32-bit counters early (tests)
    const char* e = getenv("FLIPWALK_FOLD_AT");
    const long long v = e && e[0] ? atoll(e) : 0;
    p.fold_at = v >= 64 && v <= 0x80000000ll ? (uint32_t)v : 0x80000000u;
  }
  {  // FLIPWALK_NO_BITBOARD=1: the grid kernel runs every exact search as the list search
    const char* e = getenv("FLIPWALK_NO_BITBOARD");
    p.no_bb = e && e[0] == '1' ? 1 : 0;
    const char* e2 = getenv("FLIPWALK_NO_ROWBB");
    p.no_rowbb = e2 && e2[0] == '1' ? 1 : 0;
  }
  // +8: the grid kernels read label dwords one past the last node
  p.lab_bytes = round16(((int64_t)n * lb + 7) / 8 + 8);
  // chain kernel on padded rows with pairs proposals: 2-bit per-node weights in LDS, so the
  // select reads a group's weights instead of walking its 64 padded rows in L2
  // (FLIPWALK_NO_WB=1: recompute them from the rows, as before)
  {
    const char* e = getenv("FLIPWALK_NO_WB");
    p.wb = !use16 && g->gw == 0 && g->d_ell != nullptr && (lb == 4 || lb == 5) &&
                   c->mode != FW_PROPOSE_CUTEDGE && !(e && e[0] == '1')
               ? 2
               : 0;
  }
  p.off_w = p.lab_bytes;
  p.off_gsum = p.off_w + (p.wb ? round16(((int64_t)n * p.wb + 7) / 8) : 0);
  p.off_list = p.off_gsum + round16((int64_t)fw_run_gsum_slots(G) * 2);  // u16 slots
  p.lds_bytes = p.off_list + p.qcap * 4;
  if (G > 64 * 16) {
    delete c;
    return fail(FW_EUNSUPPORTED, "graph too large (%d weight groups > 1024)", G);
  }
  if (p.lds_bytes > 160 * 1024 - 64) {
    delete c;
    return fail(FW_EUNSUPPORTED, "graph too large for LDS-resident chains (%d B)", p.lds_bytes);
  }

  // ---- initial-state validation and populations
  const int ninit = init_per_chain ? n_chains : 1;
  std::vector<int64_t> pops0((size_t)ninit * k);
  for (int i = 0; i < ninit; ++i) {
    std::string why;
    if (!plan_valid(g, init_labels + (size_t)i * n, k, pop_lo, pop_hi, pops0.data() + (size_t)i * k,
                    &why)) {
      delete c;
      return fail(FW_ESTATE, "initial plan%s invalid: %s",
                  init_per_chain ? (" " + std::to_string(i)).c_str() : "", why.c_str());
    }
  }
  // a chain's HBM record also holds its group sums (derived-state cache, FwRunParams)
  const int lab_stride = p.off_gsum + (int)round16((int64_t)4 * (use16 ? (G + 1) / 2
                                                                      : (fw_run_gsum_slots(G) + 1) / 2));
  std::vector<uint8_t> packed((size_t)n_chains * lab_stride);
  std::vector<int64_t> pops((size_t)n_chains * k);
  {
    std::vector<uint8_t> one(lab_stride);
    for (int i = 0; i < ninit; ++i) {
      pack_labels(init_labels + (size_t)i * n, n, lb, packed.data() + (size_t)i * lab_stride,
                  lab_stride);
    }
    for (int i = ninit; i < n_chains; ++i)
      std::memcpy(packed.data() + (size_t)i * lab_stride, packed.data(), lab_stride);
    for (int i = 0; i < n_chains; ++i)
      std::memcpy(pops.data() + (size_t)i * k, pops0.data() + (size_t)(init_per_chain ? i : 0) * k,
                  sizeof(int64_t) * k);
  }

  if (hipSetDevice(g->device) != hipSuccess) {
    delete c;
    return fail(FW_EHIP, "hipSetDevice failed");
  }
  p.g = g->dev();
  p.n_chains = n_chains;
  p.k = k;
  p.mode = c->mode;
  p.G = G;
  p.pop_lo = pop_lo;
  p.pop_hi = pop_hi;
  p.seed = seed;
  p.chain_id0 = chain_id0;
  p.lab_stride = lab_stride;
  p.lab_copy16 = lab_stride / 16;
  p.gcache_ok = 0;
  p.thr_stride = thr_per_chain ? 2 * D + 1 : 0;
  p.lb = lb;
  p.use16 = use16 ? 1 : 0;
  p.spec = 1;
  if ((use16 ? fw_grid16_plan(p, g->device, &c->grid)
             : fw_run_grid_size(p, lb, g->device, &c->grid)) != 0) {
    delete c;
    return fail(FW_EHIP, "occupancy query failed (LDS %d B)", use16 ? p.lds16 : p.lds_bytes);
  }
  {  // FLIPWALK_GRID_CAP=x: at most x workgroups (tests: more work units than waves)
    const char* e = getenv("FLIPWALK_GRID_CAP");
    const int v = e && e[0] ? atoi(e) : 0;
    if (v >= 1 && v < c->grid) c->grid = v;
  }
  const size_t nthr = (size_t)(thr_per_chain ? n_chains : 1) * (2 * D + 1);
  std::vector<uint64_t> thr53(nthr);
  for (size_t i = 0; i < nthr; ++i) thr53[i] = thr53_of(thr[i]);
  bool ok = hipMalloc(&c->d_labels, packed.size()) == hipSuccess &&
            hipMalloc(&c->d_stats, sizeof(fw_chain_stats) * n_chains) == hipSuccess &&
            hipMalloc(&c->d_pops, sizeof(int64_t) * pops.size()) == hipSuccess &&
            hipMalloc(&c->d_thr, sizeof(double) * nthr) == hipSuccess &&
            hipMalloc(&c->d_thr53, sizeof(uint64_t) * nthr) == hipSuccess &&
            hipMalloc(&c->d_hist_cut, sizeof(unsigned long long) * (g->nnz / 2 + 1 + FW_HIST_PAD)) ==
                hipSuccess &&
            hipMalloc(&c->d_hist_b, sizeof(unsigned long long) * (n + 1 + FW_HIST_PAD)) ==
                hipSuccess &&
            hipMalloc(&c->d_spill, sizeof(uint32_t) * (size_t)c->grid * n) ==
                hipSuccess &&
            hipMalloc(&c->d_next, sizeof(int32_t)) == hipSuccess &&
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreate(&c->ev0) == hipSuccess && hipEventCreate(&c->ev1) == hipSuccess;
  if (!ok) {
    fw_chains_destroy(c);
    return fail(FW_ENOMEM, "device allocation failed for %d chains", n_chains);
  }
  ok = hipMemcpy(c->d_labels, packed.data(), packed.size(), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(c->d_pops, pops.data(), sizeof(int64_t) * pops.size(), hipMemcpyHostToDevice) ==
           hipSuccess &&
       hipMemcpy(c->d_thr, thr, sizeof(double) * nthr, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(c->d_thr53, thr53.data(), sizeof(uint64_t) * nthr, hipMemcpyHostToDevice) ==
           hipSuccess &&
       hipMemset(c->d_stats, 0, sizeof(fw_chain_stats) * n_chains) == hipSuccess &&
       hipMemset(c->d_hist_cut, 0, sizeof(unsigned long long) * (g->nnz / 2 + 1 + FW_HIST_PAD)) ==
           hipSuccess &&
       hipMemset(c->d_hist_b, 0, sizeof(unsigned long long) * (n + 1 + FW_HIST_PAD)) == hipSuccess;
  if (!ok || hipDeviceSynchronize() != hipSuccess) {
    fw_chains_destroy(c);
    return fail(FW_EHIP, "chain upload failed");
  }
  p.labels = c->d_labels;
  p.stats = c->d_stats;
  p.pops = c->d_pops;
  p.thr = c->d_thr;
  p.thr53 = c->d_thr53;
  p.hist_cut = c->d_hist_cut;
  p.hist_b = c->d_hist_b;
  p.spill = c->d_spill;
  p.next_chain = c->d_next;
  p.slices = 1;
  p.prio_shift = 5;
  // one per chain: enough for every kernel's work units (quads, pairs or chains)
  if (hipMalloc(&c->d_segdone, sizeof(int32_t) * (size_t)n_chains) != hipSuccess) {
    fw_chains_destroy(c);
    return fail(FW_ENOMEM, "device allocation failed for %d chains", n_chains);
  }
  p.seg_done = c->d_segdone;
  // HBM visit marks of the chain kernel's list search (race_search_gscr: 5-bit labels only,
  // which run on padded rows; 3-bit labels run only on grids, whose race_search_b3 keeps its
  // marks in the labels).  Footprint: 4 B per node per resident workgroup (C4: 9,000 nodes
  // x 19 x 256 workgroups = 175 MB), beside the equally sized search-list spill buffer.
  if (!use16 && lb == 5) {
    p.gscr_words = n;  // one 32-bit mark per node (race_search_gscr)
    const size_t gb = sizeof(uint32_t) * (size_t)c->grid * (size_t)p.gscr_words;
    if (hipMalloc(&c->d_gscr, gb) != hipSuccess || hipMemset(c->d_gscr, 0, gb) != hipSuccess) {
      fw_chains_destroy(c);
      return fail(FW_ENOMEM, "device allocation failed for %d chains", n_chains);
    }
    p.gscr = c->d_gscr;
  }
  *out = c;
  return FW_OK;
}

// Slices per work unit (a quad of the grid kernel, a chain of the chain kernel) for a
// launch of `steps` steps (see fw_grid16_kernel / fw_run_kernel): with more units than
// resident waves W, the S in 1..8 that minimises a uniform-duration model of the launch,
// ceil(nu S / W) / S rounds of whole-unit time plus ~0.6% of a unit's time per extra slice
// start (measured on the grid kernel: three 333-step launches cost 1.2% more than one
// 1000-step launch net of their tails).  FLIPWALK_SLICES=x forces x (1: whole units).
static int launch_slices(const fw_chains* c, int64_t steps) {
  const char* e = getenv("FLIPWALK_SLICES");
  const int force = e && e[0] ? atoi(e) : 0;
  const long long nq = slice_units(c), W = (long long)c->grid * (c->p.use16 ? fw_grid16_launch_nw(c->p) : 1);
  // the kernels number units in int32: nq * S stays below 2^31
  const long long s_max = std::max<long long>(1, std::min<long long>(8, 0x7FFFFFFFll / std::max(nq, 1ll)));
  if (force >= 1) return (int)std::min<long long>({(long long)force, std::max<int64_t>(steps, 1), s_max});
  if (nq <= W || steps < 64) return 1;
  // chains of a small state (C2's 40x40 grid: 400 B of labels) restart a slice for almost
  // nothing, and more, shorter units even out the units' unequal durations at the end of the
  // launch: the most slices (C2 at S = 3 / 6 / 8: 1.314 / 1.340 / 1.347 x 10^9; C3 at 6 and
  // C4 at 8 lose 0.2% / 2.8%: profiles/r05/slices/)
  if (c->p.lab_bytes <= 1024) return (int)std::min<long long>(s_max, steps / 64);
  int best = 1;
  double best_t = 1e300;
  for (int S = 1; S <= s_max; ++S) {
    const double rounds = (double)((nq * S + W - 1) / W) / S;
    const double t = rounds + 0.006 * (S - 1) * (double)nq / (double)W;
    if (t < best_t - 1e-9) {
      best_t = t;
      best = S;
    }
  }
  return best;
}

// The kernels' wave-priority levels (fw_grid16_kernel, fw_run_kernel): eighths of a unit's
// steps when every unit has a wave slot of its own (the 8,192-chain shard: +1.4% over 32nds),
// quarters when waves take several units (C2 +1.2%, C3 +0.3%, C4 / C5 / Frankengraph
// +0.4-0.6%; 16ths and 128ths lose 0.5% / 1.6% on C3: profiles/r05/prio_levels/)
static int launch_prio_shift(const fw_chains* c) {
  const long long nu = slice_units(c) * (long long)c->p.slices;
  const long long W = (long long)c->grid * (c->p.use16 ? fw_grid16_launch_nw(c->p) : 1);
  return nu <= W ? 3 : 2;
}

int fw_chains_run_async(fw_chains* c, int64_t steps, int32_t max_retries) {
  if (!c || steps < 0 || max_retries <= 0) return fail(FW_EINVAL, "fw_chains_run: bad arguments");
  HIPCHK(hipSetDevice(c->g->device));
  if (steps == 0) return FW_OK;
  if (c->d_acc && c->max_yields + (uint64_t)steps + 1 >= 0xFFFFFFFFull)
    return fail(FW_EUNSUPPORTED, "spatial maps hold yield indices below 2^32");
  if (c->p.trace && steps > FW_MAX_LAUNCH_STEPS)
    return fail(FW_EUNSUPPORTED, "a traced run takes at most %lld steps", (long long)FW_MAX_LAUNCH_STEPS);
  c->max_yields += (uint64_t)steps + (c->ran ? 0 : 1);
  c->ran = true;
  c->p.max_retries = max_retries;
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  // the kernels count a launch's steps (and the per-step sums of degrees and boundary
  // changes) in 32 bits: a longer run is a sequence of launches of at most
  // FW_MAX_LAUNCH_STEPS counted steps (the trajectory does not depend on the split)
  int64_t cap = FW_MAX_LAUNCH_STEPS;
  {  // FLIPWALK_LAUNCH_STEPS=x: a smaller cap (tests of the split)
    const char* e = getenv("FLIPWALK_LAUNCH_STEPS");
    const long long v = e && e[0] ? atoll(e) : 0;
    if (v >= 1 && v < cap) cap = v;
  }
  for (int64_t left = steps; left > 0;) {
    const int64_t s = left < cap ? left : cap;
    c->p.steps = s;
    c->p.gcache_ok = c->gcache_ok ? 1 : 0;
    c->p.slices = !c->p.trace ? launch_slices(c, s) : 1;
    c->p.prio_shift = launch_prio_shift(c);
    if (c->p.slices > 1)
      HIPCHK(hipMemsetAsync(c->d_segdone, 0, sizeof(int32_t) * (size_t)slice_units(c), c->stream));
    HIPCHK(hipMemsetAsync(c->d_next, 0, sizeof(int32_t), c->stream));
    const int le = fw_launch_run(c->p, c->lb, c->grid, c->stream);
    if (le != 0) {
      c->gcache_ok = false;
      return fail(FW_EHIP, "kernel launch failed: %s", hipGetErrorString((hipError_t)le));
    }
    c->gcache_ok = true;  // this launch writes every chain's record back
    left -= s;
  }
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  return FW_OK;
}

int fw_chains_sync(fw_chains* c) {
  if (!c) return fail(FW_EINVAL, "null handle");
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  return FW_OK;
}

int fw_chains_run(fw_chains* c, int64_t steps, int32_t max_retries) {
  int rc = fw_chains_run_async(c, steps, max_retries);
  if (rc) return rc;
  return fw_chains_sync(c);
}

int fw_chains_run_traced(fw_chains* c, int64_t steps, int32_t max_retries, int32_t* host_trace,
                         size_t bytes) {
  if (!c || !host_trace || steps <= 0) return fail(FW_EINVAL, "fw_chains_run_traced: bad arguments");
  const size_t need = sizeof(int32_t) * (size_t)c->n_chains * (size_t)steps;
  if (bytes < need) return fail(FW_EINVAL, "trace needs %zu bytes", need);
  HIPCHK(hipSetDevice(c->g->device));
  int32_t* d_trace = nullptr;
  HIPCHK(hipMalloc(&d_trace, need));
  int rc = FW_OK;
  if (hipMemsetAsync(d_trace, 0xFE, need, c->stream) != hipSuccess) {
    rc = fail(FW_EHIP, "trace memset failed");
  } else {
    c->p.trace = d_trace;
    rc = fw_chains_run(c, steps, max_retries);
    c->p.trace = nullptr;
    if (rc == FW_OK && hipMemcpy(host_trace, d_trace, need, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(FW_EHIP, "trace download failed");
  }
  (void)hipFree(d_trace);
  return rc;
}

double fw_chains_last_kernel_ms(const fw_chains* c) {
  if (!c || !c->timed) return -1.0;
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.0;
  return ms;
}

int fw_chains_launch_info(const fw_chains* c, int64_t info[8]) {
  if (!c || !info) return fail(FW_EINVAL, "fw_chains_launch_info: null");
  HIPCHK(hipSetDevice(c->g->device));
  const FwRunParams& p = c->p;
  void* fn = p.use16 ? fw_grid16_fn(p) : fw_run_fn(p, c->lb);
  if (!fn) return fail(FW_EHIP, "no kernel for this plan");
  hipFuncAttributes at;
  HIPCHK(hipFuncGetAttributes(&at, fn));
  const int nw = p.use16 ? fw_grid16_launch_nw(p) : 1;
  const int lds = p.use16 ? p.lds16 : p.lds_bytes;
  int per_cu = 0;
  HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * nw, (size_t)lds));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, c->g->device));
  info[0] = c->grid;
  info[1] = nw;
  info[2] = p.use16 ? 4 / fw_grid16_launch_rows(p) : 1;
  info[3] = lds;
  info[4] = at.numRegs;
  info[5] = (int64_t)at.localSizeBytes;
  info[6] = prop.multiProcessorCount;
  info[7] = per_cu;
  return FW_OK;
}

int fw_chains_read(fw_chains* c, int32_t what, void* host_dst, size_t bytes) {
  if (!c || !host_dst) return fail(FW_EINVAL, "fw_chains_read: null");
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int n = c->g->n;
  size_t need = 0;
  switch (what) {
    case FW_READ_LABELS: {
      need = sizeof(int16_t) * (size_t)c->n_chains * n;
      if (bytes < need) return fail(FW_EINVAL, "labels need %zu bytes", need);
      std::vector<uint8_t> packed((size_t)c->n_chains * c->p.lab_stride);
      HIPCHK(hipMemcpy(packed.data(), c->d_labels, packed.size(), hipMemcpyDeviceToHost));
      for (int i = 0; i < c->n_chains; ++i)
        unpack_labels(packed.data() + (size_t)i * c->p.lab_stride, n, c->lb,
                      static_cast<int16_t*>(host_dst) + (size_t)i * n);
      return FW_OK;
    }
    case FW_READ_STATS:
      need = sizeof(fw_chain_stats) * c->n_chains;
      if (bytes < need) return fail(FW_EINVAL, "stats need %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_stats, need, hipMemcpyDeviceToHost));
      return FW_OK;
    case FW_READ_HIST_CUT:
      need = sizeof(uint64_t) * (c->g->nnz / 2 + 1);
      if (bytes < need) return fail(FW_EINVAL, "hist_cut needs %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_hist_cut, need, hipMemcpyDeviceToHost));
      return FW_OK;
    case FW_READ_HIST_B:
      need = sizeof(uint64_t) * (n + 1);
      if (bytes < need) return fail(FW_EINVAL, "hist_b needs %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_hist_b, need, hipMemcpyDeviceToHost));
      return FW_OK;
    case FW_READ_POPS:
      need = sizeof(int64_t) * (size_t)c->n_chains * c->k;
      if (bytes < need) return fail(FW_EINVAL, "pops need %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_pops, need, hipMemcpyDeviceToHost));
      return FW_OK;
    case FW_READ_HIST_RING:
      if (!c->ring_n) return fail(FW_ESTATE, "the ring observable is not enabled");
      need = sizeof(uint64_t) * ring_bins(c->ring_n);
      if (bytes < need) return fail(FW_EINVAL, "hist_ring needs %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_hist_ring, need, hipMemcpyDeviceToHost));
      return FW_OK;
    case FW_READ_RING_PAIR: {
      if (!c->ring_n) return fail(FW_ESTATE, "the ring observable is not enabled");
      need = sizeof(int32_t) * 2 * (size_t)c->n_chains;
      if (bytes < need) return fail(FW_EINVAL, "ring pairs need %zu bytes", need);
      std::vector<uint8_t> packed((size_t)c->n_chains * c->p.lab_stride);
      HIPCHK(hipMemcpy(packed.data(), c->d_labels, packed.size(), hipMemcpyDeviceToHost));
      std::vector<int16_t> lab(n);
      int32_t* out = static_cast<int32_t*>(host_dst);
      for (int i = 0; i < c->n_chains; ++i) {
        unpack_labels(packed.data() + (size_t)i * c->p.lab_stride, n, c->lb, lab.data());
        ring_pair_of(c, lab.data(), out + 2 * (size_t)i);
      }
      return FW_OK;
    }
    case FW_READ_WAITS:
      if (!c->d_wsamp) return fail(FW_ESTATE, "sampled waits are not enabled");
      need = sizeof(double) * 2 * (size_t)c->n_chains;
      if (bytes < need) return fail(FW_EINVAL, "waits need %zu bytes", need);
      HIPCHK(hipMemcpy(host_dst, c->d_wsamp, need, hipMemcpyDeviceToHost));
      return FW_OK;
    default:
      return fail(FW_EINVAL, "unknown read kind %d", what);
  }
}

int fw_chains_write(fw_chains* c, int32_t what, const void* host_src, size_t bytes) {
  if (!c || !host_src) return fail(FW_EINVAL, "fw_chains_write: null");
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int n = c->g->n;
  size_t need = 0;
  switch (what) {
    case FW_READ_LABELS: {
      need = sizeof(int16_t) * (size_t)c->n_chains * n;
      if (bytes < need) return fail(FW_EINVAL, "labels need %zu bytes", need);
      const int16_t* lab = static_cast<const int16_t*>(host_src);
      std::vector<uint8_t> packed((size_t)c->n_chains * c->p.lab_stride);
      std::vector<int64_t> pops((size_t)c->n_chains * c->k);
      for (int i = 0; i < c->n_chains; ++i) {
        std::string why;
        if (!plan_valid(c->g, lab + (size_t)i * n, c->k, c->p.pop_lo, c->p.pop_hi,
                        pops.data() + (size_t)i * c->k, &why))
          return fail(FW_ESTATE, "plan %d invalid: %s", i, why.c_str());
        pack_labels(lab + (size_t)i * n, n, c->lb, packed.data() + (size_t)i * c->p.lab_stride,
                    c->p.lab_stride);
      }
      // the spatial maps carry per-node run state of the current plans (not part of a
      // checkpoint): a new plan under them would resume with wrong maps, so refuse
      if (c->d_acc)
        return fail(FW_ESTATE, "plans cannot be written while the spatial maps are enabled");
      c->gcache_ok = false;  // group sums and counts are re-derived from the new plans
      HIPCHK(hipMemcpy(c->d_labels, packed.data(), packed.size(), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(c->d_pops, pops.data(), sizeof(int64_t) * pops.size(),
                       hipMemcpyHostToDevice));
      if (c->p.bcnt) {  // FW_ACCEPT_BOUNDARY's flagged-node counts follow the new plans
        HIPCHK(hipMemset(c->d_bcnt, 0, sizeof(int32_t) * (size_t)c->n_chains * c->k));
        if (fw_launch_bcnt_init(c->p, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
          return fail(FW_EHIP, "flag count re-init failed");
      }
      return FW_OK;
    }
    case FW_READ_STATS:
      need = sizeof(fw_chain_stats) * c->n_chains;
      if (bytes < need) return fail(FW_EINVAL, "stats need %zu bytes", need);
      c->gcache_ok = false;  // cut / bnodes / npairs come from the caller's records
      HIPCHK(hipMemcpy(c->d_stats, host_src, need, hipMemcpyHostToDevice));
      c->ran = true;  // the initial state was yielded in the run being resumed
      {  // the maps' 2^32 yield-index guard counts the yields already made
        const fw_chain_stats* st = static_cast<const fw_chain_stats*>(host_src);
        uint64_t ymax = 0;
        for (int i = 0; i < c->n_chains; ++i) ymax = std::max<uint64_t>(ymax, st[i].yields);
        c->max_yields = ymax;
      }
      return FW_OK;
    case FW_READ_HIST_CUT:
      need = sizeof(uint64_t) * (c->g->nnz / 2 + 1);
      if (bytes < need) return fail(FW_EINVAL, "hist_cut needs %zu bytes", need);
      HIPCHK(hipMemcpy(c->d_hist_cut, host_src, need, hipMemcpyHostToDevice));
      return FW_OK;
    case FW_READ_HIST_B:
      need = sizeof(uint64_t) * (n + 1);
      if (bytes < need) return fail(FW_EINVAL, "hist_b needs %zu bytes", need);
      HIPCHK(hipMemcpy(c->d_hist_b, host_src, need, hipMemcpyHostToDevice));
      return FW_OK;
    case FW_READ_HIST_RING:
      if (!c->ring_n) return fail(FW_ESTATE, "the ring observable is not enabled");
      need = sizeof(uint64_t) * ring_bins(c->ring_n);
      if (bytes < need) return fail(FW_EINVAL, "hist_ring needs %zu bytes", need);
      HIPCHK(hipMemcpy(c->d_hist_ring, host_src, need, hipMemcpyHostToDevice));
      return FW_OK;
    case FW_READ_WAITS:
      if (!c->d_wsamp) return fail(FW_ESTATE, "sampled waits are not enabled");
      need = sizeof(double) * 2 * (size_t)c->n_chains;
      if (bytes < need) return fail(FW_EINVAL, "waits need %zu bytes", need);
      HIPCHK(hipMemcpy(c->d_wsamp, host_src, need, hipMemcpyHostToDevice));
      return FW_OK;
    default:
      return fail(FW_EINVAL, "fw_chains_write: unsupported kind %d", what);
  }
}

int fw_chains_reset_observables(fw_chains* c) {
  if (!c) return fail(FW_EINVAL, "null handle");
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  std::vector<fw_chain_stats> st(c->n_chains);
  HIPCHK(hipMemcpy(st.data(), c->d_stats, sizeof(fw_chain_stats) * st.size(),
                   hipMemcpyDeviceToHost));
  for (auto& s : st) {
    s.yields = 0;
    s.sum_cut = 0;
    s.sum_bnodes = 0;
    s.sum_invb = 0.0;
  }
  HIPCHK(hipMemcpy(c->d_stats, st.data(), sizeof(fw_chain_stats) * st.size(),
                   hipMemcpyHostToDevice));
  HIPCHK(hipMemset(c->d_hist_cut, 0,
                   sizeof(unsigned long long) * (c->g->nnz / 2 + 1 + FW_HIST_PAD)));
  HIPCHK(hipMemset(c->d_hist_b, 0, sizeof(unsigned long long) * (c->g->n + 1 + FW_HIST_PAD)));
  if (c->d_hist_ring)
    HIPCHK(hipMemset(c->d_hist_ring, 0, sizeof(unsigned long long) * ring_bins(c->ring_n)));
  if (c->d_acc) {  // maps restart from the current plans (yield indices restart at 0)
    const size_t C = (size_t)c->n_chains, n = (size_t)c->g->n, E = (size_t)c->g->nnz / 2;
    HIPCHK(hipMemset(c->d_acc, 0, sizeof(int64_t) * std::max<size_t>(C * E, 1)));
    HIPCHK(hipMemset(c->d_nf, 0, sizeof(uint32_t) * C * n));
    HIPCHK(hipMemset(c->d_lf, 0, sizeof(uint32_t) * C * n));
    if (fw_launch_map_init(c->p, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return fail(FW_EHIP, "map re-init failed");
    c->max_yields = 0;
  }
  return FW_OK;
}

int fw_chains_set_accept(fw_chains* c, int32_t rule, const uint8_t* node_flags) {
  if (!c) return fail(FW_EINVAL, "null handle");
  if (rule < FW_ACCEPT_CUT || rule > FW_ACCEPT_BOUNDARY)
    return fail(FW_EINVAL, "unknown accept rule %d", rule);
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (rule == FW_ACCEPT_BOUNDARY) {
    if (!node_flags) return fail(FW_EINVAL, "FW_ACCEPT_BOUNDARY needs node flags");
    const int n = c->g->n;
    int nflag = 0;
    for (int x = 0; x < n; ++x) nflag += node_flags[x] ? 1 : 0;
    if (nflag == 0)  // boundary_condition reads blist[0] (grid_chain_sec11.py:46)
      return fail(FW_EINVAL, "boundary_condition needs at least one boundary_node");
    const size_t nb = sizeof(int32_t) * (size_t)c->n_chains * c->k;
    if (!c->d_flags) {
      if (hipMalloc(&c->d_flags, n) != hipSuccess || hipMalloc(&c->d_bcnt, nb) != hipSuccess)
        return fail(FW_ENOMEM, "flag buffers");
    }
    HIPCHK(hipMemcpy(c->d_flags, node_flags, n, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(c->d_bcnt, 0, nb));
    c->p.flags = c->d_flags;
    c->p.bcnt = c->d_bcnt;
    if (fw_launch_bcnt_init(c->p, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return fail(FW_EHIP, "flag count init failed");
  }
  c->p.accept = rule;
  return FW_OK;
}

int fw_chains_set_schedule(fw_chains* c, const double* rows, int32_t n_rows, int64_t t0) {
  if (!c) return fail(FW_EINVAL, "null handle");
  if (n_rows < 0 || (n_rows > 0 && !rows)) return fail(FW_EINVAL, "bad schedule rows");
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->d_sched) (void)hipFree(c->d_sched);
  if (c->d_sched53) (void)hipFree(c->d_sched53);
  c->d_sched = nullptr;
  c->d_sched53 = nullptr;
  c->p.sched = nullptr;
  c->p.sched53 = nullptr;
  c->p.sched_rows = 0;
  c->p.sched_t0 = 0;
  if (n_rows == 0) return FW_OK;
  const size_t m = (size_t)n_rows * (2 * c->g->maxdeg + 1);
  std::vector<uint64_t> r53(m);
  for (size_t i = 0; i < m; ++i) r53[i] = thr53_of(rows[i]);
  if (hipMalloc(&c->d_sched, sizeof(double) * m) != hipSuccess ||
      hipMalloc(&c->d_sched53, sizeof(uint64_t) * m) != hipSuccess)
    return fail(FW_ENOMEM, "schedule of %d rows", n_rows);
  HIPCHK(hipMemcpy(c->d_sched, rows, sizeof(double) * m, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_sched53, r53.data(), sizeof(uint64_t) * m, hipMemcpyHostToDevice));
  c->p.sched = c->d_sched;
  c->p.sched53 = c->d_sched53;
  c->p.sched_rows = n_rows;
  c->p.sched_t0 = t0;
  return FW_OK;
}

int fw_chains_enable_maps(fw_chains* c, const int64_t* label_values) {
  if (!c) return fail(FW_EINVAL, "null handle");
  if (c->ran) return fail(FW_ESTATE, "enable the spatial maps before the first run");
  if (c->d_acc) return FW_OK;
  HIPCHK(hipSetDevice(c->g->device));
  const size_t C = (size_t)c->n_chains, n = (size_t)c->g->n, E = (size_t)c->g->nnz / 2;
  std::vector<int64_t> lv(c->k);
  for (int d = 0; d < c->k; ++d) lv[d] = label_values ? label_values[d] : d;
  bool ok = hipMalloc(&c->d_acc, sizeof(int64_t) * std::max<size_t>(C * E, 1)) == hipSuccess &&
            hipMalloc(&c->d_nf, sizeof(uint32_t) * C * n) == hipSuccess &&
            hipMalloc(&c->d_lf, sizeof(uint32_t) * C * n) == hipSuccess &&
            hipMalloc(&c->d_ps, sizeof(int64_t) * C * n) == hipSuccess &&
            hipMalloc(&c->d_pend, sizeof(int32_t) * 4 * C) == hipSuccess &&
            hipMalloc(&c->d_labval, sizeof(int64_t) * lv.size()) == hipSuccess;
  if (!ok) {
    void* bufs[] = {c->d_acc, c->d_nf, c->d_lf, c->d_ps, c->d_pend, c->d_labval};
    for (void* b : bufs)
      if (b) (void)hipFree(b);
    c->d_acc = nullptr;
    c->d_nf = c->d_lf = nullptr;
    c->d_ps = nullptr;
    c->d_pend = nullptr;
    c->d_labval = nullptr;
    return fail(FW_ENOMEM, "spatial maps need %zu MB of device memory",
                (C * (8 * E + 16 * n)) >> 20);
  }
  HIPCHK(hipMemcpy(c->d_labval, lv.data(), sizeof(int64_t) * lv.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemsetAsync(c->d_acc, 0, sizeof(int64_t) * std::max<size_t>(C * E, 1), c->stream));
  HIPCHK(hipMemsetAsync(c->d_nf, 0, sizeof(uint32_t) * C * n, c->stream));
  HIPCHK(hipMemsetAsync(c->d_lf, 0, sizeof(uint32_t) * C * n, c->stream));
  FwRunParams& p = c->p;
  p.m_acc = c->d_acc;
  p.m_nf = c->d_nf;
  p.m_lf = c->d_lf;
  p.m_ps = c->d_ps;
  p.m_pend = c->d_pend;
  p.m_labval = c->d_labval;
  const int le = fw_launch_map_init(p, c->stream);
  if (le != 0) return fail(FW_EHIP, "map init launch failed: %s", hipGetErrorString((hipError_t)le));
  HIPCHK(hipStreamSynchronize(c->stream));
  return FW_OK;
}

int fw_chains_enable_waits(fw_chains* c, const double* p_table) {
  if (!c || !p_table) return fail(FW_EINVAL, "fw_chains_enable_waits: null");
  if (c->ran) return fail(FW_ESTATE, "enable the sampled waits before the first run");
  const int n = c->g->n;
  std::vector<double> lp((size_t)n + 1);
  for (int b = 0; b <= n; ++b) {
    if (!(p_table[b] >= 0.0 && p_table[b] < 1.0))
      return fail(FW_EINVAL, "p_table[%d] = %g outside [0, 1)", b, p_table[b]);
    lp[b] = fw_log1p(-p_table[b]);
  }
  HIPCHK(hipSetDevice(c->g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (!c->d_wsamp) {
    if (hipMalloc(&c->d_wsamp, sizeof(double) * 2 * (size_t)c->n_chains) != hipSuccess ||
        hipMalloc(&c->d_wlp, sizeof(double) * lp.size()) != hipSuccess) {
      if (c->d_wsamp) (void)hipFree(c->d_wsamp);
      c->d_wsamp = nullptr;
      return fail(FW_ENOMEM, "sampled-wait buffers");
    }
  }
  HIPCHK(hipMemcpy(c->d_wlp, lp.data(), sizeof(double) * lp.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(c->d_wsamp, 0, sizeof(double) * 2 * (size_t)c->n_chains));
  c->p.wsamp = c->d_wsamp;
  c->p.wlp = c->d_wlp;
  return FW_OK;
}

int fw_chains_enable_ring(fw_chains* c, const int32_t* ring_u, const int32_t* ring_w,
                          int32_t n_ring) {
  if (!c || !ring_u || !ring_w) return fail(FW_EINVAL, "fw_chains_enable_ring: null");
  if (n_ring < 2 || n_ring > 1024) return fail(FW_EINVAL, "n_ring = %d outside [2, 1024]", n_ring);
  const fw_graph* g = c->g;
  std::vector<uint8_t> node((size_t)g->n, 0);
  for (int r = 0; r < n_ring; ++r) {
    const int u = ring_u[r], w = ring_w[r];
    if (u < 0 || u >= g->n || w < 0 || w >= g->n ||
        !std::binary_search(g->col.begin() + g->rowptr[u], g->col.begin() + g->rowptr[u + 1], w))
      return fail(FW_EINVAL, "ring edge %d (%d, %d) is not an edge of the graph", r, u, w);
    node[u] = node[w] = 1;
  }
  HIPCHK(hipSetDevice(g->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (!c->d_ring_node && hipMalloc(&c->d_ring_node, (size_t)g->n) != hipSuccess)
    return fail(FW_ENOMEM, "ring node flags");
  // the new buffers first: on failure the handle keeps its previous ring intact
  int32_t* d_ring = nullptr;
  unsigned long long* d_hist = nullptr;
  if (hipMalloc(&d_ring, sizeof(int32_t) * 2 * (size_t)n_ring) != hipSuccess ||
      hipMalloc(&d_hist, sizeof(unsigned long long) * ring_bins(n_ring)) != hipSuccess) {
    if (d_ring) (void)hipFree(d_ring);
    return fail(FW_ENOMEM, "ring histogram of %d edges", n_ring);
  }
  if (c->d_ring) (void)hipFree(c->d_ring);
  if (c->d_hist_ring) (void)hipFree(c->d_hist_ring);
  c->d_ring = d_ring;
  c->d_hist_ring = d_hist;
  c->ring_u.assign(ring_u, ring_u + n_ring);
  c->ring_w.assign(ring_w, ring_w + n_ring);
  c->ring_n = n_ring;
  HIPCHK(hipMemcpy(c->d_ring, ring_u, sizeof(int32_t) * n_ring, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_ring + n_ring, ring_w, sizeof(int32_t) * n_ring, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_ring_node, node.data(), node.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(c->d_hist_ring, 0, sizeof(unsigned long long) * ring_bins(n_ring)));
  c->p.ring_n = n_ring;
  c->p.ring_u = c->d_ring;
  c->p.ring_w = c->d_ring + n_ring;
  c->p.ring_node = c->d_ring_node;
  c->p.hist_ring = c->d_hist_ring;
  return FW_OK;
}

int fw_chains_read_map(fw_chains* c, int32_t what, int32_t chain0, int32_t n_chains, int32_t flags,
                       int64_t* dst, size_t bytes) {
  if (!c || !dst) return fail(FW_EINVAL, "fw_chains_read_map: null");
  if (!c->d_acc) return fail(FW_ESTATE, "spatial maps are not enabled");
  if (what < FW_MAP_CUT_TIMES || what > FW_MAP_LAST_FLIPPED)
    return fail(FW_EINVAL, "unknown map %d", what);
  if (chain0 < 0 || n_chains <= 0 || (int64_t)chain0 + n_chains > c->n_chains)
    return fail(FW_EINVAL, "chain range [%d, %d) outside [0, %d)", chain0, chain0 + n_chains,
                c->n_chains);
  const int E = c->g->nnz / 2, n = c->g->n;
  const size_t M = what == FW_MAP_CUT_TIMES ? (size_t)E : (size_t)n;
  const bool sum = (flags & FW_MAP_SUM) != 0;
  const size_t need = sizeof(int64_t) * M * (sum ? 1 : (size_t)n_chains);
  if (bytes < need) return fail(FW_EINVAL, "map needs %zu bytes", need);
  if (M == 0) return FW_OK;
  HIPCHK(hipSetDevice(c->g->device));
  int64_t* d_out = nullptr;
  HIPCHK(hipMalloc(&d_out, need));
  FwMapRead m{};
  m.acc = c->d_acc;
  m.nf = c->d_nf;
  m.lf = c->d_lf;
  m.ps = c->d_ps;
  m.pend = c->d_pend;
  m.labval = c->d_labval;
  m.labels = c->d_labels;
  m.lab_stride = c->p.lab_stride;
  m.stats = c->d_stats;
  m.eu = c->g->d_eu;
  m.ew = c->g->d_ew;
  m.n = n;
  m.E = E;
  m.lb = c->lb;
  m.what = what;
  m.sum = sum ? 1 : 0;
  m.finalize = (flags & FW_MAP_FINALIZE) ? 1 : 0;
  m.chain0 = chain0;
  m.n_chains = n_chains;
  m.out = d_out;
  int rc = FW_OK;
  const int le = fw_launch_map_read(m, c->stream);
  if (le != 0)
    rc = fail(FW_EHIP, "map read launch failed: %s", hipGetErrorString((hipError_t)le));
  else if (hipMemcpyAsync(dst, d_out, need, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
           hipStreamSynchronize(c->stream) != hipSuccess)
    rc = fail(FW_EHIP, "map download failed");
  (void)hipFree(d_out);
  return rc;
}

int fw_eval_flips(fw_graph* g, const int16_t* labels, int32_t k, const int32_t* v,
                  const int16_t* target, int32_t m, int64_t pop_lo, int64_t pop_hi, int32_t* dcut,
                  uint8_t* contig, uint8_t* pop_ok, int32_t* dboundary) {
  if (!g || !labels || (m > 0 && (!v || !target || !dcut || !contig || !pop_ok || !dboundary)) ||
      m < 0)
    return fail(FW_EINVAL, "fw_eval_flips: bad arguments");
  if (m == 0) return FW_OK;
  if (k < 2 || k > FW_MAX_K) return fail(FW_EUNSUPPORTED, "k=%d outside [2, %d]", k, FW_MAX_K);
  if (g->maxdeg > FW_MAX_DEG) return fail(FW_EUNSUPPORTED, "max degree %d", g->maxdeg);
  const int lb = pick_lb(k, g->maxdeg);
  if (!lb) return fail(FW_EUNSUPPORTED, "k + maxdeg too large");
  const int n = g->n;
  std::vector<int64_t> pops(k, 0);
  for (int x = 0; x < n; ++x) {
    if (labels[x] < 0 || labels[x] >= k) return fail(FW_EINVAL, "label out of range at %d", x);
    pops[labels[x]] += g->popof(x);
  }
  for (int i = 0; i < m; ++i) {
    if (v[i] < 0 || v[i] >= n || target[i] < 0 || target[i] >= k || target[i] == labels[v[i]])
      return fail(FW_EINVAL, "flip %d (v=%d, target=%d) is not a relabelling", i, v[i], target[i]);
  }
  FwEvalParams p{};
  p.qcap = list_cap(256);
  p.lab_bytes = round16(((int64_t)n * lb + 7) / 8);
  p.off_list = p.lab_bytes;
  p.lds_bytes = p.off_list + p.qcap * 4;
  if (p.lds_bytes > 160 * 1024 - 64) return fail(FW_EUNSUPPORTED, "graph too large for LDS");
  std::vector<uint8_t> packed(p.lab_bytes);
  pack_labels(labels, n, lb, packed.data(), p.lab_bytes);
  HIPCHK(hipSetDevice(g->device));
  const int grid = std::min(m, 2048);
  uint8_t* d_lab = nullptr;
  int64_t* d_pops = nullptr;
  int32_t *d_v = nullptr, *d_dcut = nullptr, *d_db = nullptr;
  int16_t* d_t = nullptr;
  uint8_t *d_contig = nullptr, *d_pok = nullptr;
  uint32_t* d_spill = nullptr;
  bool ok = hipMalloc(&d_lab, p.lab_bytes) == hipSuccess &&
            hipMalloc(&d_pops, sizeof(int64_t) * k) == hipSuccess &&
            hipMalloc(&d_v, sizeof(int32_t) * m) == hipSuccess &&
            hipMalloc(&d_t, sizeof(int16_t) * m) == hipSuccess &&
            hipMalloc(&d_dcut, sizeof(int32_t) * m) == hipSuccess &&
            hipMalloc(&d_db, sizeof(int32_t) * m) == hipSuccess &&
            hipMalloc(&d_contig, m) == hipSuccess && hipMalloc(&d_pok, m) == hipSuccess &&
            hipMalloc(&d_spill, sizeof(uint32_t) * (size_t)grid * n) == hipSuccess;
  int rc = FW_OK;
  if (!ok) {
    rc = fail(FW_ENOMEM, "device allocation failed in fw_eval_flips");
  } else {
    ok = hipMemcpy(d_lab, packed.data(), p.lab_bytes, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(d_pops, pops.data(), sizeof(int64_t) * k, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(d_v, v, sizeof(int32_t) * m, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(d_t, target, sizeof(int16_t) * m, hipMemcpyHostToDevice) == hipSuccess;
    p.g = g->dev();
    p.labels = d_lab;
    p.pops = d_pops;
    p.k = k;
    p.m = m;
    p.v = d_v;
    p.target = d_t;
    p.pop_lo = pop_lo;
    p.pop_hi = pop_hi;
    p.dcut = d_dcut;
    p.contig = d_contig;
    p.pop_ok = d_pok;
    p.dboundary = d_db;
    p.spill = d_spill;
    if (!ok) {
      rc = fail(FW_EHIP, "upload failed in fw_eval_flips");
    } else if (const int le = fw_launch_eval(p, lb, grid, nullptr)) {
      rc = fail(FW_EHIP, "eval launch failed: %s", hipGetErrorString((hipError_t)le));
    } else if (hipDeviceSynchronize() != hipSuccess) {
      rc = fail(FW_EHIP, "eval kernel failed: %s", hipGetErrorString(hipGetLastError()));
    } else {
      ok = hipMemcpy(dcut, d_dcut, sizeof(int32_t) * m, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(dboundary, d_db, sizeof(int32_t) * m, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(contig, d_contig, m, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(pop_ok, d_pok, m, hipMemcpyDeviceToHost) == hipSuccess;
      if (!ok) rc = fail(FW_EHIP, "download failed in fw_eval_flips");
    }
  }
  void* bufs[] = {d_lab, d_pops, d_v, d_t, d_dcut, d_db, d_contig, d_pok, d_spill};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  return rc;
}

}  // extern "C"
