// fw_internal.h — structs shared by the host API (fw_api.hip) and the kernels
// (fw_kernels.hip).  Not part of the public ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/flipwalk.h"

// Kernel-variant limits (checked on the host before any launch).
#define FW_MAX_DEG 63   // lanes 1..deg of one wave hold v's neighbours during commit
#define FW_MAX_K 64     // foreign-label sets are 64-bit masks
#define FW_HIST_PAD 64  // histogram window slack past the last bin
// counted steps per kernel launch: per-launch step counters and the per-step sums of
// degrees (<= 63) and boundary changes (<= 64) stay below 2^31 in 32 bits
#define FW_MAX_LAUNCH_STEPS (1ll << 25)

struct FwGraphDev {
  const int32_t* rowptr;  // [n+1]
  const int32_t* col;     // [nnz]
  const int32_t* eid;     // [nnz] canonical edge id of each CSR entry
  const uint64_t* nbadj;  // [nnz] entry (v, i): bit j set iff neighbours i and j of v are adjacent
  const int32_t* ell;     // [n][16] neighbours padded with -1 (general graphs, max degree <= 16)
  const int32_t* dbound;  // with ell: [n] max degree over x and its neighbours, then
                          // [ceil(n/64)] max degree in each 64-node group (row loop bounds)
  const int64_t* pop;     // [n] or nullptr (unit populations)
  const double* invb;     // [n+1] 1.0 / max(b, 1), correctly rounded (no fp64 divide per step)
  int32_t n, nedges, maxdeg;
  int32_t gw, gh;         // grid width/height (gw == 0: general CSR)
  uint64_t gmagic;        // ceil(2^42 / gw): x / gw == (x * gmagic) >> 42 for x < 2^21
  uint32_t gm32;          // ceil(2^32 / gw): x / gw == mulhi(x, gm32) for x * gw < 2^32
  uint32_t gm24, gs24;    // x / gw == umul24(x, gm24) >> gs24 for x < 2^15 (0: none found)
};

struct FwRunParams {
  FwGraphDev g;
  uint8_t* labels;             // packed LB-bit labels, chain c at labels + c*lab_stride
  int64_t lab_stride;          // bytes per chain (multiple of 16)
  fw_chain_stats* stats;       // [n_chains]
  int64_t* pops;               // [n_chains][k]
  const double* thr;           // [n_chains or 1][2*maxdeg+1]
  const uint64_t* thr53;       // same shape: ceil(thr * 2^53) clamped to 2^53 (u < thr <=>
                               // u * 2^53 < thr53 for CPython's 53-bit u)
  int32_t thr_stride;          // 0 (shared table) or 2*maxdeg+1
  // threshold schedule (fw_chains_set_schedule): when set, a proposal whose step_num
  // (accepted flips so far + 1) is t uses row clamp(t - sched_t0, 0, sched_rows - 1)
  const double* sched;         // [sched_rows][2*maxdeg+1] or null
  const uint64_t* sched53;     // the same rows in the integer form of thr53
  int64_t sched_t0;
  int32_t sched_rows;
  unsigned long long* hist_cut;  // [nedges+1+FW_HIST_PAD]
  unsigned long long* hist_b;    // [n+1+FW_HIST_PAD]
  uint32_t* spill;             // [grid][n] search-list spill
  uint32_t* gscr;              // race_search_gscr (5-bit labels, padded rows): [grid][n] 32-bit visit marks (zero)
  int32_t gscr_words;
  int32_t* next_chain;         // dynamic chain counter (zeroed before launch)
  int32_t* trace;              // optional [n_chains][steps]: v*64+target if accepted, -1 if not
  int32_t n_chains, k, mode, G;  // G = ceil(n/64) weight groups
  int64_t pop_lo, pop_hi;
  uint64_t seed;
  int64_t chain_id0;
  int64_t steps;
  int32_t max_retries;
  uint32_t fold_at;             // n_sdeg at which attempt-driven 32-bit counters fold (2^31)
  int32_t qcap;                // search-list entries held in LDS
  // LDS layout (bytes from the dynamic shared base)
  int32_t lab_bytes;           // packed label bytes (multiple of 16)
  int32_t off_gsum, off_list, lds_bytes;
  // chain kernel on padded rows, pairs proposals: 2-bit per-node proposal weights at off_w
  // (between the labels and the group sums), saturated at 3 (wb = 2; 0: none)
  int32_t off_w, wb;
  int32_t off_ssum;            // grid kernel, large grids: supergroup sums in the slot
  int32_t lb;                  // label bits per node (2, 4 or 8)
  int32_t use16;               // 1: launch the four-chains-per-wave grid kernel
  // grid kernel LDS plan (fw_grid16_plan): 4*nw chain slots, shared scratch and list
  int32_t slot_stride;         // bytes between chain slots
  int32_t nw;                  // waves per workgroup (of the plan's lean kernel)
  int32_t spec;                // rows per chain of the lean kernel (speculative attempts: 1, 2, 4)
  int32_t w2;                  // 1: the lean R = 1 kernel under a 2-waves-per-SIMD register budget
                               // (launches with at most 2 waves of work per SIMD: fw_grid16_plan)
  int32_t off_scr, scr_bytes;  // 4-bit search scratch
  int32_t off_list16, qcap16;  // shared visit list
  int32_t no_bb;               // 1: exact searches skip the bitboard form (tests)
  int32_t no_rowbb;            // 1: large grids skip the row-parallel bitboard form (A/B)
  int32_t wpe5;                // 1: the 5-waves-per-SIMD chain-kernel instantiation
  int32_t lds16;               // dynamic LDS bytes per workgroup
  // derived-state cache.  A chain's HBM label record (lab_stride bytes) mirrors the start
  // of its LDS slot: labels, then the group sums (grid kernel: u16 pairs; chain kernel:
  // the padded u32 layout of gsum_slot).  Each launch writes the first
  // lab_copy16 16-B pieces back; when gcache_ok the next launch loads them all and takes
  // cut / bnodes / npairs from the stats record instead of re-deriving them from every
  // node's neighbourhood (host writes of labels or stats clear gcache_ok)
  int32_t lab_copy16;
  int32_t gcache_ok;
  // grid kernel work units: quads x slices (fw_grid16_kernel); seg_done [quads] counts a
  // quad's finished slices (zeroed before a launch with slices > 1)
  int32_t slices;
  int32_t* seg_done;
  // both kernels: a wave's priority level counts 2^-prio_shift of its unit's steps
  int32_t prio_shift;
  // spatial observables (nullptr: off).  Per chain c: acc [E] (int64: sum of -t when an
  // edge becomes cut and +t when it becomes uncut, so cut_times = acc + [cut now] * Y),
  // nf / lf [n] (num_flips, last_flipped of finished runs), ps [n] (part_sum), and the
  // pending run {node, district, first yield, -} of the current state's creating flip.
  int64_t* m_acc;
  uint32_t* m_nf;
  uint32_t* m_lf;
  int64_t* m_ps;
  int32_t* m_pend;
  const int64_t* m_labval;     // [k] GerryChain label values
  // accept rule (FW_ACCEPT_*); FW_ACCEPT_BOUNDARY: node flags and, per chain, the count
  // of flagged nodes in each district [n_chains][k]
  int32_t accept;
  const uint8_t* flags;
  int32_t* bcnt;
  // district-shape observable (fw_chains_enable_ring; ring_n == 0: off): ring edge r joins
  // ring_u[r] and ring_w[r]; ring_node[x] = 1 iff x is an endpoint of a ring edge; yields
  // counted per pair of first two cut ring edges, index i*ring_n + j (ring_n^2: < 2 cut)
  int32_t ring_n;
  const int32_t* ring_u;
  const int32_t* ring_w;
  const uint8_t* ring_node;
  unsigned long long* hist_ring;  // [ring_n^2 + 1]
  // sampled geometric waits (fw_chains_enable_waits; nullptr: off): per chain {sum over
  // yields, the current state's draw}; wlp [n+1] = log1p(-b / (N^k - 1)) (fw_math.h)
  double* wsamp;
  const double* wlp;
};

// fw_chains_read_map: finalise maps of a chain range (see include/flipwalk.h)
struct FwMapRead {
  const int64_t* acc;
  const uint32_t* nf;
  const uint32_t* lf;
  const int64_t* ps;
  const int32_t* pend;
  const int64_t* labval;
  const uint8_t* labels;
  int64_t lab_stride;
  const fw_chain_stats* stats;
  const int32_t* eu;  // [E] edge endpoints, canonical order
  const int32_t* ew;
  int32_t n, E, lb, what, sum, finalize;
  int32_t chain0, n_chains;
  int64_t* out;
};

struct FwEvalParams {
  FwGraphDev g;
  const uint8_t* labels;  // packed LB-bit labels of the one state
  int32_t lab_bytes;
  const int64_t* pops;    // [k] populations of the state
  int32_t k, m;
  const int32_t* v;
  const int16_t* target;
  int64_t pop_lo, pop_hi;
  int32_t* dcut;
  uint8_t* contig;
  uint8_t* pop_ok;
  int32_t* dboundary;
  uint32_t* spill;        // [grid][n]
  int32_t qcap;
  int32_t off_list, lds_bytes;
};

// Host-side launchers implemented in fw_kernels.hip.
int fw_launch_map_init(const FwRunParams& p, void* stream);
int fw_launch_map_read(const FwMapRead& m, void* stream);
int fw_launch_bcnt_init(const FwRunParams& p, void* stream);
int fw_launch_run(const FwRunParams& p, int lb, int grid, void* stream);
int fw_launch_eval(const FwEvalParams& p, int lb, int grid, void* stream);
int fw_run_grid_size(FwRunParams& p, int lb, int device, int* grid);
int fw_run_gsum_slots(int G);  // u16 group-sum slots of the chain kernel
// fw_grid16.hip
bool fw_grid16_candidate(int gw, int maxdeg, int G, int k, int64_t total_pop);
int fw_grid16_lb(int G, int k);
void* fw_grid16_fn(const FwRunParams& p);
void* fw_run_fn(const FwRunParams& p, int lb);  // the chain-kernel instantiation fw_launch_run takes
int fw_grid16_launch_nw(const FwRunParams& p);
int fw_grid16_launch_rows(const FwRunParams& p);
int fw_grid16_plan(FwRunParams& p, int device, int* grid);
int fw_grid16_launch(const FwRunParams& p, int grid, void* stream);
int fw_grid16_launch_rows(const FwRunParams& p);  // rows per chain of the kernel launched
int fw_grid16_launch_nw(const FwRunParams& p);    // waves per workgroup of that kernel
