/*
 * flipwalk.h — C-ABI of the MI355X-native batched single-node flip walk.
 *
 * This is the drop-in boundary for the one hot path of
 * drdeford/FlipComplexityEmpirical: GerryChain's
 *
 *   MarkovChain(proposal, Validator([single_flip_contiguous, popbound]),
 *               accept=cut_accept, initial_state, total_steps)
 *
 * as constructed at grid_chain_sec11.py:340-342 (also All_States_Chain.py:300-302,
 * Frankenstein_chain.py:370-372) and iterated at grid_chain_sec11.py:366.
 * The reference has no FFI of its own (it is pure Python over GerryChain); the
 * entry points below are what a ctypes binding of that loop binds.  Each one
 * names the reference interface it replaces.
 *
 * Conventions
 *  - Return 0 on success, a negative FW_E* code on error; fw_last_error() gives
 *    a thread-local message.
 *  - Host buffers are owned by the caller and copied in/out.  Device memory is
 *    owned by the library behind the opaque handles.
 *  - One handle is bound to one HIP device; calls on one handle must be
 *    serialised; different handles may be driven from different host threads.
 *  - Graphs are CSR with strictly ascending neighbour lists, no self loops, and
 *    symmetric adjacency (checked by fw_graph_create).  Node ids 0..n-1.
 *  - District labels are 0..k-1 (the façade maps GerryChain labels such as
 *    ±1 onto them in sorted order).
 *
 * Randomness (a deterministic restatement of the reference's unseeded
 * `random.choice` / `random.random`, grid_chain_sec11.py:143,179): proposal
 * attempt t of global chain g draws ONE Philox4x32-10 block
 *     key = (lo32(seed), hi32(seed)),  ctr = (lo32(t), hi32(t), lo32(g), hi32(g))
 * giving words x0..x3.  The proposal takes the r-th element, r =
 * floor(((x1<<32)|x0) * P / 2^64), of the proposal set in canonical order (P =
 * its size); the Metropolis draw is CPython's random() construction
 * u = ((x2>>5)*2^26 + (x3>>6)) * 2^-53.
 */
#ifndef FLIPWALK_H
#define FLIPWALK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ---------------------------------------------------------- */
#define FW_OK 0
#define FW_EINVAL (-1)      /* bad argument / malformed graph                */
#define FW_EHIP (-2)        /* HIP runtime error                             */
#define FW_ESTATE (-3)      /* invalid initial state (GerryChain ValueError) */
#define FW_EUNSUPPORTED (-4)/* configuration outside what the kernels handle */
#define FW_ENOMEM (-5)

/* ---- proposal modes -------------------------------------------------------
 * FW_PROPOSE_BI     slow_reversible_propose_bi  grid_chain_sec11.py:132-145
 *                   uniform boundary node, flipped to the other label (k==2).
 * FW_PROPOSE_PAIRS  slow_reversible_propose     grid_chain_sec11.py:117-130 with
 *                   the pair updater b_nodes :151-153 — uniform over distinct
 *                   (node, foreign-neighbour-label) pairs, ordered (node, label).
 * FW_PROPOSE_CUTEDGE gerrychain.proposals.propose_random_flip (imported
 *                   grid_chain_sec11.py:24): uniform cut edge, uniform
 *                   endpoint == uniform directed cut edge (v,u) ordered (v,u);
 *                   v takes u's label.                                        */
#define FW_PROPOSE_BI 0
#define FW_PROPOSE_PAIRS 1
#define FW_PROPOSE_CUTEDGE 2

/* ---- accept rules (fw_chains_set_accept) --------------------------------------
 * FW_ACCEPT_CUT      cut_accept grid_chain_sec11.py:171-179 (the default):
 *                    accept iff u < thr[Δcut + maxdeg]  (thr[d] = base**(-d))
 * FW_ACCEPT_BRATIO   annealing_cut_accept_backwards grid_chain_sec11.py:81-110:
 *                    accept iff u < thr[Δcut + maxdeg] * (|B'| / |B|), |B| = boundary
 *                    nodes (b_nodes_bi) before / after the flip; the host tabulates
 *                    thr[d] = base**(beta*(-d)) (the reference: base .1, beta 5)
 * FW_ACCEPT_BOUNDARY uniform_accept + boundary_condition :43-52,159-165: accept iff
 *                    the nodes flagged boundary_node span >= 2 districts after the flip
 * (u = the CPython random() draw of the attempt, include/flipwalk.h header.)        */
#define FW_ACCEPT_CUT 0
#define FW_ACCEPT_BRATIO 1
#define FW_ACCEPT_BOUNDARY 2

/* ---- what fw_chains_read can return -------------------------------------- */
#define FW_READ_LABELS 0   /* int16  [n_chains][n]                            */
#define FW_READ_STATS 1    /* fw_chain_stats [n_chains]                       */
#define FW_READ_HIST_CUT 2 /* uint64 [n_edges+1]  yields with |cut edges| = i */
#define FW_READ_HIST_B 3   /* uint64 [n+1]        yields with |B| = i         */
#define FW_READ_POPS 4     /* int64  [n_chains][k] district populations       */
#define FW_READ_HIST_RING 5 /* uint64 [n_ring*n_ring+1] yields per ring pair (below) */
#define FW_READ_RING_PAIR 6 /* int32  [n_chains][2] current ring pair (i, j), -1 = none */
#define FW_READ_WAITS 7    /* double [n_chains][2] {sum of sampled waits over yields, the
                              current state's draw} (fw_chains_enable_waits)             */

/* ---- district-shape observable (fw_chains_enable_ring) ----------------------
 * boundary_slope (grid_chain_sec11.py:55-78; Frankenstein_chain.py:57-80) collects the
 * cut edges that lie on the outer ring of the grid (both endpoints in its first/last row
 * or column, plus the four corner diagonals of the sec11 graph); the driver (:371-394)
 * takes the first two, temp[0] and temp[1], and records the slope of the line through
 * their midpoints and the angle they subtend at the grid centre, once per yield.  The
 * kernels keep, per yield, the pair (i, j), i < j, of the first two CUT ring edges in the
 * caller's ring order and count yields per pair: FW_READ_HIST_RING index i*n_ring + j,
 * index n_ring*n_ring for yields with fewer than two cut ring edges (the reference would
 * raise IndexError there).  The host turns pairs into slopes and angles with the
 * reference's own float formula.  With exactly two cut ring edges (a two-district plan
 * whose boundary crosses the ring twice) the result does not depend on the order;
 * with more, the reference picks by CPython set-iteration order, which depends on the
 * interpreter's tuple hash, and the build picks the first two in ring order.            */

/* ---- spatial observables (fw_chains_enable_maps / fw_chains_read_map) ------
 * The reference driver's per-edge and per-node maps, updated once per yield
 * (grid_chain_sec11.py:383-384 cut_times, :396-400 part_sum / last_flipped /
 * num_flips, finalised at :416-419; the same code in Frankenstein_chain.py and
 * All_States_Chain.py).  Edges are indexed canonically: undirected (u < w) pairs
 * in CSR row order.  Values are int64.                                           */
#define FW_MAP_CUT_TIMES 0    /* [n_edges] yields in which the edge was cut          */
#define FW_MAP_NUM_FLIPS 1    /* [n] yields whose state was created by flipping node */
#define FW_MAP_PART_SUM 2     /* [n] part_sum (starts at the initial label value)    */
#define FW_MAP_LAST_FLIPPED 3 /* [n] last such yield index (0: never)                */
#define FW_MAP_SUM 1          /* flag: sum over the chain range into one row          */
#define FW_MAP_FINALIZE 2     /* flag: PART_SUM of never-flipped nodes := yields*label */

/* Per-chain counters and running observables (the per-yield block of
 * grid_chain_sec11.py:366-402, reduced to sums; one struct per chain). */
typedef struct fw_chain_stats {
  uint64_t attempts;    /* proposals drawn, including invalid (retried) ones   */
  uint64_t steps;       /* valid proposals = MarkovChain counter increments    */
  uint64_t accepts;     /* Metropolis-accepted flips                           */
  uint64_t pop_fail;    /* proposals rejected by the population bound          */
  uint64_t contig_fail; /* proposals (pop-valid) rejected by contiguity        */
  uint64_t bfs_runs;    /* contiguity checks that needed a graph search        */
  uint64_t bfs_nodes;   /* nodes dequeued by those searches                    */
  uint64_t bfs_deg;     /* sum of degrees of dequeued nodes                    */
  uint64_t sum_deg;     /* sum over proposals of deg(v)                        */
  uint64_t acc_deg;     /* sum over accepts of deg(v)                          */
  uint64_t n_bchg;      /* nodes entering/leaving the boundary, over accepts   */
  uint64_t yields;      /* yielded states counted (initial state included)     */
  int64_t sum_cut;      /* sum over yields of len(cut_edges)   (rce, :367)     */
  int64_t sum_bnodes;   /* sum over yields of len(b_nodes)     (rbn, :369)     */
  double sum_invb;      /* sum over yields of 1/len(b_nodes); the expected
                           geom wait (:147-148) is (N^k-1)*sum_invb - yields   */
  int32_t cut;          /* current len(cut_edges)                              */
  int32_t bnodes;       /* current number of boundary nodes                    */
  int32_t npairs;       /* current size of the proposal set                    */
  int32_t stuck;        /* 1 once max_retries consecutive proposals failed     */
} fw_chain_stats;

typedef struct fw_graph fw_graph;
typedef struct fw_chains fw_chains;

/* Thread-local description of the last error on this thread. */
const char* fw_last_error(void);

/* Library/ABI version, e.g. 0x000600 for 0.6.0 (0.2: spatial maps; 0.3: bound
 * schedules; 0.4: ring observable, checkpoint/resume; 0.5: sampled geometric waits;
 * 0.6: fw_chains_launch_info; 0.7: fw_build_info). */
int32_t fw_version(void);

/* Provenance of this build (static string, never NULL): "src=<sha256 of every kernel,
 * header and ABI source> flags=<compiler flags, including any -D>".  Bench lines and PMC
 * profiles carry it, so a measurement names the code it measured. */
const char* fw_build_info(void);

/* Number of visible HIP devices (0 when none; never fails). */
int32_t fw_device_count(void);

/* Upload a CSR graph (replaces gerrychain.Graph / networkx adjacency,
 * grid_chain_sec11.py:191-260, All_States_Chain.py:221).  pop may be NULL
 * (every node population 1, grid_chain_sec11.py:218).  Row-major W×H grids
 * are detected and get an implicit-neighbour kernel. */
int fw_graph_create(const int32_t* rowptr, const int32_t* col, const int64_t* pop,
                    int32_t n, int32_t nnz, int device, fw_graph** out);
void fw_graph_destroy(fw_graph* g);
/* info[0]=n, info[1]=n_edges, info[2]=maxdeg, info[3]=grid width (0 = not a grid),
 * info[4]=grid height */
int fw_graph_info(const fw_graph* g, int64_t info[5]);

/* Create n_chains chains (replaces Partition(graph, assignment, updaters) +
 * within_percent_of_ideal_population + MarkovChain.__init__'s validity check,
 * grid_chain_sec11.py:316-342).
 *  init_labels  int16 [1 or n_chains][n], values 0..k-1 (init_per_chain 0/1)
 *  pop_lo/hi    integer population bounds ceil(lo), floor(hi) of Bounds
 *  thr          float64 [1 or n_chains][2*maxdeg+1]; thr[d+maxdeg] is the
 *               Metropolis bound base**(-d) for Δcut = d (cut_accept,
 *               grid_chain_sec11.py:171-179), thr_per_chain 0/1
 *  seed         Philox key; chain_id0 = global id of the first local chain
 * Fails with FW_ESTATE when an initial plan is not contiguous or violates the
 * bounds (GerryChain raises ValueError). */
int fw_chains_create(fw_graph* g, int32_t n_chains, int32_t k, const int16_t* init_labels,
                     int32_t init_per_chain, int32_t proposal_mode, int64_t pop_lo,
                     int64_t pop_hi, const double* thr, int32_t thr_per_chain, uint64_t seed,
                     int64_t chain_id0, fw_chains** out);
void fw_chains_destroy(fw_chains* c);

/* Advance every chain by `steps` counted steps (MarkovChain.__next__ called
 * `steps` times; the initial state is yielded once, on the first call).  A
 * chain that draws max_retries consecutive invalid proposals is marked stuck
 * instead of looping forever (the reference would hang).  Blocking. */
int fw_chains_run(fw_chains* c, int64_t steps, int32_t max_retries);

/* Same, asynchronous on the handle's stream; fw_chains_sync waits.  The last
 * kernel's device time (ms, HIP events on that stream) is returned by
 * fw_chains_last_kernel_ms. */
int fw_chains_run_async(fw_chains* c, int64_t steps, int32_t max_retries);
int fw_chains_sync(fw_chains* c);
double fw_chains_last_kernel_ms(const fw_chains* c);

/* The launch plan of the handle's next fw_chains_run (no reference counterpart: the
 * occupancy figures SURVEY.md §8d asks the measurement to report).
 *  info[0] workgroups of the persistent grid     info[1] waves per workgroup
 *  info[2] chains per wave                       info[3] LDS bytes per workgroup
 *  info[4] VGPRs per lane of the kernel           info[5] scratch (spill) bytes per lane
 *  info[6] compute units of the device           info[7] workgroups resident per CU */
int fw_chains_launch_info(const fw_chains* c, int64_t info[8]);

/* fw_chains_run plus a per-step trace: host_trace [n_chains][steps] receives, for
 * each counted step, v*64 + target when the flip was accepted, -1 when the
 * Metropolis draw kept the old state, and a value < -1 for steps a stuck chain
 * never took.  Used by the façade's GerryChain-style iterator to rebuild every
 * yielded Partition on the host. */
int fw_chains_run_traced(fw_chains* c, int64_t steps, int32_t max_retries, int32_t* host_trace,
                         size_t bytes);

/* Copy a state array back to the host (see FW_READ_*). */
int fw_chains_read(fw_chains* c, int32_t what, void* host_dst, size_t bytes);

/* Overwrite a state array from the host: the inverse of fw_chains_read, for exact
 * checkpoint / resume (the chain states plus the Philox attempt counter in
 * the stats record are a complete checkpoint of the counter-based RNG).  what is
 * FW_READ_LABELS (every plan is validated like an initial state, FW_ESTATE otherwise, and
 * the district populations are recomputed from it), FW_READ_STATS (counters, sums and
 * the attempt counter; the stuck flag included), FW_READ_HIST_CUT, FW_READ_HIST_B or
 * FW_READ_HIST_RING.  A chain resumed from {labels, stats} continues exactly as the
 * uninterrupted chain (same proposals, same Metropolis draws).  The FW_ACCEPT_BOUNDARY
 * flagged-node counts are recomputed from written plans; the spatial maps are not part of a
 * checkpoint, and a plan write on a handle with maps enabled fails with FW_ESTATE.  A stats
 * write also restores the yield count the maps' 2^32 index guard starts from. */
int fw_chains_write(fw_chains* c, int32_t what, const void* host_src, size_t bytes);

/* Zero the per-chain sums and the yield histograms (not the chain states). */
int fw_chains_reset_observables(fw_chains* c);

/* Select the accept rule (FW_ACCEPT_*) for every chain; node_flags [n] (1 =
 * boundary_node) is required by FW_ACCEPT_BOUNDARY and ignored otherwise.  May be
 * called between runs. */
int fw_chains_set_accept(fw_chains* c, int32_t rule, const uint8_t* node_flags);

/* Step-dependent Metropolis bounds for FW_ACCEPT_CUT / FW_ACCEPT_BRATIO, shared by
 * every chain: the commented beta schedule of annealing_cut_accept_backwards
 * (grid_chain_sec11.py:85-93, t = partition["step_num"], the step_num updater
 * :282-289 = flips accepted since the initial plan, + 1 for the proposal).  A
 * proposal with step_num t uses row clamp(t - t0, 0, n_rows - 1) of rows
 * [n_rows][2*maxdeg+1] in place of the chain's thr table (Δcut + maxdeg indexes
 * a row, as for thr).  n_rows == 0 removes the schedule.  May be called between
 * runs; the accepted-flip count is the FW_READ_STATS accepts field. */
int fw_chains_set_schedule(fw_chains* c, const double* rows, int32_t n_rows, int64_t t0);

/* Turn on the spatial observables for every chain (before the first run).
 * label_values [k] are the GerryChain assignment values of districts 0..k-1
 * (e.g. {-1, 1} for the reference's k=2 plans); NULL means 0..k-1.  Costs
 * 8*n_edges + 16*n bytes of HBM per chain.  Yields per chain must stay below 2^32. */
int fw_chains_enable_maps(fw_chains* c, const int64_t* label_values);

/* Turn on the district-shape observable for every chain: ring edge r joins nodes
 * ring_u[r] and ring_w[r] (an edge of the graph; 2 <= n_ring <= 1024), in the order that
 * picks "the first two".  Zeroes the ring histogram; may be called between runs. */
int fw_chains_enable_ring(fw_chains* c, const int32_t* ring_u, const int32_t* ring_w,
                          int32_t n_ring);

/* Turn on sampled geometric waits for every chain (before the first run): geom_wait
 * (grid_chain_sec11.py:147-148) = int(np.random.geometric(len(b_nodes)/(N**k - 1))) - 1,
 * drawn once per state object and re-used when a Metropolis rejection re-yields it
 * (:368; the Partition caches it), summed over yields (:410-411).  p_table [n+1] holds
 * b/(N^k - 1) for every boundary size b, divided as the reference divides (Python int /
 * int).  The state created by proposal attempt t of global chain g (the initial state:
 * t = 2^63 - 1) draws the Philox block key = seed, ctr = (lo32(t), hi32(t) | 2^31,
 * lo32(g), hi32(g)), takes u = CPython random() of its words (x0, x1) and waits
 * floor(log1p(-u) / log1p(-p)) (inversion; log1p evaluated in plain IEEE double
 * operations, so every implementation agrees bit for bit).  Read / write with
 * FW_READ_WAITS.  The Rao-Blackwellised expectation (stats sum_invb) stays available. */
int fw_chains_enable_waits(fw_chains* c, const double* p_table);

/* Read a map (FW_MAP_*) of chains [chain0, chain0 + n_chains) as int64
 * [n_chains][len], or with FW_MAP_SUM its sum over those chains [len]; len is
 * n_edges for FW_MAP_CUT_TIMES and n otherwise.  Values are current through the
 * last yield; FW_MAP_FINALIZE applies the reference's end-of-run rule. */
int fw_chains_read_map(fw_chains* c, int32_t what, int32_t chain0, int32_t n_chains,
                       int32_t flags, int64_t* dst, size_t bytes);

/* Batched per-flip evaluation on ONE state — the bit-exact per-step contract
 * (cut_edges updater, single_flip_contiguous, Bounds, b_nodes_bi):
 * for each i < m, flipping v[i] to target[i] gives
 *   dcut[i]      = len(cut_edges) after - before
 *   contig[i]    = 1 iff the old district of v[i] stays connected and non-empty
 *   pop_ok[i]    = 1 iff both changed districts stay inside [pop_lo, pop_hi]
 *   dboundary[i] = number of boundary nodes after - before
 * Flips with target == labels[v] or out-of-range values fail with FW_EINVAL. */
int fw_eval_flips(fw_graph* g, const int16_t* labels, int32_t k, const int32_t* v,
                  const int16_t* target, int32_t m, int64_t pop_lo, int64_t pop_hi,
                  int32_t* dcut, uint8_t* contig, uint8_t* pop_ok, int32_t* dboundary);

#ifdef __cplusplus
}
#endif

#endif /* FLIPWALK_H */
