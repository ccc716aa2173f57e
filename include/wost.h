/*
 * wost.h -- C ABI of libwost.so, the MI355X (gfx950) Walk-on-Stars solver.
 *
 * This is the drop-in boundary for the hot path of Tsuchijo/DCRMonteCarlo:
 * the per-walk loop of WostSolver_2D._solveUnified
 * (reference: solvers/WoStSolver.py:162-316) and the polyline queries it calls
 * (reference: geometry/PolylinesSimple.py:25-197). The Python facade
 * dcrmontecarlo_amd/ (WostSolver_2D, PolyLinesSimple) binds these entry points
 * through ctypes; plain pointers and sizes only, no torch types.
 *
 * Every entry point returns an int status (WOST_OK == 0, negative on error);
 * wost_last_error() returns a thread-local message for the last failure.
 * Handles are not thread-safe; distinct handles are independent.
 */
#ifndef WOST_H
#define WOST_H

#if defined(__HIPCC_RTC__)
/* compiled by hiprtc as part of a JIT-specialised walk kernel: no system headers */
typedef unsigned char uint8_t;
typedef int int32_t;
typedef unsigned int uint32_t;
typedef long long int64_t;
typedef unsigned long long uint64_t;
#else
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define WOST_ABI_VERSION 6

/* Most source fields one multi-source solve can score (wost_set_sources). */
#define WOST_MAX_SOURCES 16

/* Walks of one query point are grouped in blocks of this many consecutive
 * walk indices. Per-block partial sums are the unit of reduction and of
 * multi-GPU sharding (a shard is a contiguous range of blocks), which makes
 * the result bitwise independent of the number of GPUs. */
#define WOST_BLOCK_WALKS 4096

/* Inverse-CDF table resolution of the radial source samplers. */
#define WOST_SAMPLER_TABLE_N 4097

/* Neumann segment-tree defaults (wost_set_segment_tree). */
#define WOST_TREE_MIN_SEGMENTS_DEFAULT 64
#define WOST_TREE_LEAF_DEFAULT 10

enum wost_status {
    WOST_OK = 0,
    WOST_ERR_INVALID_ARG = -1,
    WOST_ERR_HIP = -2,
    WOST_ERR_NO_DEVICE = -3,
    WOST_ERR_UNSUPPORTED = -4,
    WOST_ERR_OOM = -5,
    WOST_ERR_COMM = -6          /* RCCL failure (multi-GPU) */
};

/* compat: "reference" reproduces the reference's estimator including its
 * quirks. "fixed" runs the corrected estimator
 * (Q1-Q5, Q7, Q12, Q13 corrected, delta tracking included). */
enum wost_compat { WOST_COMPAT_REFERENCE = 0, WOST_COMPAT_FIXED = 1 };

/* ---------------------------------------------------------------------------
 * Coefficient fields. The reference takes arbitrary Python callables for the
 * Dirichlet data g, source f, absorption sigma and diffusion alpha
 * (solvers/WoStSolver.py:22). A GPU cannot call Python, so a field is a sum
 * of terms, each a coefficient times a product of primitive factors:
 *      field(x,y) = sum_t coef_t * prod_{k in t} factor_k(x,y)
 * The factor set covers every field of the reference's scenarios
 * (tests/testWoStCorrectness.py:81-142, tests/testWostWithSource.py:42-58,
 *  tests/testWostVariableCoefficients.py:37-86,
 *  tests/testGeophysicalScenario.py:11-55, utils.py:123-129, notebook cell 17)
 * and every factor has an analytic gradient and Laplacian for sigma'.
 * ------------------------------------------------------------------------- */
enum wost_factor_kind {
    WOST_FK_MONO = 1,           /* x^p0 * y^p1, p0,p1 integers in [0,15]            */
    WOST_FK_EXP_QUAD = 2,       /* exp(p2 dx^2 + p3 dy^2 + p4 dx dy + p5 dx + p6 dy + p7),
                                   dx = x - p0, dy = y - p1                           */
    WOST_FK_SIN_LIN = 3,        /* sin(p0 x + p1 y + p2)                              */
    WOST_FK_COS_LIN = 4,        /* cos(p0 x + p1 y + p2)                              */
    WOST_FK_SIGMOID_LIN = 5,    /* 1/(1+exp(-(p0 x + p1 y + p2)))                     */
    WOST_FK_SIGMOID_RADIAL = 6, /* 1/(1+exp(-p0 (sqrt((x-p1)^2+(y-p2)^2) - p3)))
                                   (utils.py:123-129 torch_smooth_circle is p0=-100) */
    WOST_FK_IND_BOX = 7,        /* 1 if p0<=x<=p1 and p2<=y<=p3 else 0 (zero gradient) */
    WOST_FK_IND_DISK = 8,       /* 1 if (x-p0)^2+(y-p1)^2 <= p2 else 0 (zero gradient) */
    WOST_FK_GRID = 9            /* tabulated values (the fallback for a callable that is
                                   not expressible with the kinds above):
                                   Catmull-Rom bicubic interpolation of an nx x ny grid,
                                   node (i,j) at (p0 + i/p2, p1 + j/p3), values
                                   wost_field.grid[p6 + j*nx + i], nx = p4, ny = p5;
                                   the position is clamped to the grid (constant
                                   extension outside). C1, with an analytic gradient
                                   and a piecewise Laplacian for sigma'. */
};

/* Largest grid a field may carry (floats, all its FK_GRID factors together;
 * 2048 x 2048). Four fields together stay below 2^24, so offsets are exact
 * in a float parameter. */
#define WOST_MAX_GRID_VALUES (1 << 22)

typedef struct {
    int32_t kind;   /* enum wost_factor_kind */
    float p[8];
} wost_factor;

typedef struct {
    float coef;
    int32_t first_factor;   /* index into wost_field.factors */
    int32_t n_factors;      /* 0 => constant term */
} wost_term;

/* flags */
#define WOST_FIELD_DETACHED 1   /* alpha only: the reference's callable returns a value
                                   detached from autograd (or a constant), so its
                                   sigma' falls back to sigma/alpha
                                   (solvers/WoStSolver.py:123-127, quirk Q9). */

typedef struct {
    const wost_term* terms;
    int32_t n_terms;
    const wost_factor* factors;
    int32_t n_factors;
    int32_t flags;
    const float* grid;      /* values of this field's WOST_FK_GRID factors (may be NULL) */
    int64_t n_grid;         /* floats in grid, <= WOST_MAX_GRID_VALUES                 */
} wost_field;

/* A polyline: n_vertices points, xy = [x0,y0,x1,y1,...] float32
 * (reference: geometry/Polylines.py:14-21, points tensor [N,2]). */
typedef struct {
    const float* xy;
    int32_t n_vertices;
} wost_polyline;

/* Problem description == the WostSolver_2D constructor arguments
 * (solvers/WoStSolver.py:22-64). */
typedef struct {
    wost_polyline dirichlet;        /* required, >= 2 vertices                   */
    wost_polyline neumann;          /* xy == NULL or n_vertices == 0 => none     */
    const wost_field* boundary;     /* g; NULL => g == 0 (:45-46)                */
    const wost_field* source;       /* f; NULL => no source term                 */
    const wost_field* sigma;        /* NULL => 0 when alpha given (:55-56)       */
    const wost_field* alpha;        /* NULL => 1 when sigma given (:57-58)       */
    int32_t compat;                 /* enum wost_compat                          */
    int32_t device;                 /* HIP device ordinal                        */
    double sigma_bar_override;      /* > 0: use this sigma_bar instead of the
                                       50x50 grid estimate (:130-136)            */
} wost_problem;

typedef struct wost_handle wost_handle;

/* Field slots for wost_set_field. */
enum wost_field_slot { WOST_SLOT_BOUNDARY = 0, WOST_SLOT_SOURCE = 1 };

/* Timing of the last wost_solve, HIP events on the handle's stream. */
typedef struct {
    double walk_kernel_ms;      /* sum over launches of the walk kernel       */
    double reduce_kernel_ms;    /* sum over launches of the block reduction    */
    double total_ms;            /* upload -> results on host                    */
    int32_t n_launches;         /* walk-kernel launches (batches)               */
    int32_t grid_blocks;        /* workgroups per walk-kernel launch            */
    uint64_t total_steps;       /* walk-steps executed in the last solve         */
    uint64_t total_walks;
    int32_t jit;                /* 1: field-specialised (hiprtc) walk kernel,
                                   0: precompiled kernel interpreting the fields */
    int32_t tree;               /* 1: Neumann queries through the segment tree */
    /* the launch's shape -- a function of this call alone (never of an earlier solve):
     * workgroups per CU and their threads, the static first chunk of walks per wave, the
     * host's dequeue size and whether the waves then sized their dequeues from their own
     * measured walks (wost_set_option "adaptive_chunk"; never in the segment-tree kernels) */
    int32_t blocks_per_cu;
    int32_t block_threads;
    int32_t chunk0;
    int32_t chunk;
    int32_t adaptive;
    uint32_t max_walk_steps;    /* the longest walk's step count */
    double jit_ms;              /* host time compiling the field-specialised kernel in this
                                   solve (0 when the in-memory or disk cache had it) */
    /* the device's wall clock over the solve's walk launches (s_memrealtime; the last
     * launch for tail and last wave): first wave start -> last wave end; the last
     * successful dequeue -> last wave end; the wave that ended last: its duration and
     * loop iterations (one walk-step of at least one lane each); the most iterations of
     * any wave (all five 0 for the segment-tree kernels, which keep no wave records) */
    double span_ms;
    double tail_ms;
    double last_wave_ms;
    uint32_t last_wave_iters;
    uint32_t max_wave_iters;
    /* walks this solve ran on the precompiled kernel while its field-specialised kernel
     * compiled in the background (option jit_race: only the solve that starts a compile;
     * the same results either way) */
    uint64_t precompiled_walks;
} wost_timing;

int wost_version(void);
const char* wost_last_error(void);
int wost_device_count(int32_t* count);

/* WostSolver_2D.__init__ (solvers/WoStSolver.py:22-64): validates, estimates
 * sigma_bar like buildModifiedSigma (:66-138), builds the radial sampler
 * (solvers/utils.py:120-195) and uploads geometry and fields to the device. */
int wost_create(const wost_problem* problem, wost_handle** out);
void wost_destroy(wost_handle* h);

/* setBoundaryConditions (:141-148) / setSourceTerm (:150-157). Setting a
 * source on a problem without one changes the kernel variant used. */
int wost_set_field(wost_handle* h, int32_t slot, const wost_field* field);

/* The solver's sigma_bar (reference attribute WostSolver_2D.sigma_bar) and
 * whether delta tracking is on (attribute use_delta_tracking). */
int wost_get_info(const wost_handle* h, double* sigma_bar, int32_t* use_delta_tracking);

/* Number of reduction blocks of a solve: n_points * ceil(walks_per_point / WOST_BLOCK_WALKS). */
int64_t wost_num_blocks(int64_t n_points, int64_t walks_per_point);

/* _solveUnified (solvers/WoStSolver.py:162-316) over the global walk blocks
 * [block_begin, block_end) (pass 0, wost_num_blocks(...) for a full solve).
 * Walk w of point p has global id p*walks_per_point + w; its random stream is
 * Philox4x32-10 keyed by seed, subsequence = global id, one draw per step.
 *
 * Outputs (host memory, caller-owned; any may be NULL):
 *   block_stats [n_blocks_in_range][3] : sum, sum of squares, steps per block
 *   point_stats [n_points][3]          : the same, summed over the range's
 *                                        blocks in block order
 *   walk_values / walk_steps           : per-walk estimate and step count for
 *                                        every walk in the range (walk order)
 * Blocking; the result is bitwise reproducible for a given seed. */
int wost_solve(wost_handle* h, const float* points, int64_t n_points,
               int64_t walks_per_point, int64_t block_begin, int64_t block_end,
               int32_t max_steps, float eps, uint64_t seed,
               double* block_stats, double* point_stats,
               float* walk_values, uint32_t* walk_steps);

/* _solveUnified with return_history=True (solvers/WoStSolver.py:180-314): a
 * full solve (all walks of all points) that also records every walk.
 * records (host, caller-owned): [n_points * walks_per_point][max_steps + 1]
 * [WOST_REC_FLOATS] floats, walk-major in walk order. Record k < steps of a
 * walk is its step k:
 *   x, y      the point at the start of the step        (path 'point', :219)
 *   dD, dN    its Dirichlet / Neumann distance; dN = NaN without a Neumann
 *             polyline                                 (:220-221)
 *   sx, sy    the source sample point after clipping    (contributions 'point', :264)
 *   c         its source contribution (0 when clipped)  (:265)
 *   src       1 when the problem has a source (the step has a contribution)
 * Record `steps` (the walk's step count) is the end of the walk: x, y = final
 * point, c = boundary contribution g*w, src (slot 7) = the walk's total
 * (:301-306). The recorder's device buffer is bounded (1 GiB per launch);
 * solves whose single walk block does not fit fail with WOST_ERR_INVALID_ARG. */
#define WOST_REC_FLOATS 8
int wost_solve_history(wost_handle* h, const float* points, int64_t n_points,
                       int64_t walks_per_point, int32_t max_steps, float eps, uint64_t seed,
                       double* point_stats, float* walk_values, uint32_t* walk_steps, float* records);

/* Multi-source batching (beyond the reference, which solves
 * one source per WostSolver_2D.solve): a DC survey injects current through
 * many electrode pairs, each a different source f. The walks do not depend on
 * f (it only weights the source samples, solvers/WoStSolver.py:242-258), so one
 * walk can score every source at once. wost_set_sources replaces the
 * handle's source by n_sources fields (1 <= n <= WOST_MAX_SOURCES; sources[0]
 * takes the place of setSourceTerm's field). wost_solve_multi then solves
 * like wost_solve, with per-source results:
 *   block_stats [n_blocks_in_range][2*S+1], point_stats [n_points][2*S+1]:
 *       (sum_0, sumsq_0, ..., sum_{S-1}, sumsq_{S-1}, steps)
 *   walk_values [walks][S], walk_steps [walks]
 * Each source's sums are bit for bit those of a single-source solve of that
 * source with the same seed. Needs the field-specialised (hiprtc) kernel when
 * S > 1. wost_solve and wost_solve_history need S == 1. */
int wost_set_sources(wost_handle* h, const wost_field* const* sources, int32_t n_sources);
/* Compile (or fetch from the kernel caches) the field-specialised kernel that
 * wost_set_sources(h, sources, n_sources) and a wost_solve_multi / wost_solve_range of
 * n_points would launch first, without changing the handle or launching anything: a survey
 * prepares its groups' kernels from many threads at once (their compiles overlap in the
 * compile helper, wost_jit_compile) before its solves look them up. Thread-safe with other
 * wost_prepare_sources calls, also on the same handle; not with a solve, wost_set_sources or
 * an option change on that handle. No reference counterpart. */
int wost_prepare_sources(wost_handle* h, const wost_field* const* sources, int32_t n_sources, int64_t n_points);
int wost_solve_multi(wost_handle* h, const float* points, int64_t n_points,
                     int64_t walks_per_point, int64_t block_begin, int64_t block_end,
                     int32_t max_steps, float eps, uint64_t seed,
                     double* block_stats, double* point_stats,
                     float* walk_values, uint32_t* walk_steps);

int wost_last_timing(const wost_handle* h, wost_timing* out);

/* Number of source fields the handle scores (1, or n of wost_set_sources). */
int wost_num_sources(const wost_handle* h, int32_t* n_sources);

/* Walks [walk_begin, walk_end) of every point (of walks_per_point per point; the
 * ends are multiples of WOST_BLOCK_WALKS, or walk_end == walks_per_point): a shard
 * of a solve that covers every point. Global walk ids, random streams and blocks
 * are those of the full solve: block b of point p here is the full solve's block
 * walk_begin / WOST_BLOCK_WALKS + b of that point, with the same sums.
 *   block_stats [n_points][n_range_blocks][2S+1] (point-major), point_stats
 *   [n_points][2S+1], walk_values [n_points][walk_end - walk_begin][S], walk_steps
 *   [n_points][walk_end - walk_begin]  (S = wost_num_sources).
 * A range longer than one launch holds (2^26 / S walks of a point) is solved as
 * block-aligned sub-ranges, with the same results. */
int wost_solve_range(wost_handle* h, const float* points, int64_t n_points,
                     int64_t walks_per_point, int64_t walk_begin, int64_t walk_end,
                     int32_t max_steps, float eps, uint64_t seed,
                     double* block_stats, double* point_stats,
                     float* walk_values, uint32_t* walk_steps);

/* ---------------------------------------------------------------------------
 * Multi-GPU: one process per GPU, RCCL over xGMI. The reference
 * has no parallel code; walks shard trivially, and the only exchange is one
 * all-gather of the per-block partial sums.
 *   1. one rank calls wost_comm_unique_id and shares the WOST_COMM_ID_BYTES bytes
 *      with the others (any channel: a file, a TCP store, MPI);
 *   2. every rank calls wost_comm_create(id, n_ranks, rank, its device);
 *   3. every rank calls wost_solve_distributed with the same points: rank r solves
 *      the walk range wost_shard_walk_range(W, n_ranks, r) of EVERY point (each
 *      rank gets about W / n_ranks walks of each point: balanced whatever the
 *      points' walk lengths), the block sums are all-gathered, and every rank sums
 *      them per point in global block order -- point_stats is bitwise that of a
 *      one-GPU solve, for any number of ranks.
 * ------------------------------------------------------------------------- */
#define WOST_COMM_ID_BYTES 128
typedef struct wost_comm wost_comm;
enum wost_comm_op { WOST_COMM_SUM = 0, WOST_COMM_MAX = 1 };

typedef struct {
    wost_timing local;          /* this rank's solve (walk kernel time, steps) */
    int64_t walk_begin, walk_end;   /* this rank's walk range of every point */
    uint64_t total_steps;       /* walk-steps of all ranks */
    /* wall-clock phases of the protocol on this rank (wost_dist_last_phases): the local
     * solve and pack, the agreement all-reduce (it waits for the slowest rank's local
     * solve), the block all-gather and the ordered merge */
    double local_ms, agree_ms, gather_ms, merge_ms;
} wost_dist_timing;

int wost_comm_unique_id(uint8_t* id);
int wost_comm_create(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, wost_comm** out);
void wost_comm_destroy(wost_comm* c);
int wost_comm_info(const wost_comm* c, int32_t* n_ranks, int32_t* rank, int32_t* device);
const char* wost_comm_last_error(void);
/* recv[n_ranks * count] = every rank's send[count], in rank order (host buffers). */
int wost_comm_allgather(wost_comm* c, const double* send, int64_t count, double* recv);
/* inout[count] reduced over the ranks (op: WOST_COMM_SUM / WOST_COMM_MAX). */
int wost_comm_allreduce(wost_comm* c, double* inout, int64_t count, int32_t op);
int wost_comm_barrier(wost_comm* c);
/* Rank `rank`'s walk range [*walk_begin, *walk_end) of a point's walks_per_point
 * walks: whole blocks, split as evenly as possible (no device needed). */
int wost_shard_walk_range(int64_t walks_per_point, int32_t n_ranks, int32_t rank, int64_t* walk_begin,
                          int64_t* walk_end);
/* The solve of every point with walks_per_point walks across the communicator's
 * ranks (collective: every rank calls it with the same arguments); point_stats
 * [n_points][2S+1] on every rank; timing may be NULL. */
int wost_solve_distributed(wost_handle* h, wost_comm* c, const float* points, int64_t n_points,
                           int64_t walks_per_point, int32_t max_steps, float eps, uint64_t seed,
                           double* point_stats, wost_dist_timing* timing);

/* The pieces of wost_solve_distributed, host only (no device needed), so that the
 * multi-rank merge and the failure protocol run under any transport -- RCCL in
 * wost_solve_distributed, gloo in the CPU tests.
 *
 * Layout of one rank's contribution to the all-gather: [n_points][nb_max][row]
 * doubles, nb_max = wost_shard_blocks_max(W, n_ranks), the rank's blocks of each
 * point first and zero padding after them (row = 2S+1 block sums). */
int64_t wost_shard_blocks_max(int64_t walks_per_point, int32_t n_ranks);
/* blocks [n_points][n_rank_blocks][row] of rank `rank`'s walk range -> packed. */
int wost_shard_pack(const double* blocks, int64_t n_points, int64_t walks_per_point, int32_t n_ranks,
                    int32_t rank, int32_t row, double* packed);
/* gathered [n_ranks][n_points][nb_max][row] -> point_stats [n_points][row]: per point,
 * rank 0's blocks, then rank 1's, ... added to 0.0 one block at a time -- the block
 * order of a one-GPU solve, so the sums are bitwise the same for any n_ranks. */
int wost_shard_merge(const double* gathered, int64_t n_points, int64_t walks_per_point, int32_t n_ranks,
                     int32_t row, double* point_stats);

/* A transport for wost_distributed_run. Every callback returns WOST_OK or an error
 * status (and may set its message with nothing: the protocol records its own).
 *   prepare      optional: reserve transport buffers for `count` doubles per rank
 *   solve_range  this rank's walks [walk_begin, walk_end) of every point ->
 *                blocks [n_points][n_rank_blocks][row] (wost_solve_range's layout)
 *   allreduce    inout[count] reduced over ranks, op WOST_COMM_SUM / WOST_COMM_MAX
 *   allgather    recv[n_ranks][count] = every rank's send[count], in rank order
 *   key, n_key   optional (NULL / 0): up to WOST_DIST_MAX_KEY values every rank must
 *                hold identically -- the solve's other arguments (seed halves, eps,
 *                maxSteps, a checksum of the points); checked by the agreement */
#define WOST_DIST_MAX_KEY 16
typedef struct {
    void* ctx;
    int32_t (*prepare)(void* ctx, int64_t count);
    int32_t (*solve_range)(void* ctx, int64_t walk_begin, int64_t walk_end, double* blocks);
    int32_t (*allreduce)(void* ctx, double* inout, int64_t count, int32_t op);
    int32_t (*allgather)(void* ctx, const double* send, int64_t count, double* recv);
    const double* key;
    int32_t n_key;
} wost_dist_ops;

/* The agreement key wost_solve_distributed uses: {seed low 32 bits, seed high 32 bits,
 * eps, max_steps, points checksum low / high 32 bits (FNV-1a 64 of the point bytes)}
 * -> key[6]. Host only. */
int wost_dist_solve_key(uint64_t seed, float eps, int32_t max_steps, const float* points, int64_t n_points,
                        double* key);

/* The distributed solve's protocol over a transport (collective). Every rank makes
 * exactly two collective calls, in the same order, whatever fails locally:
 *   1. allreduce(MAX) of (failed, n_points, row, walks_per_point, key) and their
 *      negatives -- so a rank whose solve or buffers failed, or whose arguments
 *      differ, is known to all;
 *   2. only if no rank failed and all agree: allgather of the packed blocks,
 *      then wost_shard_merge.
 * A rank that failed returns its own status; the others return WOST_ERR_COMM
 * ("another rank failed"); disagreeing shapes give WOST_ERR_INVALID_ARG on all.
 * walk_begin / walk_end / total_steps (all ranks' walk-steps) may be NULL. */
int wost_distributed_run(const wost_dist_ops* ops, int32_t n_ranks, int32_t rank, int64_t n_points,
                         int64_t walks_per_point, int32_t row, double* point_stats,
                         int64_t* walk_begin, int64_t* walk_end, uint64_t* total_steps);
/* The calling thread's last wost_distributed_run, in wall-clock ms: ms[0] the local
 * solve and pack, ms[1] the agreement all-reduce, ms[2] the block all-gather, ms[3] the
 * merge (a phase not reached is 0). Per thread, so concurrent protocols on other threads
 * do not overwrite it. */
int wost_dist_last_phases(double* ms);

/* Walk kernels: by default libwost compiles a field-specialised walk kernel per
 * handle and kernel variant with hiprtc (cached in memory and in
 * $WOST_JIT_CACHE, default ~/.cache/wost) and falls back to the precompiled
 * interpreting kernel if that fails. enable = 0 forces the precompiled kernel.
 * Both give identical results. */
int wost_set_jit(wost_handle* h, int32_t enable);

/* The walk direction's cos and sin (solvers/WoStSolver.py:230-232). The reference's
 * torch.cos/torch.sin return the exact values rounded to float32 within their own ulp;
 * on a walk that hits a curved Neumann boundary a one-ulp change of a direction sends it
 * elsewhere (C5: ~20% of the walks), so:
 *   WOST_TRIG_EXACT  correctly rounded, evaluated in double precision (C5: 93% of the
 *                    reference's replayed walks identical, as the oracle; 3% slower there,
 *                    13-24% on the short-step scenarios);
 *   WOST_TRIG_FAST   the hardware's v_sin/v_cos (a few ulps; C5: 83% identical);
 *   WOST_TRIG_AUTO   (default) exact when the Neumann polyline has >= 3 segments (a
 *                    curved boundary: C3's circle, C5's topography), fast otherwise
 *                    (Dirichlet-only problems and the DCR scenarios' straight top, whose
 *                    walks match the reference's either way).
 * (Study builds only: environment WOST_TRIG = auto | exact | fast, the default of new
 * handles; the product library reads no environment variable that changes a kernel.) */
enum wost_trig { WOST_TRIG_AUTO = 0, WOST_TRIG_EXACT = 1, WOST_TRIG_FAST = 2 };
int wost_set_trig(wost_handle* h, int32_t mode);

/* compat="fixed" with delta tracking: the corrected screened law moves a walk
 * ~2/sqrt(sigma_bar) per collision, so a point at Dirichlet distance d needs
 * ~d^2 sigma_bar / 4 steps. Every solve entry point refuses (WOST_ERR_INVALID_ARG)
 * when that estimate at the median query point exceeds maxSteps -- the walks would
 * all end truncated (the DCR configurations: sigma_bar = 10, d ~ 100). enable = 0
 * turns the check off (default on). No reference counterpart. */
int wost_set_fixed_step_check(wost_handle* h, int32_t enable);

/* Neumann segment tree: for a Neumann polyline of at least min_segments
 * segments (default WOST_TREE_MIN_SEGMENTS_DEFAULT; < 0: never, 0: always)
 * the walk kernel's closest-silhouette and ray queries (geometry/
 * PolylinesSimple.py:83-102, :134-197, which scan every segment) go through an
 * implicit 4-ary tree of oriented boxes and direction arcs with leaf_segments
 * (1..32) segments per leaf (0 keeps the current value), under both estimators (compat="fixed":
 * the nearest-crossing ray query). Results are bit-identical to the scans. */
int wost_set_segment_tree(wost_handle* h, int32_t min_segments, int32_t leaf_segments);

/* Kernel and launch options of a handle (no reference counterpart). Each selects HOW the
 * walks run -- workgroup size, LDS staging, work-queue chunks, the segment tree's walk
 * pools and hand-outs -- never what they compute: every walk's value and step count
 * depend only on (seed, walk id), and the GPU tests check each option against the
 * default walk for walk. Names (dcrmontecarlo_amd/csrc/wost_options.h): tree_pool,
 * pool_near, pool_slots, pool_near_waves, pool_min_push, tree_lds, tree_lds_block,
 * tree_share, tree_share_min, tree_share_descent, tree_batch, tree_qmargin, jit_waves,
 * const_vertices, jit_slp, walk_block, fused_scan, refill_min, philox_ahead, param_sources, jit_process, jit_race,
 * chunk0,
 * chunk_min, chunk_max, adaptive_chunk, grid_blocks_per_cu, lds_pad_bytes.
 * WOST_ERR_INVALID_ARG for an unknown name or a value out of range; WOST_ERR_UNSUPPORTED
 * for a study-build-only name (exp_flags, tree_iter_stats) in the product library. The
 * product library reads no environment variable that changes a kernel or a result
 * (study builds, build/libwost_study.so, seed options from the tools' A/B variables). */
int wost_set_option(wost_handle* h, const char* name, double value);
int wost_get_option(const wost_handle* h, const char* name, double* value);
/* {"build": "product"|"study", "non_default": {name: value, ...}} as JSON (NUL-terminated,
 * truncated to capacity - 1; *length = its full length). h may be NULL: the options a new
 * handle would get. */
int wost_options_report(const wost_handle* h, char* out, int64_t capacity, int64_t* length);

/* HIP source of the field-specialised walk kernel wost_create would build for
 * this problem (host only, no device needed): for offline ISA study and for
 * checking on a build machine that the generator's output compiles.
 * *length = source length; the source (NUL-terminated, truncated to
 * capacity - 1) is copied to out when out != NULL. Compile it against
 * wost.h, dcrmontecarlo_amd/csrc/wost_device.h and wost_walk.h. */
int wost_kernel_source(const wost_problem* problem, char* out, int64_t capacity, int64_t* length);
/* The same for a multi-source solve (wost_set_sources' n_sources fields; 0: the problem's
 * own source, as wost_kernel_source), with the sources compiled in as literals (the
 * default; option param_sources = 1 reads them from the program buffer instead). */
int wost_kernel_source_sources(const wost_problem* problem, const wost_field* const* sources, int32_t n_sources,
                               char* out, int64_t capacity, int64_t* length);

/* Compiles a generated walk-kernel source (wost_kernel_source) for the gfx target `arch`
 * ("gfx950") with the compile options of a new handle, without a device: in the compile
 * helper wost_jitc (installed next to libwost.so) unless in_process, else -- or when the
 * helper is missing or fails -- in this process; *used_helper (optional) says which ran.
 * Handles compile their kernels the same way (option jit_process, default 1): ROCm's
 * compiler library serialises one process's compiles, so concurrent handles (a survey's
 * threads) overlap theirs only in helpers. *length = the code object's size; it is copied
 * to out when out != NULL (WOST_ERR_INVALID_ARG when capacity is smaller). No reference
 * counterpart (the reference's TorchScript kernels compile in the interpreter). */
int wost_jit_compile(const char* source, const char* arch, int32_t in_process, uint8_t* out, int64_t capacity,
                     int64_t* length, int32_t* used_helper);

/* Device evaluation of the handle's fields at points (for tests and for the
 * host API): which = 0 g, 1 f, 2 sigma, 3 alpha (value, d/dx, d/dy, Laplacian
 * per point -> out[n][4]), 4 sigma' (solvers/WoStSolver.py:88-127 -> out[n][4],
 * value in column 0). */
int wost_eval_field(wost_handle* h, int32_t which, const float* points, int64_t n, float* out);

/* The radial sampler's inverse-CDF nodes (WOST_SAMPLER_TABLE_N floats). */
int wost_sampler_table(const wost_handle* h, float* out, int32_t n);

/* The walk kernels' screened Green's norm G_norm(R) for this sigma_bar
 * (replaces screenedGreensNorm2D, solvers/utils.py:29-44, at
 * solvers/WoStSolver.py:250), evaluated on the host with the kernels' own
 * table and arithmetic: out[i] = G_norm(radii[i]). No device needed. */
int wost_greens_norm(double sigma_bar, const float* radii, int64_t n, float* out);

/* compat="fixed" delta tracking's radial sampler (quirks Q4/Q5 of
 * ScreenedGreensDistribution2D, solvers/utils.py:154-195, corrected): the radius
 * fraction rho[i] the walk kernels draw for uniform u[i] at the shape s[i] = R
 * sqrt(sigma_bar), evaluated on the host with the kernels' table and arithmetic;
 * and the exact CDF F_s(rho) of the ball's screened Green's radial law that it
 * samples (closed form in I0, I1, K0, K1). No device needed. */
int wost_screened_sample_fixed(const float* s, const float* u, int64_t n, float* rho);
int wost_screened_cdf_fixed(double s, const double* rho, int64_t n, double* cdf);

/* Batched polyline queries on the device (geometry/PolylinesSimple.py).
 *   op 0 distance          (:25-49, :214-224)   out_f[n]
 *   op 1 isSilhouette      (:51-81, :242-253)   out_mask[n][nv-2]
 *   op 2 silhouetteDistance(:83-102, :255-265)  out_f[n]
 *   op 3 rayIntersection   (:104-132, :281-292) out_f[n][nv-1]  (dirs used)
 *   op 4 intersectPolylines(:134-197, :294-307) out_f[n][5] = x, y, nx, ny, found
 *                                                (dirs and radii used)
 * op | WOST_GEOM_TREE (ops 2 and 4, >= 2 segments): the same query answered by the
 * walk kernels' Neumann segment tree (wost_set_segment_tree; default leaf size) one
 * query per lane instead of the full scan -- bit-identical to the scan, which the
 * tests check at the reference's own outputs (tests/golden/geometry_kats_c5.npz). */
enum wost_geom_op {
    WOST_GEOM_DISTANCE = 0,
    WOST_GEOM_IS_SILHOUETTE = 1,
    WOST_GEOM_SILHOUETTE_DISTANCE = 2,
    WOST_GEOM_RAY_INTERSECTION = 3,
    WOST_GEOM_INTERSECT_POLYLINES = 4,
    WOST_GEOM_TREE = 256
};
int wost_geometry_query(int32_t device, int32_t op, const wost_polyline* poly,
                        const float* points, const float* dirs, const float* radii,
                        int64_t n, float* out_f, uint8_t* out_mask);

#ifdef __cplusplus
}
#endif

#endif /* WOST_H */
