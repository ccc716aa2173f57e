// wost_walk.h -- the walk loop of WostSolver_2D._solveUnified
// (reference: solvers/WoStSolver.py:182-311) as a device function template,
// instantiated by the precompiled kernels (wost_kernels.hip, fields read from
// a program buffer) and by the hiprtc-specialised kernels (wost_jit.cpp,
// fields compiled in). Compiled by hipcc and by hiprtc: no system headers.
//
// One walk per lane:
//  * persistent waves; each lane holds one walk's state in registers;
//  * when walks finish, the wave re-fills those lanes by __ballot / __popcll
//    rank from a chunk of walk ids it dequeued with one atomic (active-mask
//    compaction, so short walks never idle a lane for long);
//  * polyline vertices, the sampler's inverse-CDF table and (up to 1024) query
//    points staged in LDS; the segment loops are wave-uniform (LDS broadcasts);
//  * Philox4x32-10 counters derived from (seed, walk id, step): no RNG state.
#pragma once

#include "wost_device.h"

namespace wost {

// Arguments of the walk kernel, passed by value in the kernarg segment.
struct WalkArgs {
    const float2* points;        // [n_points] query points
    const float2* dverts;        // Dirichlet polyline vertices
    const float2* nverts;        // Neumann polyline vertices (may be null)
    const float* table;          // sampler inverse-CDF nodes (may be null)
    const char* prog;            // DProgram + terms + factors (interpreted fields)
    float* out_val;              // [count] per-walk estimate
    uint32_t* out_steps;         // [count] per-walk step count
    unsigned long long* counter; // the launch's control words (kCtlWords, zeroed before launch): [0] the
                                 // work-queue head; the per-wave launch statistics after them
    int64_t wid_begin;           // global id of local walk 0
    int64_t count;               // walks in this launch
    int64_t walks_per_point;     // W: point of global walk g is g / W
    int32_t nd, nn;              // vertex counts
    int32_t max_steps;
    float eps;
    float rmin;                  // eps / 2 (solvers/WoStSolver.py:167)
    uint32_t key0, key1;         // Philox key = seed
    int32_t chunk;               // walks claimed per work-queue dequeue
    int32_t n_points;            // query points
    double inv_walks_per_point;  // 1/W for the point index of a walk id
    const float* seg_phi;        // [nn-1] atan2 of each Neumann segment's left normal
    float* rec;                  // walk recorder (return_history), or null: kRecFloats floats per
                                 // record, rec_stride records per local walk
    int32_t rec_stride;          // max_steps + 1
    const float4* tree;          // Neumann segment tree (TREE kernels; wost_device.h SegTree)
    int32_t tree_first_leaf;
    int32_t tree_leaf;
    float tree_tol;
    float tree_stop2;            // largest float whose sqrtf is <= rmin (< 0: none); silhouette_distance_tree
    float tree_kmax;             // SegmentTreeHost::kmax
    int32_t tree_lds_records;    // records staged in LDS (the first ones, 128 B each; field-specialised
                                 // kernels with kTreeStageBlock-thread workgroups), or 0: read through L1/L2
    int32_t tree_depth;          // level of the tree's leaves
    int32_t tree_lds_verts;      // Neumann vertices staged in LDS after the records (kTreeStageVertsBlock
                                 // workgroups, WOST_TREE_VSTAGED kernels), or 0
    // walk-range batches (wost_solve_range): when range_walks > 0, local walk l is walk
    // range_offset + l % range_walks of point range_point0 + l / range_walks, i.e. global
    // id (range_point0 + l / range_walks) * walks_per_point + range_offset + l % range_walks
    int64_t range_walks;
    int64_t range_offset;
    int64_t range_point0;
    double inv_range_walks;
    // delta tracking: alpha at each query point (point_alpha_body, same fields and
    // arithmetic as the walk's own alpha), read at a walk's start instead of
    // evaluating the field there
    const float* point_alpha;
    // 32-bit point index of a walk (the refill's quotient): wid_begin = base_pid * W +
    // base_off, and when base_off + count < 2^31 (small32) the quotient of base_off +
    // local index by W is taken in 32 bits (a double estimate and one correction)
    int64_t base_pid;
    uint32_t base_off;
    int32_t small32;
    // walk pools (TREE kernels, WOST_TREE_POOL; null: none): pool_wg_words words per
    // workgroup, a 4-word header (lock, walks parked near, walks parked far) and then
    // per class pool_slots parked walks of pool_fields(NS) words each (field-major);
    // a walk is "near" while its point lies in pool_box (x0, y0, x1, y1)
    uint32_t* pool;
    int32_t pool_slots;
    int32_t pool_wg_words;
    float4 pool_box;
    int32_t pool_near_waves;     // the workgroup's first pool_near_waves waves take the near walks
                                 // (0: each wave takes the class most of its walks are in)
    int32_t exact_trig;          // precompiled kernels: the direction's cos/sin correctly rounded
                                 // (wost_set_trig; the field-specialised kernels fix it at compile time)
    // the work queue's static first fill: wave v of the grid starts with local walks
    // [v * chunk0, (v + 1) * chunk0) (clamped to count) without touching the counter, and
    // the counter's dequeues start at queue_base = waves * chunk0 (>= count: none)
    int32_t chunk0;
    int64_t queue_base;
    // adaptive dequeues (chunk_share > 0; walk_body's refill): a wave's dynamic dequeue takes
    // at least the walks that keep the whole grid below ~4e7 dequeues per second at the
    // grid's walk completion rate as this wave measures it -- the walks it has completed
    // since it started, over the wall-clock ticks, times the grid's `waves` -- and at most
    // chunk_share (count / (waves * 4): a quarter of a wave's even share). The launch shape
    // is thus a function of this call alone, never of an earlier one.
    uint32_t chunk_share;
    uint32_t waves;
};

// The walk launch's control words (WalkArgs::counter): [0] the work-queue head, [1] the
// block reduce's finished-workgroup count, [2] its longest walk (kernels without wave
// records), [3] unused; then per wave two uint4 of launch statistics: {start tick low, high,
// last dequeue - start, end - start} and {loop iterations, longest walk, 0, 0} (wave index
// as in the static chunks). Derived from the
// queue's own pointer so that the walk loop keeps no extra pointer live.
constexpr int kCtlWords = 4;
WOST_HD constexpr size_t ctl_words(int64_t waves) { return (size_t)kCtlWords + 4 * (size_t)waves; }

// words of one parked walk: global id (2), local index (2), x, y, dD, step | onB << 31,
// phi, w, alpha(x), then the NS source totals
WOST_HD constexpr int pool_fields(int ns) { return 11 + ns; }
WOST_HD constexpr int pool_wg_words(int ns, int slots) { return 4 + 2 * pool_fields(ns) * slots; }

// The GPU's constant-rate wall clock (s_memrealtime, 100 MHz on gfx950: hipDeviceAttribute-
// WallClockRate), low 32 bits: differences are exact for launches shorter than ~42 s.
__device__ __forceinline__ uint64_t wall_ticks64() {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint64_t)__builtin_amdgcn_s_memrealtime();
#else
    return 0ull;
#endif
}
__device__ __forceinline__ uint32_t wall_ticks() { return (uint32_t)wall_ticks64(); }
// the grid's dequeue budget (~4e7 per second) per tick of the 100 MHz wall clock, inverted
constexpr float kDequeuesPerTickInv = 1.0e8f / 4.0e7f;
// The scan kernels' adaptive dequeues and launch statistics (walk_body). The segment-tree
// kernels compile neither: their registers are full (96 VGPRs at 5 waves per SIMD, with
// spills), their long walks take the host's 16-walk chunks, and the wave state they need
// cost the C5 kernel ~4% (profiles/r06_ab/).
#ifndef WOST_ADAPTIVE_DEQ
#define WOST_ADAPTIVE_DEQ 1
#endif
#ifndef WOST_WAVE_STATS
#define WOST_WAVE_STATS 1
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define WOST_KEEP_VGPR(v) __asm__ volatile("" : "+v"(v))
#else
#define WOST_KEEP_VGPR(v) ((void)0)
#endif

// Sum over the wave's lanes (every lane active), as a wave-uniform value.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// alpha at the query points with the walk kernel's own Fields policy (the same
// function the walk would evaluate at its start point, hence the same bits).
template <class F>
__device__ __forceinline__ void point_alpha_body(const float2* pts, int64_t n, float* out, const F& fld) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float2 q = pts[i];
        out[i] = fld.alpha(q.x, q.y);
    }
}

constexpr int kWalkBlock = 256;
// workgroup of the field-specialised tree kernels that stage the tree's records in LDS:
// 8 waves, two per SIMD, so two workgroups per CU place 4 waves on every SIMD (a
// 640-thread workgroup places 3-3-2-2 and a second one no longer fits 5 per SIMD:
// profiles/r03_tree/tree_lds_block_ab.log; WOST_TREE_LDS_BLOCK for A/B)
constexpr int kTreeStageBlock = 512;
// ... and of those that stage the polyline's vertices as well: one 16-wave workgroup per CU
constexpr int kTreeStageVertsBlock = 1024;

// Walk recorder (solvers/WoStSolver.py:197-309, return_history). Record k < steps
// of a walk is its step k: the pre-step point and its distances (:218-222), the
// source sample point after clipping and its contribution (:261-266).
// Record `steps` is the end: final point (REC_X, REC_Y), boundary contribution
// (REC_C) and the walk's total (REC_AUX) (:301-306). A step record's REC_AUX is
// 1 when the step sampled the source.
constexpr int kRecFloats = WOST_REC_FLOATS;   // include/wost.h, wost_solve_history
enum RecField { REC_X = 0, REC_Y, REC_DD, REC_DN, REC_SX, REC_SY, REC_C, REC_AUX };

WOST_HD size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

// LDS scratch of one wave for the cooperative tree queries (below): the hand-out
// slots and one result slot per owner lane
struct TreeWaveScratch {
    uint32_t task[64];             // owner | level << 6 | position << 10
    unsigned long long slot[64];   // silhouette: float bits of the squared distance; ray: s bits << 32 | segment
};
constexpr size_t kTreeWaveScratchBytes = sizeof(TreeWaveScratch);

// Bytes of dynamic LDS a walk-kernel workgroup needs, in layout order:
//  * G_norm cells (delta tracking; else a 16-byte pad): sample_rho_tail reads the
//    word before the sampler's tail;
//  * the sampler's nodes 1..N-1 (node 0 is a kernel argument);
//  * the Dirichlet vertices, unless the Fields policy has them compiled in;
//  * the Neumann vertices and segment angles (scan kernels), unless compiled in;
//  * with the segment tree, its first tree_lds records (128 B each), the tree_verts
//    staged Neumann vertices, then one TreeWaveScratch per wave (the cooperative
//    tree queries) of the `block`-thread workgroup.
// Query points are read from global memory (once per walk, at refill).
WOST_HD size_t walk_lds_bytes_for(bool neu, bool src, int nd, int nn, int n_points, bool tree = false,
                                  bool delta = false, int tree_lds = 0, bool const_d = false, bool const_n = false,
                                  bool global_polylines = false, int block = kWalkBlock, int tree_verts = 0) {
    if (global_polylines) const_d = const_n = true;   // nothing of the polylines is staged
    (void)n_points;
    size_t b = 0;
    if (src) b += delta ? sizeof(float4) * (size_t)kGnormCells : 16;
    if (src) b += sizeof(float) * (size_t)kSamplerTailFloats;
    b = align16(b);
    if (!const_d) b += align16(sizeof(float2) * (size_t)nd);
    if (neu && !tree && !const_n)
        b += align16(sizeof(float2) * (size_t)nn) + align16(sizeof(float) * (size_t)(nn > 1 ? nn - 1 : 0));
    if (tree)
        b += 8 * sizeof(float4) * (size_t)tree_lds + align16(sizeof(float2) * (size_t)tree_verts) +
             kTreeWaveScratchBytes * (size_t)((block + 63) / 64);
    return b;
}

// ---------------------------------------------------------------------------
// Wave-cooperative segment-tree queries (TREE kernels; compat="fixed" too, its ray
// query keyed by the nearest crossing's (t, segment)). The records and, when they
// fit, the vertices are read from LDS (WOST_TREE_STAGED / WOST_TREE_VSTAGED kernels).
//
// silhouette_distance_tree / intersect_polylines_tree run one query per lane, and a
// wave iterates until its slowest lane is done: at C5's walk positions ~89% of the
// queries end after one or two record visits while the few near the surface need
// 20-40, so a tree instruction ran on ~12-19% of the lanes. Here the lanes of a wave
// share the work: when at most WOST_TREE_SHARE lanes still search, the searching
// lanes hand the subtrees pending in their traversal state (pend bits: the children
// of an ancestor still to visit) to idle lanes, which search them for the same query
// (the owner's registers, read with a lane shuffle) and leave their result in the
// owner's LDS slot. Both queries are minima that do not depend on the visiting order
// (the silhouette query's squared distance, the ray query's lexicographic (s, segment)
// -- the scan's first argmin), so the answer is bit for bit the per-lane search's.
// Shared bounds only prune more: at each hand-out the silhouette searches of one
// owner take the smallest squared distance found so far by any of them.
// Every lane of the wave calls these together (no lane may have left the loop body).
// ---------------------------------------------------------------------------
#ifndef WOST_TREE_SHARE   // hand out pending subtrees when at most this many lanes search
#define WOST_TREE_SHARE 32
#endif
#ifndef WOST_TREE_SHARE_DESCENT   // also at every level of the descent (else once per leaf round)
#define WOST_TREE_SHARE_DESCENT 1
#endif
#ifndef WOST_TREE_SHARE_MIN   // ... and at least this many subtrees are pending
#define WOST_TREE_SHARE_MIN 1
#endif
#ifndef WOST_TREE_BATCH   // children of a record whose words are loaded together (1, 2 or 4)
#define WOST_TREE_BATCH 4
#endif

// the LDS writes of the wave's lanes visible to its other lanes (a wave's LDS
// operations complete in order; this keeps the compiler from moving them)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The pending subtrees of the wave: per bit b of each lane's count n < 32 of pend
// bits, the ballot of that bit (so the total is scalar work and a lane's prefix
// offset is taken only when a hand-out happens).
struct PendCount {
    uint64_t m[5];
    uint32_t total;
};
__device__ __forceinline__ PendCount wave_pend_count(uint32_t n) {
    PendCount c;
    c.total = 0u;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        c.m[b] = __ballot((n >> b) & 1u);
        c.total += (uint32_t)__popcll(c.m[b]) << b;
    }
    return c;
}

// Hand out pending subtrees: searching lanes (`live`, n = popcount(pend)) list their
// pend bits (the shallowest levels, i.e. the largest subtrees, first) into the idle
// lanes' slots; an idle lane that receives one becomes a helper: *owner, d, pos of the
// subtree's root, pend = 0. Returns true on the lanes that became helpers.
__device__ __forceinline__ bool tree_hand_out(TreeWaveScratch* ws, uint64_t live_mask, bool live, uint32_t n,
                                              const PendCount& pc, uint64_t lanes_below, int& owner, int& d, int& pos,
                                              uint32_t& pend) {
    const uint64_t idle = ~live_mask;
    const uint32_t nidle = (uint32_t)__popcll(idle);
    uint32_t off = 0u;   // exclusive prefix sum of n over the lanes below
#pragma unroll
    for (int b = 0; b < 5; ++b) off += (uint32_t)__popcll(pc.m[b] & lanes_below) << b;
    if (live && off < nidle) {
        const uint32_t give = n < nidle - off ? n : nidle - off;
        for (uint32_t i = 0; i < give; ++i) {
            const int b = lowest_bit(pend);
            pend &= pend - 1u;
            const int p = b >> 2, child = 4 * (pos >> (2 * (d - p))) + (b & 3);
            ws->task[off + i] = (uint32_t)owner | (uint32_t)(p + 1) << 6 | (uint32_t)child << 10;
        }
    }
    wave_lds_sync();
    const uint32_t rank = (uint32_t)__popcll(idle & lanes_below);
    const bool helper = !live && rank < (pc.total < nidle ? pc.total : nidle);
    if (helper) {
        const uint32_t tk = ws->task[rank];
        owner = (int)(tk & 63u);
        d = (int)((tk >> 6) & 15u);
        pos = (int)(tk >> 10);
        pend = 0u;
    }
    return helper;
}

// silhouette_distance_tree (wost_device.h), the wave's lanes sharing the search;
// `want`: this lane has a query. Same use contract (exact below dd and above rmin).
// (ic: loop counters of a WOST_TREE_ITER_STATS study build, else null and compiled away)
__device__ __forceinline__ float silhouette_distance_tree_wave(const SegTree& t, float px, float py, float dd,
                                                               float stop2, bool want, TreeWaveScratch* ws,
                                                               int lane, uint32_t* ic = nullptr) {
#pragma clang fp contract(off)
    const uint64_t lanes_below = (1ull << lane) - 1ull;
    const int nv = t.nv, nseg = nv - 1;
    const float Town = (dd * dd) * 1.002f;
    ws->slot[lane] = (unsigned long long)__builtin_bit_cast(uint32_t, WOST_INF);
    // the query this lane searches for (its own, or its owner's as a helper)
    float qx = px, qy = py, T = Town;
    // its rounding scales (silhouette_child_keep_q, WOST_TREE_QMARGIN)
    auto qscale = [&]() { return ((fabsf(qx) + fabsf(qy)) + t.kmax) * 1.001f; };
    float qsl = 9.5367431640625e-07f * qscale(), qmc = kConeMargin * qscale();   // 2^-20 W, 1e-5 W
    int owner = lane;
    float best = WOST_INF;
    bool live = want && nv >= 3;
    int d = 0, pos = 0;
    uint32_t pend = 0u;
    float plb0 = WOST_INF, plb1 = WOST_INF, plb2 = WOST_INF, plb3 = WOST_INF, plb4 = WOST_INF;
    auto plb_get = [&](int l) {
        float v = -WOST_INF;
        v = l == 0 ? plb0 : v; v = l == 1 ? plb1 : v; v = l == 2 ? plb2 : v;
        v = l == 3 ? plb3 : v; v = l == 4 ? plb4 : v;
        return v;
    };
    auto plb_set = [&](int l, float x) {
        plb0 = l == 0 ? x : plb0; plb1 = l == 1 ? x : plb1; plb2 = l == 2 ? x : plb2;
        plb3 = l == 3 ? x : plb3; plb4 = l == 4 ? x : plb4;
    };
    auto visit = [&](int lvl, int at, uint32_t cand, int& nj, float& nb2) {
        if (ic) {
            ic[3] += 1u;                                                     // lane-visits
            if (lane == (int)__builtin_ctzll(__ballot(1))) ic[15] += 1u;    // the wave's visit issues
        }
        const int k = tree_level_offset(lvl) + at;
        const float bound = best < T ? best : T;
        uint32_t kept = 0u;
        float nb = WOST_INF;
        nb2 = WOST_INF;
        nj = 0;
        // the children's words loaded WOST_TREE_BATCH children at a time before any test
        // (one round trip per batch; tested one by one the loads waited in turn)
#pragma unroll
        for (int j0 = 0; j0 < 4; j0 += WOST_TREE_BATCH) {
            float4 w[2 * WOST_TREE_BATCH];
#pragma unroll
            for (int i = 0; i < 2 * WOST_TREE_BATCH; ++i) w[i] = t.word(k, 2 * j0 + i);
#pragma unroll
            for (int u = 0; u < WOST_TREE_BATCH; ++u) {
                const int j = j0 + u;
                float lb;
#if WOST_TREE_QMARGIN
                const bool keep = silhouette_child_keep_q(w[2 * u], w[2 * u + 1], qx, qy, bound, qsl, qmc, &lb);
#else
                const bool keep = silhouette_child_keep(w[2 * u], w[2 * u + 1], qx, qy, bound, &lb);
#endif
                if (((cand >> j) & 1u) && keep) {
                    kept |= 1u << j;
                    if (lb < nb) { nb2 = nb; nb = lb; nj = j; }
                    else if (lb < nb2) nb2 = lb;
                }
            }
        }
        return kept;
    };
    auto resume = [&]() {
        while (pend != 0u) {
            const int p = highest_bit(pend) >> 2;
            const uint32_t m = (pend >> (4 * p)) & 15u;
            pend &= ~(15u << (4 * p));
            const float bound = best < T ? best : T;
            if (plb_get(p) > bound) continue;
            const int anc = pos >> (2 * (d - p));
            int nj;
            float nb2;
            const uint32_t kept = visit(p, anc, m, nj, nb2);
            if (kept) {
                pend |= (kept & ~(1u << nj)) << (4 * p);
                plb_set(p, nb2);
                pos = 4 * anc + nj;
                d = p + 1;
                return true;
            }
        }
        return false;
    };
    // hand out pending subtrees when few lanes still search (a uniform branch)
    auto share = [&](uint64_t L) {
        if (!(__popcll(L) <= WOST_TREE_SHARE) || __ballot(live && pend != 0u) == 0ull) return;
        const uint32_t n = live ? (uint32_t)__popcll(pend) : 0u;
        const PendCount pc = wave_pend_count(n);
        if (WOST_TREE_SHARE_MIN > 1 && pc.total < WOST_TREE_SHARE_MIN) return;
        if (ic) ic[4] += 1u;
        // every lane leaves what it found in its owner's slot, then takes the owner's
        // best so far as its bound
        if (best < WOST_INF) atomicMin(&ws->slot[owner], (unsigned long long)__builtin_bit_cast(uint32_t, best));
        if (tree_hand_out(ws, L, live, n, pc, lanes_below, owner, d, pos, pend)) {
            live = true;
            best = WOST_INF;
            plb0 = plb1 = plb2 = plb3 = plb4 = WOST_INF;
        }
        qx = __shfl(px, owner);
        qy = __shfl(py, owner);
        T = __shfl(Town, owner);
        qsl = 9.5367431640625e-07f * qscale();
        qmc = kConeMargin * qscale();
        const float sb = __builtin_bit_cast(float, (uint32_t)ws->slot[owner]);
        best = sb < best ? sb : best;
        if (live && best <= stop2) { live = false; pend = 0u; }
    };
    if (ic) ic[0] += 1u;
    wave_lds_sync();
    for (;;) {
        const uint64_t L = __ballot(live);
        if (L == 0ull) break;
        if (ic) ic[1] += 1u;
        share(L);
#if WOST_TREE_SHARE_DESCENT
        // the descent as a uniform loop, so that a hand-out can run at every level
        for (;;) {
            const bool down = live && d < t.depth;
            if (!__any(down)) break;
            if (ic) ic[2] += 1u;
            if (down) {
#else
        {
            while (live && d < t.depth) {
#endif
                int nj;
                float nb2;
                const uint32_t kept = visit(d, pos, 15u, nj, nb2);
                if (kept) {
                    pend |= (kept & ~(1u << nj)) << (4 * d);
                    plb_set(d, nb2);
                    pos = 4 * pos + nj;
                    ++d;
                } else {
                    live = resume();
                }
            }
#if WOST_TREE_SHARE_DESCENT
            share(__ballot(live));
#endif
        }
        // (no `continue` in this loop: every lane must reach the next ballot)
        if (ic && __any(live)) ic[6] += 1u;
        if (live) {
            if (ic) ic[5] += 1u;
            const int s0 = pos * t.leaf;
            const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
            const int j1 = s1 < nv - 2 ? s1 : nv - 2;
            bool stop = false;
            if (s0 + 1 <= j1) {
                const float2 va = t.vert(s0);
                float2 vb = t.vert(s0 + 1);
                float cprev = (vb.x - va.x) * (qy - va.y) - (vb.y - va.y) * (qx - va.x);
                // vertices loaded four at a time (indices clamped in range), then scanned
                for (int j0 = s0 + 1; j0 <= j1; j0 += 4) {
                    float2 vcs[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) vcs[u] = t.vert(j0 + 1 + u < nv ? j0 + 1 + u : nv - 1);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (j0 + u <= j1) {
                            const float2 vc = vcs[u];
                            const float bpx = qx - vb.x, bpy = qy - vb.y;
                            const float ccur = (vc.x - vb.x) * bpy - (vc.y - vb.y) * bpx;
                            if (cprev * ccur < 0.0f) {
                                const float d2 = bpx * bpx + bpy * bpy;
                                best = d2 < best ? d2 : best;
                            }
                            cprev = ccur;
                            vb = vc;
                        }
                    }
                }
                stop = best <= stop2;
            }
            if (stop) {
                live = false;
                pend = 0u;
            } else {
                live = resume();
            }
        }
    }
    if (best < WOST_INF) atomicMin(&ws->slot[owner], (unsigned long long)__builtin_bit_cast(uint32_t, best));
    wave_lds_sync();
    const float res = __builtin_bit_cast(float, (uint32_t)ws->slot[lane]);
    wave_lds_sync();   // the slots are rewritten by the next query
    return res == WOST_INF ? res : sqrt_rn(res);
}

// intersect_polylines_tree<NORMAL> (wost_device.h, reference mode), the wave's lanes
// sharing the search; `want`: this lane has a query.
// NEAREST (compat="fixed"): the nearest crossing of intersect_polylines_tree<.., true>,
// the lexicographic minimum of (t, segment), t > 0.
template <bool NORMAL = true, bool NEAREST = false>
__device__ __forceinline__ Hit intersect_polylines_tree_wave(const SegTree& t, float px, float py, float dxi,
                                                             float dyi, float r, bool want, TreeWaveScratch* ws,
                                                             int lane, uint32_t* ic = nullptr) {
#pragma clang fp contract(off)
    const uint64_t lanes_below = (1ull << lane) - 1ull;
    float dn, dx, dy;
    unit_direction(dxi, dyi, dn, dx, dy);
    const bool degenerate = dn < 1e-10f;
    const float qx0 = px + 1e-6f * dx, qy0 = py + 1e-6f * dy;
    const float tol0 = t.tol + 7.62939453125e-06f * (fabsf(qx0) + fabsf(qy0));   // + 2^-17 |q|_1
    const int nseg = t.nv - 1;
    ws->slot[lane] = ~0ull;
    float qx = qx0, qy = qy0, ddx = dx, ddy = dy, tol = tol0;
    int owner = lane;
    float best = WOST_INF;
    int bi = -1;
    bool live = want && !degenerate;
    // the pruning of intersect_polylines_tree's keep()
    auto keep = [&](float4 cu, float4 ab) {
        if (ab.x < 0.0f) return false;
        const float cx = cu.x - qx, cy = cu.y - qy;
        const float cr = ddx * cu.w - ddy * cu.z, dt = ddx * cu.z + ddy * cu.w;
        if (fabsf(ddx * cy - ddy * cx) > (ab.x * fabsf(cr) + ab.y * fabsf(dt)) + tol) return false;
#if !defined(WOST_NO_TREE_BEHIND)
        if (ab.z == 3.0f) return true;
        const float ahead = (ddx * cx + ddy * cy) + (ab.x * fabsf(dt) + ab.y * fabsf(cr));
        if (!(ahead < -(512.0f * tol + 1e-2f * ((fabsf(cx) + fabsf(cy)) + (ab.x + ab.y))))) return true;
        if (ab.z == 2.0f) return false;
        return !(ab.z * fabsf(cr) - ab.w * fabsf(dt) > 1e-3f);
#else
        return true;
#endif
    };
    int d = 0, pos = 0;
    uint32_t pend = 0u;
    auto resume = [&]() {
        if (pend == 0u) return false;
        const int p = highest_bit(pend) >> 2;
        const int j = lowest_bit((pend >> (4 * p)) & 15u);
        pend &= ~(1u << (4 * p + j));
        pos = 4 * (pos >> (2 * (d - p))) + j;
        d = p + 1;
        return true;
    };
    // (s, segment) as one 64-bit key: s >= 0 here, so its bits order like the floats
    // (s + 0 makes a -0 the +0 it ties with, leaving the segment index to decide)
    auto deposit = [&]() {
        if (bi >= 0)
            atomicMin(&ws->slot[owner], (unsigned long long)__builtin_bit_cast(uint32_t, best + 0.0f) << 32 |
                                            (unsigned long long)(uint32_t)bi);
    };
    auto share = [&](uint64_t L) {
        if (!(__popcll(L) <= WOST_TREE_SHARE) || __ballot(live && pend != 0u) == 0ull) return;
        const uint32_t n = live ? (uint32_t)__popcll(pend) : 0u;
        const PendCount pc = wave_pend_count(n);
        if (WOST_TREE_SHARE_MIN > 1 && pc.total < WOST_TREE_SHARE_MIN) return;
        if (ic) ic[11] += 1u;
        deposit();
        if (tree_hand_out(ws, L, live, n, pc, lanes_below, owner, d, pos, pend)) {
            live = true;
            best = WOST_INF;
            bi = -1;
        }
        qx = __shfl(qx0, owner);
        qy = __shfl(qy0, owner);
        ddx = __shfl(dx, owner);
        ddy = __shfl(dy, owner);
        tol = __shfl(tol0, owner);
    };
    if (ic) ic[7] += 1u;
    wave_lds_sync();
    for (;;) {
        const uint64_t L = __ballot(live);
        if (L == 0ull) break;
        if (ic) ic[8] += 1u;
        share(L);
#if WOST_TREE_SHARE_DESCENT
        for (;;) {
            const bool down = live && d < t.depth;
            if (!__any(down)) break;
            if (ic) ic[9] += 1u;
            if (down) {
#else
        {
            while (live && d < t.depth) {
#endif
                if (ic) ic[10] += 1u;
                const int k = tree_level_offset(d) + pos;
                uint32_t kept = 0u;
#pragma unroll
                for (int j0 = 0; j0 < 4; j0 += WOST_TREE_BATCH) {
                    float4 w[2 * WOST_TREE_BATCH];
#pragma unroll
                    for (int i = 0; i < 2 * WOST_TREE_BATCH; ++i) w[i] = t.word(k, 2 * j0 + i);
#pragma unroll
                    for (int u = 0; u < WOST_TREE_BATCH; ++u)
                        if (keep(w[2 * u], w[2 * u + 1])) kept |= 1u << (j0 + u);
                }
                if (kept) {
                    const int j = lowest_bit(kept);
                    pend |= (kept & ~(1u << j)) << (4 * d);
                    pos = 4 * pos + j;
                    ++d;
                } else {
                    live = resume();
                }
            }
#if WOST_TREE_SHARE_DESCENT
            share(__ballot(live));
#endif
        }
        const int s0 = pos * t.leaf;
        const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
        if (ic && __any(live && s0 < s1)) ic[13] += 1u;
        if (ic && live && s0 < s1) ic[12] += 1u;
        if (NEAREST && live && s0 < s1) {
            float2 a = t.vert(s0);
            for (int i0 = s0; i0 < s1; i0 += 4) {   // vertices loaded four at a time
                float2 bs[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) bs[u] = t.vert(i0 + 1 + u <= nseg ? i0 + 1 + u : nseg);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (i0 + u < s1) {
                        const int i = i0 + u;
                        // t <= best (ties too: the lower segment index wins them)
                        const float bq = best < WOST_INF ? bits_to_float(__builtin_bit_cast(int32_t, best) + 1) : best;
                        const float tt = ray_segment_nearest_t(a, bs[u], qx, qy, ddx, ddy, bq);
                        if (tt < best || (tt == best && i < bi)) { best = tt; bi = i; }
                        a = bs[u];
                    }
                }
            }
        } else if (live && s0 < s1) {
            const float S = 2.0f * tol;
            const float m = fmaf(ddx, qy, -(ddy * qx));
            const float hi = m + S, lo = m - S;     // the thresholds of intersect_polylines_lines
            const float2 a = t.vert(s0);
            const float ca = fmaf(ddx, a.y, -(ddy * a.x));
            bool aprev = ca > hi, bprev = ca < lo;   // the filter of intersect_polylines_lines
            uint32_t cand = 0u;
            for (int i0 = s0; i0 < s1; i0 += 4) {   // vertices loaded four at a time
                float2 bs[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) bs[u] = t.vert(i0 + 1 + u <= nseg ? i0 + 1 + u : nseg);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (i0 + u < s1) {
                        const float cb = fmaf(ddx, bs[u].y, -(ddy * bs[u].x));
                        const bool ab = cb > hi, bb = cb < lo;
                        if (!((aprev && ab) || (bprev && bb))) cand |= 1u << (i0 + u - s0);
                        aprev = ab;
                        bprev = bb;
                    }
                }
            }
            while (cand != 0u) {
                const int i = s0 + lowest_bit(cand);
                cand &= cand - 1u;
                const float s = ray_segment_time_filtered(t.vert(i), t.vert(i + 1), qx, qy, ddx, ddy);
                if (s < best || (s == best && i < bi)) { best = s; bi = i; }
            }
        }
        if (live) live = resume();
    }
    deposit();
    wave_lds_sync();
    const unsigned long long key = ws->slot[lane];
    wave_lds_sync();   // the slots are rewritten by the next query
    if (degenerate) {
        Hit h;
        h.x = px; h.y = py; h.nx = 1.f; h.ny = 0.f; h.hit = false; h.seg = -1;
        return h;
    }
    const int wbi = key == ~0ull ? -1 : (int)(uint32_t)key;
    const float wbest = key == ~0ull ? WOST_INF : __builtin_bit_cast(float, (uint32_t)(key >> 32));
    if (NEAREST) return ray_nearest_finish(wbi, wbest, px, py, dx, dy, qx0, qy0, r);
    return intersect_finish<NORMAL>(t.v, wbi, wbest, px, py, dx, dy, qx0, qy0, r);
}

// The Fields policy F provides: has_g(), g(x,y), f(x,y), sigma(x,y),
// alpha(x,y), alpha_jet(x,y), detached(), sigma_bar(), sqrt_sigma_bar(),
// inv_sigma_bar(), and the polyline scans dirichlet_distance(sD,
// nd, x, y), neumann_silhouette_distance(sN, nn, x, y), neumann_intersect(sN,
// nn, x, y, dx, dy, r), neumann_intersect_nearest(...) (compat="fixed"),
// neumann_phi(sPhi, seg) (the interpreted kernels scan the
// staged vertices; the specialised ones may have them compiled in:
// F::kConstDirichlet / F::kConstNeumann, and then nothing is staged for them). TREE: Neumann queries through
// the segment tree. REC: the kernel can record walks (A.rec).
// NS > 1 (multi-source batching): the walk scores NS source
// fields at once -- the walk itself does not depend on the source, so every
// source's total is bit for bit what a single-source solve of it gives. The
// Fields policy then provides f_multi(x, y, float out[NS]); per-walk values go
// to out_val[local walk * NS + k].
// FIX (compat="fixed"): the estimator with the reference's quirks corrected
// (SURVEY 8a):
//  Q7/Q12 the walk stops when the CURRENT point's Dirichlet distance is <= eps
//         (no extra step inside the eps-shell; eps >= 1 no longer skips walks);
//  Q1     the Neumann ray query takes the nearest crossing along the ray;
//  Q2     after a Neumann hit the direction is uniform on the hemisphere of the
//         INWARD normal (the side the ray came from);
//  Q3     the source radius follows the Green's density with its Jacobian,
//         rho ln(1/rho) (the host builds that sampler table);
//  Q13    (Laplace / Poisson / mixed) the source sample takes its own direction
//         (Philox word w) and counts only if it is visible from x (no Neumann
//         crossing before it); on a Neumann boundary point that direction, like
//         the step's, is uniform on the inward hemisphere (the star-shaped region
//         is then a half-ball: the full ball's radial law over a half-circle of
//         directions gives the factor 2 of the boundary representation);
//  Q4/Q5  delta tracking draws the sample from the ball's screened Green's
//         function of THIS radius (shape s = R sqrt(sigma_bar), Jacobian
//         included, no clipped envelope; sample_rho_screened_fixed).
//  Delta tracking with Neumann boundaries needs more than the reference's
//  collision rule: along a ray that meets the boundary at distance d < R, the
//  screened Poisson kernel's weight there is t (K1(t) + c I1(t)) (t = d
//  sqrt(sigma_bar)), not 1/I0(R sqrt(sigma_bar)) -- per direction, the
//  no-collision probability must be 1 - sigma_bar |G| F_s(d / R). FIX draws the
//  sample on the step's ray and collides only when mu <= sigma_bar |G| AND the
//  sample lies before the ray's boundary point (probability F_s(d / R)), which is
//  exactly that, with the collision point from the truncated law; otherwise the
//  walk moves to the ray's point with weight 1. A collision leaves the Neumann
//  boundary, and its weight 1 - sigma'/sigma_bar is kept signed (unbiased for
//  any sigma_bar; the reference's max(., 0) at solvers/WoStSolver.py:282 is
//  biased wherever sigma' > sigma_bar).
// GL: the polylines (and segment angles) are read from global memory instead of being
// staged in LDS -- field-specialised kernels for polylines too long for the LDS budget
// (wost_api.hip kGlobalPolylineLdsBytes).
// Walk pools (TREE kernels): see the exchange in walk_body. WOST_TREE_POOL 0 compiles
// them out; WOST_POOL_MIN_PUSH: fewest mismatched walks a wave parks at once.
#ifndef WOST_TREE_POOL
#define WOST_TREE_POOL 1
#endif
#ifndef WOST_POOL_MIN_PUSH
#define WOST_POOL_MIN_PUSH 1
#endif
__device__ __forceinline__ bool pool_near(float4 b, float x, float y) {
    return x >= b.x && x <= b.z && y >= b.y && y <= b.w;
}
// walks parked in class c (header word 1 + c), read with an atomic load so that every
// read goes to memory (under the lock: exact; outside it: a hint)
// A pool count as a wave-uniform value: the first active lane's load, broadcast. The
// callers branch on it around pool_lock/pool_unlock, which must run with the whole wave
// (lane 0 takes the lock for it), so no lane may see a different count.
__device__ __forceinline__ uint32_t pool_count(uint32_t* pool, int c) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(pool + 1 + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// the pool lock (header word 0), taken by the wave's first lane for the whole wave; the
// fences order the wave's slot reads and writes inside it
__device__ __forceinline__ void pool_lock(uint32_t* pool, int lane) {
    if (lane == 0) {
        while (__hip_atomic_exchange(pool, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u)
            __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void pool_unlock(uint32_t* pool, int lane, uint32_t n_near, uint32_t n_far) {
    if (lane == 0) {
        __hip_atomic_store(pool + 1, n_near, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(pool + 2, n_far, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) __hip_atomic_store(pool, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Phase markers of the walk step for the offline ISA budget (tools/r05/phase_isa.py,
// WOST_PHASE_MARKS builds only): an assembly comment, which also bounds the instruction
// scheduler's regions, so the marked kernel is a study build, never the one that runs.
#if defined(WOST_PHASE_MARKS)
#define WOST_PHASE(name) asm volatile("; @phase " name)
#else
#define WOST_PHASE(name)
#endif

// Study builds (tools/r05/phase_dup.sh; WOST_EXP_FLAGS bits 2^18 and up, A/B only): a
// phase of the walk step computed a second time from opaque copies of its inputs and
// merged so that it cannot be removed yet changes no bit (x | (y & opaque 0)), so the
// walks are the same walks and the dynamic VALU counter grows by that phase's cost plus
// the merge's ~3 instructions. 1 Dirichlet distance, 2 Philox draw, 4 direction cos/sin,
// 8 Neumann ray query (scan kernels), 16 radial sampler, 32 screened G_norm, 64 alpha jet
// at the sample, 128 alpha at the ray's point, 256 the source f, 512 sigma'.
#ifndef WOST_ABL_DUP
#define WOST_ABL_DUP 0
#endif
__device__ __forceinline__ float dup_opq(float v) {
    __asm__ volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t dup_zero() {
    uint32_t z = 0u;
    __asm__ volatile("" : "+v"(z));
    return z;
}
__device__ __forceinline__ float dup_merge(float a, float b) {   // a, depending on b
    return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, a) | (__builtin_bit_cast(uint32_t, b) & dup_zero()));
}

// The direction's cos and sin (wost_set_trig): correctly rounded (sincos_rn, the
// reference's values but for its own ulp errors; double-precision arithmetic) or the
// hardware's v_sin/v_cos (a few ulps, tens near the zeros). The field-specialised kernels
// fix the choice at compile time (WOST_JIT_TRIG_EXACT 1 / 0), the precompiled ones take
// it per launch (a uniform branch).
__device__ __forceinline__ void walk_sincos(float theta, float& sn, float& cs, bool exact) {
#if defined(WOST_JIT_TRIG_EXACT)
    exact = WOST_JIT_TRIG_EXACT != 0;
#endif
    if (exact) {
        sincos_rn(theta, sn, cs);
    } else {
        cs = f_cos(theta);
        sn = f_sin(theta);
    }
}

#ifndef WOST_REFILL_MIN   // idle lanes that trigger a refill (tools/ab_refill.sh; 1 = every iteration)
#define WOST_REFILL_MIN 4
#endif
// Philox one step ahead: step k's random words are drawn during step k - 1 (at the
// refill for step 0), right after that step's direction, where the ten dependent
// multiply rounds can overlap the step's geometry and field arithmetic instead of
// heading the next step's dependency chain. The words depend only on (seed, walk id,
// step), so the bits are unchanged.
// (1: where the compiler puts it -- it sinks the draw to the loop latch; 2: pinned
// right after the direction; 3: pinned before the source sample's clip test)
#ifndef WOST_PHILOX_AHEAD
#define WOST_PHILOX_AHEAD 0
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define WOST_PIN_U4(u) __asm__ volatile("" : "+v"((u).x), "+v"((u).y), "+v"((u).z), "+v"((u).w))
#else
#define WOST_PIN_U4(u) ((void)0)
#endif
template <bool NEU, bool SRC, bool DELTA, bool TREE, bool REC, int NS = 1, bool FIX = false, bool GL = false,
          class F>
__device__ __forceinline__ void walk_body(const WalkArgs& A, const F& fld, unsigned char* smem) {
    // the walk's position updates round op by op like the reference (torch CPU
    // has no FMA contraction); the field math it calls keeps its own setting
#pragma clang fp contract(off)
    static_assert(NS >= 1 && (NS == 1 || SRC) && (NS == 1 || !REC), "multi-source walks need a source, no recorder");
    constexpr bool kStageD = !F::kConstDirichlet && !GL;
    // the Neumann polyline is staged also when compiled in (FIX scans sN itself; a few
    // hundred bytes otherwise)
    constexpr bool kStageN = NEU && !TREE && !GL;
    unsigned char* lds = smem;
    float4* sG = reinterpret_cast<float4*>(lds);                          // G_norm cells
    float* sT = reinterpret_cast<float*>(lds + (DELTA ? sizeof(float4) * (size_t)kGnormCells : 16));  // sampler tail
    lds += SRC ? align16((DELTA ? sizeof(float4) * (size_t)kGnormCells : 16) + sizeof(float) * kSamplerTailFloats) : 0;
    float2* sD = reinterpret_cast<float2*>(lds);
    lds += kStageD ? align16(sizeof(float2) * (size_t)A.nd) : 0;
    float2* sN = reinterpret_cast<float2*>(lds);
    lds += kStageN ? align16(sizeof(float2) * (size_t)A.nn) : 0;
    float* sPhi = reinterpret_cast<float*>(lds);
    lds += kStageN ? align16(sizeof(float) * (size_t)(A.nn > 1 ? A.nn - 1 : 0)) : 0;
    // the cooperative tree queries (the silhouette and the step's ray query; compat="fixed"
    // keeps the per-lane search for the source sample's visibility)
    constexpr bool kWaveTree = TREE;
    float4* const sRec = reinterpret_cast<float4*>(lds);   // staged tree records (TREE, tree_lds_records > 0)
    const int n_rec = TREE ? A.tree_lds_records : 0;
    lds += 8 * sizeof(float4) * (size_t)n_rec;
    float2* const sVert = reinterpret_cast<float2*>(lds);  // staged Neumann vertices (TREE, tree_lds_verts > 0)
    const int n_vert = TREE ? A.tree_lds_verts : 0;
    lds += align16(sizeof(float2) * (size_t)n_vert);
    TreeWaveScratch* const tws = reinterpret_cast<TreeWaveScratch*>(lds) + (threadIdx.x >> 6);
    for (int i = threadIdx.x; i < 8 * n_rec; i += blockDim.x) sRec[i] = A.tree[i];
    for (int i = threadIdx.x; i < n_vert; i += blockDim.x) sVert[i] = A.nverts[i];

    if (kStageD)
        for (int i = threadIdx.x; i < A.nd; i += blockDim.x) sD[i] = A.dverts[i];
    if (kStageN) {
        for (int i = threadIdx.x; i < A.nn; i += blockDim.x) sN[i] = A.nverts[i];
        for (int i = threadIdx.x; i < A.nn - 1; i += blockDim.x) sPhi[i] = A.seg_phi[i];
    }
    // the polylines the queries read: the LDS copies, or (GL) global memory
    const float2* const dP = GL ? A.dverts : sD;
    const float2* const nP = GL ? A.nverts : sN;
    const float* const phiP = GL ? A.seg_phi : sPhi;
    const SegTree tree{A.tree, A.nverts, A.nn, A.tree_first_leaf, A.tree_depth, A.tree_leaf, A.tree_tol, A.tree_kmax,
                       sRec, n_rec, sVert};
    float node0 = 0.0f;
    if (SRC) {
        node0 = A.table[0];
        for (int i = threadIdx.x; i < kSamplerTailFloats; i += blockDim.x) sT[i] = A.table[i + 1];
    }
    if (DELTA) {
        const float4* g = reinterpret_cast<const float4*>(A.table + kSamplerFloatsPadded);
        for (int i = threadIdx.x; i < kGnormCells; i += blockDim.x) sG[i] = g[i];
    }
    // this workgroup's walk pools (header: lock, walks parked near, walks parked far)
    uint32_t* const pool = (TREE && WOST_TREE_POOL && A.pool != nullptr)
                               ? A.pool + (size_t)blockIdx.x * (size_t)A.pool_wg_words : nullptr;
    if (pool != nullptr && threadIdx.x < 4) pool[threadIdx.x] = 0u;
    __syncthreads();

    const float sigma_bar = fld.sigma_bar();
    const float inv_sb = fld.inv_sigma_bar();
    const float sqrt_sb = fld.sqrt_sigma_bar();

    const int lane = threadIdx.x & 63;
    const uint64_t lanebit = 1ull << lane;
    const uint64_t lanes_below = lanebit - 1ull;

    // wave-uniform work-queue state
    uint64_t c_next = 0, c_end = 0;
    bool exhausted = false;
    // the wave's own measurements (adaptive dequeues, launch statistics): its start and
    // last dequeue on the wall clock and its loop iterations (wave-uniform values kept in
    // VGPRs: the SGPR file is full, and a uniform scalar here would spill into VGPR lanes
    // through v_writelane / v_readlane inside the loop)
    constexpr bool kAdaptive = WOST_ADAPTIVE_DEQ && !TREE;
    constexpr bool kWaveStats = WOST_WAVE_STATS && !TREE;
    uint32_t q_t0 = (kAdaptive || kWaveStats) ? wall_ticks() : 0u;
    WOST_KEEP_VGPR(q_t0);
    uint32_t q_tdeq = q_t0;   // (WOST_WAVE_STATS)
    uint32_t q_iters = 0u;
    WOST_KEEP_VGPR(q_iters);
    uint32_t q_taken = 0u;   // walks this wave took from its static chunk and the queue (kAdaptive)
    WOST_KEEP_VGPR(q_taken);
    uint32_t my_kmax = 0u;   // the longest walk this lane finished (kWaveStats)
    {   // the wave's static first chunk (no atomic at the launch's start, when every wave
        // would hit the one counter at once)
        const uint64_t wv = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        const uint64_t cnt = (uint64_t)A.count;
        c_next = min(wv * (uint64_t)A.chunk0, cnt);
        c_end = min(c_next + (uint64_t)A.chunk0, cnt);
    }

    // per-lane walk state (solvers/WoStSolver.py:188-195)
    bool active = false;
    uint64_t wid = 0;           // global walk id: the Philox subsequence
    PhiloxWalk pw{0u, 0u, 0u, 0u};   // its per-walk Philox words (philox_walk)
    uint64_t lid = 0;           // local walk index: the output slot
    float px = 0.f, py = 0.f;
    float dD = 1.0f;            // dDirichlet seeded with 1.0 (:190, quirk Q12)
    int k = 0;                  // step_count
    bool onB = false;           // onBoundary
    float phi = 0.f;            // atan2 of currentNormal (:228), set when onB
    float w = 1.f;              // attenuation_coef
    float ax = 1.f;             // alpha(current_point), cached
    U4 rn_ahead{0u, 0u, 0u, 0u};   // (WOST_PHILOX_AHEAD) the words of this walk's step k
    float total[NS];            // this walk's contributions (one per source)
#pragma unroll
    for (int s = 0; s < NS; ++s) total[s] = 0.f;
#if defined(WOST_TREE_ITER_STATS)   // study build: the tree queries' loop counters (WOST_IC)
    uint32_t ic_arr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ic_arr[i] = 0u;
#define WOST_IC (TREE ? ic_arr : nullptr)
#else
#define WOST_IC nullptr
#endif

    // Tree kernels (long walks) also defer a finished walk's end record and output
    // into the refill batch: it idles until WOST_REFILL_MIN lanes are finished or
    // idle, or no lane is still stepping (C5 +4%; C3 and Laplace -2%, C4 neutral:
    // profiles/r02_ab/termination_batch.log). Its state does not change meanwhile,
    // so neither do its bits.
    constexpr bool kBatchEnd = TREE;
    for (;;) {
        const bool done = active && !((k < A.max_steps) && (dD > A.eps));
        bool batch = true;
        if (kBatchEnd) batch = __popcll(__ballot(done || !active)) >= WOST_REFILL_MIN || !__any(active && !done);
        // --- walk termination: while-condition of :206, boundary term :295-298
        if (batch && done) {
            float g = fld.has_g() ? fld.g(px, py) : 0.0f;
            if (DELTA) g = g * w;
#pragma unroll
            for (int s = 0; s < NS; ++s) total[s] = total[s] + g;
            const int64_t li = (int64_t)lid;
            if (REC && A.rec != nullptr) {
                float* rr = A.rec + ((size_t)li * (size_t)A.rec_stride + (size_t)k) * kRecFloats;
                rr[REC_X] = px; rr[REC_Y] = py; rr[REC_C] = g; rr[REC_AUX] = total[0];   // end record
            }
#pragma unroll
            for (int s = 0; s < NS; ++s) A.out_val[li * NS + s] = total[s];
            A.out_steps[li] = (uint32_t)k;
            if (kWaveStats) my_kmax = (uint32_t)k > my_kmax ? (uint32_t)k : my_kmax;
            active = false;
        }

        // --- refill idle lanes from the wave's chunk (active-mask compaction), in
        // batches: the refill runs on the few lanes it starts while the wave's other
        // lanes wait, so finished lanes idle until WOST_REFILL_MIN of them (or all
        // the wave's live ones) can start together. Each walk's result depends only
        // on its id, so the batching changes no bits.
        // --- walk pools (TREE kernels): a wave pays its slowest lane's tree queries, and the
        // lanes whose walks are near the Neumann polyline are the slow ones (C5: ~5% of the
        // positions within 30 units of the topography cost ~5x the others). A wave whose
        // walks are mostly far parks its near walks in the workgroup's near pool, and one
        // whose walks are mostly near parks its far ones; freed lanes take parked walks of
        // the wave's own class first, then new walks from the queue. A walk's state moves
        // with it whole and its result depends only on its id: the bits do not change.
        if (pool != nullptr && batch) {
            const uint64_t act = __ballot(active);
            const uint64_t nm = __ballot(active && pool_near(A.pool_box, px, py));
            const int nact = __popcll(act), nnear = __popcll(nm);
            const uint32_t hn = pool_count(pool, 0), hf = pool_count(pool, 1);
            const int role = A.pool_near_waves > 0 ? ((int)(threadIdx.x >> 6) < A.pool_near_waves ? 0 : 1)
                             : nact > 0 ? (2 * nnear > nact ? 0 : 1) : (hn >= hf ? 0 : 1);
            uint64_t mis = role == 0 ? (act & ~nm) : nm;
            if (exhausted || __popcll(mis) < WOST_POOL_MIN_PUSH) mis = 0ull;
            if (mis != 0ull || (act != ~0ull && (role == 0 ? hn : hf) > 0u)) {
                pool_lock(pool, lane);
                uint32_t cnt[2] = {pool_count(pool, 0), pool_count(pool, 1)};
                const int cm = 1 - role;
                const uint32_t npush = min((uint32_t)__popcll(mis), (uint32_t)A.pool_slots - cnt[cm]);
                const uint32_t rk = (uint32_t)__popcll(mis & lanes_below);
                if ((mis & lanebit) && rk < npush) {
                    uint32_t* const r = pool + 4 + (size_t)cm * pool_fields(NS) * A.pool_slots + cnt[cm] + rk;
                    const int P = A.pool_slots;
                    r[0 * P] = (uint32_t)wid; r[1 * P] = (uint32_t)(wid >> 32);
                    r[2 * P] = (uint32_t)lid; r[3 * P] = (uint32_t)(lid >> 32);
                    r[4 * P] = __builtin_bit_cast(uint32_t, px); r[5 * P] = __builtin_bit_cast(uint32_t, py);
                    r[6 * P] = __builtin_bit_cast(uint32_t, dD);
                    r[7 * P] = (uint32_t)k | (onB ? 0x80000000u : 0u);
                    r[8 * P] = __builtin_bit_cast(uint32_t, phi); r[9 * P] = __builtin_bit_cast(uint32_t, w);
                    r[10 * P] = __builtin_bit_cast(uint32_t, ax);
#pragma unroll
                    for (int s = 0; s < NS; ++s) r[(11 + s) * P] = __builtin_bit_cast(uint32_t, total[s]);
                    active = false;
                }
                cnt[cm] += npush;
                const uint64_t fr = __ballot(!active);
                const uint32_t npull = min((uint32_t)__popcll(fr), cnt[role]);
                const uint32_t rf = (uint32_t)__popcll(fr & lanes_below);
                if (!active && rf < npull) {
                    const uint32_t* const r =
                        pool + 4 + (size_t)role * pool_fields(NS) * A.pool_slots + (cnt[role] - npull) + rf;
                    const int P = A.pool_slots;
                    wid = (uint64_t)r[0 * P] | (uint64_t)r[1 * P] << 32;
                    lid = (uint64_t)r[2 * P] | (uint64_t)r[3 * P] << 32;
                    px = __builtin_bit_cast(float, r[4 * P]); py = __builtin_bit_cast(float, r[5 * P]);
                    dD = __builtin_bit_cast(float, r[6 * P]);
                    const uint32_t kb = r[7 * P];
                    k = (int)(kb & 0x7fffffffu); onB = (kb >> 31) != 0u;
                    phi = __builtin_bit_cast(float, r[8 * P]); w = __builtin_bit_cast(float, r[9 * P]);
                    ax = __builtin_bit_cast(float, r[10 * P]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) total[s] = __builtin_bit_cast(float, r[(11 + s) * P]);
                    pw = philox_walk(wid, A.key0, A.key1);
                    if (WOST_PHILOX_AHEAD) rn_ahead = philox_draw(pw, (uint32_t)k, A.key0, A.key1);
                    active = true;
                }
                cnt[role] -= npull;
                pool_unlock(pool, lane, cnt[0], cnt[1]);
            }
        }
        uint64_t need = batch ? __ballot(!active) : 0ull;
        if (!kBatchEnd && __popcll(need) < WOST_REFILL_MIN && __any(active)) need = 0ull;
        while (need != 0ull && !exhausted) {
            if (c_next >= c_end) {
                if (A.queue_base >= A.count) {   // the static chunks covered every walk
                    exhausted = true;
                    break;
                }
                // the dequeue's size: the host's (WalkArgs::chunk), raised (adaptive) to
                // keep the grid below ~4e7 dequeues per second at the walk completion rate
                // seen so far (cheap short walks: a counter dequeue per 64 walks would set
                // the pace, 2.1e11 -> 7.0e10 walk-steps/s on Laplace), within chunk_share
                uint32_t chunk = (uint32_t)A.chunk;
                const uint32_t now = (kAdaptive || kWaveStats) ? wall_ticks() : 0u;
                if (kAdaptive && A.chunk_share > 0u) {
                    // the walks this wave completed: taken, less its lanes still walking
                    const float done = (float)(q_taken - (64u - (uint32_t)__popcll(need)));
                    // grid walks per second / 4e7 per second, at the 100 MHz wall clock
                    const float lo = fminf((float)A.chunk_share, ceilf(done * (float)A.waves * kDequeuesPerTickInv /
                                                                       ((float)(now - q_t0) + 1.0f)));
                    chunk = (uint32_t)__builtin_amdgcn_readfirstlane((int)fmaxf(lo, (float)chunk));
                }
                unsigned long long c = 0;
                if (lane == 0) c = atomicAdd(A.counter, (unsigned long long)chunk);
                c += (unsigned long long)A.queue_base;
                // lane 0's value as a scalar (every lane runs the refill): the queue
                // state stays in SGPRs and the refill loop's control flow uniform
                c = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(c >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c);
                if (c >= (unsigned long long)A.count) {
                    exhausted = true;
                    break;
                }
                if (kWaveStats) {
                    q_tdeq = now;
                    WOST_KEEP_VGPR(q_tdeq);
                }
                c_next = c;
                c_end = c + (uint64_t)chunk;
                if (c_end > (uint64_t)A.count) c_end = (uint64_t)A.count;
            }
            const uint64_t avail = c_end - c_next;
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t take = avail < (uint64_t)n ? (uint32_t)avail : n;
            const uint32_t rank = (uint32_t)__popcll(need & lanes_below);
            if ((need & lanebit) && rank < take) {
                lid = c_next + rank;
                // integer quotients without a 64-bit division: a double estimate
                // (exact operands below 2^53) and one correction
                uint64_t pid;
                if (A.range_walks > 0) {
                    // local index < 2^26 (one launch): a 32-bit quotient
                    const uint32_t l32 = (uint32_t)lid, rw = (uint32_t)A.range_walks;
                    uint32_t q = (uint32_t)((double)l32 * A.inv_range_walks);
                    int32_t rem = (int32_t)(l32 - q * rw);
                    if (rem < 0) { --q; rem += (int32_t)rw; }
                    else if (rem >= (int32_t)rw) { ++q; rem -= (int32_t)rw; }
                    pid = (uint64_t)A.range_point0 + q;
                    wid = pid * (uint64_t)A.walks_per_point + (uint64_t)A.range_offset + (uint64_t)rem;
                } else if (A.small32) {
                    const uint32_t local = A.base_off + (uint32_t)lid, w32 = (uint32_t)A.walks_per_point;
                    uint32_t q = (uint32_t)((double)local * A.inv_walks_per_point);
                    const int32_t rem = (int32_t)(local - q * w32);
                    if (rem < 0) --q;
                    else if (rem >= (int32_t)w32) ++q;
                    pid = (uint64_t)A.base_pid + q;
                    wid = (uint64_t)A.wid_begin + lid;
                } else {
                    wid = (uint64_t)A.wid_begin + lid;
                    pid = (uint64_t)((double)wid * A.inv_walks_per_point);
                    const int64_t rem = (int64_t)(wid - pid * (uint64_t)A.walks_per_point);
                    if (rem < 0) --pid;
                    else if (rem >= A.walks_per_point) ++pid;
                }
                pw = philox_walk(wid, A.key0, A.key1);
                if (WOST_PHILOX_AHEAD) rn_ahead = philox_draw(pw, 0u, A.key0, A.key1);
                const float2 q = A.points[pid];
                px = q.x; py = q.y;
                k = 0; dD = FIX ? WOST_INF : 1.0f; onB = false; phi = 0.f; w = 1.f;
#pragma unroll
                for (int s = 0; s < NS; ++s) total[s] = 0.f;
                if (DELTA) ax = A.point_alpha[pid];                // alpha(x0), precomputed per point
                active = true;
            }
            c_next += take;
            if (kAdaptive) {
                q_taken += take;
                WOST_KEEP_VGPR(q_taken);
            }
            need = __ballot(!active);
        }
        // the queue is exhausted: idle lanes take parked walks of either class, and the
        // wave ends only when both pools are empty (a wave parks walks only while the
        // queue is not exhausted for it, and drains the pools itself before it ends)
        if (pool != nullptr && exhausted && batch && __ballot(!active) != 0ull &&
            (!__any(active) || pool_count(pool, 0) + pool_count(pool, 1) > 0u)) {
            pool_lock(pool, lane);
            uint32_t cnt[2] = {pool_count(pool, 0), pool_count(pool, 1)};
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const uint64_t fr = __ballot(!active);
                const uint32_t npull = min((uint32_t)__popcll(fr), cnt[c]);
                const uint32_t rf = (uint32_t)__popcll(fr & lanes_below);
                if (!active && rf < npull) {
                    const uint32_t* const r =
                        pool + 4 + (size_t)c * pool_fields(NS) * A.pool_slots + (cnt[c] - npull) + rf;
                    const int P = A.pool_slots;
                    wid = (uint64_t)r[0 * P] | (uint64_t)r[1 * P] << 32;
                    lid = (uint64_t)r[2 * P] | (uint64_t)r[3 * P] << 32;
                    px = __builtin_bit_cast(float, r[4 * P]); py = __builtin_bit_cast(float, r[5 * P]);
                    dD = __builtin_bit_cast(float, r[6 * P]);
                    const uint32_t kb = r[7 * P];
                    k = (int)(kb & 0x7fffffffu); onB = (kb >> 31) != 0u;
                    phi = __builtin_bit_cast(float, r[8 * P]); w = __builtin_bit_cast(float, r[9 * P]);
                    ax = __builtin_bit_cast(float, r[10 * P]);
#pragma unroll
                    for (int s = 0; s < NS; ++s) total[s] = __builtin_bit_cast(float, r[(11 + s) * P]);
                    pw = philox_walk(wid, A.key0, A.key1);
                    if (WOST_PHILOX_AHEAD) rn_ahead = philox_draw(pw, (uint32_t)k, A.key0, A.key1);
                    active = true;
                }
                cnt[c] -= npull;
            }
            pool_unlock(pool, lane, cnt[0], cnt[1]);
        }
        if (!__any(active)) break;
        if (kWaveStats) {
            q_iters += 1u;
            WOST_KEEP_VGPR(q_iters);
        }
        // a freshly refilled walk may already fail the while-condition (eps >= 1,
        // maxSteps == 0): it takes no step and is finished at the next iteration
        bool stepping = active && (k < A.max_steps) && (dD > A.eps);
        // the cooperative tree queries need every lane of the wave: the others run the
        // step's pure arithmetic up to the ray query with them and leave after it
        if (kWaveTree ? !__any(stepping) : !stepping) continue;

        // --- one walk-step (:206-291)
#if defined(WOST_TREE_ITER_STATS)
        ic_arr[14] += 1u;
#endif
        WOST_PHASE("dirichlet_distance");
        float dd = fld.dirichlet_distance(dP, A.nd, px, py);        // :208
        if (WOST_ABL_DUP & 1) dd = dup_merge(dd, fld.dirichlet_distance(dP, A.nd, dup_opq(px), py));
        if (FIX && stepping && !(dd > A.eps)) {   // Q7/Q12 fixed: stop here, g at this point
            dD = dd;
            if (!kWaveTree) continue;
            stepping = false;   // (it only helps the wave's tree queries)
        }
        // the step's random words and direction (:226-232)
        U4 rn;
        float cs = 0.f, sn = 0.f;
        bool onB0 = false;                                           // the current point's, for FIX's
        float phi0 = 0.f;                                            // source direction
        auto draw_direction = [&]() {
#if defined(WOST_ABL_NO_PHILOX)   // ablation (timing only): a cheap hash
            const uint32_t hh = (pw.b ^ (uint32_t)k * 0x9E3779B9u) * 0x85EBCA6Bu;
            rn = U4{hh, hh * 0xC2B2AE35u, (hh ^ pw.d) * 0x27D4EB2Fu, hh ^ pw.c};
#else
            // the key enters each step opaque, so its round schedule (key + r * W) is
            // formed by scalar adds here instead of 16 loop-invariant SGPRs, which the
            // register allocator would otherwise spill to VGPR lanes (a v_readlane each)
            if (WOST_PHILOX_AHEAD) {
                rn = rn_ahead;                                       // drawn during the previous step
            } else {
                uint32_t key0 = A.key0, key1 = A.key1;
                WOST_OPAQUE_SGPR(key0);
                WOST_OPAQUE_SGPR(key1);
                rn = philox_draw(pw, (uint32_t)k, key0, key1);       // philox4x32_10({k, 0, wid})
                if (WOST_ABL_DUP & 2) {
                    const U4 r2 = philox_draw(pw, (uint32_t)k | dup_zero(), key0, key1);
                    rn.x |= (r2.x ^ r2.y ^ r2.z ^ r2.w) & dup_zero();
                }
            }
#endif
            float theta = (u01(rn.x) * 2.0f) * kPiF;                 // :226
            // :227-228 (quirk Q2): atan2(normal) is a property of the segment that
            // was hit, precomputed per segment on the host (the C library's atan2f)
            if (NEU && onB) theta = FIX ? theta / 2.0f + (phi - kPiF / 2.0f) : theta / 2.0f + phi;
            onB0 = onB;
            phi0 = phi;
            walk_sincos(theta, sn, cs, A.exact_trig != 0);           // :230-232
            if (WOST_ABL_DUP & 4) {
                float s2, c2;
                walk_sincos(dup_opq(theta), s2, c2, A.exact_trig != 0);
                sn = dup_merge(sn, s2);
                cs = dup_merge(cs, c2);
            }
        };
        float r;
        float dnv = WOST_NAN;                                        // recorder: None without Neumann
        // a long polyline's brute-force scans in one pass (neumann_scan_both): the direction
        // first, the ray query's finish after r
#if defined(WOST_ABL_NO_SILHOUETTE)   // (the ablation skips the fused scan, which draws the direction)
        constexpr bool kFused = false;
#else
        constexpr bool kFused = NEU && !TREE && !FIX && F::kFusedNeumann;
#endif
        ScanBoth sb{};
        WOST_PHASE("silhouette");
        if (NEU) {
#if defined(WOST_ABL_NO_SILHOUETTE)   // ablation (timing only)
            const float dn = WOST_INF;
#else
            float dn;
            if constexpr (kFused) {
                draw_direction();
                sb = fld.neumann_scan_both(nP, A.nn, px, py, cs, sn);
                dn = scan_both_silhouette(sb);                        // :211
            } else {
                dn = kWaveTree ? silhouette_distance_tree_wave(tree, px, py, dd, A.tree_stop2, stepping, tws, lane,
                                                               WOST_IC)
                     : TREE    ? silhouette_distance_tree(tree, px, py, dd, A.tree_stop2)
                               : fld.neumann_silhouette_distance(nP, A.nn, px, py);  // :211
            }
#endif
            dnv = dn;
            const float m = dn < dd ? dn : dd;                       // Python min()
            r = m > A.rmin ? m : A.rmin;                             // Python max() (:212)
        } else {
            r = dd > A.rmin ? dd : A.rmin;                           // :215
        }
        WOST_PHASE("philox_direction");
        if (!kFused) draw_direction();
#if !defined(WOST_ABL_NO_PHILOX)
        if (WOST_PHILOX_AHEAD) {   // the next step's words, overlapping this step's arithmetic
            uint32_t key0 = A.key0, key1 = A.key1;
            WOST_OPAQUE_SGPR(key0);
            WOST_OPAQUE_SGPR(key1);
            rn_ahead = philox_draw(pw, (uint32_t)(k + 1), key0, key1);
            if (WOST_PHILOX_AHEAD == 2) WOST_PIN_U4(rn_ahead);
        }
#endif

        float xnx, xny;
        WOST_PHASE("ray_query");
        if (NEU) {                                                   // :235-236
#if defined(WOST_ABL_NO_RAY)
            Hit h; h.x = px + r * cs; h.y = py + r * sn; h.hit = false; h.seg = -1;
#else
            Hit h = kFused    ? scan_both_finish(nP, sb, px, py, r)
                    : kWaveTree ? intersect_polylines_tree_wave<false, FIX>(tree, px, py, cs, sn, r, stepping, tws,
                                                                            lane, WOST_IC)
                    : FIX       ? fld.neumann_intersect_nearest(nP, A.nn, px, py, cs, sn, r)
                                : fld.neumann_intersect(nP, A.nn, px, py, cs, sn, r);
            if ((WOST_ABL_DUP & 8) && !kWaveTree && !FIX && !kFused) {
                const Hit h2 = fld.neumann_intersect(nP, A.nn, dup_opq(px), py, cs, sn, r);
                h.x = dup_merge(h.x, h2.x);
                h.y = dup_merge(h.y, h2.y);
                h.seg |= h2.seg & (int)dup_zero();
                h.hit = h.hit || (h2.hit && dup_zero() != 0u);
            }
#endif
            if (kWaveTree && !stepping) continue;   // the lanes that only helped
            xnx = h.x; xny = h.y; onB = h.hit;
            if (h.hit) phi = TREE ? A.seg_phi[h.seg] : fld.neumann_phi(phiP, h.seg);
            if (FIX && h.hit) {
                // inward normal: the left normal when the ray crossed the segment from
                // its left side, i.e. cross(d, u) > 0 (then dot(left normal, d) < 0)
                const float2* const sv = TREE ? A.nverts : nP;   // the tree kernels stage none
                const float2 a = sv[h.seg], b = sv[h.seg + 1];
                if (!(cs * (b.y - a.y) - sn * (b.x - a.x) > 0.0f)) phi = phi + kPiF;
            }
        } else {                                                     // :238-239
            xnx = px + r * cs;
            xny = py + r * sn;
        }

        float yx = xnx, yy = xny;
        float cv = 0.0f;                                             // recorder: source contribution
        bool clipped = false;
        float gnorm = 0.f;
        Jet aj{0.f, 0.f, 0.f, 0.f};
        WOST_PHASE("sample_and_clip");
        if (SRC) {                                                   // :242-258
            float rs;
            if constexpr (FIX && DELTA)                              // Q4/Q5 fixed: this ball's law
                rs = sample_rho_screened_fixed(A.table + kFixTableOffset, u01(rn.y), r * sqrt_sb) * r;
            else
                rs = sample_rho_tail(sT, node0, u01(rn.y)) * r;      // :244 (sampler, quirks Q3-Q5)
            if (WOST_ABL_DUP & 16) rs = dup_merge(rs, sample_rho_tail(sT, node0, u01(rn.y | dup_zero())) * r);
            if constexpr (FIX && !DELTA) {                           // Q13 fixed: own direction
                float ts = (u01(rn.w) * 2.0f) * kPiF;
                if (NEU && onB0) ts = ts / 2.0f + (phi0 - kPiF / 2.0f);   // the inward hemisphere
                float cs2, sn2;
                walk_sincos(ts, sn2, cs2, A.exact_trig != 0);
                yx = px + rs * cs2;
                yy = py + rs * sn2;
                if (NEU)   // not visible
                    clipped = TREE ? intersect_polylines_tree<false, true>(tree, px, py, cs2, sn2, rs).hit
                                   : fld.neumann_intersect_nearest(nP, A.nn, px, py, cs2, sn2, rs).hit;
            } else {
                // :245 (quirk Q13). FIX delta keeps the sample on the step's ray: with the
                // nearest crossing (Q1) the clip below is exactly "y is in the star-shaped
                // region", and a collision is taken only there, so it lands at a radius
                // drawn from the Green's law truncated at the ray's boundary point
                yx = px + rs * cs;
                yy = py + rs * sn;
                const float e1x = yx - px, e1y = yy - py;
                const float e2x = xnx - px, e2y = xny - py;
                // :248 compares the two norms. sqrt is monotone, so sqrt(a2) > sqrt(b2)
                // needs a2 > b2 (rare: only Neumann hits make the next point closer);
                // only then evaluate the reference's exact comparison.
                const float a2 = e1x * e1x + e1y * e1y, b2 = e2x * e2x + e2y * e2y;
                if (WOST_PHILOX_AHEAD == 3) WOST_PIN_U4(rn_ahead);
                // a real branch (the compiler otherwise evaluates both correctly rounded
                // square roots for every lane and selects, ~35 instructions per step)
                if (WOST_ANY(a2 > b2)) {
                    WOST_NO_SPECULATION();
                    if (a2 > b2) clipped = sqrtf(a2) > sqrtf(b2);
                }
                if (clipped) { yx = xnx; yy = xny; }
            }
            if (DELTA) {
                WOST_PHASE("greens_norm");
                gnorm = greens_norm_from_table(sG, r * sqrt_sb, r, inv_sb);   // solvers/utils.py:29-44
                if (WOST_ABL_DUP & 32) gnorm = dup_merge(gnorm, greens_norm_from_table(sG, dup_opq(r) * sqrt_sb, r, inv_sb));
                WOST_PHASE("alpha_jet");
                aj = fld.alpha_jet(yx, yy);
                if (WOST_ABL_DUP & 64) {
                    const Jet a2 = fld.alpha_jet(dup_opq(yx), yy);
                    aj.v = dup_merge(aj.v, a2.v);
                    aj.gx = dup_merge(aj.gx, a2.gx);
                    aj.gy = dup_merge(aj.gy, a2.gy);
                    aj.lap = dup_merge(aj.lap, a2.lap);
                }
            }
            WOST_PHASE("source_contribution");
            if constexpr (NS == 1) {
                float c = 0.0f;
                if (!clipped) {
                    float f = fld.f(yx, yy);
                    if (WOST_ABL_DUP & 256) f = dup_merge(f, fld.f(dup_opq(yx), yy));
                    if (DELTA)
                        c = (f * gnorm) * f_rsq(aj.v * ax) * w;  // :253-254
                    else
                        c = f * ((r * r) / 4.0f);                        // :256, utils.py:61
                }
                total[0] = total[0] + c;                                 // :258
                cv = c;
            } else if (!clipped) {                                       // the same per source
                float fv[NS];
                fld.f_multi(yx, yy, fv);
                const float sa = DELTA ? f_rsq(aj.v * ax) : 0.0f;
                const float q = DELTA ? 0.0f : ((r * r) / 4.0f);
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const float c = DELTA ? ((fv[s] * gnorm) * sa * w) : fv[s] * q;
                    total[s] = total[s] + c;
                }
            } else {
#pragma unroll
                for (int s = 0; s < NS; ++s) total[s] = total[s] + 0.0f;
            }
        }
        if (REC && A.rec != nullptr) {                               // :218-222, :261-266
            // the tree's silhouette distance is exact only below dD: recompute it
            if (TREE) dnv = silhouette_distance_tree(tree, px, py, WOST_INF);
            const int64_t li = (int64_t)lid;
            float4* rr = reinterpret_cast<float4*>(A.rec + ((size_t)li * (size_t)A.rec_stride + (size_t)k) * kRecFloats);
            rr[0] = float4{px, py, dd, dnv};
            rr[1] = float4{yx, yy, cv, SRC ? 1.0f : 0.0f};
        }

        WOST_PHASE("delta_update");
        if (DELTA && FIX) {
            const float mu = u01(rn.z);
            // collision: mu <= sigma_bar |G| and the sample before the ray's boundary point
            const bool collide = !(mu > sigma_bar * gnorm) && !clipped;
            float anew = aj.v;                                       // a collision, or a clipped sample (y = z)
            if (!collide && !clipped) anew = fld.alpha(xnx, xny);
            float sc = 1.0f;
            if (collide) sc = 1.0f - sigma_prime_from(aj, fld.sigma(yx, yy), fld.detached()) * inv_sb;
            const float wt = w * f_sqrt(f_div(anew, ax));
            w = collide ? wt * sc : wt;
            px = collide ? yx : xnx;
            py = collide ? yy : xny;
            onB = collide ? false : onB;                             // a collision point is interior
            ax = anew;
        } else if (DELTA) {                                          // :271-284
            const float mu = u01(rn.z);
            const bool accept = mu > sigma_bar * gnorm;              // :273-275
            // the two branches share the weight update w * sqrt(a_new / alpha(x));
            // only the field evaluations stay divergent
            float anew = aj.v;                                       // collision, or a clipped accept
#if !defined(WOST_ABL_NO_ALPHA_Z)
            if (accept && !clipped) {
                anew = fld.alpha(xnx, xny);                          // :277
                if (WOST_ABL_DUP & 128) anew = dup_merge(anew, fld.alpha(dup_opq(xnx), xny));
            }
#endif
            float sc = 1.0f;
#if defined(WOST_ABL_NO_SIGMA_PRIME)
            if (false) {
#else
            if (!accept) {
#endif
                float spv = sigma_prime_from(aj, fld.sigma(yx, yy), fld.detached());  // :281
                if (WOST_ABL_DUP & 512)
                    spv = dup_merge(spv, sigma_prime_from(Jet{dup_opq(aj.v), aj.gx, aj.gy, aj.lap},
                                                          fld.sigma(dup_opq(yx), yy), fld.detached()));
                sc = 1.0f - spv * inv_sb;
                sc = (0.0f > sc) ? 0.0f : sc;                        // Python max(., 0.0) (:282)
            }
            const float wt = w * f_sqrt(f_div(anew, ax));           // :277 / :283
            w = accept ? wt : wt * sc;
            px = accept ? xnx : yx;
            py = accept ? xny : yy;
            ax = anew;
        } else {
            px = xnx; py = xny;                                      // :287
        }
        k += 1;                                                      // :291
        dD = dd;   // the loop tests the distance of the pre-step point (quirk Q7)
        WOST_PHASE("loop_head");
    }
    if (kWaveStats) {   // the wave's longest walk (every lane is here)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t other = (uint32_t)__shfl_xor((int)my_kmax, o);
            my_kmax = other > my_kmax ? other : my_kmax;
        }
    }
    if (kWaveStats && lane == 0) {   // the launch statistics (wost_block_reduce sums them up)
        uint4* const wave_stats = reinterpret_cast<uint4*>(A.counter + kCtlWords);
        const uint64_t wv = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        const uint64_t end = wall_ticks64();
        const uint32_t dur = (uint32_t)end - q_t0;
        const uint64_t start = end - dur;                   // the start's high word, from the end's
        wave_stats[2 * wv] = uint4{(uint32_t)start, (uint32_t)(start >> 32), q_tdeq - q_t0, dur};
        wave_stats[2 * wv + 1] = uint4{q_iters, my_kmax, 0u, 0u};
    }
#if defined(WOST_TREE_ITER_STATS)
    // each lane's counters into the workgroup's study words after its pools (the host
    // sizes A.pool for them when WOST_TREE_ITER_STATS is set)
    if (pool != nullptr) {
        uint32_t* const st = pool + 4 + 2 * (size_t)pool_fields(NS) * A.pool_slots;
#pragma unroll
        for (int i = 0; i < 16; ++i) atomicAdd(st + i, ic_arr[i]);
    }
#endif
#undef WOST_IC
}

}  // namespace wost
