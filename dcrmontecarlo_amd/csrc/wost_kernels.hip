// wost_kernels.hip -- precompiled gfx950 kernels of the Walk-on-Stars hot path.
//
// wost_walk_kernel<NEU,SRC,DELTA,TREE>: the walk loop of wost_walk.h with the
// coefficient fields interpreted from a program buffer read through the
// constant address space with uniform indices (scalar loads). wost_jit.cpp
// builds the same loop with the fields compiled in.
// Per-walk results go to HBM; wost_block_reduce then sums them per block of
// WOST_BLOCK_WALKS walks in a fixed order (deterministic, GPU-count
// independent).
#include "wost_device.h"
#include "wost_internal.h"

namespace wost {

#if defined(__HIP_DEVICE_COMPILE__)
#define WOST_AS_CONST __attribute__((address_space(4)))
#else
#define WOST_AS_CONST
#endif

template <class T>
using cptr = const WOST_AS_CONST T*;

// Constant-address-space views of the program buffer. Members are read one
// by one (a reference cannot bind across address spaces); with a uniform
// index each read is an s_load.
struct TermsC {
    cptr<DTerm> p;
    __device__ __forceinline__ DTerm operator[](int i) const {
        DTerm t;
        t.coef = p[i].coef;
        t.first = p[i].first;
        t.nf = p[i].nf;
        t.pad = 0;
        return t;
    }
};
struct FactorsC {
    cptr<DFactor> p;
    __device__ __forceinline__ DFactor operator[](int i) const {
        DFactor f;
        f.kind = p[i].kind;
#pragma unroll
        for (int k = 0; k < 8; ++k) f.p[k] = p[i].p[k];
        return f;
    }
};
struct FloatsC {
    cptr<float> p;
    __device__ __forceinline__ float operator[](int i) const { return p[i]; }
};

struct ProgView {
    cptr<DProgram> hdr;
    TermsC terms;
    FactorsC factors;
    const float* grid;   // tabulated values: per-lane gathers, so a plain global pointer
    __device__ __forceinline__ explicit ProgView(const char* prog) {
        hdr = (cptr<DProgram>)prog;
        terms.p = (cptr<DTerm>)(prog + sizeof(DProgram));
        factors.p = (cptr<DFactor>)(prog + sizeof(DProgram) + sizeof(DTerm) * hdr->n_terms_total);
        grid = reinterpret_cast<const float*>(prog + program_grid_offset(hdr->n_terms_total, hdr->n_factors_total));
    }
    __device__ __forceinline__ DField field(int slot) const {
        DField f;
        f.n_terms = hdr->field[slot].n_terms;
        f.first_term = hdr->field[slot].first_term;
        f.flags = hdr->field[slot].flags;
        f.present = hdr->field[slot].present;
        return f;
    }
    __device__ __forceinline__ float value(const DField& f, float x, float y) const {
        return field_value(f, terms, factors, grid, x, y);
    }
    __device__ __forceinline__ Jet jet(const DField& f, float x, float y) const {
        return field_jet(f, terms, factors, grid, x, y);
    }
};

// Fields read from the program buffer (the precompiled, interpreted path).
struct InterpFields {
    static constexpr bool kConstDirichlet = false;   // polylines are staged in LDS
    static constexpr bool kConstNeumann = false;
    static constexpr bool kFusedNeumann = false;      // (the field-specialised kernels' long-polyline scan)
    ProgView P;
    DField fG, fF, fS, fA;
    bool det;
    float sb, sqsb, isb;
    __device__ __forceinline__ explicit InterpFields(const char* prog) : P(prog) {
        fG = P.field(SLOT_G);
        fF = P.field(SLOT_F);
        fS = P.field(SLOT_SIGMA);
        fA = P.field(SLOT_ALPHA);
        det = (fA.flags & WOST_FIELD_DETACHED) != 0;
        sb = P.hdr->sigma_bar;
        sqsb = P.hdr->sqrt_sigma_bar;
        isb = P.hdr->inv_sigma_bar;
    }
    __device__ __forceinline__ bool has_g() const { return fG.present != 0; }
    __device__ __forceinline__ float g(float x, float y) const { return P.value(fG, x, y); }
    __device__ __forceinline__ float f(float x, float y) const { return P.value(fF, x, y); }
    __device__ __forceinline__ float sigma(float x, float y) const { return fS.present ? P.value(fS, x, y) : 0.0f; }
    __device__ __forceinline__ float alpha(float x, float y) const { return P.value(fA, x, y); }
    __device__ __forceinline__ Jet alpha_jet(float x, float y) const { return P.jet(fA, x, y); }
    __device__ __forceinline__ bool detached() const { return det; }
    __device__ __forceinline__ float sigma_bar() const { return sb; }
    __device__ __forceinline__ float sqrt_sigma_bar() const { return sqsb; }
    __device__ __forceinline__ float inv_sigma_bar() const { return isb; }
    __device__ __forceinline__ float dirichlet_distance(const float2* sD, int nd, float x, float y) const {
        return poly_distance(sD, nd, x, y);
    }
    __device__ __forceinline__ float neumann_silhouette_distance(const float2* sN, int nn, float x, float y) const {
        return silhouette_distance(sN, nn, x, y);
    }
    __device__ __forceinline__ Hit neumann_intersect(const float2* sN, int nn, float x, float y, float dx, float dy,
                                                     float r) const {
        return intersect_polylines<false>(sN, nn, x, y, dx, dy, r);
    }
    __device__ __forceinline__ Hit neumann_intersect_nearest(const float2* sN, int nn, float x, float y, float dx,
                                                             float dy, float r) const {
        return intersect_polylines_ray(sN, nn, x, y, dx, dy, r);
    }
    __device__ __forceinline__ float neumann_phi(const float* sPhi, int seg) const { return sPhi[seg]; }
};

#ifndef WOST_WALK_MIN_WAVES
#define WOST_WALK_MIN_WAVES 6   // 6 waves/SIMD: measured best (tools/ab_bench.sh)
#endif

// One walk-step of _solveUnified (solvers/WoStSolver.py:206-291) for every
// active lane, with the finish/refill logic of loops 1-2 (:182-188, :294-311)
// around it: see wost_walk.h.
template <bool NEU, bool SRC, bool DELTA, bool TREE, bool FIX>
__global__ void __launch_bounds__(kWalkBlock, WOST_WALK_MIN_WAVES)
wost_walk_kernel(const WalkArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const InterpFields fld(A.prog);
    walk_body<NEU, SRC, DELTA, TREE, true, 1, FIX>(A, fld, smem);   // records when A.rec is set
}

// alpha at the query points (WalkArgs::point_alpha) with the interpreted fields
__global__ void __launch_bounds__(256) wost_point_alpha_kernel(const char* prog, const float2* pts, int64_t n,
                                                               float* out) {
    const InterpFields fld(prog);
    point_alpha_body(pts, n, out, fld);
}

hipError_t launch_point_alpha(const char* prog, const float2* pts, int64_t n, float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
    wost_point_alpha_kernel<<<grid, 256, 0, s>>>(prog, pts, n, out);
    return hipGetLastError();
}

// mode -> kernel instantiation (MODE_* of wost_internal.h)
#define WOST_FOR_MODE(mode, X)                                   \
    switch (mode) {                                              \
    case MODE_DIRICHLET: X(false, false, false, false, false);        \
    case MODE_POISSON: X(false, true, false, false, false);           \
    case MODE_MIXED: X(true, false, false, false, false);             \
    case MODE_MIXED_POISSON: X(true, true, false, false, false);      \
    case MODE_DELTA: X(false, true, true, false, false);              \
    case MODE_MIXED_DELTA: X(true, true, true, false, false);         \
    case MODE_MIXED_TREE: X(true, false, false, true, false);         \
    case MODE_MIXED_POISSON_TREE: X(true, true, false, true, false);  \
    case MODE_MIXED_DELTA_TREE: X(true, true, true, true, false);     \
    case MODE_FIX_DIRICHLET: X(false, false, false, false, true);     \
    case MODE_FIX_POISSON: X(false, true, false, false, true);        \
    case MODE_FIX_MIXED: X(true, false, false, false, true);          \
    case MODE_FIX_MIXED_POISSON: X(true, true, false, false, true);   \
    case MODE_FIX_DELTA: X(false, true, true, false, true);           \
    case MODE_FIX_MIXED_DELTA: X(true, true, true, false, true);      \
    case MODE_FIX_MIXED_TREE: X(true, false, false, true, true);      \
    case MODE_FIX_MIXED_POISSON_TREE: X(true, true, false, true, true); \
    case MODE_FIX_MIXED_DELTA_TREE: X(true, true, true, true, true);  \
    default: return hipErrorInvalidValue;                        \
    }

hipError_t walk_occupancy(int mode, int nd, int nn, int n_points, int* blocks_per_cu) {
    (void)n_points;
    const size_t lds = walk_lds_bytes(mode, nd, nn, n_points);
#define OCC(n, s, d, t, x) \
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<n, s, d, t, x>, kWalkBlock, lds)
    WOST_FOR_MODE(mode, OCC)
#undef OCC
}

hipError_t launch_walk(int mode, const WalkArgs& a, int grid, hipStream_t s) {
    const size_t lds = walk_lds_bytes(mode, a.nd, a.nn, a.n_points);
#define LAUNCH(n, sr, d, t, x)                                       \
    wost_walk_kernel<n, sr, d, t, x><<<grid, kWalkBlock, lds, s>>>(a); \
    return hipGetLastError()
    WOST_FOR_MODE(mode, LAUNCH)
#undef LAUNCH
}

// ---------------------------------------------------------------------------
// Deterministic per-block sums (sum, sum of squares, steps) in float64. The
// thread -> walk assignment and the LDS tree are fixed, so the bits depend
// only on the walk values.
// ---------------------------------------------------------------------------
constexpr int kReduceBlock = 256;

// The walk launch's statistics (the per-wave records after the control words, wost_walk.h
// kCtlWords) summed up by one workgroup: lstats[0] earliest wave start, [1] latest dequeue,
// [2] latest wave end (wall-clock ticks), [3] the longest walk, [4] loop iterations of the
// wave that ended last and [5] its duration, [6] the most iterations of any wave, [7] waves.
// A later launch of the same solve combines with the earlier ones' values ([0] the first
// start, [1]/[2]/[4]/[5] the last launch's, [3]/[6] the maximum).
__device__ void reduce_wave_stats(const uint4* __restrict__ ws, int64_t n_waves, unsigned long long* lstats,
                                  int first_batch) {
    __shared__ unsigned long long s_start[kReduceBlock], s_deq[kReduceBlock], s_end[kReduceBlock];
    __shared__ uint32_t s_it[kReduceBlock], s_dur[kReduceBlock], s_itmax[kReduceBlock], s_kmax[kReduceBlock];
    unsigned long long st = ~0ull, dq = 0ull, en = 0ull;
    uint32_t it = 0u, dur = 0u, itmax = 0u, kmax = 0u;
    for (int64_t i = threadIdx.x; i < n_waves; i += kReduceBlock) {
        const uint4 a = ws[2 * i], b = ws[2 * i + 1];
        const unsigned long long t0 = (unsigned long long)a.y << 32 | a.x;
        st = t0 < st ? t0 : st;
        dq = t0 + a.z > dq ? t0 + a.z : dq;
        if (t0 + a.w >= en) {
            en = t0 + a.w;
            it = b.x;
            dur = a.w;
        }
        itmax = b.x > itmax ? b.x : itmax;
        kmax = b.y > kmax ? b.y : kmax;
    }
    s_start[threadIdx.x] = st; s_deq[threadIdx.x] = dq; s_end[threadIdx.x] = en;
    s_it[threadIdx.x] = it; s_dur[threadIdx.x] = dur; s_itmax[threadIdx.x] = itmax; s_kmax[threadIdx.x] = kmax;
    __syncthreads();
    for (int h = kReduceBlock / 2; h > 0; h >>= 1) {
        const int t = (int)threadIdx.x;
        if (t < h) {
            s_start[t] = s_start[t + h] < s_start[t] ? s_start[t + h] : s_start[t];
            s_deq[t] = s_deq[t + h] > s_deq[t] ? s_deq[t + h] : s_deq[t];
            if (s_end[t + h] > s_end[t]) {
                s_end[t] = s_end[t + h];
                s_it[t] = s_it[t + h];
                s_dur[t] = s_dur[t + h];
            }
            s_itmax[t] = s_itmax[t + h] > s_itmax[t] ? s_itmax[t + h] : s_itmax[t];
            s_kmax[t] = s_kmax[t + h] > s_kmax[t] ? s_kmax[t + h] : s_kmax[t];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        unsigned long long start = s_start[0], itm = s_itmax[0], km = s_kmax[0];
        if (!first_batch) {
            start = lstats[0] < start ? lstats[0] : start;
            itm = lstats[6] > itm ? lstats[6] : itm;
            km = lstats[3] > km ? lstats[3] : km;
        }
        lstats[3] = km;
        lstats[0] = start;
        lstats[1] = s_deq[0];
        lstats[2] = s_end[0];
        lstats[4] = s_it[0];
        lstats[5] = s_dur[0];
        lstats[6] = itm;
        lstats[7] = (unsigned long long)n_waves;
    }
    __syncthreads();
}

// ns values per walk (multi-source solves): for each its sum and sum of
// squares, then the steps -- rows of 2*ns+1 doubles. The summation order is
// the same for every ns, so source k's sums do not depend on the other sources.
// ctl (may be null): the walk launch's control words (wost_walk.h kCtlWords): workgroup 0
// resets the queue head for the next launch and, with lstats, sums up the n_waves
// launch statistics into lstats (the longest walk among them). Without wave records
// (n_waves = 0: the segment-tree kernels) every workgroup adds its longest walk to ctl[2]
// (atomicMax, skipped when not above the value already there), and the last one to finish
// moves it to lstats[3] and resets ctl[1..2]. (With per-workgroup atomics on every launch
// C4's 11,760-workgroup reduce took 0.40 ms instead of 0.09: profiles/r06_ab/r06s5.)
__global__ void __launch_bounds__(kReduceBlock)
wost_block_reduce(const float* __restrict__ val, const uint32_t* __restrict__ steps,
                  const int64_t* __restrict__ begin, int64_t nblocks, int ns, double* __restrict__ out,
                  unsigned long long* ctl, int64_t n_waves, unsigned long long* lstats, int first_batch) {
    __shared__ double s_sum[kReduceBlock], s_sq[kReduceBlock], s_st[kReduceBlock];
    __shared__ uint32_t s_mx[kReduceBlock];
    __shared__ int s_last;
    const int row = 2 * ns + 1;
    if (ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) ctl[0] = 0ull;   // (a vector store)
    // the waves' records (scan kernels): reduced by one extra workgroup, the last, beside the
    // block sums (C2: its 4,096 records held up workgroup 0's sums); the segment-tree kernels
    // keep none (n_waves 0: workgroup 0 writes their empty statistics)
    const bool stats_wg = ctl != nullptr && lstats != nullptr && n_waves > 0;
    const int64_t nred = (int64_t)gridDim.x - (stats_wg ? 1 : 0);   // workgroups that sum blocks
    if (stats_wg && (int64_t)blockIdx.x == nred) {
        reduce_wave_stats(reinterpret_cast<const uint4*>(ctl + kCtlWords), n_waves, lstats, first_batch);
        return;
    }
    if (!stats_wg && ctl != nullptr && lstats != nullptr && blockIdx.x == 0)
        reduce_wave_stats(reinterpret_cast<const uint4*>(ctl + kCtlWords), n_waves, lstats, first_batch);
    uint32_t mx_all = 0u;
    for (int64_t b = blockIdx.x; b < nblocks; b += nred) {
        const int64_t lo = begin[b], hi = begin[b + 1];
        for (int k = 0; k < ns; ++k) {
            double s = 0.0, q = 0.0;
            uint64_t st = 0;
            for (int64_t i = lo + threadIdx.x; i < hi; i += kReduceBlock) {
                const double v = (double)val[i * ns + k];
                s += v;
                q += v * v;
                if (k == 0) {
                    const uint32_t si = steps[i];
                    st += si;
                    mx_all = si > mx_all ? si : mx_all;
                }
            }
            s_sum[threadIdx.x] = s;
            s_sq[threadIdx.x] = q;
            s_st[threadIdx.x] = (double)st;
            __syncthreads();
            for (int h = kReduceBlock / 2; h > 0; h >>= 1) {
                if ((int)threadIdx.x < h) {
                    s_sum[threadIdx.x] += s_sum[threadIdx.x + h];
                    s_sq[threadIdx.x] += s_sq[threadIdx.x + h];
                    if (k == 0) s_st[threadIdx.x] += s_st[threadIdx.x + h];
                }
                __syncthreads();
            }
            if (threadIdx.x == 0) {
                out[row * b + 2 * k] = s_sum[0];
                out[row * b + 2 * k + 1] = s_sq[0];
                if (k == 0) out[row * b + row - 1] = s_st[0];
            }
            __syncthreads();
        }
    }
    if (ctl == nullptr || lstats == nullptr || n_waves > 0) return;
    // the longest walk: one atomic per workgroup, then the last workgroup to finish moves it
    s_mx[threadIdx.x] = mx_all;
    __syncthreads();
    for (int h = kReduceBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h && s_mx[threadIdx.x + h] > s_mx[threadIdx.x]) s_mx[threadIdx.x] = s_mx[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if ((unsigned long long)s_mx[0] > *(volatile unsigned long long*)(ctl + 2))
            atomicMax(ctl + 2, (unsigned long long)s_mx[0]);
        __threadfence();
        s_last = atomicAdd(ctl + 1, 1ull) == (unsigned long long)gridDim.x - 1ull;
    }
    __syncthreads();
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        const unsigned long long mx = atomicAdd(ctl + 2, 0ull);
        lstats[3] = first_batch ? mx : (lstats[3] > mx ? lstats[3] : mx);
        ctl[1] = 0ull;
        ctl[2] = 0ull;
    }
}

hipError_t launch_block_reduce(const float* val, const uint32_t* steps, const int64_t* begin,
                               int64_t nblocks, int ns, double* out, unsigned long long* ctl,
                               hipStream_t s, int64_t n_waves, unsigned long long* lstats, int first_batch) {
    if (nblocks <= 0) return ctl ? hipMemsetAsync(ctl, 0, sizeof(unsigned long long) * kCtlWords, s) : hipSuccess;
    // (one more workgroup for the waves' records: wost_block_reduce)
    const int grid = (int)(nblocks < 65536 ? nblocks : 65536) + ((ctl && lstats && n_waves > 0) ? 1 : 0);
    wost_block_reduce<<<grid, kReduceBlock, 0, s>>>(val, steps, begin, nblocks, ns, out, ctl, n_waves, lstats,
                                                    first_batch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Batched polyline queries (geometry/PolylinesSimple.py:214-307), one query
// per thread, vertices read from global memory.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
wost_geometry_query_kernel(int op, const float2* __restrict__ verts, int nv,
                           const float2* __restrict__ pts, const float2* __restrict__ dirs,
                           const float* __restrict__ radii, int64_t n,
                           float* __restrict__ out_f, uint8_t* __restrict__ out_mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 p = pts[i];
    switch (op) {
    case WOST_GEOM_DISTANCE:
        out_f[i] = poly_distance(verts, nv, p.x, p.y);
        break;
    case WOST_GEOM_IS_SILHOUETTE:
        for (int j = 1; j + 1 < nv; ++j)
            out_mask[i * (int64_t)(nv - 2) + (j - 1)] =
                is_silhouette(verts[j - 1], verts[j], verts[j + 1], p.x, p.y) ? 1 : 0;
        break;
    case WOST_GEOM_SILHOUETTE_DISTANCE:
        out_f[i] = silhouette_distance(verts, nv, p.x, p.y);
        break;
    case WOST_GEOM_RAY_INTERSECTION: {
        const float2 d = dirs[i];
        for (int j = 0; j + 1 < nv; ++j)
            out_f[i * (int64_t)(nv - 1) + j] = ray_segment_time(verts[j], verts[j + 1], p.x, p.y, d.x, d.y);
        break;
    }
    case WOST_GEOM_INTERSECT_POLYLINES: {
        const float2 d = dirs[i];
        const Hit h = intersect_polylines(verts, nv, p.x, p.y, d.x, d.y, radii[i]);
        out_f[5 * i + 0] = h.x;
        out_f[5 * i + 1] = h.y;
        out_f[5 * i + 2] = h.nx;
        out_f[5 * i + 3] = h.ny;
        out_f[5 * i + 4] = h.hit ? 1.f : 0.f;
        break;
    }
    default:
        break;
    }
}

hipError_t launch_geometry_query(int op, const float2* verts, int nv, const float2* pts,
                                 const float2* dirs, const float* radii, int64_t n,
                                 float* out_f, uint8_t* out_mask, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t grid = (n + 255) / 256;
    wost_geometry_query_kernel<<<(unsigned)grid, 256, 0, s>>>(op, verts, nv, pts, dirs, radii, n, out_f, out_mask);
    return hipGetLastError();
}

// The same queries answered by the Neumann segment tree of the walk kernels, one
// query per lane (silhouette_distance_tree without a Dirichlet bound: exact;
// intersect_polylines_tree, reference mode): wost_geometry_query(op | WOST_GEOM_TREE).
__global__ void __launch_bounds__(256)
wost_geometry_tree_kernel(int op, SegTree t, const float2* __restrict__ pts, const float2* __restrict__ dirs,
                          const float* __restrict__ radii, int64_t n, float* __restrict__ out_f) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 p = pts[i];
    if (op == WOST_GEOM_SILHOUETTE_DISTANCE) {
        out_f[i] = silhouette_distance_tree(t, p.x, p.y, WOST_INF);
    } else {
        const float2 d = dirs[i];
        const Hit h = intersect_polylines_tree(t, p.x, p.y, d.x, d.y, radii[i]);
        out_f[5 * i + 0] = h.x;
        out_f[5 * i + 1] = h.y;
        out_f[5 * i + 2] = h.nx;
        out_f[5 * i + 3] = h.ny;
        out_f[5 * i + 4] = h.hit ? 1.f : 0.f;
    }
}

hipError_t launch_geometry_tree_query(int op, const float2* verts, int nv, const float4* rec, int first_leaf,
                                      int depth, int leaf, float tol, float kmax, const float2* pts,
                                      const float2* dirs, const float* radii, int64_t n, float* out_f,
                                      hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (op != WOST_GEOM_SILHOUETTE_DISTANCE && op != WOST_GEOM_INTERSECT_POLYLINES) return hipErrorInvalidValue;
    SegTree t{rec, verts, nv, first_leaf, depth, leaf, tol, kmax};
    const int64_t grid = (n + 255) / 256;
    wost_geometry_tree_kernel<<<(unsigned)grid, 256, 0, s>>>(op, t, pts, dirs, radii, n, out_f);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Field evaluation at points: value + gradient + Laplacian, or sigma'.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
wost_eval_field_kernel(const char* prog, int which, const float2* __restrict__ pts, int64_t n,
                       float4* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ProgView P(prog);
    const float2 p = pts[i];
    if (which < N_SLOTS) {
        const DField f = P.field(which);
        const Jet j = P.jet(f, p.x, p.y);
        out[i] = make_float4(j.v, j.gx, j.gy, j.lap);
    } else {
        const DField fa = P.field(SLOT_ALPHA);
        const DField fs = P.field(SLOT_SIGMA);
        const Jet aj = P.jet(fa, p.x, p.y);
        const float sg = fs.present ? P.value(fs, p.x, p.y) : 0.f;
        const float sp = sigma_prime_from(aj, sg, (fa.flags & WOST_FIELD_DETACHED) != 0);
        out[i] = make_float4(sp, aj.v, sg, 0.f);
    }
}

hipError_t launch_eval_field(const char* prog, int which, const float2* pts, int64_t n,
                             float4* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t grid = (n + 255) / 256;
    wost_eval_field_kernel<<<(unsigned)grid, 256, 0, s>>>(prog, which, pts, n, out);
    return hipGetLastError();
}

}  // namespace wost
