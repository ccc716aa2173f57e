// wost_kernels.hip -- gfx950 kernels of the Walk-on-Stars hot path.
//
// wost_walk_kernel restates the per-walk loop of WostSolver_2D._solveUnified
// (reference: solvers/WoStSolver.py:182-311) as one walk per lane:
//  * persistent waves, each lane holding one walk's state in registers;
//  * when walks finish, the wave re-fills those lanes by __ballot /
//    __popcll rank from a chunk of walk ids it dequeued with one atomic
//    (active-mask compaction, so short walks never idle a lane for long);
//  * polyline vertices and the sampler's inverse-CDF table staged in LDS
//    (wave-uniform segment loops read them as LDS broadcasts);
//  * coefficient-field programs read through the constant address space
//    with uniform indices (scalar loads);
//  * Philox4x32-10 counters derived from (seed, walk id, step), no RNG state
//    in memory.
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
    __device__ __forceinline__ explicit ProgView(const char* prog) {
        hdr = (cptr<DProgram>)prog;
        terms.p = (cptr<DTerm>)(prog + sizeof(DProgram));
        factors.p = (cptr<DFactor>)(prog + sizeof(DProgram) + sizeof(DTerm) * hdr->n_terms_total);
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
        return field_value(f, terms, factors, x, y);
    }
    __device__ __forceinline__ Jet jet(const DField& f, float x, float y) const {
        return field_jet(f, terms, factors, x, y);
    }
};

constexpr size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

size_t walk_lds_bytes(int mode, int nd, int nn, int n_points) {
    bool neu = mode == MODE_MIXED || mode == MODE_MIXED_POISSON || mode == MODE_MIXED_DELTA;
    bool src = mode == MODE_POISSON || mode == MODE_MIXED_POISSON || mode == MODE_DELTA ||
               mode == MODE_MIXED_DELTA;
    size_t b = align16(sizeof(float2) * (size_t)nd);
    if (neu) b += align16(sizeof(float2) * (size_t)nn);
    if (src) b += align16(sizeof(float) * WOST_SAMPLER_TABLE_N);
    if (n_points <= kLdsPointsMax) b += align16(sizeof(float2) * (size_t)n_points);
    return b;
}

// One walk-step of _solveUnified (solvers/WoStSolver.py:206-291) for every
// active lane, with the finish/refill logic of loops 1-2 (:182-188, :294-311)
// around it.
#ifndef WOST_WALK_MIN_WAVES
#define WOST_WALK_MIN_WAVES 6   // 6 waves/SIMD: measured best (tools/ab_bench.sh)
#endif
template <bool NEU, bool SRC, bool DELTA>
__global__ void __launch_bounds__(kWalkBlock, WOST_WALK_MIN_WAVES)
wost_walk_kernel(const WalkArgs A) {
    // the walk's position updates round op by op like the reference (torch CPU
    // has no FMA contraction); the field math it calls keeps FMAs
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* sD = reinterpret_cast<float2*>(smem);
    float2* sN = reinterpret_cast<float2*>(smem + align16(sizeof(float2) * (size_t)A.nd));
    float* sT = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(sN) +
                                         (NEU ? align16(sizeof(float2) * (size_t)A.nn) : 0));
    float2* sP = reinterpret_cast<float2*>(reinterpret_cast<unsigned char*>(sT) +
                                           (SRC ? align16(sizeof(float) * WOST_SAMPLER_TABLE_N) : 0));
    const bool points_in_lds = A.n_points <= kLdsPointsMax;

    for (int i = threadIdx.x; i < A.nd; i += blockDim.x) sD[i] = A.dverts[i];
    if (NEU)
        for (int i = threadIdx.x; i < A.nn; i += blockDim.x) sN[i] = A.nverts[i];
    if (SRC)
        for (int i = threadIdx.x; i < WOST_SAMPLER_TABLE_N; i += blockDim.x) sT[i] = A.table[i];
    if (points_in_lds)
        for (int i = threadIdx.x; i < A.n_points; i += blockDim.x) sP[i] = A.points[i];
    __syncthreads();

    const ProgView P(A.prog);
    const DField fG = P.field(SLOT_G);
    const DField fF = P.field(SLOT_F);
    const DField fS = P.field(SLOT_SIGMA);
    const DField fA = P.field(SLOT_ALPHA);
    const bool detached = (fA.flags & WOST_FIELD_DETACHED) != 0;
    const float sigma_bar = P.hdr->sigma_bar;
    const float sqrt_sb = P.hdr->sqrt_sigma_bar;
    const float inv_sb = P.hdr->inv_sigma_bar;
    const FloatsC cheb_a{(cptr<float>)P.hdr->cheb_a};
    const FloatsC cheb_b{(cptr<float>)P.hdr->cheb_b};

    const int lane = threadIdx.x & 63;
    const uint64_t lanebit = 1ull << lane;
    const uint64_t lanes_below = lanebit - 1ull;

    // wave-uniform work-queue state
    uint64_t c_next = 0, c_end = 0;
    bool exhausted = false;

    // per-lane walk state (solvers/WoStSolver.py:188-195)
    bool active = false;
    uint64_t wid = 0;
    float px = 0.f, py = 0.f;
    float dD = 1.0f;            // dDirichlet seeded with 1.0 (:190, quirk Q12)
    int k = 0;                  // step_count
    bool onB = false;           // onBoundary
    float nx = 0.f, ny = 1.f;   // normal
    float w = 1.f;              // attenuation_coef
    float ax = 1.f;             // alpha(current_point), cached
    float total = 0.f;          // this walk's contributions

    for (;;) {
        // --- walk termination: while-condition of :206, boundary term :295-298
        if (active && !((k < A.max_steps) && (dD > A.eps))) {
            float g = fG.present ? P.value(fG, px, py) : 0.0f;
            if (DELTA) g = g * w;
            total = total + g;
            const int64_t li = (int64_t)(wid - (uint64_t)A.wid_begin);
            A.out_val[li] = total;
            A.out_steps[li] = (uint32_t)k;
            active = false;
        }

        // --- refill idle lanes from the wave's chunk (active-mask compaction)
        uint64_t need = __ballot(!active);
        while (need != 0ull && !exhausted) {
            if (c_next >= c_end) {
                unsigned long long c = 0;
                if (lane == 0) c = atomicAdd(A.counter, (unsigned long long)A.chunk);
                c = __shfl(c, 0);
                if (c >= (unsigned long long)A.count) {
                    exhausted = true;
                    break;
                }
                c_next = c;
                c_end = c + (uint64_t)A.chunk;
                if (c_end > (uint64_t)A.count) c_end = (uint64_t)A.count;
            }
            const uint64_t avail = c_end - c_next;
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t take = avail < (uint64_t)n ? (uint32_t)avail : n;
            const uint32_t rank = (uint32_t)__popcll(need & lanes_below);
            if ((need & lanebit) && rank < take) {
                wid = (uint64_t)A.wid_begin + c_next + rank;
                // pid = wid / W without a 64-bit integer division: a double
                // estimate (exact operands below 2^53) and one correction
                uint64_t pid = (uint64_t)((double)wid * A.inv_walks_per_point);
                const int64_t rem = (int64_t)(wid - pid * (uint64_t)A.walks_per_point);
                if (rem < 0) --pid;
                else if (rem >= A.walks_per_point) ++pid;
                float2 q;
                if (points_in_lds) q = sP[pid];
                else q = A.points[pid];
                px = q.x; py = q.y;
                k = 0; dD = 1.0f; onB = false; nx = 0.f; ny = 1.f; w = 1.f; total = 0.f;
                if (DELTA) ax = P.value(fA, px, py);
                active = true;
            }
            c_next += take;
            need = __ballot(!active);
        }
        if (!__any(active)) break;
        // a freshly refilled walk may already fail the while-condition (eps >= 1,
        // maxSteps == 0): it takes no step and is finished at the next iteration
        if (!(active && (k < A.max_steps) && (dD > A.eps))) continue;

        // --- one walk-step (:206-291)
        const float dd = poly_distance(sD, A.nd, px, py);           // :208
        float r;
        if (NEU) {
            const float dn = silhouette_distance(sN, A.nn, px, py);  // :211
            const float m = dn < dd ? dn : dd;                       // Python min()
            r = m > A.rmin ? m : A.rmin;                             // Python max() (:212)
        } else {
            r = dd > A.rmin ? dd : A.rmin;                           // :215
        }

        const U4 rn = philox4x32_10(U4{(uint32_t)k, 0u, (uint32_t)wid, (uint32_t)(wid >> 32)},
                                    A.key0, A.key1);
        float theta = (u01(rn.x) * 2.0f) * kPiF;                     // :226
        if (NEU && onB) theta = theta / 2.0f + atan2f(ny, nx);       // :227-228 (quirk Q2)
        const float cs = f_cos(theta), sn = f_sin(theta);            // :230-232

        float xnx, xny;
        if (NEU) {                                                   // :235-236
            const Hit h = intersect_polylines(sN, A.nn, px, py, cs, sn, r);
            xnx = h.x; xny = h.y; nx = h.nx; ny = h.ny; onB = h.hit;
        } else {                                                     // :238-239
            xnx = px + r * cs;
            xny = py + r * sn;
        }

        float yx = xnx, yy = xny;
        bool clipped = false;
        float gnorm = 0.f;
        Jet aj{0.f, 0.f, 0.f, 0.f};
        if (SRC) {                                                   // :242-258
            const float rs = sample_rho(sT, u01(rn.y)) * r;          // :244 (sampler, quirks Q3-Q5)
            yx = px + rs * cs;                                       // :245 (quirk Q13)
            yy = py + rs * sn;
            const float e1x = yx - px, e1y = yy - py;
            const float e2x = xnx - px, e2y = xny - py;
            clipped = sqrtf(e1x * e1x + e1y * e1y) > sqrtf(e2x * e2x + e2y * e2y);  // :248
            if (clipped) { yx = xnx; yy = xny; }
            if (DELTA) {
                gnorm = inv_sb * (1.0f - inv_i0(cheb_a, cheb_b, r * sqrt_sb));  // solvers/utils.py:43-44
                aj = P.jet(fA, yx, yy);
            }
            float c = 0.0f;
            if (!clipped) {
                const float f = P.value(fF, yx, yy);
                if (DELTA)
                    c = (f * gnorm) * f_rcp(f_sqrt(aj.v * ax)) * w;  // :253-254
                else
                    c = f * ((r * r) / 4.0f);                        // :256, utils.py:61
            }
            total = total + c;                                       // :258
        }

        if (DELTA) {                                                 // :271-284
            const float mu = u01(rn.z);
            if (mu > sigma_bar * gnorm) {
                const float an = clipped ? aj.v : P.value(fA, xnx, xny);
                w = w * f_sqrt(f_div(an, ax));                       // :277
                px = xnx; py = xny; ax = an;
            } else {
                const float sg = fS.present ? P.value(fS, yx, yy) : 0.0f;
                const float spv = sigma_prime_from(aj, sg, detached);    // :281
                float sc = 1.0f - spv * inv_sb;
                sc = (0.0f > sc) ? 0.0f : sc;                        // Python max(., 0.0) (:282)
                w = (w * f_sqrt(f_div(aj.v, ax))) * sc;              // :283
                px = yx; py = yy; ax = aj.v;
            }
        } else {
            px = xnx; py = xny;                                      // :287
        }
        k += 1;                                                      // :291
        dD = dd;   // the loop tests the distance of the pre-step point (quirk Q7)
    }
}

hipError_t walk_occupancy(int mode, int nd, int nn, int n_points, int* blocks_per_cu) {
    const size_t lds = walk_lds_bytes(mode, nd, nn, n_points);
    switch (mode) {
    case MODE_DIRICHLET:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<false, false, false>, kWalkBlock, lds);
    case MODE_POISSON:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<false, true, false>, kWalkBlock, lds);
    case MODE_MIXED:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<true, false, false>, kWalkBlock, lds);
    case MODE_MIXED_POISSON:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<true, true, false>, kWalkBlock, lds);
    case MODE_DELTA:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<false, true, true>, kWalkBlock, lds);
    case MODE_MIXED_DELTA:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wost_walk_kernel<true, true, true>, kWalkBlock, lds);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_walk(int mode, const WalkArgs& a, int grid, hipStream_t s) {
    const size_t lds = walk_lds_bytes(mode, a.nd, a.nn, a.n_points);
    switch (mode) {
    case MODE_DIRICHLET: wost_walk_kernel<false, false, false><<<grid, kWalkBlock, lds, s>>>(a); break;
    case MODE_POISSON: wost_walk_kernel<false, true, false><<<grid, kWalkBlock, lds, s>>>(a); break;
    case MODE_MIXED: wost_walk_kernel<true, false, false><<<grid, kWalkBlock, lds, s>>>(a); break;
    case MODE_MIXED_POISSON: wost_walk_kernel<true, true, false><<<grid, kWalkBlock, lds, s>>>(a); break;
    case MODE_DELTA: wost_walk_kernel<false, true, true><<<grid, kWalkBlock, lds, s>>>(a); break;
    case MODE_MIXED_DELTA: wost_walk_kernel<true, true, true><<<grid, kWalkBlock, lds, s>>>(a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Deterministic per-block sums (sum, sum of squares, steps) in float64. The
// thread -> walk assignment and the LDS tree are fixed, so the bits depend
// only on the walk values.
// ---------------------------------------------------------------------------
constexpr int kReduceBlock = 256;

__global__ void __launch_bounds__(kReduceBlock)
wost_block_reduce(const float* __restrict__ val, const uint32_t* __restrict__ steps,
                  const int64_t* __restrict__ begin, int64_t nblocks, double* __restrict__ out) {
    __shared__ double s_sum[kReduceBlock], s_sq[kReduceBlock], s_st[kReduceBlock];
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const int64_t lo = begin[b], hi = begin[b + 1];
        double s = 0.0, q = 0.0;
        uint64_t st = 0;
        for (int64_t i = lo + threadIdx.x; i < hi; i += kReduceBlock) {
            const double v = (double)val[i];
            s += v;
            q += v * v;
            st += steps[i];
        }
        s_sum[threadIdx.x] = s;
        s_sq[threadIdx.x] = q;
        s_st[threadIdx.x] = (double)st;
        __syncthreads();
        for (int h = kReduceBlock / 2; h > 0; h >>= 1) {
            if ((int)threadIdx.x < h) {
                s_sum[threadIdx.x] += s_sum[threadIdx.x + h];
                s_sq[threadIdx.x] += s_sq[threadIdx.x + h];
                s_st[threadIdx.x] += s_st[threadIdx.x + h];
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            out[3 * b + 0] = s_sum[0];
            out[3 * b + 1] = s_sq[0];
            out[3 * b + 2] = s_st[0];
        }
        __syncthreads();
    }
}

hipError_t launch_block_reduce(const float* val, const uint32_t* steps, const int64_t* begin,
                               int64_t nblocks, double* out, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    const int grid = (int)(nblocks < 65536 ? nblocks : 65536);
    wost_block_reduce<<<grid, kReduceBlock, 0, s>>>(val, steps, begin, nblocks, out);
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
