// wost_device.h -- arithmetic of one walk-step, shared by the gfx950 kernels
// and by libwost's host-side setup (sigma_bar grid, table checks).
//
// Everything here restates a piece of the reference's hot path; each function
// cites the reference lines it follows. The arithmetic is float32 like the
// reference's tensors (geometry/PolylinesSimple.py, solvers/WoStSolver.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "wost.h"

#define WOST_HD __host__ __device__ __forceinline__

namespace wost {

constexpr float kPiF = 3.14159265358979323846f;
constexpr int kChebA = 17;   // i0e on [0,8], t = x/4 - 1           (max rel. error 5e-7 in float)
constexpr int kChebB = 8;    // sqrt(x) i0e(x) on (8,inf), t = 16/x - 1 (max rel. error 2e-7 in float)

// ---------------------------------------------------------------------------
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11), the bijection of
// rocRAND's philox4x32_10_engine (rocrand/rocrand_philox4x32_10.h). A walk
// with global id g uses subsequence g: draw k of the walk is
// philox({k, 0, g_lo, g_hi}, {seed_lo, seed_hi}), i.e. the k-th rocrand4()
// of rocrand_init(seed, g, 0). One draw per walk-step gives the step's
// direction, source radius and collision uniforms. Replaces torch.rand(1)
// (solvers/WoStSolver.py:226,272) and the numpy sampler cache
// (solvers/utils.py:109-117).
// ---------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

WOST_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

WOST_HD U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c.x, hi0, lo0);
        mulhilo(0xCD9E8D57u, c.z, hi1, lo1);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// 24-bit uniform in [0,1), exactly representable in float32 (torch.rand's range).
WOST_HD float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------------------
// Fields (include/wost.h, "Coefficient fields"). Device layout of one field:
// header + terms + factors inside one program buffer.
// ---------------------------------------------------------------------------
struct alignas(16) DFactor {
    int32_t kind;
    int32_t pad[3];
    float p[8];
};
struct alignas(16) DTerm {
    float coef;
    int32_t first;   // absolute index into the program's factor array
    int32_t nf;
    int32_t pad;
};
struct alignas(16) DField {
    int32_t n_terms;
    int32_t first_term;  // absolute index into the program's term array
    int32_t flags;
    int32_t present;
};

// Program buffer header (uploaded once per handle, read with uniform indices).
enum { SLOT_G = 0, SLOT_F = 1, SLOT_SIGMA = 2, SLOT_ALPHA = 3, N_SLOTS = 4 };
struct alignas(16) DProgram {
    DField field[N_SLOTS];
    float cheb_a[kChebA];
    float cheb_b[kChebB];
    float sigma_bar;
    float sqrt_sigma_bar;
    float inv_sigma_bar;
    int32_t n_terms_total;
    // DTerm terms[n_terms_total] follows at offset sizeof(DProgram), then DFactor[]
};

struct Jet { float v, gx, gy, lap; };

WOST_HD Jet jet_mul(const Jet& a, const Jet& b) {
    Jet r;
    r.v = a.v * b.v;
    r.gx = a.v * b.gx + b.v * a.gx;
    r.gy = a.v * b.gy + b.v * a.gy;
    r.lap = a.v * b.lap + b.v * a.lap + 2.0f * (a.gx * b.gx + a.gy * b.gy);
    return r;
}

// ---------------------------------------------------------------------------
// Arithmetic of the coefficient fields, the Green's norm and the walk
// direction. On the device these use the hardware transcendental / reciprocal
// / square-root instructions (v_exp_f32, v_rcp_f32, v_sqrt_f32, v_sin_f32,
// v_cos_f32: a few ulp) instead of the correctly rounded library sequences.
// They feed values (contributions, weights), not the walk's geometric branch
// decisions, which stay IEEE (see the polyline queries below). The host build
// (sigma_bar grid) uses the C library.
// ---------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
WOST_HD float f_exp(float x) { return __expf(x); }
WOST_HD float f_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
WOST_HD float f_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
WOST_HD float f_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
WOST_HD float f_sin(float x) { return __sinf(x); }
WOST_HD float f_cos(float x) { return __cosf(x); }
#else
WOST_HD float f_exp(float x) { return expf(x); }
WOST_HD float f_rcp(float x) { return 1.0f / x; }
WOST_HD float f_div(float a, float b) { return a / b; }
WOST_HD float f_sqrt(float x) { return sqrtf(x); }
WOST_HD float f_sin(float x) { return sinf(x); }
WOST_HD float f_cos(float x) { return cosf(x); }
#endif

// torch.sigmoid in float32
WOST_HD float sigmoidf(float z) { return f_rcp(1.0f + f_exp(-z)); }

WOST_HD float ipowf(float x, int n) {
    float r = 1.0f;
    for (int i = 0; i < n; ++i) r *= x;
    return r;
}

WOST_HD float factor_value(const DFactor& f, float x, float y) {
    const float* p = f.p;
    switch (f.kind) {
    case WOST_FK_MONO:
        return ipowf(x, (int)p[0]) * ipowf(y, (int)p[1]);
    case WOST_FK_EXP_QUAD: {
        float dx = x - p[0], dy = y - p[1];
        float q = p[2] * (dx * dx) + p[3] * (dy * dy) + p[4] * (dx * dy) + p[5] * dx + p[6] * dy + p[7];
        return f_exp(q);
    }
    case WOST_FK_SIN_LIN:
        return f_sin(p[0] * x + p[1] * y + p[2]);
    case WOST_FK_COS_LIN:
        return f_cos(p[0] * x + p[1] * y + p[2]);
    case WOST_FK_SIGMOID_LIN:
        return sigmoidf(p[0] * x + p[1] * y + p[2]);
    case WOST_FK_SIGMOID_RADIAL: {
        // utils.py:128-129: sdf = ||x - c|| - R ; sigmoid(k * sdf)
        float dx = x - p[1], dy = y - p[2];
        float d = f_sqrt(dx * dx + dy * dy);
        return sigmoidf(p[0] * (d - p[3]));
    }
    case WOST_FK_IND_BOX:
        return (x >= p[0] && x <= p[1] && y >= p[2] && y <= p[3]) ? 1.0f : 0.0f;
    case WOST_FK_IND_DISK: {
        float dx = x - p[0], dy = y - p[1];
        return (dx * dx + dy * dy <= p[2]) ? 1.0f : 0.0f;
    }
    default:
        return NAN;
    }
}

WOST_HD Jet factor_jet(const DFactor& f, float x, float y) {
    const float* p = f.p;
    Jet j{0.f, 0.f, 0.f, 0.f};
    switch (f.kind) {
    case WOST_FK_MONO: {
        int a = (int)p[0], b = (int)p[1];
        float xa2 = a >= 2 ? ipowf(x, a - 2) : 0.f;
        float xa1 = a >= 1 ? (a >= 2 ? xa2 * x : 1.f) : 0.f;
        float xa = a >= 1 ? xa1 * x : 1.f;
        float yb2 = b >= 2 ? ipowf(y, b - 2) : 0.f;
        float yb1 = b >= 1 ? (b >= 2 ? yb2 * y : 1.f) : 0.f;
        float yb = b >= 1 ? yb1 * y : 1.f;
        j.v = xa * yb;
        j.gx = (float)a * xa1 * yb;
        j.gy = (float)b * xa * yb1;
        j.lap = (float)(a * (a - 1)) * xa2 * yb + (float)(b * (b - 1)) * xa * yb2;
        return j;
    }
    case WOST_FK_EXP_QUAD: {
        float dx = x - p[0], dy = y - p[1];
        float q = p[2] * (dx * dx) + p[3] * (dy * dy) + p[4] * (dx * dy) + p[5] * dx + p[6] * dy + p[7];
        float e = f_exp(q);
        float qx = 2.f * p[2] * dx + p[4] * dy + p[5];
        float qy = 2.f * p[3] * dy + p[4] * dx + p[6];
        j.v = e;
        j.gx = e * qx;
        j.gy = e * qy;
        j.lap = e * (qx * qx + qy * qy + 2.f * (p[2] + p[3]));
        return j;
    }
    case WOST_FK_SIN_LIN:
    case WOST_FK_COS_LIN: {
        float l = p[0] * x + p[1] * y + p[2];
        float s = f_sin(l), c = f_cos(l);
        float aa = p[0] * p[0] + p[1] * p[1];
        if (f.kind == WOST_FK_SIN_LIN) {
            j.v = s; j.gx = c * p[0]; j.gy = c * p[1]; j.lap = -s * aa;
        } else {
            j.v = c; j.gx = -s * p[0]; j.gy = -s * p[1]; j.lap = -c * aa;
        }
        return j;
    }
    case WOST_FK_SIGMOID_LIN: {
        float s = sigmoidf(p[0] * x + p[1] * y + p[2]);
        float s1 = s * (1.f - s);
        float s2 = s1 * (1.f - 2.f * s);
        j.v = s; j.gx = s1 * p[0]; j.gy = s1 * p[1];
        j.lap = s2 * (p[0] * p[0] + p[1] * p[1]);
        return j;
    }
    case WOST_FK_SIGMOID_RADIAL: {
        float dx = x - p[1], dy = y - p[2];
        float d = f_sqrt(dx * dx + dy * dy);
        float k = p[0];
        float s = sigmoidf(k * (d - p[3]));
        float s1 = s * (1.f - s);          // ds/dz
        float s2 = s1 * (1.f - 2.f * s);   // d2s/dz2
        float inv = f_rcp(d);
        // z = k (d - R): grad z = k (x-c)/d, lap z = k/d (2-D), |grad z|^2 = k^2
        j.v = s;
        j.gx = s1 * k * dx * inv;
        j.gy = s1 * k * dy * inv;
        j.lap = s2 * k * k + s1 * k * inv;
        return j;
    }
    case WOST_FK_IND_BOX:
    case WOST_FK_IND_DISK:
        j.v = factor_value(f, x, y);
        return j;
    default:
        j.v = NAN;
        return j;
    }
}

// Field evaluation. TP/FP are pointer types to DTerm/DFactor: plain pointers
// on the host, constant-address-space pointers on the device so that the
// wave-uniform reads become scalar (SMEM) loads.
template <class TP, class FP>
WOST_HD float field_value(const DField& fd, TP terms, FP factors, float x, float y) {
    float acc = 0.0f;
    for (int t = 0; t < fd.n_terms; ++t) {
        DTerm tm = terms[fd.first_term + t];
        float prod = tm.coef;
        for (int k = 0; k < tm.nf; ++k) {
            DFactor f = factors[tm.first + k];
            prod = prod * factor_value(f, x, y);
        }
        acc = acc + prod;
    }
    return acc;
}

template <class TP, class FP>
WOST_HD Jet field_jet(const DField& fd, TP terms, FP factors, float x, float y) {
    Jet acc{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < fd.n_terms; ++t) {
        DTerm tm = terms[fd.first_term + t];
        Jet prod{tm.coef, 0.f, 0.f, 0.f};
        for (int k = 0; k < tm.nf; ++k) {
            DFactor f = factors[tm.first + k];
            prod = jet_mul(prod, factor_jet(f, x, y));
        }
        acc.v += prod.v; acc.gx += prod.gx; acc.gy += prod.gy; acc.lap += prod.lap;
    }
    return acc;
}

// sigma'(y) of buildModifiedSigma (solvers/WoStSolver.py:74-127):
//   alpha_c = clamp(alpha, 1e-8)                                   (:80-86)
//   sigma/alpha_c + 0.5 * ((lap alpha_c + 1e-8)/alpha_c
//                          - |grad log(alpha_c + 1e-8)|^2 / 2)     (:102-121, utils.py:54)
// A detached or constant alpha makes autograd raise, and the reference falls
// back to sigma/alpha_c (:123-127, quirk Q9).
WOST_HD float sigma_prime_from(const Jet& alpha, float sigma, bool detached) {
    float ac = alpha.v < 1e-8f ? 1e-8f : alpha.v;
    float ratio = f_div(sigma, ac);
    if (detached) return ratio;
    bool clamped = !(alpha.v >= 1e-8f);
    float gx = clamped ? 0.f : alpha.gx, gy = clamped ? 0.f : alpha.gy;
    float lap = 1e-8f + (clamped ? 0.f : alpha.lap);
    float rden = f_rcp(ac + 1e-8f);
    float lx = gx * rden, ly = gy * rden;
    float gn = lx * lx + ly * ly;
    return ratio + 0.5f * (f_div(lap, ac) - gn / 2.0f);
}

// ---------------------------------------------------------------------------
// Screened Green's function norm (solvers/utils.py:29-44):
//   G_norm(R) = (1/sigma_bar) (1 - 1/I0(R sqrt(sigma_bar)))
// with 1/I0(x) = exp(-x) / i0e(x); i0e from Chebyshev series whose
// coefficients the host fits in double precision (wost_api.hip).
// ---------------------------------------------------------------------------
template <class CP>
WOST_HD float cheb_eval(CP c, int n, float t) {
    float b1 = 0.f, b2 = 0.f, t2 = 2.f * t;
    for (int k = n - 1; k >= 1; --k) {
        float b0 = t2 * b1 - b2 + c[k];
        b2 = b1;
        b1 = b0;
    }
    return t * b1 - b2 + c[0];
}

template <class CP>
WOST_HD float inv_i0(CP ca, CP cb, float x) {
    float i0e;
    if (x <= 8.0f) {
        i0e = cheb_eval(ca, kChebA, x * 0.25f - 1.0f);
    } else {
        i0e = cheb_eval(cb, kChebB, 16.0f * f_rcp(x) - 1.0f) * f_rcp(f_sqrt(x));
    }
    return f_exp(-x) * f_rcp(i0e);
}

// ---------------------------------------------------------------------------
// Radial sampler: inverse CDF of the reference's rejection samplers
// (GreensDistribution2D solvers/utils.py:138-151: density ~ -log rho on
// [1e-6,1); ScreenedGreensDistribution2D :181-195: density ~
// min(|G_sigmabar(rho; R=1)|, G_norm(1)) on [1e-6,1)), as WOST_SAMPLER_TABLE_N
// nodes F^-1(i/(N-1)) interpolated linearly. The sample is rho * r (:117).
// ---------------------------------------------------------------------------
template <class TabP>
WOST_HD float sample_rho(TabP tab, float u) {
#pragma clang fp contract(off)
    float pos = u * (float)(WOST_SAMPLER_TABLE_N - 1);
    int i = (int)pos;
    if (i > WOST_SAMPLER_TABLE_N - 2) i = WOST_SAMPLER_TABLE_N - 2;
    float f = pos - (float)i;
    float a = tab[i], b = tab[i + 1];
    return a + f * (b - a);
}

// ---------------------------------------------------------------------------
// Polyline queries (geometry/PolylinesSimple.py). VP is a pointer type to
// float2 vertices (LDS or constant address space); the loops are wave-uniform.
// Their branch decisions (clamps, silhouette signs, ray validity) must round
// op by op like the reference's torch CPU ops, so FMA contraction is off here.
// ---------------------------------------------------------------------------

// distance_to_polyline_jit (:25-49): min over segments of the distance to the
// clamped projection; a zero-length segment yields NaN which torch.min
// propagates. sqrt is monotonic, so min(sqrt) == sqrt(min) bit for bit.
template <class VP>
WOST_HD float poly_distance(VP v, int nv, float px, float py) {
#pragma clang fp contract(off)
    float best = INFINITY;
    bool nan = false;
    float2 a = v[0];
    for (int i = 1; i < nv; ++i) {
        float2 b = v[i];
        float ux = b.x - a.x, uy = b.y - a.y;
        float vx = px - a.x, vy = py - a.y;
        float duv = vx * ux + vy * uy;
        float duu = ux * ux + uy * uy;
        float t = duv / duu;
        t = t < 0.f ? 0.f : t;   // torch.clamp keeps NaN
        t = t > 1.f ? 1.f : t;
        float cx = (1.0f - t) * a.x + t * b.x;
        float cy = (1.0f - t) * a.y + t * b.y;
        float ex = cx - px, ey = cy - py;
        float d2 = ex * ex + ey * ey;
        nan |= (d2 != d2);
        best = d2 < best ? d2 : best;
        a = b;
    }
    return nan ? NAN : sqrtf(best);
}

// is_silhouette_jit (:51-81) for interior vertex j in [1, nv-2].
WOST_HD bool is_silhouette(float2 a, float2 b, float2 c, float px, float py) {
#pragma clang fp contract(off)
    float abx = b.x - a.x, aby = b.y - a.y;
    float bcx = c.x - b.x, bcy = c.y - b.y;
    float apx = px - a.x, apy = py - a.y;
    float bpx = px - b.x, bpy = py - b.y;
    float c1 = abx * apy - aby * apx;
    float c2 = bcx * bpy - bcy * bpx;
    return c1 * c2 < 0.0f;
}

// silhouette_distance_jit (:83-102): inf when no vertex is a silhouette; the
// first and last vertex are never tested (quirk Q6).
template <class VP>
WOST_HD float silhouette_distance(VP v, int nv, float px, float py) {
#pragma clang fp contract(off)
    float best = INFINITY;
    if (nv < 3) return best;
    float2 a = v[0], b = v[1];
    for (int j = 1; j + 1 < nv; ++j) {
        float2 c = v[j + 1];
        if (is_silhouette(a, b, c, px, py)) {
            float ex = b.x - px, ey = b.y - py;
            float d2 = ex * ex + ey * ey;
            best = d2 < best ? d2 : best;
        }
        a = b;
        b = c;
    }
    return best == INFINITY ? best : sqrtf(best);
}

// ray_intersection_jit (:104-132) for one segment: returns the SEGMENT
// parameter s as the "time" (quirk Q1), +inf when invalid.
WOST_HD float ray_segment_time(float2 a, float2 b, float qx, float qy, float dx, float dy) {
#pragma clang fp contract(off)
    float ux = b.x - a.x, uy = b.y - a.y;
    float wx = qx - a.x, wy = qy - a.y;
    float den = dx * uy - dy * ux;
    float s = (dx * wy - dy * wx) / den;
    float t = (ux * wy - uy * wx) / den;
    bool valid = (s >= 0.0f) && (s <= 1.0f) && (t > 0.0f);
    return valid ? s : INFINITY;
}

// The same test with the two IEEE divisions done only for candidate segments.
// The candidate filter uses the hardware reciprocal and is a strict superset
// of the reference's validity (slack 1e-6 on s >= 0 / s <= 1, t >= 0), and the
// candidates are then decided with the exact divisions, so the result is bit
// for bit that of ray_segment_time.
WOST_HD float ray_segment_time_filtered(float2 a, float2 b, float qx, float qy, float dx, float dy) {
#pragma clang fp contract(off)
    float ux = b.x - a.x, uy = b.y - a.y;
    float wx = qx - a.x, wy = qy - a.y;
    float den = dx * uy - dy * ux;
    float ns = dx * wy - dy * wx;
    float nt = ux * wy - uy * wx;
    float rd = f_rcp(den);
    float sa = ns * rd, ta = nt * rd;
    float res = INFINITY;
    if (sa >= -1e-6f && sa <= 1.000001f && ta >= 0.0f) {
        float s = ns / den;
        float t = nt / den;
        if ((s >= 0.0f) && (s <= 1.0f) && (t > 0.0f)) res = s;
    }
    return res;
}

struct Hit { float x, y, nx, ny; bool hit; };

// intersect_polylines_jit (:134-197).
template <class VP>
WOST_HD Hit intersect_polylines(VP v, int nv, float px, float py, float dxi, float dyi, float r) {
#pragma clang fp contract(off)
    Hit h;
    float dn = sqrtf(dxi * dxi + dyi * dyi);
    if (dn < 1e-10f) {
        h.x = px; h.y = py; h.nx = 1.f; h.ny = 0.f; h.hit = false;
        return h;
    }
    float dx = dxi / dn, dy = dyi / dn;
    float qx = px + 1e-6f * dx, qy = py + 1e-6f * dy;
    float best = INFINITY;
    int bi = -1;
    float2 a = v[0];
    for (int i = 1; i < nv; ++i) {
        float2 b = v[i];
        float s = ray_segment_time_filtered(a, b, qx, qy, dx, dy);
        if (s < best) { best = s; bi = i - 1; }   // first argmin (:177-178)
        a = b;
    }
    if (bi < 0 || best > r || best <= 0.0f) {
        h.x = px + r * dx; h.y = py + r * dy; h.nx = 0.f; h.ny = 0.f; h.hit = false;
        return h;
    }
    float2 sa = v[bi], sb = v[bi + 1];
    float ux = sb.x - sa.x, uy = sb.y - sa.y;
    float len = sqrtf(ux * ux + uy * uy);
    if (len < 1e-10f) {
        h.nx = 0.f; h.ny = 1.f;
    } else {
        float ex = ux / len, ey = uy / len;
        h.nx = -ey; h.ny = ex;    // left normal (:191-194)
    }
    h.x = qx + best * dx;
    h.y = qy + best * dy;
    h.hit = true;
    return h;
}

}  // namespace wost
