// TEST HARNESS -- host build of wost_device.h: poly_distance_const (compiled-in
// polylines, Markstein division, no NaN bookkeeping) against poly_distance, bit
// for bit, on caller-supplied polylines and points. Built by
// tests/test_poly_distance_const.py.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"

namespace {
uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
float bf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// y = RN(1/duu) when the Markstein step is exact for every dividend mantissa, else 0
// (the rule of wost_jit.cpp markstein_reciprocal, restated for the test)
float checked_reciprocal(float d) {
    if (!(d >= 0x1p-40f && d <= 0x1p40f) || (fb(d) & 0x7FFFFFu) == 0) return 0.0f;
    const float b = bf(0x3F800000u | (fb(d) & 0x7FFFFFu));
    volatile float one = 1.0f, vb = b;
    const float y = one / vb;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        const float a = bf(0x3F800000u | m);
        const float q = a * y;
        volatile float va = a;
        if (fb(std::fma(std::fma(-q, b, a), y, q)) != fb(va / vb)) return 0.0f;
    }
    volatile float vd = d;
    return one / vd;
}
}  // namespace

extern "C" int polydist_check(const float* verts, int nv, const float* pts, long n, long* mismatches,
                              int* n_markstein) {
    std::vector<float2> v(nv);
    for (int i = 0; i < nv; ++i) v[i] = float2{verts[2 * i], verts[2 * i + 1]};
    std::vector<float> rcp(nv > 1 ? nv - 1 : 1, 0.0f);
    *n_markstein = 0;
    for (int i = 0; i + 1 < nv; ++i) {
        volatile float ux = v[i + 1].x - v[i].x, uy = v[i + 1].y - v[i].y;
        volatile float duu = ux * ux + uy * uy;
        rcp[i] = checked_reciprocal(duu);
        *n_markstein += rcp[i] != 0.0f;
    }
    long bad = 0;
    for (long k = 0; k < n; ++k) {
        const float px = pts[2 * k], py = pts[2 * k + 1];
        const float a = wost::poly_distance(v.data(), nv, px, py);
        const float b = wost::poly_distance_const(v.data(), rcp.data(), nv, px, py);
        if (fb(a) != fb(b)) ++bad;
    }
    *mismatches = bad;
    return 0;
}

// ray_segment_time_filtered (candidate filter, sign-only t test) against
// ray_segment_time (both IEEE divisions), bit for bit: segs[n][4], rays[n][4].
extern "C" int raytime_check(const float* segs, const float* rays, long n, long* mismatches, long* valid) {
    long bad = 0, ok = 0;
    for (long k = 0; k < n; ++k) {
        const float2 a{segs[4 * k], segs[4 * k + 1]}, b{segs[4 * k + 2], segs[4 * k + 3]};
        const float qx = rays[4 * k], qy = rays[4 * k + 1], dx = rays[4 * k + 2], dy = rays[4 * k + 3];
        const float s0 = wost::ray_segment_time(a, b, qx, qy, dx, dy);
        const float s1 = wost::ray_segment_time_filtered(a, b, qx, qy, dx, dy);
        if (fb(s0) != fb(s1)) ++bad;
        ok += s0 != WOST_INF;
    }
    *mismatches = bad;
    *valid = ok;
    return 0;
}
