// TEST HARNESS -- host build of wost_device.h: the two-pass scans over compiled-in
// Neumann polylines (intersect_polylines_lines: per-vertex line filter;
// silhouette_distance_compact: squared distances of the marked silhouettes only)
// against the one-pass scans they replace, bit for bit, on caller-supplied polylines
// and queries. Built by tests/test_compiled_scans.py.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
namespace {
bool same(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}

template <int NV>
void check(const float2* v, const float* pts, const float* dirs, const float* radii, long n, float c1, long* out) {
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const Hit a = intersect_polylines<false>(v, NV, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        const Hit b = intersect_polylines_lines<NV>(v, v, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i], c1);
        if (!same(a.x, b.x) || !same(a.y, b.y) || a.hit != b.hit || (a.hit && a.seg != b.seg)) ++out[0];
        if (a.hit) ++out[2];
        const float s1 = silhouette_distance(v, NV, px, py);
        const float s2 = silhouette_distance_compact<NV>(v, v, px, py);
        if (!same(s1, s2)) ++out[1];
        if (s1 < WOST_INF) ++out[3];
    }
}
}  // namespace

// out[0] ray mismatches, out[1] silhouette mismatches, out[2] ray hits, out[3] queries with a silhouette
extern "C" int scan_check(const float* verts, int nv, const float* pts, const float* dirs, const float* radii, long n,
                          long* out) {
    std::vector<float2> v(nv);
    float c1 = 0.0f;
    for (int i = 0; i < nv; ++i) {
        v[i] = float2{verts[2 * i], verts[2 * i + 1]};
        c1 = std::fmax(c1, std::fabs(verts[2 * i]) + std::fabs(verts[2 * i + 1]));
    }
    c1 *= 1.0001f;   // as wost_jit.cpp passes it
    out[0] = out[1] = out[2] = out[3] = 0;
    switch (nv) {
        case 9: check<9>(v.data(), pts, dirs, radii, n, c1, out); break;
        case 17: check<17>(v.data(), pts, dirs, radii, n, c1, out); break;
        case 33: check<33>(v.data(), pts, dirs, radii, n, c1, out); break;
        case 65: check<65>(v.data(), pts, dirs, radii, n, c1, out); break;
        default: return 1;
    }
    return 0;
}

// neumann_scan_both (both queries in one pass, the brute-force kernels) against
// silhouette_distance and intersect_polylines<false> on a runtime polyline of any length.
// out[0] ray mismatches, out[1] silhouette mismatches, out[2] ray hits, out[3] silhouettes.
extern "C" int scan_both_check(const float* verts, int nv, const float* pts, const float* dirs, const float* radii,
                               long n, long* out) {
    std::vector<float2> v(nv + 16);   // the LDS variant reads up to a batch past the last vertex
    float c1 = 0.0f;
    for (int i = 0; i < nv + 16; ++i) {
        const int k = i < nv ? i : nv - 1;
        v[i] = float2{verts[2 * k], verts[2 * k + 1]};
        if (i < nv) c1 = std::fmax(c1, std::fabs(verts[2 * i]) + std::fabs(verts[2 * i + 1]));
    }
    c1 *= 1.0001f;   // as wost_jit.cpp passes it
    out[0] = out[1] = out[2] = out[3] = 0;
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const ScanBoth o = neumann_scan_both<false>(v.data(), nv, c1, px, py, dirs[2 * i], dirs[2 * i + 1]);
        const Hit a = intersect_polylines<false>(v.data(), nv, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        const Hit b = scan_both_finish(v.data(), o, px, py, radii[i]);
        if (!same(a.x, b.x) || !same(a.y, b.y) || a.hit != b.hit || (a.hit && a.seg != b.seg)) ++out[0];
        if (a.hit) ++out[2];
        const float s1 = silhouette_distance(v.data(), nv, px, py);
        if (!same(s1, scan_both_silhouette(o))) ++out[1];
        if (s1 < WOST_INF) ++out[3];
    }
    return 0;
}
#endif
