// TEST HARNESS -- host build of the walk kernels' geometry (wost_device.h)
// comparing the segment-tree queries with the full scans they replace, bit for
// bit, on caller-supplied queries. Built by tests/test_segment_tree.py.
#include <cstring>
#include <vector>

#define WOST_TREE_STATS 1

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
long wost::g_tree_stats[4];
#endif

namespace {
bool same(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}
}  // namespace

extern "C" {

// Depth of the tree built over xy[2 * nv] with `leaf` segments per leaf, or -1 when
// build_segment_tree refuses it (degenerate input, deeper than kTreeMaxDepth).
int tree_build_depth(const float* xy, int nv, int leaf) {
    SegmentTreeHost th;
    return build_segment_tree(xy, nv, leaf, &th) ? th.depth : -1;
}

// Node / leaf visits of the tree queries since the last call (4 counters).
void tree_stats(long* out) {
#if !defined(__HIP_DEVICE_COMPILE__)
    for (int i = 0; i < 4; ++i) {
        out[i] = g_tree_stats[i];
        g_tree_stats[i] = 0;
    }
#endif
}

// For query i: point pts[i], direction dirs[i] (unnormalised), radius radii[i],
// Dirichlet distance dd[i]. Counts mismatches of min(silhouette, dd) (:212)
// into out[0] and of the ray hit (x, y, nx, ny, hit) into out[1]; out[2] =
// queries with a silhouette closer than dd, out[3] = ray hits (coverage).
int tree_check(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* radii,
               const float* dd, long n, long* out) {
    SegmentTreeHost th;
    if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    const float2* v = reinterpret_cast<const float2*>(xy);
    out[0] = out[1] = out[2] = out[3] = 0;
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float dn_b = silhouette_distance(v, nv, px, py);
        const float dn_t = silhouette_distance_tree(t, px, py, dd[i]);
        const float mb = dn_b < dd[i] ? dn_b : dd[i];
        const float mt = dn_t < dd[i] ? dn_t : dd[i];
        if (!same(mb, mt)) ++out[0];
        if (dn_b < dd[i]) ++out[2];
        const Hit hb = intersect_polylines(v, nv, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        const Hit ht = intersect_polylines_tree(t, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        if (!same(hb.x, ht.x) || !same(hb.y, ht.y) || !same(hb.nx, ht.nx) || !same(hb.ny, ht.ny) || hb.hit != ht.hit)
            ++out[1];
        if (hb.hit) ++out[3];
    }
    return 0;
}

// The walk's use r = max(rmin, min(dn, dd)) (:210-215) with the tree's early stop
// at stop2 (the largest float whose sqrtf is <= rmin) against the full scan.
// out[0] = mismatches of r, out[1] = queries where the early stop decided r
// (the scan found a silhouette at <= rmin), out[2] = tree node visits.
int tree_check_stop(const float* xy, int nv, int leaf, const float* pts, const float* dd, float rmin, float stop2,
                    long n, long* out) {
    SegmentTreeHost th;
    if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    const float2* v = reinterpret_cast<const float2*>(xy);
    out[0] = out[1] = out[2] = 0;
#if !defined(__HIP_DEVICE_COMPILE__)
    for (int i = 0; i < 4; ++i) g_tree_stats[i] = 0;
#endif
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float dn_b = silhouette_distance(v, nv, px, py);
        const float dn_t = silhouette_distance_tree(t, px, py, dd[i], stop2);
        const float mb = dn_b < dd[i] ? dn_b : dd[i], mt = dn_t < dd[i] ? dn_t : dd[i];
        const float rb = mb > rmin ? mb : rmin, rt = mt > rmin ? mt : rmin;
        if (!same(rb, rt)) ++out[0];
        if (dn_b <= rmin) ++out[1];
    }
#if !defined(__HIP_DEVICE_COMPILE__)
    out[2] = g_tree_stats[0];
#endif
    return 0;
}

// compat="fixed": the nearest-crossing ray query over the tree
// (intersect_polylines_tree<false, true>) against intersect_polylines_ray's scan,
// bit for bit (x, y, hit, segment). out[0] = mismatches, out[1] = hits.
int tree_check_nearest(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* radii,
                       long n, long* out) {
    SegmentTreeHost th;
    if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    const float2* v = reinterpret_cast<const float2*>(xy);
    out[0] = out[1] = 0;
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const Hit hb = intersect_polylines_ray(v, nv, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        const Hit ht = intersect_polylines_tree<false, true>(t, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        if (!same(hb.x, ht.x) || !same(hb.y, ht.y) || hb.hit != ht.hit || hb.seg != ht.seg) ++out[0];
        if (hb.hit) ++out[1];
    }
    return 0;
}

// The tree's raw answers (what wost_geometry_query(op | WOST_GEOM_TREE) returns on the
// device): silhouette_distance_tree without a Dirichlet bound -> sil[n], and
// intersect_polylines_tree (reference mode) -> hit[n][5] = x, y, nx, ny, found.
int tree_query(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* radii, long n,
               float* sil, float* hit) {
    SegmentTreeHost th;
    if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    for (long i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        sil[i] = silhouette_distance_tree(t, px, py, WOST_INF);
        const Hit h = intersect_polylines_tree(t, px, py, dirs[2 * i], dirs[2 * i + 1], radii[i]);
        hit[5 * i + 0] = h.x;
        hit[5 * i + 1] = h.y;
        hit[5 * i + 2] = h.nx;
        hit[5 * i + 3] = h.ny;
        hit[5 * i + 4] = h.hit ? 1.f : 0.f;
    }
    return 0;
}

}  // extern "C"
