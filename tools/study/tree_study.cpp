// STUDY HARNESS (host only, not shipped): per-query visit counts of the segment-tree
// queries of wost_device.h on caller-supplied queries, for sizing the C5 traversal.
#include <cstring>
#include <vector>

#define WOST_TREE_STATS 1

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
long wost::g_tree_stats[4];
#endif

#if !defined(__HIP_DEVICE_COMPILE__)
extern "C" {

// out[4*i..]: silhouette records, silhouette leaves, ray records, ray leaves of query i;
// res[2*i..]: r (the star radius) and the ray's hit flag
int tree_counts(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* dd, float rmin,
                float stop2, long n, long* out, float* res) {
    SegmentTreeHost th;
    if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    for (long i = 0; i < n; ++i) {
        for (int k = 0; k < 4; ++k) g_tree_stats[k] = 0;
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float dn = silhouette_distance_tree(t, px, py, dd[i], stop2);
        const float m = dn < dd[i] ? dn : dd[i];
        const float r = m > rmin ? m : rmin;
        const Hit h = intersect_polylines_tree<false>(t, px, py, dirs[2 * i], dirs[2 * i + 1], r);
        for (int k = 0; k < 4; ++k) out[4 * i + k] = g_tree_stats[k];
        res[2 * i] = r;
        res[2 * i + 1] = h.hit ? 1.f : 0.f;
    }
    return 0;
}
}
#endif
