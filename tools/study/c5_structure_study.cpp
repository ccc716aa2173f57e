// STUDY HARNESS (host only, not shipped; round 6): the work a wave of
// C5 Neumann queries costs under the current 4-ary segment tree and under the two
// structural candidates -- (a) waves of walks from one of K spatial classes (the walk
// pools generalised), (b) a wide node: 16-ary nodes whose 16 children are tested by 16 lanes
// at once (4 queries per wave instruction). The tree, its child tests and the silhouette
// bound are wost_device.h's (the kernels' code built for the host). A 16-ary node is the
// 4-ary tree with every other level removed: its children are the 4-ary grandchildren,
// whose oriented boxes and arcs are the 4-ary records one level down (so the same tests,
// and the same leaves reached).
//
// Per query q and kind (silhouette: depth-first, nearest child first, the bound tightening
// as leaves are scanned, as silhouette_distance_tree; ray: every record the line keeps):
//   v4  record visits of the 4-ary search (each: one lane tests the record's 4 children)
//   c4  = 4 v4 child tests;   leaves  leaf scans
//   c16 child tests of the 16-ary search (16 per wide-node visit, 4 per visit of the last
//       4-ary level when the depth is odd)
//   path the longest root-to-leaf chain of visits (a lower bound on any search's rounds)
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
namespace {

bool ray_keep(float4 cu, float4 ab, float qx, float qy, float dx, float dy, float tol) {
    if (ab.x < 0.0f) return false;
    const float cx = cu.x - qx, cy = cu.y - qy;
    const float cr = dx * cu.w - dy * cu.z, dt = dx * cu.z + dy * cu.w;
    if (fabsf(dx * cy - dy * cx) > (ab.x * fabsf(cr) + ab.y * fabsf(dt)) + tol) return false;
    if (ab.z == 3.0f) return true;
    const float ahead = (dx * cx + dy * cy) + (ab.x * fabsf(dt) + ab.y * fabsf(cr));
    if (!(ahead < -(512.0f * tol + 1e-2f * ((fabsf(cx) + fabsf(cy)) + (ab.x + ab.y))))) return true;
    if (ab.z == 2.0f) return false;
    return !(ab.z * fabsf(cr) - ab.w * fabsf(dt) > 1e-3f);
}

struct Q {
    const SegTree* t;
    float px, py, T, sl, mc, best;
    long v4, c16, leaves, path;
};

// the record of node (lvl, pos): child j's box and arc words
inline float4 cw(const SegTree& t, int lvl, int pos, int j, int w) {
    return t.word(tree_level_offset(lvl) + pos, 2 * j + w);
}

void leaf_scan(Q& q, int pos) {
    const SegTree& t = *q.t;
    const int nseg = t.nv - 1, s0 = pos * t.leaf, s1 = std::min(s0 + t.leaf, nseg), j1 = std::min(s1, t.nv - 2);
    ++q.leaves;
    for (int j = std::max(s0, 1); j <= j1; ++j) {
        const float2 a = t.v[j - 1], c = t.v[j], d = t.v[j + 1];
        if (is_silhouette(a, c, d, q.px, q.py)) {
            const float bx = q.px - c.x, by = q.py - c.y;
            q.best = std::min(q.best, bx * bx + by * by);
        }
    }
}

// 4-ary silhouette search from node (lvl, pos), depth-first, nearest child first
void sil4(Q& q, int lvl, int pos, int chain) {
    const SegTree& t = *q.t;
    ++q.v4;
    q.path = std::max<long>(q.path, chain + 1);
    struct K { float lb; int j; };
    K kept[4];
    int n = 0;
    for (int j = 0; j < 4; ++j) {
        float lb;
        if (silhouette_child_keep_q(cw(t, lvl, pos, j, 0), cw(t, lvl, pos, j, 1), q.px, q.py, std::min(q.best, q.T),
                                    q.sl, q.mc, &lb))
            kept[n++] = {lb, j};
    }
    std::sort(kept, kept + n, [](const K& a, const K& b) { return a.lb < b.lb; });
    for (int i = 0; i < n; ++i) {
        if (kept[i].lb > std::min(q.best, q.T)) continue;   // pruned when resumed
        const int c = 4 * pos + kept[i].j;
        if (lvl + 1 == t.depth) leaf_scan(q, c);
        else sil4(q, lvl + 1, c, chain + 1);
    }
}

// 16-ary silhouette search: at even levels a wide node tests its 16 grandchildren (a
// grandchild is kept when its parent's test and its own keep it -- the parent test is what
// a 16-ary node's child box would be looser than; we credit the wide node with the
// grandchild's own, tighter box alone); at the last odd level a 4-ary step
void sil16(Q& q, int lvl, int pos, int chain) {
    const SegTree& t = *q.t;
    q.path = std::max<long>(q.path, chain + 1);
    if (lvl + 1 == t.depth) {   // last level: a 4-ary node
        q.c16 += 4;
        struct K { float lb; int j; };
        K kept[4];
        int n = 0;
        for (int j = 0; j < 4; ++j) {
            float lb;
            if (silhouette_child_keep_q(cw(t, lvl, pos, j, 0), cw(t, lvl, pos, j, 1), q.px, q.py,
                                        std::min(q.best, q.T), q.sl, q.mc, &lb))
                kept[n++] = {lb, j};
        }
        std::sort(kept, kept + n, [](const K& a, const K& b) { return a.lb < b.lb; });
        for (int i = 0; i < n; ++i)
            if (!(kept[i].lb > std::min(q.best, q.T))) leaf_scan(q, 4 * pos + kept[i].j);
        return;
    }
    q.c16 += 16;
    struct K { float lb; int g; };
    K kept[16];
    int n = 0;
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
            float lb;
            const int c = 4 * pos + j;
            if (silhouette_child_keep_q(cw(t, lvl + 1, c, k, 0), cw(t, lvl + 1, c, k, 1), q.px, q.py,
                                        std::min(q.best, q.T), q.sl, q.mc, &lb))
                kept[n++] = {lb, 4 * c + k};
        }
    std::sort(kept, kept + n, [](const K& a, const K& b) { return a.lb < b.lb; });
    for (int i = 0; i < n; ++i) {
        if (kept[i].lb > std::min(q.best, q.T)) continue;
        if (lvl + 2 == t.depth) leaf_scan(q, kept[i].g);
        else sil16(q, lvl + 2, kept[i].g, chain + 1);
    }
}

struct R {
    const SegTree* t;
    float qx, qy, ux, uy, tol;
    long v4, c16, leaves, path;
};

void ray4(R& r, int lvl, int pos, int chain) {
    const SegTree& t = *r.t;
    ++r.v4;
    r.path = std::max<long>(r.path, chain + 1);
    for (int j = 0; j < 4; ++j)
        if (ray_keep(cw(t, lvl, pos, j, 0), cw(t, lvl, pos, j, 1), r.qx, r.qy, r.ux, r.uy, r.tol)) {
            if (lvl + 1 == t.depth) ++r.leaves;
            else ray4(r, lvl + 1, 4 * pos + j, chain + 1);
        }
}

void ray16(R& r, int lvl, int pos, int chain) {
    const SegTree& t = *r.t;
    r.path = std::max<long>(r.path, chain + 1);
    if (lvl + 1 == t.depth) {
        r.c16 += 4;
        for (int j = 0; j < 4; ++j)
            if (ray_keep(cw(t, lvl, pos, j, 0), cw(t, lvl, pos, j, 1), r.qx, r.qy, r.ux, r.uy, r.tol)) ++r.leaves;
        return;
    }
    r.c16 += 16;
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
            const int c = 4 * pos + j;
            if (ray_keep(cw(t, lvl + 1, c, k, 0), cw(t, lvl + 1, c, k, 1), r.qx, r.qy, r.ux, r.uy, r.tol)) {
                if (lvl + 2 == t.depth) ++r.leaves;
                else ray16(r, lvl + 2, 4 * c + k, chain + 1);
            }
        }
}

}  // namespace

extern "C" {

// n queries: out[i*8 + 0..7] = silhouette v4, c16, leaves, path(4-ary), ray v4, c16, leaves, path(4-ary)
int structure_queries(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* dd, int n,
                      long* out) {
    static SegmentTreeHost th;
    static std::vector<float> key;
    if (key.size() != (size_t)(2 * nv) || std::memcmp(key.data(), xy, sizeof(float) * 2 * nv) != 0 ||
        th.leaf != leaf) {
        if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
        key.assign(xy, xy + 2 * nv);
    }
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    for (int i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float s = ((fabsf(px) + fabsf(py)) + t.kmax) * 1.001f;
        Q a{&t, px, py, (dd[i] * dd[i]) * 1.002f, 9.5367431640625e-07f * s, kConeMargin * s, WOST_INF, 0, 0, 0, 0};
        sil4(a, 0, 0, 0);
        Q b = a;
        b.best = WOST_INF;
        b.v4 = b.c16 = b.leaves = b.path = 0;
        sil16(b, 0, 0, 0);
        float dn, ux, uy;
        unit_direction(dirs[2 * i], dirs[2 * i + 1], dn, ux, uy);
        const float qx = px + 1e-6f * ux, qy = py + 1e-6f * uy;
        R r{&t, qx, qy, ux, uy, t.tol + 7.62939453125e-06f * (fabsf(qx) + fabsf(qy)), 0, 0, 0, 0};
        ray4(r, 0, 0, 0);
        R r2 = r;
        r2.v4 = r2.c16 = r2.leaves = r2.path = 0;
        ray16(r2, 0, 0, 0);
        long* o = out + 8 * i;
        o[0] = a.v4; o[1] = b.c16; o[2] = a.leaves; o[3] = a.path;
        o[4] = r.v4; o[5] = r2.c16; o[6] = r.leaves; o[7] = r.path;
    }
    return 0;
}
}
#endif
