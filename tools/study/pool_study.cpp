// STUDY HARNESS (host only, not shipped; round 5): how many rounds a
// wave would need if each Neumann query kind drained a wave-wide task pool (a breadth-first
// pool of (query, record) and (query, leaf) tasks, every lane taking one task per round)
// instead of the per-lane stackless searches with hand-outs. The segment tree, its child
// tests and leaf scans are wost_device.h's (the kernels' code built for the host); the
// silhouette pruning bound of a query tightens as its leaf scans finish (FIFO: breadth
// first; LIFO: the newest tasks first, closer to the per-lane depth-first order).
#include <algorithm>
#include <cstring>
#include <deque>
#include <vector>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
namespace {

struct Task {
    int owner, lvl, pos;   // lvl == depth: a leaf scan of leaf pos
    float lb;              // silhouette: the child's lower bound when it was kept
};

// the ray query's child test of intersect_polylines_tree_wave (reference mode)
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

}  // namespace

extern "C" {

// One wave (n <= 64 queries). out[0..7]: silhouette rounds with internal tasks, rounds with
// leaf tasks, internal tasks, leaf tasks; the same four for the ray query. lifo: pop newest.
int pool_wave(const float* xy, int nv, int leaf, const float* pts, const float* dirs, const float* dd, int n,
              int lifo, long* out) {
    static SegmentTreeHost th;
    static std::vector<float> key;
    if (key.size() != (size_t)(2 * nv) || std::memcmp(key.data(), xy, sizeof(float) * 2 * nv) != 0 ||
        th.leaf != leaf) {
        if (!build_segment_tree(xy, nv, leaf, &th)) return 1;
        key.assign(xy, xy + 2 * nv);
    }
    const SegTree t{reinterpret_cast<const float4*>(th.rec.data()), reinterpret_cast<const float2*>(xy), nv,
                    th.first_leaf, th.depth, th.leaf, th.tol, th.kmax};
    const int nseg = nv - 1;
    for (int i = 0; i < 8; ++i) out[i] = 0;
    // --- silhouette
    std::vector<float> best(n, WOST_INF), T(n), sl(n), mc(n);
    std::deque<Task> q;
    for (int i = 0; i < n; ++i) {
        const float px = pts[2 * i], py = pts[2 * i + 1];
        T[i] = (dd[i] * dd[i]) * 1.002f;
        const float s = ((fabsf(px) + fabsf(py)) + t.kmax) * 1.001f;
        sl[i] = 9.5367431640625e-07f * s;
        mc[i] = kConeMargin * s;
        q.push_back({i, 0, 0, -WOST_INF});
    }
    while (!q.empty()) {
        std::vector<Task> round;
        while (!q.empty() && (int)round.size() < 64) {
            Task tk = lifo ? q.back() : q.front();
            if (lifo) q.pop_back(); else q.pop_front();
            const float bound = std::min(best[tk.owner], T[tk.owner]);
            if (tk.lb > bound) continue;   // pruned when popped: a lane's cheap test, not a task
            round.push_back(tk);
        }
        if (round.empty()) break;
        bool inner = false, leafr = false;
        std::vector<Task> born;
        for (const Task& tk : round) {
            const float px = pts[2 * tk.owner], py = pts[2 * tk.owner + 1];
            if (tk.lvl < t.depth) {
                inner = true;
                ++out[2];
                const int k = tree_level_offset(tk.lvl) + tk.pos;
                const float bound = std::min(best[tk.owner], T[tk.owner]);
                for (int j = 0; j < 4; ++j) {
                    float lb;
                    if (silhouette_child_keep_q(t.word(k, 2 * j), t.word(k, 2 * j + 1), px, py, bound, sl[tk.owner],
                                                mc[tk.owner], &lb))
                        born.push_back({tk.owner, tk.lvl + 1, 4 * tk.pos + j, lb});
                }
            } else {
                leafr = true;
                ++out[3];
                const int s0 = tk.pos * t.leaf, s1 = std::min(s0 + t.leaf, nseg), j1 = std::min(s1, nv - 2);
                float b = best[tk.owner];
                for (int j = std::max(s0, 1); j <= j1; ++j) {
                    const float2 a = t.v[j - 1], c = t.v[j], d = t.v[j + 1];
                    if (is_silhouette(a, c, d, px, py)) {
                        const float bx = px - c.x, by = py - c.y;
                        b = std::min(b, bx * bx + by * by);
                    }
                }
                best[tk.owner] = b;
            }
        }
        out[0] += inner;
        out[1] += leafr;
        for (const Task& b : born) q.push_back(b);
    }
    // --- ray (no bound: every record along the line)
    for (int i = 0; i < n; ++i) q.push_back({i, 0, 0, 0.f});
    std::vector<float> qx(n), qy(n), ux(n), uy(n), tol(n);
    for (int i = 0; i < n; ++i) {
        float dn;
        unit_direction(dirs[2 * i], dirs[2 * i + 1], dn, ux[i], uy[i]);
        qx[i] = pts[2 * i] + 1e-6f * ux[i];
        qy[i] = pts[2 * i + 1] + 1e-6f * uy[i];
        tol[i] = t.tol + 7.62939453125e-06f * (fabsf(qx[i]) + fabsf(qy[i]));
    }
    while (!q.empty()) {
        std::vector<Task> round;
        while (!q.empty() && (int)round.size() < 64) {
            round.push_back(lifo ? q.back() : q.front());
            if (lifo) q.pop_back(); else q.pop_front();
        }
        bool inner = false, leafr = false;
        std::vector<Task> born;
        for (const Task& tk : round) {
            const int o = tk.owner;
            if (tk.lvl < t.depth) {
                inner = true;
                ++out[6];
                const int k = tree_level_offset(tk.lvl) + tk.pos;
                for (int j = 0; j < 4; ++j)
                    if (ray_keep(t.word(k, 2 * j), t.word(k, 2 * j + 1), qx[o], qy[o], ux[o], uy[o], tol[o]))
                        born.push_back({o, tk.lvl + 1, 4 * tk.pos + j, 0.f});
            } else {
                leafr = true;
                ++out[7];
            }
        }
        out[4] += inner;
        out[5] += leafr;
        for (const Task& b : born) q.push_back(b);
    }
    return 0;
}
}
#endif
