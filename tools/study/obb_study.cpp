// STUDY HARNESS (host only, not shipped): oriented-box (OBB) child bounds for the
// segment tree, against the AABB tree of wost_device.h and the full scans: visit counts
// and bit-exactness on caller-supplied queries.
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define WOST_TREE_STATS 1

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"

using namespace wost;

#if !defined(__HIP_DEVICE_COMPILE__)
long wost::g_tree_stats[4];

namespace {

struct ObbTree {
    std::vector<float> nd;   // per node: cx, cy, ux, uy, a, b, ch, sh   (a < 0: padding)
    int first_leaf = 0, leaf = 0;
    float tol = 0.f;
    const float2* v = nullptr;
    int nv = 0;
};

float g_margin = 1e-5f;
float g_tolscale = 1.0f;

int g_pow4 = 0;
int g_arity = 2;

bool build_obb(const float* xy, int nv, int leaf, ObbTree* t) {
    const int nseg = nv - 1;
    const int nleaves = (nseg + leaf - 1) / leaf;
    const int A = g_arity;
    int P = A;
    while (P < nleaves) P *= A;
    const int first_leaf = (P - 1) / (A - 1);
    const int n_nodes = first_leaf + P;
    t->first_leaf = first_leaf;
    t->leaf = leaf;
    t->v = reinterpret_cast<const float2*>(xy);
    t->nv = nv;
    t->nd.assign(8 * (size_t)n_nodes, 0.f);
    std::vector<int> lo(n_nodes, -1), hi(n_nodes, -1);
    for (int l = 0; l < P; ++l) {
        const int k = first_leaf + l;
        if (l * leaf < nseg) { lo[k] = l * leaf; hi[k] = std::min((l + 1) * leaf, nseg - 1); }
    }
    for (int k = first_leaf - 1; k >= 0; --k)
        for (int j = 0; j < A; ++j) {
            const int c = A * k + 1 + j;
            if (lo[c] < 0) continue;
            if (lo[k] < 0) lo[k] = lo[c];
            hi[k] = hi[c];
        }
    float cmax = 0.f;
    for (int i = 0; i < 2 * nv; ++i) cmax = std::max(cmax, std::fabs(xy[i]));
    t->tol = std::ldexp(1.0f + cmax, -14);
    std::vector<double> ang;
    for (int k = 0; k < n_nodes; ++k) {
        float* o = &t->nd[8 * (size_t)k];
        if (lo[k] < 0) { o[4] = -1.f; o[6] = 2.f; continue; }
        ang.clear();
        for (int s = lo[k]; s <= hi[k]; ++s) {
            const double ux = (double)xy[2 * s + 2] - xy[2 * s], uy = (double)xy[2 * s + 3] - xy[2 * s + 1];
            if (ux != 0.0 || uy != 0.0) ang.push_back(std::atan2(uy, ux));
        }
        double axis = 0.0, half = 0.0;
        int code = 0;
        if (ang.empty()) code = 2;
        else {
            std::sort(ang.begin(), ang.end());
            double gap = ang.front() + 2 * M_PI - ang.back();
            size_t st = 0;
            for (size_t i = 1; i < ang.size(); ++i) if (ang[i] - ang[i - 1] > gap) { gap = ang[i] - ang[i - 1]; st = i; }
            half = 0.5 * (2 * M_PI - gap);
            axis = ang[st] + half;
            if (half >= 0.5 * M_PI - 0.01) code = 3;
        }
        double ux = 1.0, uy = 0.0;
        if (code == 0) { ux = std::cos(axis); uy = std::sin(axis); }
        // store u in float and build the box around the float axis
        const float fux = (float)ux, fuy = (float)uy;
        ux = fux; uy = fuy;
        const double nx = -uy, ny = ux;
        double tmin = 1e300, tmax = -1e300, smin = 1e300, smax = -1e300;
        for (int v = lo[k]; v <= hi[k] + 1; ++v) {
            const double x = xy[2 * v], y = xy[2 * v + 1];
            const double tt = x * ux + y * uy, ss = x * nx + y * ny;
            tmin = std::min(tmin, tt); tmax = std::max(tmax, tt); smin = std::min(smin, ss); smax = std::max(smax, ss);
        }
        const double tc = 0.5 * (tmin + tmax), sc = 0.5 * (smin + smax);
        const double cx = tc * ux + sc * nx, cy = tc * uy + sc * ny;
        double a = 0.5 * (tmax - tmin), b = 0.5 * (smax - smin);
        const double slack = 16.0 * std::ldexp(1.0, -24) * (std::fabs(cx) + std::fabs(cy) + a + b) + 1e-30;
        a += slack; b += slack;
        o[0] = (float)cx; o[1] = (float)cy; o[2] = fux; o[3] = fuy;
        o[4] = (float)(a * (1 + 1e-6)); o[5] = (float)(b * (1 + 1e-6)) + (float)slack;
        if (code == 0) { half += 1e-6; o[6] = (float)std::cos(half); o[7] = (float)std::sin(half); }
        else { o[6] = (float)code; o[7] = 0.f; }
    }
    return true;
}

inline const float* node(const ObbTree& t, int k) { return &t.nd[8 * (size_t)k]; }

// lower bound of every vertex's computed squared distance
float obb_lb2(const float* o, float px, float py) {
    if (o[4] < 0.f) return WOST_INF;
    const float wx = px - o[0], wy = py - o[1];
    const float pu = wx * o[2] + wy * o[3], pn = wy * o[2] - wx * o[3];
    const float sl = 1.0f / 1048576.0f * (fabsf(wx) + fabsf(wy) + o[4] + o[5]);
    float gu = fabsf(pu) - o[4] - sl, gn = fabsf(pn) - o[5] - sl;
    gu = gu > 0.f ? gu : 0.f;
    gn = gn > 0.f ? gn : 0.f;
    return (gu * gu + gn * gn) * (1.0f - 1.0f / 1048576.0f);
}

bool obb_cone_excludes(const float* o, float px, float py) {
    if (o[6] == 2.0f) return true;
    if (o[6] == 3.0f) return false;
    const float ux = o[2], uy = o[3], nx = -uy, ny = ux;
    float qx[4], qy[4];
    int i = 0;
    for (int su = -1; su <= 1; su += 2)
        for (int sn = -1; sn <= 1; sn += 2) {
            qx[i] = o[0] + su * o[4] * ux + sn * o[5] * nx;
            qy[i] = o[1] + su * o[4] * uy + sn * o[5] * ny;
            ++i;
        }
    const float ch = o[6], sh = o[7];
    const float e1x = ch * ux + sh * uy, e1y = -sh * ux + ch * uy;   // u rotated by -h
    const float e2x = ch * ux - sh * uy, e2y = sh * ux + ch * uy;    // u rotated by +h
    float lo = WOST_INF, hi = -WOST_INF, mx = 0.f, my = 0.f;
    for (int j = 0; j < 4; ++j) {
        const float wx = px - qx[j], wy = py - qy[j];
        mx = fmaxf(mx, fabsf(wx)); my = fmaxf(my, fabsf(wy));
        const float v1 = e1x * wy - e1y * wx, v2 = e2x * wy - e2y * wx;
        lo = fminf(lo, fminf(v1, v2)); hi = fmaxf(hi, fmaxf(v1, v2));
    }
    const float m = g_margin * (mx + my);
    return lo > m || hi < -m;
}

float sil_obb(const ObbTree& t, float px, float py, float dd, float stop2, long* cnt) {
    float best = WOST_INF;
    const int nv = t.nv, nseg = nv - 1;
    if (nv < 3) return best;
    const float T = (dd * dd) * 1.002f;
    // nearest-first DFS with an explicit stack (study: visit counts only matter)
    std::vector<std::pair<float, int>> st;
    st.push_back({0.f, 0});
    while (!st.empty()) {
        auto [lb, k] = st.back();
        st.pop_back();
        const float bound = best < T ? best : T;
        if (lb > bound) continue;
        if (k < t.first_leaf) {
            ++cnt[0];
            const int c[2] = {2 * k + 1, 2 * k + 2};
            float l[2];
            bool ok[2];
            for (int j = 0; j < 2; ++j) {
                const float* o = node(t, c[j]);
                l[j] = obb_lb2(o, px, py);
                ok[j] = !(l[j] > bound) && !obb_cone_excludes(o, px, py);
            }
            // push far first so that near is popped first
            const int nearj = (ok[1] && (!ok[0] || l[1] < l[0])) ? 1 : 0;
            if (ok[1 - nearj]) st.push_back({l[1 - nearj], c[1 - nearj]});
            if (ok[nearj]) st.push_back({l[nearj], c[nearj]});
            continue;
        }
        ++cnt[1];
        const int s0 = (k - t.first_leaf) * t.leaf;
        const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
        const int j1 = s1 < nv - 2 ? s1 : nv - 2;
        if (s0 + 1 <= j1) {
            const float2 va = t.v[s0];
            float2 vb = t.v[s0 + 1];
            float cprev = (vb.x - va.x) * (py - va.y) - (vb.y - va.y) * (px - va.x);
            for (int j = s0 + 1; j <= j1; ++j) {
                const float2 vc = t.v[j + 1];
                const float bpx = px - vb.x, bpy = py - vb.y;
                const float ccur = (vc.x - vb.x) * bpy - (vc.y - vb.y) * bpx;
                if (cprev * ccur < 0.0f) {
                    const float d2 = bpx * bpx + bpy * bpy;
                    best = d2 < best ? d2 : best;
                }
                cprev = ccur;
                vb = vc;
            }
            if (best <= stop2) break;
        }
    }
    return best == WOST_INF ? best : sqrt_rn(best);
}

Hit ray_obb(const ObbTree& t, float px, float py, float dxi, float dyi, float r, long* cnt) {
    Hit h;
    float dn, dx, dy;
    unit_direction(dxi, dyi, dn, dx, dy);
    if (dn < 1e-10f) { h.x = px; h.y = py; h.nx = 1.f; h.ny = 0.f; h.hit = false; h.seg = -1; return h; }
    const float qx = px + 1e-6f * dx, qy = py + 1e-6f * dy;
    const float tol = g_tolscale * (t.tol + 6.103515625e-05f * (fabsf(qx) + fabsf(qy)));
    const int nseg = t.nv - 1;
    float best = WOST_INF;
    int bi = -1;
    auto keep = [&](const float* o) {
        if (o[4] < 0.f) return false;
        const float cx = o[0] - qx, cy = o[1] - qy;
        const float cu = dx * o[3] - dy * o[2], du = dx * o[2] + dy * o[3];
        if (fabsf(dx * cy - dy * cx) > o[4] * fabsf(cu) + o[5] * fabsf(du) + tol) return false;
        if (o[6] == 3.0f) return true;
        const float ahead = dx * cx + dy * cy + o[4] * fabsf(du) + o[5] * fabsf(cu);
        if (!(ahead < -(64.0f * tol + 1e-2f * (fabsf(cx) + fabsf(cy) + o[4] + o[5])))) return true;
        if (o[6] == 2.0f) return false;
        const float ux = o[2], uy = o[3], ch = o[6], sh = o[7];
        const float e1x = ch * ux + sh * uy, e1y = -sh * ux + ch * uy;
        const float e2x = ch * ux - sh * uy, e2y = sh * ux + ch * uy;
        const float c1 = e1x * dy - e1y * dx, c2 = e2x * dy - e2y * dx;
        return !((c1 > 1e-3f && c2 > 1e-3f) || (c1 < -1e-3f && c2 < -1e-3f));
    };
    std::vector<int> st;
    st.push_back(0);
    while (!st.empty()) {
        const int k = st.back();
        st.pop_back();
        if (k < t.first_leaf) {
            ++cnt[2];
            const bool l = keep(node(t, 2 * k + 1)), rr = keep(node(t, 2 * k + 2));
            if (rr) st.push_back(2 * k + 2);
            if (l) st.push_back(2 * k + 1);
            continue;
        }
        ++cnt[3];
        const int s0 = (k - t.first_leaf) * t.leaf;
        const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
        float2 a = t.v[s0];
        for (int i = s0; i < s1; ++i) {
            const float2 b = t.v[i + 1];
            const float s = ray_segment_time_filtered(a, b, qx, qy, dx, dy);
            if (s < best) { best = s; bi = i; }
            a = b;
        }
    }
    return intersect_finish<false>(t.v, bi, best, px, py, dx, dy, qx, qy, r);
}

// 4-ary traversals over the same nodes: node k (even binary depth) has children
// 4k+3 .. 4k+6 (its grandchildren). Order-independent results: silhouette min d2,
// ray lexicographic (s, segment) min.
float sil_obb4(const ObbTree& t, float px, float py, float dd, float stop2, long* cnt) {
    float best = WOST_INF;
    const int nv = t.nv, nseg = nv - 1;
    if (nv < 3) return best;
    const float T = (dd * dd) * 1.002f;
    std::vector<std::pair<float, int>> st;
    st.push_back({0.f, 0});
    while (!st.empty()) {
        auto [lb, k] = st.back();
        st.pop_back();
        const float bound = best < T ? best : T;
        if (lb > bound) continue;
        if (k < t.first_leaf) {
            ++cnt[0];
            std::pair<float, int> ch[64];
            int nk = 0;
            for (int j = 0; j < g_arity; ++j) {
                const int c = g_arity * k + 1 + j;
                const float* o = node(t, c);
                const float l = obb_lb2(o, px, py);
                if (!(l > bound) && !obb_cone_excludes(o, px, py)) ch[nk++] = {l, c};
            }
            std::sort(ch, ch + nk, [](auto a, auto b) { return a.first > b.first; });   // far first on the stack
            for (int j = 0; j < nk; ++j) st.push_back(ch[j]);
            continue;
        }
        ++cnt[1];
        const int s0 = (k - t.first_leaf) * t.leaf;
        const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
        const int j1 = s1 < nv - 2 ? s1 : nv - 2;
        if (s0 + 1 <= j1) {
            const float2 va = t.v[s0];
            float2 vb = t.v[s0 + 1];
            float cprev = (vb.x - va.x) * (py - va.y) - (vb.y - va.y) * (px - va.x);
            for (int j = s0 + 1; j <= j1; ++j) {
                const float2 vc = t.v[j + 1];
                const float bpx = px - vb.x, bpy = py - vb.y;
                const float ccur = (vc.x - vb.x) * bpy - (vc.y - vb.y) * bpx;
                if (cprev * ccur < 0.0f) {
                    const float d2 = bpx * bpx + bpy * bpy;
                    best = d2 < best ? d2 : best;
                }
                cprev = ccur;
                vb = vc;
            }
            if (best <= stop2) break;
        }
    }
    return best == WOST_INF ? best : sqrt_rn(best);
}

Hit ray_obb4(const ObbTree& t, float px, float py, float dxi, float dyi, float r, long* cnt) {
    Hit h;
    float dn, dx, dy;
    unit_direction(dxi, dyi, dn, dx, dy);
    if (dn < 1e-10f) { h.x = px; h.y = py; h.nx = 1.f; h.ny = 0.f; h.hit = false; h.seg = -1; return h; }
    const float qx = px + 1e-6f * dx, qy = py + 1e-6f * dy;
    const float tol = g_tolscale * (t.tol + 6.103515625e-05f * (fabsf(qx) + fabsf(qy)));
    const int nseg = t.nv - 1;
    float best = WOST_INF;
    int bi = -1;
    auto keep = [&](const float* o) {
        if (o[4] < 0.f) return false;
        const float cx = o[0] - qx, cy = o[1] - qy;
        const float cu = dx * o[3] - dy * o[2], du = dx * o[2] + dy * o[3];
        if (fabsf(dx * cy - dy * cx) > o[4] * fabsf(cu) + o[5] * fabsf(du) + tol) return false;
        if (o[6] == 3.0f) return true;
        const float ahead = dx * cx + dy * cy + o[4] * fabsf(du) + o[5] * fabsf(cu);
        if (!(ahead < -(64.0f * tol + 1e-2f * (fabsf(cx) + fabsf(cy) + o[4] + o[5])))) return true;
        if (o[6] == 2.0f) return false;
        const float ux = o[2], uy = o[3], ch = o[6], sh = o[7];
        const float e1x = ch * ux + sh * uy, e1y = -sh * ux + ch * uy;
        const float e2x = ch * ux - sh * uy, e2y = sh * ux + ch * uy;
        const float c1 = e1x * dy - e1y * dx, c2 = e2x * dy - e2y * dx;
        return !((c1 > 1e-3f && c2 > 1e-3f) || (c1 < -1e-3f && c2 < -1e-3f));
    };
    std::vector<int> st;
    st.push_back(0);
    while (!st.empty()) {
        const int k = st.back();
        st.pop_back();
        if (k < t.first_leaf) {
            ++cnt[2];
            for (int j = g_arity - 1; j >= 0; --j) if (keep(node(t, g_arity * k + 1 + j))) st.push_back(g_arity * k + 1 + j);
            continue;
        }
        ++cnt[3];
        const int s0 = (k - t.first_leaf) * t.leaf;
        const int s1 = s0 + t.leaf < nseg ? s0 + t.leaf : nseg;
        float2 a = t.v[s0];
        for (int i = s0; i < s1; ++i) {
            const float2 b = t.v[i + 1];
            const float s = ray_segment_time_filtered(a, b, qx, qy, dx, dy);
            if (s < best || (s == best && i < bi)) { best = s; bi = i; }
            a = b;
        }
    }
    return intersect_finish<false>(t.v, bi, best, px, py, dx, dy, qx, qy, r);
}

bool same(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}

}  // namespace

extern "C" {

// per query: counts[4] (OBB: sil records, sil leaves, ray records, ray leaves);
// mism[0] = r mismatches vs the scan, mism[1] = ray-hit mismatches vs the scan
int obb_counts(const float* xy, int nv, int leaf, float margin, const float* pts, const float* dirs, const float* dd,
               float rmin, float stop2, long n, long* out, long* mism, int arity) {
    ObbTree t;
    g_margin = margin;
    g_arity = arity;
    if (getenv("TOLSCALE")) g_tolscale = atof(getenv("TOLSCALE"));
    build_obb(xy, nv, leaf, &t);
    const float2* v = reinterpret_cast<const float2*>(xy);
    mism[0] = mism[1] = 0;
    for (long i = 0; i < n; ++i) {
        long* c = out + 4 * i;
        c[0] = c[1] = c[2] = c[3] = 0;
        const float px = pts[2 * i], py = pts[2 * i + 1];
        const float dn_t = arity > 2 ? sil_obb4(t, px, py, dd[i], stop2, c) : sil_obb(t, px, py, dd[i], stop2, c);
        const float dn_b = silhouette_distance(v, nv, px, py);
        const float mb = dn_b < dd[i] ? dn_b : dd[i], mt = dn_t < dd[i] ? dn_t : dd[i];
        const float rb = mb > rmin ? mb : rmin, rt = mt > rmin ? mt : rmin;
        if (!same(rb, rt)) ++mism[0];
        const Hit hb = intersect_polylines(v, nv, px, py, dirs[2 * i], dirs[2 * i + 1], rb);
        const Hit ht = arity > 2 ? ray_obb4(t, px, py, dirs[2 * i], dirs[2 * i + 1], rb, c)
                                  : ray_obb(t, px, py, dirs[2 * i], dirs[2 * i + 1], rb, c);
        if (!same(hb.x, ht.x) || !same(hb.y, ht.y) || hb.hit != ht.hit || (hb.hit && hb.seg != ht.seg)) {
            if (mism[1] < 3)
                fprintf(stderr, "q %ld p (%.9g, %.9g) d (%.9g, %.9g) r %g: scan hit %d seg %d (%.9g,%.9g)  obb hit %d seg %d (%.9g,%.9g)\n",
                       i, px, py, dirs[2 * i], dirs[2 * i + 1], rb, hb.hit, hb.seg, hb.x, hb.y, ht.hit, ht.seg, ht.x, ht.y);
            ++mism[1];
        }
    }
    return 0;
}
}
#endif
