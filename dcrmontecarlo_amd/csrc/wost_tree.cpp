// wost_tree.cpp -- builds the implicit segment tree of a Neumann polyline
// (see wost_device.h for how the kernels traverse it and why the queries stay
// bit-identical to the reference's full scans).
#include "wost_tree.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace wost {

namespace {

// Smallest arc of directions holding all the angles: (axis, half-angle).
// Returns false when there is no angle.
bool enclosing_arc(std::vector<double>& ang, double* axis, double* half) {
    if (ang.empty()) return false;
    std::sort(ang.begin(), ang.end());
    const double two_pi = 2.0 * M_PI;
    double gap = ang.front() + two_pi - ang.back();   // wrap-around gap
    size_t start = 0;                                 // arc starts after the largest gap
    for (size_t i = 1; i < ang.size(); ++i) {
        const double g = ang[i] - ang[i - 1];
        if (g > gap) {
            gap = g;
            start = i;
        }
    }
    *half = 0.5 * (two_pi - gap);
    *axis = ang[start] + *half;
    return true;
}

}  // namespace

bool build_segment_tree(const float* xy, int nv, int leaf, SegmentTreeHost* out) {
    if (nv < 2 || leaf < 1) return false;
    const int nseg = nv - 1;
    const int nleaves = (nseg + leaf - 1) / leaf;
    int P = 1;
    while (P < nleaves) P <<= 1;
    const int n_nodes = 2 * P - 1;
    out->first_leaf = P - 1;
    out->leaf = leaf;
    std::vector<float> node(8 * (size_t)n_nodes, 0.f);   // per node: box, cone

    // segment range [lo, hi] of every node (hi includes the right neighbour's
    // first segment: a vertex's silhouette test reads both adjacent segments)
    std::vector<int> lo(n_nodes, -1), hi(n_nodes, -1);
    for (int l = 0; l < P; ++l) {
        const int k = P - 1 + l;
        if (l * leaf < nseg) {
            lo[k] = l * leaf;
            hi[k] = std::min((l + 1) * leaf, nseg - 1);
        }
    }
    for (int k = P - 2; k >= 0; --k) {
        const int a = 2 * k + 1, b = 2 * k + 2;
        if (lo[a] < 0) continue;
        lo[k] = lo[a];
        hi[k] = lo[b] < 0 ? hi[a] : hi[b];
    }

    const float inf = std::numeric_limits<float>::infinity();
    float cmax = 0.f;
    for (int i = 0; i < 2 * nv; ++i) cmax = std::max(cmax, std::fabs(xy[i]));
    out->tol = std::ldexp(1.0f + cmax, -14);

    std::vector<double> ang;
    for (int k = 0; k < n_nodes; ++k) {
        float* box = &node[8 * (size_t)k];
        float* cone = box + 4;
        if (lo[k] < 0) {   // padding: inverted box, "no segment" cone
            box[0] = inf; box[1] = inf; box[2] = -inf; box[3] = -inf;
            cone[0] = 2.f; cone[1] = 0.f; cone[2] = 0.f; cone[3] = 0.f;
            continue;
        }
        float xmin = inf, ymin = inf, xmax = -inf, ymax = -inf;
        for (int v = lo[k]; v <= hi[k] + 1; ++v) {
            xmin = std::min(xmin, xy[2 * v]); xmax = std::max(xmax, xy[2 * v]);
            ymin = std::min(ymin, xy[2 * v + 1]); ymax = std::max(ymax, xy[2 * v + 1]);
        }
        box[0] = xmin; box[1] = ymin; box[2] = xmax; box[3] = ymax;

        ang.clear();
        for (int s = lo[k]; s <= hi[k]; ++s) {
            const double ux = (double)xy[2 * s + 2] - xy[2 * s], uy = (double)xy[2 * s + 3] - xy[2 * s + 1];
            if (ux != 0.0 || uy != 0.0) ang.push_back(std::atan2(uy, ux));
        }
        double axis = 0.0, half = 0.0;
        if (!enclosing_arc(ang, &axis, &half)) {
            cone[0] = 2.f; cone[1] = 0.f; cone[2] = 0.f; cone[3] = 0.f;   // only zero-length segments
        } else if (half >= 0.5 * M_PI - 0.01) {
            cone[0] = 3.f; cone[1] = 0.f; cone[2] = 0.f; cone[3] = 0.f;   // too wide to prune
        } else {
            half += 1e-6;   // cover the float rounding of the stored edges
            cone[0] = (float)std::cos(axis - half);
            cone[1] = (float)std::sin(axis - half);
            cone[2] = (float)std::cos(axis + half);
            cone[3] = (float)std::sin(axis + half);
        }
    }
    // child records of the internal nodes: {box(2k+1), box(2k+2), cone(2k+1), cone(2k+2)}
    out->rec.assign(16 * (size_t)(P - 1), 0.f);
    for (int k = 0; k < P - 1; ++k) {
        float* r = &out->rec[16 * (size_t)k];
        for (int c = 0; c < 2; ++c) {
            const float* nd = &node[8 * (size_t)(2 * k + 1 + c)];
            for (int q = 0; q < 4; ++q) {
                r[4 * c + q] = nd[q];          // box
                r[8 + 4 * c + q] = nd[4 + q];  // cone
            }
        }
    }
    return true;
}

}  // namespace wost
