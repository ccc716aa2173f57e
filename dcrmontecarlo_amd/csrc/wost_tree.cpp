// wost_tree.cpp -- builds the implicit segment tree of a Neumann polyline
// (see wost_device.h for how the kernels traverse it and why the queries stay
// bit-identical to the reference's full scans).
#include "wost_tree.h"

#include <algorithm>
#include <cmath>
#include <cstring>
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
    int D = 1, P = 4;                       // leaves at level D, P = 4^D leaf slots
    while (P < nleaves) { P *= 4; ++D; }
    if (D > kTreeMaxDepth) return false;
    const int first_leaf = (P - 1) / 3;     // (4^D - 1) / 3 internal nodes
    const int n_nodes = first_leaf + P;
    out->first_leaf = first_leaf;
    out->depth = D;
    out->leaf = leaf;

    // segment range [lo, hi] of every node (hi includes the right neighbour's
    // first segment: a vertex's silhouette test reads both adjacent segments)
    std::vector<int> lo(n_nodes, -1), hi(n_nodes, -1);
    for (int l = 0; l < P; ++l) {
        const int k = first_leaf + l;
        if (l * leaf < nseg) {
            lo[k] = l * leaf;
            hi[k] = std::min((l + 1) * leaf, nseg - 1);
        }
    }
    for (int k = first_leaf - 1; k >= 0; --k) {
        for (int j = 0; j < kTreeArity; ++j) {
            const int c = kTreeArity * k + 1 + j;
            if (lo[c] < 0) continue;
            if (lo[k] < 0) lo[k] = lo[c];
            hi[k] = hi[c];
        }
    }

    float cmax = 0.f;
    for (int i = 0; i < 2 * nv; ++i) cmax = std::max(cmax, std::fabs(xy[i]));
    out->tol = std::ldexp(1.0f + cmax, -17);

    // per node: the oriented box around the arc's axis and the arc (see the header)
    std::vector<float> node((size_t)kTreeChildFloats * (size_t)n_nodes, 0.f);
    std::vector<double> ang;
    for (int k = 1; k < n_nodes; ++k) {   // (the root has no parent record)
        float* o = &node[(size_t)kTreeChildFloats * (size_t)k];
        if (lo[k] < 0) {                  // padding: never kept
            o[0] = o[1] = 0.f; o[2] = 1.f; o[3] = 0.f; o[4] = -1.f; o[5] = -1.f; o[6] = 2.f; o[7] = 0.f;
            continue;
        }
        ang.clear();
        for (int sg = lo[k]; sg <= hi[k]; ++sg) {
            const double ux = (double)xy[2 * sg + 2] - xy[2 * sg], uy = (double)xy[2 * sg + 3] - xy[2 * sg + 1];
            if (ux != 0.0 || uy != 0.0) ang.push_back(std::atan2(uy, ux));
        }
        double axis = 0.0, half = 0.0;
        int code = 0;
        if (!enclosing_arc(ang, &axis, &half)) code = 2;                 // only zero-length segments
        else if (half >= 0.5 * M_PI - 0.01) code = 3;                    // too wide to prune
        // the box is built around the float axis the kernels read
        const float fux = code == 0 ? (float)std::cos(axis) : 1.0f, fuy = code == 0 ? (float)std::sin(axis) : 0.0f;
        const double ux = fux, uy = fuy, nx = -uy, ny = ux;
        double tmin = 1e300, tmax = -1e300, smin = 1e300, smax = -1e300;
        for (int v = lo[k]; v <= hi[k] + 1; ++v) {
            const double x = xy[2 * v], y = xy[2 * v + 1];
            const double tt = x * ux + y * uy, ss = x * nx + y * ny;
            tmin = std::min(tmin, tt); tmax = std::max(tmax, tt);
            smin = std::min(smin, ss); smax = std::max(smax, ss);
        }
        const double tc = 0.5 * (tmin + tmax), sc = 0.5 * (smin + smax);
        const double cx = tc * ux + sc * nx, cy = tc * uy + sc * ny;
        // inflate by far more than the rounding of the stored centre and of the
        // kernels' corner arithmetic, so that the float box holds every vertex
        const double slack = 16.0 * std::ldexp(1.0, -24) * (std::fabs(cx) + std::fabs(cy) + 0.5 * (tmax - tmin) +
                                                             0.5 * (smax - smin)) + 1e-30;
        const double a = (0.5 * (tmax - tmin) + slack) * (1.0 + std::ldexp(1.0, -20));
        const double b = (0.5 * (smax - smin) + slack) * (1.0 + std::ldexp(1.0, -20));
        o[0] = (float)cx; o[1] = (float)cy; o[2] = fux; o[3] = fuy; o[4] = (float)a; o[5] = (float)b;
        if (code == 0) {
            half += 1e-6;   // cover the float rounding of the axis and of the kernels' edge vectors
            o[6] = (float)std::cos(half);
            o[7] = (float)std::sin(half);
        } else {
            o[6] = (float)code;
            o[7] = 0.f;
        }
    }
    double kmax = 0.0;
    for (int k = 1; k < n_nodes; ++k) {
        const float* o = &node[(size_t)kTreeChildFloats * (size_t)k];
        if (o[4] < 0.f) continue;
        kmax = std::max(kmax, std::fabs((double)o[0]) + std::fabs((double)o[1]) + 2.0 * ((double)o[4] + o[5]));
    }
    out->kmax = (float)(kmax * (1.0 + std::ldexp(1.0, -10)));
    // child records of the internal nodes
    out->rec.assign((size_t)kTreeNodeFloats * (size_t)first_leaf, 0.f);
    for (int k = 0; k < first_leaf; ++k)
        for (int j = 0; j < kTreeArity; ++j)
            std::memcpy(&out->rec[(size_t)kTreeNodeFloats * k + (size_t)kTreeChildFloats * j],
                        &node[(size_t)kTreeChildFloats * (size_t)(kTreeArity * k + 1 + j)],
                        sizeof(float) * kTreeChildFloats);
    return true;
}

}  // namespace wost
