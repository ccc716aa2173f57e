// wost_tree.h -- host construction of the Neumann segment tree that the
// walk kernels' TREE variants query (layout and exactness argument:
// wost_device.h, "Segment tree over a long Neumann polyline").
#pragma once

#include <vector>

namespace wost {

// floats per child description (oriented box + direction arc) and per internal node
constexpr int kTreeChildFloats = 8;
constexpr int kTreeArity = 4;
constexpr int kTreeNodeFloats = kTreeArity * kTreeChildFloats;
// the traversals keep 4 pending-child bits per level in 32 bits: at most 8 levels
// below the root (4^8 leaves, 2^21 segments at 32 per leaf)
constexpr int kTreeMaxDepth = 8;

struct SegmentTreeHost {
    std::vector<float> rec;    // kTreeNodeFloats per internal node k: for child j = 0..3 (node 4k+1+j)
                               // {cx, cy, ux, uy, a, b, cos h, sin h}: the oriented box centred at c
                               // with unit axis u, half-length a along u and half-width b across it,
                               // and the half-angle h of the arc of segment directions around u
                               // (cos h = 2: no segment direction; 3: arc too wide to use; a < 0: padding)
    int first_leaf = 0;        // index of the first leaf node = number of internal nodes
    int depth = 0;             // level of the leaves (the root is level 0)
    int leaf = 0;              // segments per leaf
    float tol = 0.f;           // line-test tolerance at the origin; grows with |q|
    float kmax = 0.f;          // max over the child boxes of |cx| + |cy| + 2 (a + b), rounded up: with
                               // |p|_1 it bounds every per-child rounding scale of the silhouette tests
};

// Builds the 4-ary tree of the polyline xy[2*nv] (nv >= 2) with `leaf` segments per
// leaf (the leaf count padded to a power of 4). Returns false for a degenerate input
// or a tree deeper than kTreeMaxDepth.
bool build_segment_tree(const float* xy, int nv, int leaf, SegmentTreeHost* out);

}  // namespace wost
