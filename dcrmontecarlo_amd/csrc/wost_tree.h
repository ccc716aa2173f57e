// wost_tree.h -- host construction of the Neumann segment tree that the
// walk kernels' TREE variants query (layout and exactness argument:
// wost_device.h, "Segment tree over a long Neumann polyline").
#pragma once

#include <vector>

namespace wost {

struct SegmentTreeHost {
    std::vector<float> node;   // 8 floats per node: box (xmin, ymin, xmax, ymax), direction-arc edges (e1, e2)
    int first_leaf = 0;        // index of the first leaf node
    int leaf = 0;              // segments per leaf
    float tol = 0.f;           // line-test tolerance at the origin
};

// Builds the tree of the polyline xy[2*nv] (nv >= 2) with `leaf` segments per
// leaf. Returns false for a degenerate input.
bool build_segment_tree(const float* xy, int nv, int leaf, SegmentTreeHost* out);

}  // namespace wost
