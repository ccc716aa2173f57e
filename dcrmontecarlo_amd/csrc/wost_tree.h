// wost_tree.h -- host construction of the Neumann segment tree that the
// walk kernels' TREE variants query (layout and exactness argument:
// wost_device.h, "Segment tree over a long Neumann polyline").
#pragma once

#include <vector>

namespace wost {

struct SegmentTreeHost {
    std::vector<float> rec;    // 16 floats per internal node k: its children's boxes (xmin, ymin, xmax, ymax)
                               // then their direction-arc edges (e1, e2): box(2k+1), box(2k+2), cone(2k+1), cone(2k+2)
    int first_leaf = 0;        // index of the first leaf node = number of internal nodes
    int leaf = 0;              // segments per leaf
    float tol = 0.f;           // line-test tolerance at the origin
};

// Builds the tree of the polyline xy[2*nv] (nv >= 2) with `leaf` segments per
// leaf. Returns false for a degenerate input.
bool build_segment_tree(const float* xy, int nv, int leaf, SegmentTreeHost* out);

}  // namespace wost
