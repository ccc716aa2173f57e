// wost_internal.h -- launch interface between libwost's host code (wost_api.hip,
// wost_jit.cpp) and its gfx950 kernels (wost_kernels.hip). Not part of the
// public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wost_walk.h"

namespace wost {

enum WalkMode : int {
    MODE_DIRICHLET = 0,      // Laplace, Dirichlet only
    MODE_POISSON = 1,        // + source, Green's sampler
    MODE_MIXED = 2,          // + Neumann polyline
    MODE_MIXED_POISSON = 3,  // + Neumann + source
    MODE_DELTA = 4,          // delta tracking (source required), Dirichlet only
    MODE_MIXED_DELTA = 5,    // delta tracking + Neumann
    // the mixed modes with the Neumann queries through the segment tree
    MODE_MIXED_TREE = 6,
    MODE_MIXED_POISSON_TREE = 7,
    MODE_MIXED_DELTA_TREE = 8,
    // compat="fixed" estimators (wost_walk.h FIX): Laplace, Poisson, mixed (Neumann scans)
    MODE_FIX_DIRICHLET = 9,
    MODE_FIX_POISSON = 10,
    MODE_FIX_MIXED = 11,
    MODE_FIX_MIXED_POISSON = 12,
    // compat="fixed" delta tracking (Q4/Q5 corrected sampler), Dirichlet only / + Neumann
    MODE_FIX_DELTA = 13,
    MODE_FIX_MIXED_DELTA = 14,
    // compat="fixed" mixed modes with the Neumann queries through the segment tree
    MODE_FIX_MIXED_TREE = 15,
    MODE_FIX_MIXED_POISSON_TREE = 16,
    MODE_FIX_MIXED_DELTA_TREE = 17,
    MODE_COUNT = 18
};

inline bool mode_fix(int m) { return m >= MODE_FIX_DIRICHLET && m <= MODE_FIX_MIXED_DELTA_TREE; }
inline bool mode_tree(int m) {
    return (m >= MODE_MIXED_TREE && m <= MODE_MIXED_DELTA_TREE) ||
           (m >= MODE_FIX_MIXED_TREE && m <= MODE_FIX_MIXED_DELTA_TREE);
}
inline bool mode_neu(int m) {
    return m == MODE_MIXED || m == MODE_MIXED_POISSON || m == MODE_MIXED_DELTA || mode_tree(m) ||
           m == MODE_FIX_MIXED || m == MODE_FIX_MIXED_POISSON || m == MODE_FIX_MIXED_DELTA;
}
inline bool mode_src(int m) {
    return m == MODE_POISSON || m == MODE_MIXED_POISSON || m == MODE_DELTA || m == MODE_MIXED_DELTA ||
           m == MODE_MIXED_POISSON_TREE || m == MODE_MIXED_DELTA_TREE || m == MODE_FIX_POISSON ||
           m == MODE_FIX_MIXED_POISSON || m == MODE_FIX_DELTA || m == MODE_FIX_MIXED_DELTA ||
           m == MODE_FIX_MIXED_POISSON_TREE || m == MODE_FIX_MIXED_DELTA_TREE;
}
inline bool mode_delta(int m) {
    return m == MODE_DELTA || m == MODE_MIXED_DELTA || m == MODE_MIXED_DELTA_TREE || m == MODE_FIX_DELTA ||
           m == MODE_FIX_MIXED_DELTA || m == MODE_FIX_MIXED_DELTA_TREE;
}

// const_d: the kernel has the Dirichlet polyline compiled in (field-specialised
// kernels, wost_jit.cpp), so it stages no copy; a Neumann polyline is always staged
// (const_n is kept for the callers).
inline size_t walk_lds_bytes(int mode, int nd, int nn, int n_points, int tree_lds = 0, bool const_d = false,
                             bool const_n = false, bool global_polylines = false, int block = kWalkBlock,
                             int tree_verts = 0) {
    (void)const_n;   // the Neumann polyline is always staged (unless global_polylines)
    return walk_lds_bytes_for(mode_neu(mode), mode_src(mode), nd, nn, n_points, mode_tree(mode), mode_delta(mode),
                              tree_lds, const_d, false, global_polylines, block, tree_verts);
}
// floats of the sampler / G_norm table buffer (WalkArgs::table); compat="fixed" delta
// tracking appends the corrected screened sampler's [kFixRows][kFixCols] nodes
inline size_t table_floats(bool delta, bool fixed_delta = false) {
    return (size_t)kSamplerFloatsPadded + (delta ? 4 * (size_t)kGnormCells : 0) +
           (fixed_delta ? (size_t)kFixTableFloats : 0);
}


// alpha at the query points with the interpreted fields (delta tracking)
hipError_t launch_point_alpha(const char* prog, const float2* pts, int64_t n, float* out, hipStream_t s);

// precompiled (interpreted-field) walk kernels
hipError_t walk_occupancy(int mode, int nd, int nn, int n_points, int* blocks_per_cu);
hipError_t launch_walk(int mode, const WalkArgs& a, int grid, hipStream_t s);

// Per-block reduction: block b covers local walks [begin[b], begin[b+1]).
// ns values per walk (multi-source: val[walk * ns + k]); rows of 2*ns+1 doubles
// (sum_k, sumsq_k for each k, then steps).
// ctl (may be null): the walk launch's control words (wost_walk.h kCtlWords), the queue
// head reset for the next walk launch. lstats (may be null): the solve's launch statistics
// [8] (wost_kernels.hip reduce_wave_stats) from the walk launch's n_waves per-wave records
// and its walks' step counts; first_batch: the solve's first launch.
hipError_t launch_block_reduce(const float* val, const uint32_t* steps, const int64_t* begin,
                               int64_t nblocks, int ns, double* out, unsigned long long* ctl,
                               hipStream_t s, int64_t n_waves = 0, unsigned long long* lstats = nullptr,
                               int first_batch = 1);

hipError_t launch_geometry_query(int op, const float2* verts, int nv, const float2* pts,
                                 const float2* dirs, const float* radii, int64_t n,
                                 float* out_f, uint8_t* out_mask, hipStream_t s);
// op 2 / 4 through the segment tree (records rec of SegmentTreeHost), one query per lane
hipError_t launch_geometry_tree_query(int op, const float2* verts, int nv, const float4* rec, int first_leaf,
                                      int depth, int leaf, float tol, float kmax, const float2* pts,
                                      const float2* dirs, const float* radii, int64_t n, float* out_f,
                                      hipStream_t s);

hipError_t launch_eval_field(const char* prog, int which, const float2* pts, int64_t n,
                             float4* out, hipStream_t s);

}  // namespace wost
