// wost_internal.h -- launch interface between libwost's host code (wost_api.hip)
// and its gfx950 kernels (wost_kernels.hip). Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wost {

// Arguments of the walk kernel, passed by value in the kernarg segment.
struct WalkArgs {
    const float2* points;        // [n_points] query points
    const float2* dverts;        // Dirichlet polyline vertices
    const float2* nverts;        // Neumann polyline vertices (may be null)
    const float* table;          // sampler inverse-CDF nodes (may be null)
    const char* prog;            // DProgram + terms + factors
    float* out_val;              // [count] per-walk estimate
    uint32_t* out_steps;         // [count] per-walk step count
    unsigned long long* counter; // work-queue head (zeroed before launch)
    int64_t wid_begin;           // global id of local walk 0
    int64_t count;               // walks in this launch
    int64_t walks_per_point;     // W: point of global walk g is g / W
    int32_t nd, nn;              // vertex counts
    int32_t max_steps;
    float eps;
    float rmin;                  // eps / 2 (solvers/WoStSolver.py:167)
    uint32_t key0, key1;         // Philox key = seed
    int32_t chunk;               // walks claimed per work-queue dequeue
    int32_t n_points;            // query points (staged in LDS when <= kLdsPointsMax)
    double inv_walks_per_point;  // 1/W for the point index of a walk id
};

constexpr int kLdsPointsMax = 1024;

enum WalkMode : int {
    MODE_DIRICHLET = 0,      // Laplace, Dirichlet only
    MODE_POISSON = 1,        // + source, Green's sampler
    MODE_MIXED = 2,          // + Neumann polyline
    MODE_MIXED_POISSON = 3,  // + Neumann + source
    MODE_DELTA = 4,          // delta tracking (source required), Dirichlet only
    MODE_MIXED_DELTA = 5     // delta tracking + Neumann
};

size_t walk_lds_bytes(int mode, int nd, int nn, int n_points);
hipError_t walk_occupancy(int mode, int nd, int nn, int n_points, int* blocks_per_cu);
hipError_t launch_walk(int mode, const WalkArgs& a, int grid, hipStream_t s);

// Per-block reduction: block b covers local walks [begin[b], begin[b+1]).
hipError_t launch_block_reduce(const float* val, const uint32_t* steps, const int64_t* begin,
                               int64_t nblocks, double* out, hipStream_t s);

hipError_t launch_geometry_query(int op, const float2* verts, int nv, const float2* pts,
                                 const float2* dirs, const float* radii, int64_t n,
                                 float* out_f, uint8_t* out_mask, hipStream_t s);

hipError_t launch_eval_field(const char* prog, int which, const float2* pts, int64_t n,
                             float4* out, hipStream_t s);

constexpr int kWalkBlock = 256;

}  // namespace wost
