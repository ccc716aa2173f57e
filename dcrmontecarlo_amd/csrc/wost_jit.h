// wost_jit.h -- field-specialised walk kernels compiled at run time (hiprtc).
//
// The precompiled walk kernel interprets each handle's coefficient fields
// from a program buffer (a term/factor loop with a kind switch per factor).
// For a given handle and kernel variant, libwost instead generates HIP source
// in which the fields are straight-line calls to the same per-kind functions
// (wost_device.h) with their parameters as literals, compiles it for the
// device's gfx target with hiprtc, caches the code object (in memory and on
// disk) and launches it with the same WalkArgs. Results are identical to the
// interpreted kernel; the interpretation overhead disappears.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "wost_device.h"
#include "wost_options.h"

namespace wost {

// Which polylines a specialised kernel of `mode` compiles in (at most
// Options::const_vertices vertices, default kJitMaxConstVertices; they are then not
// staged in LDS).
bool jit_const_dirichlet(const Options& o, int nd);
bool jit_const_neumann(const Options& o, int mode, int nn);
// a long Neumann polyline scanned without the segment tree (the brute-force kernel, reference
// mode): both queries of a step in one pass (wost_device.h neumann_scan_both)
bool jit_fused_neumann_scan(const Options& o, int mode, int nn);

// HIP source of a walk kernel named "wost_walk_jit" for walk mode `mode`
// (wost_internal.h WalkMode) with the fields of `prog` and short polylines
// (Dirichlet dverts[2*nd], Neumann nverts[2*nn]) compiled in; `record`: the
// kernel can record walks (return_history); `n_sources` > 1: the walk scores
// sources SLOT_F, SLOT_EXTRA.. (multi-source batching).
// `block`: threads per workgroup the kernel is launched with; seg_phi: the
// device's per-segment normal angles of a compiled-in Neumann polyline (nn - 1
// floats, read back from the setup kernel so the constants carry its bits);
// global_polylines: the kernel reads polylines that are not compiled in from
// global memory instead of staging them in LDS (wost_walk.h GL). tree_stage (tree
// modes): 0 = the segment tree through L1/L2, 1 = its records staged in LDS
// (WOST_TREE_STAGED), 2 = its records and the Neumann vertices (WOST_TREE_VSTAGED) --
// the caller's staging decision, independent of the workgroup size.
// `opt`: the handle's kernel options (wost_options.h).
std::string jit_generate(const Options& opt, int mode, const DProgram& hdr, const DTerm* terms, const DFactor* factors,
                         const float* dverts, int nd, const float* nverts, int nn, bool record,
                         int n_sources = 1, int block = 256, const float* seg_phi = nullptr,
                         bool global_polylines = false, int tree_stage = 0, bool exact_trig = true);

// Compiles (or fetches from the caches) the source for `device` and returns
// the kernel. On failure returns false and a message in *err.
// alpha_fn (optional): the source's wost_point_alpha_jit kernel (delta tracking), or null.
// opt: the compile options it selects (the SLP vectoriser; study builds: the scheduler).
// *compile_ms: host time of the hiprtc compile (0 when a cache had the code).
bool jit_get_kernel(const Options& opt, int device, const std::string& source, hipFunction_t* fn, std::string* err,
                    hipFunction_t* alpha_fn = nullptr, double* compile_ms = nullptr);

// Background compiles for a solve that can run on the precompiled kernel meanwhile
// (option jit_race, wost_api.hip solve_race): jit_try_kernel returns
//   kReady   -- *fn is the kernel (in memory, on disk, or a finished background compile);
//   kStarted -- it was nowhere and nothing compiled it: a compile started now in a helper
//               process (a detached thread waits for it and fills the disk cache); *ticket
//               says when it is done, and jit_get_kernel then loads it without compiling;
//   kWait    -- only a blocking jit_get_kernel gets it (a compile of it is already running,
//               or failed, or there is no helper).
enum class JitTry { kReady, kStarted, kWait };
struct JitTicket {
    const void* p = nullptr;
    bool done() const;
};
JitTry jit_try_kernel(const Options& opt, int device, const std::string& source, hipFunction_t* fn,
                      hipFunction_t* alpha_fn, JitTicket* ticket, std::string* err);

// A compile of `source` for `arch` with the options `opt` selects, without a device (the
// helper process wost_jitc when there is one and opt.jit_process is set, else in this
// process; *in_helper says which ran). For wost_jit_compile and the tests.
bool jit_compile_host(const Options& opt, const std::string& source, const std::string& arch,
                      std::vector<char>* code, std::string* err, bool* in_helper);
// Whether the compile helper is installed next to this library (and runs).
bool jit_helper_available();
// Starts finding the helper's compiler in the background (once per process; wost_create),
// so that the first compile does not wait for the helper's start.
void jit_start_identity_probe();

}  // namespace wost
