// wost_options.h -- a handle's kernel and launch choices (wost_set_option).
//
// Every option here selects HOW the walks run -- workgroup size, LDS staging, work-queue
// chunks, the walk pools, the tree queries' hand-outs -- never WHAT they compute: each
// walk's value and step count depend only on (seed, walk id), and the GPU tests check
// every option below against the default walk for walk (tests/test_gpu_c5.py,
// test_segment_tree.py, test_gpu_queue.py). The product library reads them from the
// handle only (wost_set_option); it reads no environment variable that changes a kernel
// or a result. Non-default values are reported by wost_options_report, and bench.py
// refuses to print a metric when any is set.
//
// Study builds (make study: build/libwost_study.so, -DWOST_STUDY) additionally seed the
// options from the A/B environment variables of tools/ (WOST_POOL_SLOTS, WOST_CHUNK0, ...)
// and accept the result-changing ablations (WOST_EXP_FLAGS, timing studies only: their
// walks are wrong by design) and the tree queries' loop counters (WOST_TREE_ITER_STATS).
#pragma once

#include <cstddef>
#include <string>

namespace wost {

// Polylines of at most this many vertices are compiled into the specialised kernel.
constexpr int kJitMaxConstVertices = 40;

struct Options {
    // walk pools of the tree kernels (wost_walk.h): on/off, near margin (fraction of the
    // Neumann polyline's largest extent), parked walks per class and workgroup, the waves
    // that take the near class (0: each wave takes its majority class)
    int tree_pool = 1;
    double pool_near = 0.1;
    int pool_slots = 128;
    int pool_near_waves = 2;
    int pool_min_push = 1;          // fewest walks a wave parks (WOST_POOL_MIN_PUSH)
    // segment-tree staging level cap (2: records + vertices, 1: records, 0: none) and the
    // workgroup of level 1
    int tree_lds = 2;
    int tree_lds_block = 512;
    // the tree queries' hand-outs of pending subtrees and record batches (wost_walk.h)
    int tree_share = -1;            // -1: the kernel's default (WOST_TREE_SHARE)
    int tree_share_min = -1;
    int tree_share_descent = -1;
    int tree_batch = -1;
    int tree_qmargin = -1;
    // field-specialised kernels: waves per SIMD of the register budget (0: by kernel kind),
    // polylines compiled in up to this many vertices, the SLP vectoriser, the scan
    // kernels' workgroup (0: 256), both brute-force Neumann queries in one pass
    int jit_waves = 0;
    int const_vertices = kJitMaxConstVertices;
    int jit_slp = 0;
    int walk_block = 0;
    int fused_scan = 1;
    int refill_min = -1;            // idle lanes that trigger a refill (-1: WOST_REFILL_MIN)
    int philox_ahead = -1;          // Philox words one step ahead (-1: off)
    int param_sources = 0;          // multi-source kernels read the sources' parameters from the
                                    // program buffer (one compile per source structure; wost_jit.cpp)
    int jit_process = 1;            // compile in the helper process wost_jitc (the same code object;
                                    // concurrent handles' compiles overlap), 0: in this process
    int jit_race = 1;               // a whole solve whose specialised kernel is in no cache runs on the
                                    // precompiled kernel while it compiles (wost_api.hip solve_race)
    // work queue (wost_api.hip solve_impl; -1 / 0: the call's own shape)
    int chunk0 = -1;
    int chunk_min = -1;
    int chunk_max = -1;
    int adaptive_chunk = 1;         // waves size their dequeues from their own measured walks
    int grid_blocks_per_cu = 0;
    int lds_pad_bytes = 0;
    // study builds only (never settable in the product library)
    int exp_flags = 0;              // result-changing ablations (wost_jit.cpp)
    int tree_iter_stats = 0;        // the tree queries' loop counters
    std::string jit_sched;          // -mllvm -amdgpu-sched-strategy=<...>
};

// 1 in study builds (-DWOST_STUDY), else 0.
int options_study_build();
// The option `name` := value (range-checked). Returns 0, -1 unknown name, -2 bad value,
// -3 a study-only option in the product library. *kernel_changed: the option changes the
// generated kernel source (the handle's cached kernel must be rebuilt).
int options_set(Options& o, const char* name, double value, bool* kernel_changed);
int options_get(const Options& o, const char* name, double* value);
// {"build": "product"|"study", "non_default": {name: value, ...}}
std::string options_report(const Options& o);
// Study builds: seed o from the tools' A/B environment variables (no-op otherwise).
void options_from_study_env(Options& o);

}  // namespace wost
