// wost_options.cpp -- see wost_options.h.
#include "wost_options.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace wost {
namespace {

// One named option: an int or double member, its range, whether it changes the
// generated kernel source, and whether only study builds accept it.
struct Spec {
    const char* name;
    int Options::* i;
    double Options::* d;
    double lo, hi;
    bool kernel;
    bool study;
    const char* env;   // the tools' A/B environment variable (study builds)
};

const Spec kSpecs[] = {
    {"tree_pool", &Options::tree_pool, nullptr, 0, 1, false, false, "WOST_TREE_POOL"},
    {"pool_near", nullptr, &Options::pool_near, 0, 1e30, false, false, "WOST_POOL_NEAR"},
    {"pool_slots", &Options::pool_slots, nullptr, 1, 4096, false, false, "WOST_POOL_SLOTS"},
    {"pool_near_waves", &Options::pool_near_waves, nullptr, 0, 16, false, false, "WOST_POOL_NEAR_WAVES"},
    {"pool_min_push", &Options::pool_min_push, nullptr, 1, 64, true, false, "WOST_JIT_POOL_MIN_PUSH"},
    {"tree_lds", &Options::tree_lds, nullptr, 0, 2, true, false, "WOST_TREE_LDS"},
    {"tree_lds_block", &Options::tree_lds_block, nullptr, 64, 1024, true, false, "WOST_TREE_LDS_BLOCK"},
    {"tree_share", &Options::tree_share, nullptr, -1, 64, true, false, "WOST_JIT_TREE_SHARE"},
    {"tree_share_min", &Options::tree_share_min, nullptr, -1, 64, true, false, "WOST_JIT_TREE_SHARE_MIN"},
    {"tree_share_descent", &Options::tree_share_descent, nullptr, -1, 1, true, false, "WOST_JIT_TREE_SHARE_DESCENT"},
    {"tree_batch", &Options::tree_batch, nullptr, -1, 4, true, false, "WOST_JIT_TREE_BATCH"},
    {"tree_qmargin", &Options::tree_qmargin, nullptr, -1, 1, true, false, "WOST_JIT_TREE_QMARGIN"},
    {"jit_waves", &Options::jit_waves, nullptr, 0, 8, true, false, "WOST_JIT_WAVES"},
    {"const_vertices", &Options::const_vertices, nullptr, 0, 256, true, false, "WOST_JIT_CONST_VERTICES"},
    {"jit_slp", &Options::jit_slp, nullptr, 0, 1, true, false, "WOST_JIT_SLP"},
    {"walk_block", &Options::walk_block, nullptr, 0, 1024, true, false, "WOST_WALK_BLOCK"},
    {"fused_scan", &Options::fused_scan, nullptr, 0, 1, true, false, nullptr},
    {"refill_min", &Options::refill_min, nullptr, -1, 64, true, false, "WOST_JIT_REFILL_MIN"},
    {"philox_ahead", &Options::philox_ahead, nullptr, -1, 3, true, false, "WOST_JIT_PHILOX_AHEAD"},
    {"param_sources", &Options::param_sources, nullptr, 0, 1, true, false, nullptr},
    {"jit_process", &Options::jit_process, nullptr, 0, 1, false, false, nullptr},
    {"jit_race", &Options::jit_race, nullptr, 0, 1, false, false, nullptr},
    {"chunk0", &Options::chunk0, nullptr, -1, 1024, false, false, "WOST_CHUNK0"},
    {"chunk_min", &Options::chunk_min, nullptr, -1, 1024, false, false, "WOST_CHUNK_MIN"},
    {"chunk_max", &Options::chunk_max, nullptr, -1, 1 << 20, false, false, "WOST_CHUNK_MAX"},
    {"adaptive_chunk", &Options::adaptive_chunk, nullptr, 0, 1, false, false, nullptr},
    {"grid_blocks_per_cu", &Options::grid_blocks_per_cu, nullptr, 0, 64, false, false, "WOST_GRID_BLOCKS_PER_CU"},
    {"lds_pad_bytes", &Options::lds_pad_bytes, nullptr, 0, 1 << 17, false, false, "WOST_LDS_PAD_BYTES"},
    {"exp_flags", &Options::exp_flags, nullptr, 0, 0x3FFFFFFF, true, true, "WOST_EXP_FLAGS"},
    {"tree_iter_stats", &Options::tree_iter_stats, nullptr, 0, 1, true, true, "WOST_TREE_ITER_STATS"},
};

const Spec* find(const char* name) {
    if (!name) return nullptr;
    for (const Spec& s : kSpecs)
        if (std::strcmp(s.name, name) == 0) return &s;
    return nullptr;
}

double value_of(const Options& o, const Spec& s) { return s.i ? (double)(o.*(s.i)) : o.*(s.d); }

}  // namespace

int options_study_build() {
#if defined(WOST_STUDY)
    return 1;
#else
    return 0;
#endif
}

int options_set(Options& o, const char* name, double value, bool* kernel_changed) {
    if (kernel_changed) *kernel_changed = false;
    const Spec* s = find(name);
    if (!s) return -1;
    if (s->study && !options_study_build()) return -3;
    if (!(value >= s->lo && value <= s->hi)) return -2;
    if (s->i && value != std::floor(value)) return -2;
    if (s->i && std::strcmp(s->name, "walk_block") == 0 && (int)value % 64 != 0) return -2;   // whole waves
    if (s->i && std::strcmp(s->name, "tree_lds_block") == 0 && (int)value % 64 != 0) return -2;
    const double old = value_of(o, *s);
    if (s->i) o.*(s->i) = (int)value;
    else o.*(s->d) = value;
    if (kernel_changed) *kernel_changed = s->kernel && old != value;
    return 0;
}

int options_get(const Options& o, const char* name, double* value) {
    const Spec* s = find(name);
    if (!s) return -1;
    if (value) *value = value_of(o, *s);
    return 0;
}

std::string options_report(const Options& o) {
    static const Options def;
    std::string out = std::string("{\"build\": \"") + (options_study_build() ? "study" : "product") +
                      "\", \"non_default\": {";
    bool first = true;
    char buf[96];
    for (const Spec& s : kSpecs) {
        const double v = value_of(o, s);
        if (v == value_of(def, s)) continue;
        std::snprintf(buf, sizeof(buf), "%s\"%s\": %.17g", first ? "" : ", ", s.name, v);
        out += buf;
        first = false;
    }
    if (o.jit_sched != def.jit_sched) {
        out += std::string(first ? "" : ", ") + "\"jit_sched\": \"" + o.jit_sched + "\"";
        first = false;
    }
    out += "}}";
    return out;
}

void options_from_study_env(Options& o) {
#if defined(WOST_STUDY)
    for (const Spec& s : kSpecs) {
        const char* e = s.env ? std::getenv(s.env) : nullptr;
        if (!e || !*e) continue;
        double v = std::atof(e);
        if (std::strcmp(s.name, "walk_block") == 0 || std::strcmp(s.name, "tree_lds_block") == 0)
            v = std::floor(v / 64.0) * 64.0;   // whole waves
        v = std::fmax(s.lo, std::fmin(s.hi, s.i ? std::floor(v) : v));
        if (s.i) o.*(s.i) = (int)v;
        else o.*(s.d) = v;
    }
    if (const char* e = std::getenv("WOST_JIT_SCHED")) o.jit_sched = e;
#else
    (void)o;
#endif
}

}  // namespace wost
