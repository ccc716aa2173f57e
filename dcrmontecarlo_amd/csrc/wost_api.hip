// wost_api.hip -- host side of libwost.so: the C ABI of include/wost.h.
//
// Mirrors the control flow around the reference's hot loop:
//   wost_create  <- WostSolver_2D.__init__ / buildModifiedSigma (solvers/WoStSolver.py:22-138)
//   wost_solve   <- WostSolver_2D.solve / _solveUnified        (solvers/WoStSolver.py:162-353)
// and owns the device state: geometry, field programs, sampler table,
// per-walk workspace and the walk/reduce launches on a private HIP stream.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <map>
#include <thread>
#include <set>
#include <mutex>
#include <string>
#include <vector>

#include "wost_device.h"
#include "wost_internal.h"
#include "wost_jit.h"
#include "wost_options.h"
#include "wost_tables.h"
#include "wost_tree.h"

using namespace wost;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(WOST_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

struct HostField {
    bool present = false;
    int flags = 0;
    std::vector<DTerm> terms;      // first = index into this field's factors
    std::vector<DFactor> factors;
    std::vector<float> grid;       // FK_GRID values; p6 = offset into this field's grid
};

int convert_field(const wost_field* in, HostField& out, const char* name) {
    out = HostField();
    if (!in) return WOST_OK;
    if (in->n_terms < 0 || in->n_factors < 0 || (in->n_terms > 0 && !in->terms) ||
        (in->n_factors > 0 && !in->factors))
        return fail(WOST_ERR_INVALID_ARG, "field %s: bad term/factor arrays", name);
    if (in->n_terms > 4096 || in->n_factors > 16384)
        return fail(WOST_ERR_INVALID_ARG, "field %s: too many terms/factors", name);
    if (in->n_grid < 0 || in->n_grid > WOST_MAX_GRID_VALUES || (in->n_grid > 0 && !in->grid))
        return fail(WOST_ERR_INVALID_ARG, "field %s: bad grid array (%lld values)", name, (long long)in->n_grid);
    out.present = true;
    out.flags = in->flags;
    for (int i = 0; i < in->n_factors; ++i) {
        const wost_factor& f = in->factors[i];
        if (f.kind < WOST_FK_MONO || f.kind > WOST_FK_GRID)
            return fail(WOST_ERR_INVALID_ARG, "field %s: factor %d has unknown kind %d", name, i, f.kind);
        if (f.kind == WOST_FK_GRID) {
            const float nx = f.p[4], ny = f.p[5], off = f.p[6];
            const bool ints = nx == std::floor(nx) && ny == std::floor(ny) && off == std::floor(off);
            if (!ints || !(nx >= 2.f && ny >= 2.f && off >= 0.f) ||
                (double)off + (double)nx * (double)ny > (double)in->n_grid)
                return fail(WOST_ERR_INVALID_ARG, "field %s: grid factor %d (%g x %g at %g) exceeds the %lld grid values",
                            name, i, nx, ny, off, (long long)in->n_grid);
            if (!(std::isfinite(f.p[0]) && std::isfinite(f.p[1]) && f.p[2] > 0.f && f.p[3] > 0.f &&
                  std::isfinite(f.p[2]) && std::isfinite(f.p[3])))
                return fail(WOST_ERR_INVALID_ARG, "field %s: grid factor %d has a bad origin or spacing", name, i);
        }
        if (f.kind == WOST_FK_MONO) {
            for (int q = 0; q < 2; ++q) {
                float e = f.p[q];
                if (!(e >= 0.f && e <= 15.f) || e != std::floor(e))
                    return fail(WOST_ERR_INVALID_ARG, "field %s: monomial exponent %g not an integer in [0,15]", name, e);
            }
        }
        DFactor d{};
        d.kind = f.kind;
        for (int q = 0; q < 8; ++q) d.p[q] = f.p[q];
        out.factors.push_back(d);
    }
    for (int t = 0; t < in->n_terms; ++t) {
        const wost_term& tm = in->terms[t];
        if (tm.n_factors < 0 || tm.first_factor < 0 || tm.first_factor + tm.n_factors > in->n_factors)
            return fail(WOST_ERR_INVALID_ARG, "field %s: term %d references factors out of range", name, t);
        DTerm d{};
        d.coef = tm.coef;
        d.first = tm.first_factor;
        d.nf = tm.n_factors;
        out.terms.push_back(d);
    }
    if (in->n_grid > 0) out.grid.assign(in->grid, in->grid + in->n_grid);
    return WOST_OK;
}

// Flattened program for the device (and for host-side evaluation).
struct Program {
    std::vector<unsigned char> bytes;
    const DProgram* hdr() const { return reinterpret_cast<const DProgram*>(bytes.data()); }
    const DTerm* terms() const { return reinterpret_cast<const DTerm*>(bytes.data() + sizeof(DProgram)); }
    const DFactor* factors() const {
        return reinterpret_cast<const DFactor*>(bytes.data() + sizeof(DProgram) +
                                                sizeof(DTerm) * hdr()->n_terms_total);
    }
    const float* grid() const {
        return reinterpret_cast<const float*>(bytes.data() +
                                              program_grid_offset(hdr()->n_terms_total, hdr()->n_factors_total));
    }
};

// f: N_FIELDS fields (absent ones empty)
void build_program(const HostField* f, double sigma_bar, Program& out) {
    DProgram hdr{};
    std::vector<DTerm> terms;
    std::vector<DFactor> factors;
    std::vector<float> grid;
    for (int s = 0; s < N_FIELDS; ++s) {
        hdr.field[s].present = f[s].present ? 1 : 0;
        hdr.field[s].flags = f[s].flags;
        hdr.field[s].first_term = (int)terms.size();
        hdr.field[s].n_terms = (int)f[s].terms.size();
        const int fbase = (int)factors.size();
        const float gbase = (float)grid.size();   // exact: < 2^24 per field, checked on input
        for (DTerm t : f[s].terms) {
            t.first += fbase;
            terms.push_back(t);
        }
        for (DFactor d : f[s].factors) {
            if (d.kind == WOST_FK_GRID) d.p[6] += gbase;
            factors.push_back(d);
        }
        grid.insert(grid.end(), f[s].grid.begin(), f[s].grid.end());
    }
    hdr.sigma_bar = (float)sigma_bar;
    hdr.sqrt_sigma_bar = (float)std::sqrt(sigma_bar > 0 ? sigma_bar : 0.0);
    hdr.inv_sigma_bar = sigma_bar > 0 ? (float)(1.0 / sigma_bar) : 0.f;
    hdr.n_terms_total = (int)terms.size();
    hdr.n_factors_total = (int)factors.size();
    hdr.n_grid_total = (int)grid.size();
    const size_t goff = program_grid_offset(hdr.n_terms_total, hdr.n_factors_total);
    out.bytes.assign(goff + sizeof(float) * grid.size(), 0);
    std::memcpy(out.bytes.data(), &hdr, sizeof(hdr));
    if (!terms.empty())
        std::memcpy(out.bytes.data() + sizeof(DProgram), terms.data(), sizeof(DTerm) * terms.size());
    if (!factors.empty())
        std::memcpy(out.bytes.data() + sizeof(DProgram) + sizeof(DTerm) * terms.size(), factors.data(),
                    sizeof(DFactor) * factors.size());
    if (!grid.empty()) std::memcpy(out.bytes.data() + goff, grid.data(), sizeof(float) * grid.size());
}

// torch.linspace(start, end, steps) in float32 (ATen CPU kernel: the first half
// counts up from start, the second half down from end).
std::vector<float> torch_linspace(float start, float end, int steps) {
    std::vector<float> v(steps);
    if (steps == 1) { v[0] = start; return v; }
    const float step = (end - start) / (float)(steps - 1);
    const int half = steps / 2;
    for (int i = 0; i < steps; ++i)
        v[i] = i < half ? start + step * (float)i : end - step * (float)(steps - i - 1);
    return v;
}

}  // namespace

struct wost_handle {
    int device = 0;
    int compat = WOST_COMPAT_REFERENCE;
    int num_cus = 0;
    std::vector<float> dverts, nverts;
    HostField fields[N_FIELDS];   // N_SLOTS problem fields, then sources 1.. of wost_set_sources
    int n_sources = 1;
    bool delta = false;
    double sigma_bar = 0.0;
    Program prog;
    std::vector<float> table;   // sampler nodes (built on first use)
    bool table_ready = false;
    bool prog_dirty = true;
    uint64_t prog_version = 0;  // bumped whenever the program is rebuilt

    // compat="fixed" delta tracking: refuse solves whose walks would all hit maxSteps
    bool fixed_step_check = true;
    int trig_mode = WOST_TRIG_AUTO;       // wost_set_trig

    // kernel and launch options (wost_set_option; study builds: also the A/B environment)
    Options opt;

    // field-specialised walk kernel (wost_jit.cpp)
    bool jit_enabled = true;
    hipFunction_t jit_fn = nullptr;
    hipFunction_t jit_alpha_fn = nullptr;   // the same module's wost_point_alpha_jit (delta modes)
    int jit_mode = -1;
    uint64_t jit_version = ~0ull;
    std::string jit_error;

    // Neumann segment tree (wost_tree.h): used when the Neumann polyline has at
    // least tree_min_segments segments (< 0: never)
    int tree_min_segments = WOST_TREE_MIN_SEGMENTS_DEFAULT;
    int tree_leaf = WOST_TREE_LEAF_DEFAULT;
    bool tree_ready = false;
    SegmentTreeHost tree;
    float* d_tree = nullptr;

    hipStream_t stream = nullptr;
    hipEvent_t ev[6] = {};
    float2* d_dverts = nullptr;
    float2* d_nverts = nullptr;
    float* d_seg_phi = nullptr;
    float* d_table = nullptr;
    char* d_prog = nullptr;
    size_t d_prog_cap = 0;
    unsigned long long* d_counter = nullptr;   // the walk launches' control words (wost_walk.h kCtlWords)
    int64_t ctl_cap = 0;                       // ... words allocated
    float* d_val = nullptr;
    uint32_t* d_steps = nullptr;
    int64_t ws_cap = 0, ws_val_cap = 0;
    int64_t* d_begin = nullptr;       // (d_points and d_begin point into d_stage)
    char* d_stage = nullptr;          // device image of the pinned staging's [points | block ranges]
    size_t stage_cap = 0;
    double* d_bstats = nullptr;
    int64_t bstats_cap = 0;
    float2* d_points = nullptr;
    float* d_point_alpha = nullptr;   // alpha at the query points (delta tracking)
    int64_t point_alpha_cap = 0;
    uint32_t* d_pool = nullptr;       // walk pools of the tree kernels' workgroups (WalkArgs::pool)
    int64_t pool_cap = 0;
    double tick_khz = 100000.0;       // the device wall clock (hipDeviceAttributeWallClockRate)
    // pinned host staging of a solve's small copies (points, block ranges, block sums):
    // a pageable hipMemcpyAsync costs ~9 us of host time each (profiles/r05_ab/host_path/)
    char* h_pin = nullptr;
    size_t pin_cap = 0;
    bool counter_zero = false;        // d_counter is 0 (the block reduce resets it after each walk launch)
    wost_timing timing{};
};

namespace {

constexpr int64_t kMaxBatchWalks = int64_t(1) << 26;   // 64 Mi walks = 512 MiB of per-walk results
// Above this many bytes of staged polylines per workgroup (4 workgroups of 256 on a
// 160 KiB CU, 4 waves per SIMD) the field-specialised kernel reads the polylines from
// global memory instead (wost_walk.h GL): long Dirichlet polylines, and long Neumann
// polylines under compat="fixed" (which scans them), work at any length.
constexpr size_t kGlobalPolylineLdsBytes = 40 * 1024;

// The solve's launch statistics (the walk kernel's per-wave records, wost_block_reduce)
// ride in front of the block sums in d_bstats, so that one copy brings both to the host.
constexpr int64_t kLstatsWords = 8;

int upload_program(wost_handle* h) {
    if (!h->prog_dirty) return WOST_OK;
    build_program(h->fields, h->sigma_bar, h->prog);
    if (h->prog.bytes.size() > h->d_prog_cap) {
        if (h->d_prog) (void)hipFree(h->d_prog);
        h->d_prog = nullptr;
        HIP_TRY(hipMalloc(&h->d_prog, h->prog.bytes.size()));
        h->d_prog_cap = h->prog.bytes.size();
    }
    HIP_TRY(hipMemcpy(h->d_prog, h->prog.bytes.data(), h->prog.bytes.size(), hipMemcpyHostToDevice));
    h->prog_dirty = false;
    ++h->prog_version;
    return WOST_OK;
}

// The field-specialised kernel for `mode` (with the walk recorder compiled in
// when `record`), or nullptr when it is disabled or could not be built (the
// precompiled kernel is used then; same results).
// wost_set_trig's choice for this handle: WOST_TRIG_AUTO is exact for a Neumann polyline
// of >= 3 segments (a curved boundary, where a direction's last ulp decides where the
// walk goes), the hardware's sin/cos otherwise
bool exact_trig_of(const wost_handle* h) {
    if (h->trig_mode != WOST_TRIG_AUTO) return h->trig_mode == WOST_TRIG_EXACT;
    return (int)(h->nverts.size() / 2) - 1 >= 3;
}

// The source of the field-specialised kernel for `mode` with the program `prog` (the
// handle's own, or wost_prepare_multi's with other sources): the handle's polylines,
// options and trig choice, the launch's workgroup, staging and polyline placement.
int jit_source(const wost_handle* h, const Program& prog, int mode, bool record, int ns, int block,
               bool global_polylines, int tree_stage, std::string* src) {
    const int nn = (int)(h->nverts.size() / 2);
    std::vector<float> phi;   // a compiled-in Neumann polyline carries the device's segment angles
    if (jit_const_neumann(h->opt, mode, nn) && nn >= 2) {
        phi.resize(nn - 1);
        HIP_TRY(hipMemcpy(phi.data(), h->d_seg_phi, sizeof(float) * phi.size(), hipMemcpyDeviceToHost));
    }
    *src = jit_generate(h->opt, mode, *prog.hdr(), prog.terms(), prog.factors(), h->dverts.data(),
                        (int)(h->dverts.size() / 2), h->nverts.data(), nn, record, ns, block,
                        phi.empty() ? nullptr : phi.data(), global_polylines, tree_stage, exact_trig_of(h));
    return WOST_OK;
}

// The handle's key of a kernel variant: everything its source depends on besides the
// program (prog_version): the staging level, the exact workgroup size (a multiple of 64,
// at most 1024) and the trig choice
int jit_key(const wost_handle* h, int mode, bool record, int ns, int block, bool global_polylines, int tree_stage) {
    const bool exact = exact_trig_of(h);
    return (((((2 * mode + (record ? 1 : 0)) * (WOST_MAX_SOURCES + 1) + ns) * 3 + tree_stage) * 17 + block / 64) * 2 +
            (global_polylines ? 1 : 0)) * 2 + (exact ? 1 : 0);
}

// jit_kernel without blocking on a compile (option jit_race): kReady with the handle's
// kernel set, kStarted when its compile began now in the background (ticket), else kWait.
JitTry jit_kernel_try(wost_handle* h, int mode, int block, bool global_polylines, int tree_stage, JitTicket* ticket) {
    if (!h->jit_enabled) return JitTry::kWait;
    const int key = jit_key(h, mode, false, 1, block, global_polylines, tree_stage);
    if (h->jit_mode == key && h->jit_version == h->prog_version && h->jit_fn) return JitTry::kReady;
    std::string src, err;
    if (jit_source(h, h->prog, mode, false, 1, block, global_polylines, tree_stage, &src) != WOST_OK)
        return JitTry::kWait;
    hipFunction_t fn = nullptr, afn = nullptr;
    const JitTry r = jit_try_kernel(h->opt, h->device, src, &fn, &afn, ticket, &err);
    if (r == JitTry::kReady && (!mode_delta(mode) || afn)) {
        h->jit_mode = key;
        h->jit_version = h->prog_version;
        h->jit_fn = fn;
        h->jit_alpha_fn = afn;
    }
    return r;
}

hipFunction_t jit_kernel(wost_handle* h, int mode, bool record, int ns = 1, int block = kWalkBlock,
                         bool global_polylines = false, int tree_stage = 0, double* compile_ms = nullptr) {
    if (!h->jit_enabled) return nullptr;
    const int key = jit_key(h, mode, record, ns, block, global_polylines, tree_stage);
    if (h->jit_mode == key && h->jit_version == h->prog_version) return h->jit_fn;
    h->jit_fn = nullptr;
    h->jit_alpha_fn = nullptr;
    h->jit_mode = key;
    h->jit_version = h->prog_version;
    std::string src;
    if (jit_source(h, h->prog, mode, record, ns, block, global_polylines, tree_stage, &src) != WOST_OK) return nullptr;
    std::string err;
    hipFunction_t fn = nullptr;
    hipFunction_t afn = nullptr;
    double cms = 0.0;
    const bool ok = jit_get_kernel(h->opt, h->device, src, &fn, &err, &afn, &cms);
    if (compile_ms) *compile_ms += cms;
    if (!ok) {
        h->jit_error = err;
        std::fprintf(stderr, "libwost: field-specialised kernel unavailable, using the precompiled one: %s\n",
                     err.c_str());
        return nullptr;
    }
    if (mode_delta(mode) && !afn) {
        h->jit_error = "the specialised module has no wost_point_alpha_jit";
        return nullptr;
    }
    h->jit_fn = fn;
    h->jit_alpha_fn = afn;
    return fn;
}

// The corrected screened sampler's nodes do not depend on sigma_bar (only on the
// shape s = R sqrt(sigma_bar)): built once per process (~0.5 s of Bessel series).
const std::vector<float>& fixed_screened_table() {
    static const std::vector<float> t = [] {
        std::vector<float> v((size_t)kFixTableFloats);
        screened_fixed_nodes(v.data(), kFixRows, kFixCols, kFixXMax);
        return v;
    }();
    return t;
}

// The radial sampler's nodes depend only on the sampler and (screened) sigma_bar: each
// table is computed once per process (8-14 ms of host time, which every fresh handle's
// first solve paid; a survey's handles share one sigma_bar). kind 0: Green's, 1: the
// Jacobian-corrected Green's (compat fixed), 2: screened.
// (the cache and its lock are never destroyed: a prefetch thread may outlive the statics)
struct NodeCache {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<int, uint64_t>, std::vector<float>> done;
    std::set<std::pair<int, uint64_t>> running;
};
NodeCache& node_cache() {
    static NodeCache* c = new NodeCache;
    return *c;
}

std::pair<int, uint64_t> node_key(int kind, double sigma_bar) {
    uint64_t bits = 0;
    if (kind == 2) std::memcpy(&bits, &sigma_bar, sizeof(bits));
    return std::make_pair(kind, bits);
}

void compute_nodes(int kind, double sigma_bar, std::vector<float>& v) {
    v.resize(WOST_SAMPLER_TABLE_N);
    if (kind == 2) screened_sampler_nodes(v.data(), WOST_SAMPLER_TABLE_N, sigma_bar);
    else if (kind == 1) greens_sampler_nodes_jacobian(v.data(), WOST_SAMPLER_TABLE_N);
    else greens_sampler_nodes(v.data(), WOST_SAMPLER_TABLE_N);
}

void store_nodes(const std::pair<int, uint64_t>& key, std::vector<float>&& v) {
    NodeCache& c = node_cache();
    std::lock_guard<std::mutex> lock(c.mu);
    if (c.done.size() >= 64) c.done.clear();
    c.done.emplace(key, std::move(v));
    c.running.erase(key);
    c.cv.notify_all();
}

void sampler_nodes_once(int kind, double sigma_bar, float* out) {
    NodeCache& c = node_cache();
    const auto key = node_key(kind, sigma_bar);
    {
        std::unique_lock<std::mutex> lock(c.mu);
        c.cv.wait(lock, [&] { return !c.running.count(key); });   // (a prefetch computing them)
        auto it = c.done.find(key);
        if (it != c.done.end()) {
            std::memcpy(out, it->second.data(), sizeof(float) * WOST_SAMPLER_TABLE_N);
            return;
        }
        c.running.insert(key);
    }
    std::vector<float> v;
    compute_nodes(kind, sigma_bar, v);
    std::memcpy(out, v.data(), sizeof(float) * WOST_SAMPLER_TABLE_N);
    store_nodes(key, std::move(v));
}

// wost_create: the nodes a first solve of this handle needs, computed in the background
// while the handle's device setup runs (a fresh process's first HIP calls take ~0.1 s).
void sampler_nodes_prefetch(int kind, double sigma_bar) {
    NodeCache& c = node_cache();
    const auto key = node_key(kind, sigma_bar);
    {
        std::lock_guard<std::mutex> lock(c.mu);
        if (c.running.count(key) || c.done.count(key)) return;
        c.running.insert(key);
    }
    try {
        std::thread([kind, sigma_bar, key]() {
            std::vector<float> v;
            compute_nodes(kind, sigma_bar, v);
            store_nodes(key, std::move(v));
        }).detach();
    } catch (...) {
        std::vector<float> v;
        compute_nodes(kind, sigma_bar, v);
        store_nodes(key, std::move(v));
    }
}

// The sampler kind ensure_table builds for a handle.
int sampler_kind(const wost_handle* h) {
    if (h->delta && h->compat == WOST_COMPAT_FIXED) return 1;
    if (h->delta) return 2;
    return h->compat == WOST_COMPAT_FIXED ? 1 : 0;
}

int ensure_table(wost_handle* h) {
    if (h->table_ready) return WOST_OK;
    // sampler nodes, then (delta tracking) the G_norm cells (wost_device.h), then
    // (compat="fixed" delta tracking) the corrected screened sampler's nodes
    const bool fix_delta = h->delta && h->compat == WOST_COMPAT_FIXED;
    const size_t n = table_floats(h->delta, fix_delta);
    h->table.assign(n, 0.f);
    if (fix_delta) {
        sampler_nodes_once(sampler_kind(h), 0.0, h->table.data());   // staged, unused
        greens_norm_cells(h->table.data() + kSamplerFloatsPadded, kGnormCells, (double)kGnormCells / kGnormInvH);
        const std::vector<float>& fx = fixed_screened_table();
        std::memcpy(h->table.data() + kFixTableOffset, fx.data(), sizeof(float) * fx.size());
    } else if (h->delta) {
        sampler_nodes_once(2, h->sigma_bar, h->table.data());
        greens_norm_cells(h->table.data() + kSamplerFloatsPadded, kGnormCells, (double)kGnormCells / kGnormInvH);
    } else if (h->compat == WOST_COMPAT_FIXED) {
        sampler_nodes_once(1, 0.0, h->table.data());
    } else {
        sampler_nodes_once(0, 0.0, h->table.data());
    }
    if (!h->d_table) HIP_TRY(hipMalloc(&h->d_table, sizeof(float) * std::max(n, table_floats(true))));
    HIP_TRY(hipMemcpy(h->d_table, h->table.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    h->table_ready = true;
    return WOST_OK;
}

// buildModifiedSigma's sigma_bar (solvers/WoStSolver.py:129-136 with
// utils.py:65-120): max - min of sigma' on a 50x50 ij-grid over the bounding
// box of all boundary vertices; NaN/inf samples skipped; a range <= 0 or
// > 1e3 falls back to 10.0 (quirk Q8).
double estimate_sigma_bar(const wost_handle* h, const Program& prog) {
    float xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    auto scan = [&](const std::vector<float>& v) {
        for (size_t i = 0; i + 1 < v.size(); i += 2) {
            xmin = std::min(xmin, v[i]); xmax = std::max(xmax, v[i]);
            ymin = std::min(ymin, v[i + 1]); ymax = std::max(ymax, v[i + 1]);
        }
    };
    scan(h->dverts);
    scan(h->nverts);
    const std::vector<float> gx = torch_linspace(xmin, xmax, 50), gy = torch_linspace(ymin, ymax, 50);
    const DProgram* hd = prog.hdr();
    const DField& fa = hd->field[SLOT_ALPHA];
    const DField& fs = hd->field[SLOT_SIGMA];
    const bool detached = (fa.flags & WOST_FIELD_DETACHED) != 0;
    bool any = false;
    float lo = INFINITY, hi = -INFINITY;
    for (float x : gx) {
        for (float y : gy) {
            Jet aj = field_jet(fa, prog.terms(), prog.factors(), prog.grid(), x, y);
            float sg = fs.present ? field_value(fs, prog.terms(), prog.factors(), prog.grid(), x, y) : 0.f;
            float sp = sigma_prime_from(aj, sg, detached);
            if (std::isnan(sp) || std::isinf(sp)) continue;
            any = true;
            lo = std::min(lo, sp);
            hi = std::max(hi, sp);
        }
    }
    if (!any) return NAN;
    double sb = (double)hi - (double)lo;
    if (sb <= 0.0 || sb > 1e3) sb = 10.0;
    return sb;
}

// The largest float x with sqrtf(x) <= rmin (IEEE sqrt, as the kernels take it): a
// silhouette vertex at squared distance <= x makes r = max(rmin, min(dn, dd)) equal
// rmin whatever the other vertices are (silhouette_distance_tree's early stop).
float silhouette_stop2(float rmin) {
    if (!(rmin > 0.0f) || !std::isfinite(rmin)) return -1.0f;
    float x = rmin * rmin;
    while (x > 0.0f && std::sqrt(x) > rmin) x = std::nextafter(x, 0.0f);
    while (std::sqrt(std::nextafter(x, INFINITY)) <= rmin) x = std::nextafter(x, INFINITY);
    return x;
}

// What of the segment tree the field-specialised kernels stage in LDS, by level:
// 2 = its records and the Neumann vertices (one kTreeStageVertsBlock-thread workgroup
// per CU), 1 = its records (two kTreeStageBlock-thread workgroups per CU), 0 = nothing
// (256-thread workgroups, records and vertices through L1/L2). The option tree_lds caps
// the level (A/B; the results are the same bits at every level). Returns the records to
// stage and sets the workgroup size and the vertices to stage.
constexpr size_t kTreeLdsMaxBytes = 64 * 1024;
constexpr int kTreeLdsDefaultLevel = 2;
int tree_lds_records(const wost_handle* h, int mode, int level, int* block, int* verts) {
    *block = kWalkBlock;
    *verts = 0;
    if (!mode_tree(mode) || !h->tree_ready) return 0;
    level = std::min(level, h->opt.tree_lds);
    const int n = h->tree.first_leaf;
    if (level <= 0 || n <= 0 || (size_t)n * 8 * sizeof(float4) > kTreeLdsMaxBytes) return 0;
    if (level >= 2) {
        *block = kTreeStageVertsBlock;
        *verts = (int)(h->nverts.size() / 2);
        return n;
    }
    *block = h->opt.tree_lds_block;
    return n;
}

bool use_tree(const wost_handle* h) {
    const int nseg = (int)(h->nverts.size() / 2) - 1;
    return nseg >= 1 && h->tree_min_segments >= 0 && nseg >= h->tree_min_segments;
}

int walk_mode_src(const wost_handle* h, bool src) {
    const bool neu = !h->nverts.empty();
    const bool tree = neu && use_tree(h);
    if (h->compat == WOST_COMPAT_FIXED) {   // the nearest-crossing ray queries (scan or tree)
        if (h->delta) return neu ? (tree ? MODE_FIX_MIXED_DELTA_TREE : MODE_FIX_MIXED_DELTA) : MODE_FIX_DELTA;
        if (neu) return src ? (tree ? MODE_FIX_MIXED_POISSON_TREE : MODE_FIX_MIXED_POISSON)
                            : (tree ? MODE_FIX_MIXED_TREE : MODE_FIX_MIXED);
        return src ? MODE_FIX_POISSON : MODE_FIX_DIRICHLET;
    }
    if (h->delta) return neu ? (tree ? MODE_MIXED_DELTA_TREE : MODE_MIXED_DELTA) : MODE_DELTA;
    if (neu) return src ? (tree ? MODE_MIXED_POISSON_TREE : MODE_MIXED_POISSON) : (tree ? MODE_MIXED_TREE : MODE_MIXED);
    return src ? MODE_POISSON : MODE_DIRICHLET;
}

int walk_mode(const wost_handle* h) { return walk_mode_src(h, h->fields[SLOT_F].present); }

int ensure_tree(wost_handle* h) {
    if (h->tree_ready) return WOST_OK;
    const int nv = (int)(h->nverts.size() / 2);
    // a polyline too long for kTreeMaxDepth levels at the chosen leaf size takes 32 per leaf
    if (!build_segment_tree(h->nverts.data(), nv, h->tree_leaf, &h->tree) &&
        !build_segment_tree(h->nverts.data(), nv, 32, &h->tree))
        return fail(WOST_ERR_UNSUPPORTED, "cannot build the Neumann segment tree of %d segments (at most %d levels "
                    "of 32-segment leaves)", nv - 1, kTreeMaxDepth);
    if (h->d_tree) (void)hipFree(h->d_tree);
    h->d_tree = nullptr;
    const size_t n = std::max<size_t>(h->tree.rec.size(), 16);
    HIP_TRY(hipMalloc(&h->d_tree, sizeof(float) * n));
    if (!h->tree.rec.empty())
        HIP_TRY(hipMemcpy(h->d_tree, h->tree.rec.data(), sizeof(float) * h->tree.rec.size(), hipMemcpyHostToDevice));
    h->tree_ready = true;
    return WOST_OK;
}

template <class T>
int ensure_cap(T*& p, int64_t& cap, int64_t need) {
    if (need <= cap) return WOST_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, sizeof(T) * (size_t)need);
    if (e != hipSuccess) return fail(WOST_ERR_OOM, "hipMalloc(%lld bytes): %s", (long long)(sizeof(T) * need), hipGetErrorString(e));
    cap = need;
    return WOST_OK;
}

// pinned host staging of at least `need` bytes
int ensure_pin(wost_handle* h, size_t need) {
    if (need <= h->pin_cap) return WOST_OK;
    if (h->h_pin) {   // (a solve that failed mid-way may have left copies from it queued)
        (void)hipStreamSynchronize(h->stream);
        (void)hipHostFree(h->h_pin);
    }
    h->h_pin = nullptr;
    h->pin_cap = 0;
    need = std::max<size_t>(need, 4096);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&h->h_pin), need, hipHostMallocDefault);
    if (e != hipSuccess) return fail(WOST_ERR_OOM, "hipHostMalloc(%zu bytes): %s", need, hipGetErrorString(e));
    h->pin_cap = need;
    return WOST_OK;
}

// per-walk value and step buffers, always of equal capacity
// Per-walk results of `need` walks with `ns` values each.
int ensure_workspace(wost_handle* h, int64_t need, int ns = 1) {
    if (need <= h->ws_cap && need * ns <= h->ws_val_cap && h->d_val && h->d_steps) return WOST_OK;
    if (h->d_val) (void)hipFree(h->d_val);
    if (h->d_steps) (void)hipFree(h->d_steps);
    h->d_val = nullptr;
    h->d_steps = nullptr;
    h->ws_cap = h->ws_val_cap = 0;
    hipError_t e = hipMalloc(&h->d_val, sizeof(float) * (size_t)need * (size_t)ns);
    if (e == hipSuccess) e = hipMalloc(&h->d_steps, sizeof(uint32_t) * (size_t)need);
    if (e != hipSuccess) return fail(WOST_ERR_OOM, "per-walk workspace of %lld walks: %s", (long long)need, hipGetErrorString(e));
    h->ws_cap = need;
    h->ws_val_cap = need * ns;
    return WOST_OK;
}

int check_polyline(const wost_polyline& p, const char* name, bool required, std::vector<float>& out) {
    out.clear();
    if (!p.xy || p.n_vertices == 0) {
        if (required) return fail(WOST_ERR_INVALID_ARG, "%s polyline is required", name);
        return WOST_OK;
    }
    if (p.n_vertices < 2) return fail(WOST_ERR_INVALID_ARG, "%s polyline needs >= 2 vertices (got %d)", name, p.n_vertices);
    out.assign(p.xy, p.xy + 2 * (size_t)p.n_vertices);
    for (float v : out)
        if (!std::isfinite(v)) return fail(WOST_ERR_INVALID_ARG, "%s polyline has a non-finite coordinate", name);
    return WOST_OK;
}

}  // namespace

extern "C" {

int wost_version(void) { return WOST_ABI_VERSION; }

const char* wost_last_error(void) { return g_err.c_str(); }

int wost_device_count(int32_t* count) {
    if (!count) return fail(WOST_ERR_INVALID_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(WOST_ERR_NO_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return WOST_OK;
}

int64_t wost_num_blocks(int64_t n_points, int64_t walks_per_point) {
    if (n_points <= 0 || walks_per_point <= 0) return 0;
    return n_points * ((walks_per_point + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS);
}

void wost_destroy(wost_handle* h) {
    if (!h) return;
    if (h->device >= 0) (void)hipSetDevice(h->device);
    void* ptrs[] = {h->d_dverts, h->d_nverts, h->d_table, h->d_prog, h->d_counter, h->d_val,
                    h->d_steps, h->d_stage, h->d_bstats, h->d_tree, h->d_seg_phi, h->d_point_alpha, h->d_pool};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (h->h_pin) (void)hipHostFree(h->h_pin);
    for (hipEvent_t& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

}  // extern "C"

namespace {

// The host half of wost_create: validation, field conversion, sigma_bar. No
// HIP call; the handle's device is -1 until wost_create takes a device.
int create_host(const wost_problem* pb, wost_handle** out) {
    *out = nullptr;
    if (pb->compat != WOST_COMPAT_REFERENCE && pb->compat != WOST_COMPAT_FIXED)
        return fail(WOST_ERR_INVALID_ARG, "unknown compat %d", pb->compat);
    wost_handle* h = new wost_handle();
    h->device = -1;
    int rc;
    if ((rc = check_polyline(pb->dirichlet, "dirichlet", true, h->dverts)) != WOST_OK ||
        (rc = check_polyline(pb->neumann, "neumann", false, h->nverts)) != WOST_OK ||
        (rc = convert_field(pb->boundary, h->fields[SLOT_G], "boundary")) != WOST_OK ||
        (rc = convert_field(pb->source, h->fields[SLOT_F], "source")) != WOST_OK ||
        (rc = convert_field(pb->sigma, h->fields[SLOT_SIGMA], "sigma")) != WOST_OK ||
        (rc = convert_field(pb->alpha, h->fields[SLOT_ALPHA], "alpha")) != WOST_OK) {
        delete h;
        return rc;
    }
    h->compat = pb->compat;
#if defined(WOST_STUDY)
    // study builds only: the tools' A/B environment (the product library reads none of it;
    // wost_set_jit / wost_set_trig / wost_set_segment_tree / wost_set_option instead)
    if (const char* e = std::getenv("WOST_JIT")) h->jit_enabled = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("WOST_TREE_MIN_SEGMENTS")) h->tree_min_segments = std::atoi(e);
    if (const char* e = std::getenv("WOST_TRIG"))
        h->trig_mode = std::strcmp(e, "exact") == 0 ? WOST_TRIG_EXACT : std::strcmp(e, "fast") == 0 ? WOST_TRIG_FAST
                                                                                                   : WOST_TRIG_AUTO;
    if (const char* e = std::getenv("WOST_TREE_LEAF")) h->tree_leaf = std::min(32, std::max(1, std::atoi(e)));
#endif
    options_from_study_env(h->opt);
    // solvers/WoStSolver.py:54-64: any of sigma/alpha turns on delta tracking,
    // the missing one defaults to sigma = 0 / alpha = 1 (constant => Q9 fallback).
    h->delta = h->fields[SLOT_SIGMA].present || h->fields[SLOT_ALPHA].present;
    if (h->delta) {
        if (!h->fields[SLOT_ALPHA].present) {
            HostField& a = h->fields[SLOT_ALPHA];
            a.present = true;
            a.flags = WOST_FIELD_DETACHED;
            a.terms.push_back(DTerm{1.0f, 0, 0, 0});
        }
        if (!h->fields[SLOT_SIGMA].present) {
            HostField& s = h->fields[SLOT_SIGMA];
            s.present = true;
            s.terms.push_back(DTerm{0.0f, 0, 0, 0});
        }
        if (pb->sigma_bar_override > 0.0) {
            h->sigma_bar = pb->sigma_bar_override;
        } else {
            Program tmp;
            build_program(h->fields, 1.0, tmp);
            h->sigma_bar = estimate_sigma_bar(h, tmp);
            if (!(h->sigma_bar > 0.0)) {
                delete h;
                return fail(WOST_ERR_INVALID_ARG,
                            "sigma' could not be evaluated at any grid point (reference raises ValueError, utils.py:108-109)");
            }
        }
    }
    *out = h;
    return WOST_OK;
}

}  // namespace

extern "C" {

int wost_create(const wost_problem* pb, wost_handle** out) {
    if (!pb || !out) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    jit_start_identity_probe();   // (the compile helper's start, in the background)
    wost_handle* h = nullptr;
    int rc = create_host(pb, &h);
    if (rc != WOST_OK) return rc;
    *out = nullptr;
    if (h->fields[SLOT_F].present || h->delta)   // the first solve's sampler nodes, meanwhile
        sampler_nodes_prefetch(sampler_kind(h), h->sigma_bar);

    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        wost_destroy(h);
        return fail(WOST_ERR_NO_DEVICE, "no HIP device available (%s)", hipGetErrorString(e));
    }
    if (pb->device < 0 || pb->device >= ndev) {
        wost_destroy(h);
        return fail(WOST_ERR_INVALID_ARG, "device %d out of range [0,%d)", pb->device, ndev);
    }
    h->device = pb->device;
#define CREATE_TRY(expr)                                              \
    do {                                                              \
        hipError_t e_ = (expr);                                       \
        if (e_ != hipSuccess) {                                       \
            int rc_ = fail(WOST_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
            wost_destroy(h);                                          \
            return rc_;                                               \
        }                                                             \
    } while (0)
    CREATE_TRY(hipSetDevice(h->device));
    CREATE_TRY(hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, h->device));
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) == hipSuccess && khz > 0)
            h->tick_khz = (double)khz;
    }
    CREATE_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    for (hipEvent_t& ev : h->ev) CREATE_TRY(hipEventCreate(&ev));
    h->ctl_cap = (int64_t)ctl_words(8192);   // 8,192 waves: 256 CUs x 32
    CREATE_TRY(hipMalloc(&h->d_counter, sizeof(unsigned long long) * (size_t)h->ctl_cap));
    CREATE_TRY(hipMemset(h->d_counter, 0, sizeof(unsigned long long) * (size_t)h->ctl_cap));
    CREATE_TRY(hipMalloc(&h->d_dverts, sizeof(float) * h->dverts.size()));
    CREATE_TRY(hipMemcpy(h->d_dverts, h->dverts.data(), sizeof(float) * h->dverts.size(), hipMemcpyHostToDevice));
    if (!h->nverts.empty()) {
        CREATE_TRY(hipMalloc(&h->d_nverts, sizeof(float) * h->nverts.size()));
        CREATE_TRY(hipMemcpy(h->d_nverts, h->nverts.data(), sizeof(float) * h->nverts.size(), hipMemcpyHostToDevice));
        // atan2 of each segment's left normal (:227-228, quirk Q2) on the host: the C
        // library's atan2f is what torch.atan2 of the reference's 0-d tensors calls, and
        // the device's atan2f differs from it on ~half of the C5 topography's segments
        // (tools/r05/trig_compare.py), each a different direction after a Neumann hit
        const int nseg = (int)(h->nverts.size() / 2) - 1;
        std::vector<float> phi((size_t)std::max(nseg, 1), 0.0f);
        for (int i = 0; i < nseg; ++i) {
            const float2 a{h->nverts[2 * i], h->nverts[2 * i + 1]}, b{h->nverts[2 * i + 2], h->nverts[2 * i + 3]};
            const float2 n = segment_left_normal(a, b);
            phi[i] = std::atan2(n.y, n.x);
        }
        CREATE_TRY(hipMalloc(&h->d_seg_phi, sizeof(float) * phi.size()));
        CREATE_TRY(hipMemcpy(h->d_seg_phi, phi.data(), sizeof(float) * phi.size(), hipMemcpyHostToDevice));
    }
#undef CREATE_TRY
    if ((rc = upload_program(h)) != WOST_OK) {
        wost_destroy(h);
        return rc;
    }
    *out = h;
    return WOST_OK;
}

int wost_set_field(wost_handle* h, int32_t slot, const wost_field* field) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    int s;
    if (slot == WOST_SLOT_BOUNDARY) s = SLOT_G;
    else if (slot == WOST_SLOT_SOURCE) s = SLOT_F;
    else return fail(WOST_ERR_INVALID_ARG, "unknown field slot %d", slot);
    HostField hf;
    int rc = convert_field(field, hf, s == SLOT_G ? "boundary" : "source");
    if (rc != WOST_OK) return rc;
    h->fields[s] = hf;
    if (s == SLOT_F) {   // setSourceTerm: back to a single source
        for (int k = SLOT_EXTRA; k < N_FIELDS; ++k) h->fields[k] = HostField();
        h->n_sources = 1;
    }
    h->prog_dirty = true;
    HIP_TRY(hipSetDevice(h->device));
    return upload_program(h);
}

int wost_get_info(const wost_handle* h, double* sigma_bar, int32_t* use_delta) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    if (sigma_bar) *sigma_bar = h->sigma_bar;
    if (use_delta) *use_delta = h->delta ? 1 : 0;
    return WOST_OK;
}

int wost_sampler_table(const wost_handle* hc, float* out, int32_t n) {
    wost_handle* h = const_cast<wost_handle*>(hc);
    if (!h || !out || n != WOST_SAMPLER_TABLE_N)
        return fail(WOST_ERR_INVALID_ARG, "need a handle and a %d-float buffer", WOST_SAMPLER_TABLE_N);
    HIP_TRY(hipSetDevice(h->device));
    int rc = ensure_table(h);
    if (rc != WOST_OK) return rc;
    std::memcpy(out, h->table.data(), sizeof(float) * WOST_SAMPLER_TABLE_N);
    return WOST_OK;
}

int wost_greens_norm(double sigma_bar, const float* radii, int64_t n, float* out) {
    if (!(sigma_bar > 0.0) || n < 0 || (n > 0 && (!radii || !out)))
        return fail(WOST_ERR_INVALID_ARG, "need sigma_bar > 0 and n >= 0 radii");
    std::vector<float4> cells(kGnormCells);
    greens_norm_cells(reinterpret_cast<float*>(cells.data()), kGnormCells, (double)kGnormCells / kGnormInvH);
    // the kernels' constants (build_program)
    const float sqrt_sb = (float)std::sqrt(sigma_bar), inv_sb = (float)(1.0 / sigma_bar);
    for (int64_t i = 0; i < n; ++i) {
        const float r = radii[i];
        out[i] = greens_norm_from_table(cells.data(), r * sqrt_sb, r, inv_sb);
    }
    return WOST_OK;
}

int wost_screened_sample_fixed(const float* s, const float* u, int64_t n, float* rho) {
    if (n < 0 || (n > 0 && (!s || !u || !rho))) return fail(WOST_ERR_INVALID_ARG, "need n >= 0 and buffers");
    const std::vector<float>& t = fixed_screened_table();
    for (int64_t i = 0; i < n; ++i) rho[i] = sample_rho_screened_fixed(t.data(), u[i], s[i]);
    return WOST_OK;
}

int wost_screened_cdf_fixed(double s, const double* rho, int64_t n, double* cdf) {
    if (!(s >= 0.0) || n < 0 || (n > 0 && (!rho || !cdf))) return fail(WOST_ERR_INVALID_ARG, "need s >= 0, n >= 0");
    for (int64_t i = 0; i < n; ++i) cdf[i] = screened_fixed_cdf(rho[i], s);
    return WOST_OK;
}

int wost_num_sources(const wost_handle* h, int32_t* n_sources) {
    if (!h || !n_sources) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    *n_sources = h->n_sources;
    return WOST_OK;
}

int wost_last_timing(const wost_handle* h, wost_timing* out) {
    if (!h || !out) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    *out = h->timing;
    return WOST_OK;
}

}  // extern "C"

namespace {

constexpr int64_t kMaxRecordBatchBytes = int64_t(1) << 30;   // device buffer of the walk recorder

// wost_solve, and with `records` != null also the walk recorder
// (wost_solve_history): records[walk][max_steps + 1][kRecFloats] on the host.
// Walk-range mode (wost_solve_range): walk_begin/walk_end != 0/W solves walks
// [walk_begin, walk_end) of every point; blocks are then (point, block of the
// range), point-major, and block_begin/block_end are ignored.
// The kernel a solve of n_points launches first (its occupancy fallback may then stage
// less): the workgroup, the segment tree's staging, and whether the polylines are read
// from global memory. Shared by solve_impl and wost_prepare_multi, so that a prepared
// kernel is the one the solve looks up.
struct KernelShape {
    int block = kWalkBlock, tree_verts = 0, tree_level = kTreeLdsDefaultLevel, tree_lds = 0;
    bool gpoly = false;
};

int first_kernel_shape(const wost_handle* h, int mode, int64_t n_points, KernelShape* ks) {
    *ks = KernelShape{};
    ks->tree_lds = h->jit_enabled ? tree_lds_records(h, mode, ks->tree_level, &ks->block, &ks->tree_verts) : 0;
    // option walk_block: the workgroup of the field-specialised scan kernels (a multiple of
    // 64 up to 1024): larger workgroups share one LDS copy of the sampler and G_norm tables,
    // so more waves fit a CU than 256-thread workgroups allow (results are the same bits)
    if (h->jit_enabled && !mode_tree(mode) && h->opt.walk_block > 0) ks->block = h->opt.walk_block;
    const int nd_ = (int)(h->dverts.size() / 2), nn_ = (int)(h->nverts.size() / 2);
    const Options& O = h->opt;
    // polylines whose LDS copy would cost the walk kernel its occupancy are read from
    // global memory instead (field-specialised kernels; the precompiled ones stage them)
    // (the staged tree records have their own budget, kTreeLdsMaxBytes)
    ks->gpoly = h->jit_enabled && walk_lds_bytes(mode, nd_, nn_, (int)n_points, 0,
                                                 jit_const_dirichlet(O, nd_)) > kGlobalPolylineLdsBytes;
    // the brute-force scan of a long Neumann polyline (neumann_scan_both) reads every vertex
    // at every step: staged in LDS with one 1024-thread workgroup per CU when it fits (a
    // broadcast LDS read per vertex), else from global memory
    if (ks->gpoly && h->jit_enabled && jit_fused_neumann_scan(O, mode, nn_)) {
        int cap = 0;
        HIP_TRY(hipDeviceGetAttribute(&cap, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device));
        if (walk_lds_bytes(mode, nd_, nn_, (int)n_points, 0, jit_const_dirichlet(O, nd_), false, false,
                           kTreeStageVertsBlock) <= (size_t)cap) {
            ks->gpoly = false;
            ks->block = kTreeStageVertsBlock;
        }
    }
    return WOST_OK;
}

int solve_impl(wost_handle* h, const float* points, int64_t n_points, int64_t W, int64_t block_begin,
               int64_t block_end, int32_t max_steps, float eps, uint64_t seed, double* block_stats,
               double* point_stats, float* walk_values, uint32_t* walk_steps, float* records, bool multi = false,
               int64_t walk_begin = 0, int64_t walk_end = -1) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    const int ns = h->n_sources;
    if (ns != 1 && !multi)
        return fail(WOST_ERR_INVALID_ARG, "the handle has %d sources (wost_set_sources): use wost_solve_multi", ns);
    const int row = 2 * ns + 1;   // doubles per block / point row
    if (n_points < 0 || (n_points > 0 && !points)) return fail(WOST_ERR_INVALID_ARG, "bad points");
    if (W <= 0) return fail(WOST_ERR_INVALID_ARG, "nWalks must be >= 1 (got %lld)", (long long)W);
    if (max_steps < 0) return fail(WOST_ERR_INVALID_ARG, "maxSteps must be >= 0");
    if (!(eps == eps)) return fail(WOST_ERR_INVALID_ARG, "eps is NaN");
    if (n_points > 0 && W > (int64_t(1) << 53) / n_points)
        return fail(WOST_ERR_INVALID_ARG, "n_points * nWalks must stay below 2^53 walks");
    const int64_t nbpp = (W + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    const int64_t nb_total = n_points * nbpp;
    if (walk_end < 0) walk_end = W;
    const bool range = walk_begin != 0 || walk_end != W;
    if (range && (walk_begin < 0 || walk_end <= walk_begin || walk_end > W || walk_begin % WOST_BLOCK_WALKS != 0 ||
                  (walk_end % WOST_BLOCK_WALKS != 0 && walk_end != W)))
        return fail(WOST_ERR_INVALID_ARG,
                    "walk range [%lld,%lld) of %lld walks must be non-empty with block-aligned ends (multiples of %d, "
                    "or the end at W)", (long long)walk_begin, (long long)walk_end, (long long)W, WOST_BLOCK_WALKS);
    const int64_t Wr = walk_end - walk_begin;                            // walks per point solved
    const int64_t nbr = (Wr + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;   // blocks per point solved
    if (range) {
        block_begin = 0;
        block_end = n_points * nbr;
    } else if (block_begin < 0 || block_end < block_begin || block_end > nb_total)
        return fail(WOST_ERR_INVALID_ARG, "block range [%lld,%lld) outside [0,%lld)", (long long)block_begin,
                    (long long)block_end, (long long)nb_total);
    for (int64_t i = 0; i < 2 * n_points; ++i)
        if (!std::isfinite(points[i])) return fail(WOST_ERR_INVALID_ARG, "solve point %lld is not finite", (long long)(i / 2));
    if (h->delta && !h->fields[SLOT_F].present)
        return fail(WOST_ERR_INVALID_ARG,
                    "delta tracking (sigma/alpha given) needs a source term: the reference raises "
                    "UnboundLocalError at solvers/WoStSolver.py:281 (quirk Q14)");
    if (h->compat == WOST_COMPAT_FIXED && h->delta && h->fixed_step_check && n_points > 0 && max_steps > 0 &&
        h->dverts.size() >= 4) {
        // compat="fixed" delta tracking draws each collision from the ball's own screened
        // law: with R sqrt(sigma_bar) >> 1 a step moves ~2/sqrt(sigma_bar) (E[l^2] = 4 /
        // sigma_bar), so leaving a point at Dirichlet distance d takes ~d^2 sigma_bar / 4
        // steps. When that exceeds maxSteps at the median point, every walk would end
        // truncated at maxSteps (the DCR configurations: sigma_bar = 10, d ~ 100): refuse.
        std::vector<double> est((size_t)n_points);
        const auto* dv = reinterpret_cast<const float2*>(h->dverts.data());
        const int nd = (int)(h->dverts.size() / 2);
        for (int64_t i = 0; i < n_points; ++i) {
            const double d = poly_distance(dv, nd, points[2 * i], points[2 * i + 1]);
            est[(size_t)i] = d * d * h->sigma_bar / 4.0;
        }
        std::nth_element(est.begin(), est.begin() + n_points / 2, est.end());
        const double med = est[(size_t)(n_points / 2)];
        if (med > (double)max_steps)
            return fail(WOST_ERR_INVALID_ARG,
                        "compat=\"fixed\" delta tracking would truncate the walks: at the median query point a walk "
                        "needs ~%.3g steps (d^2 sigma_bar / 4, sigma_bar = %g) to reach the Dirichlet boundary, "
                        "maxSteps is %d; raise maxSteps, lower sigma_bar, or disable this check "
                        "(wost_set_fixed_step_check / WostSolver_2D.set_fixed_step_check(False))",
                        med, h->sigma_bar, (int)max_steps);
    }
    const int mode = walk_mode(h);
    const bool src = h->fields[SLOT_F].present;

    HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = upload_program(h)) != WOST_OK) return rc;
    if (src && (rc = ensure_table(h)) != WOST_OK) return rc;
    if (mode_tree(mode) && (rc = ensure_tree(h)) != WOST_OK) return rc;

    h->timing = wost_timing{};
    const int64_t nblk = block_end - block_begin;
    if (point_stats) std::fill(point_stats, point_stats + row * n_points, 0.0);
    if (nblk == 0) return WOST_OK;

    // block -> global walk range
    auto blk_begin = [&](int64_t j) { return (j / nbpp) * W + (j % nbpp) * WOST_BLOCK_WALKS; };
    auto blk_end = [&](int64_t j) {
        const int64_t p = j / nbpp, b = j % nbpp;
        return p * W + std::min<int64_t>((b + 1) * WOST_BLOCK_WALKS, W);
    };

    const int64_t walks_total = range ? n_points * Wr : blk_end(block_end - 1) - blk_begin(block_begin);
    // walks per launch: the recorder's device buffer bounds it
    int64_t batch_limit = kMaxBatchWalks / ns;
    const int64_t rec_stride = (int64_t)max_steps + 1;
    const int64_t rec_walk_bytes = rec_stride * kRecFloats * (int64_t)sizeof(float);
    if (records) {
        batch_limit = std::min<int64_t>(kMaxBatchWalks, kMaxRecordBatchBytes / rec_walk_bytes);
        if (batch_limit < std::min<int64_t>(W, WOST_BLOCK_WALKS))
            return fail(WOST_ERR_INVALID_ARG,
                        "return_history: %lld recorded steps per walk need more than %lld bytes per walk block; "
                        "lower maxSteps or nWalks", (long long)rec_stride, (long long)kMaxRecordBatchBytes);
    }
    if (range && Wr > batch_limit)
        return fail(WOST_ERR_INVALID_ARG, "walk range of %lld walks per point exceeds one launch (%lld walks)",
                    (long long)Wr, (long long)batch_limit);
    // pinned staging: [points | one batch's block ranges | the block sums], 64-byte aligned;
    // the device holds the first two parts in one buffer of the same layout, so that one copy
    // brings the points and the first batch's block ranges (C2: a copy and its ~6 us gap less)
    auto al64 = [](size_t b) { return (b + 63) / 64 * 64; };
    const size_t pin_pts = al64(sizeof(float2) * (size_t)std::max<int64_t>(n_points, 1));
    const size_t pin_beg = al64(sizeof(int64_t) * (size_t)(nblk + 1));
    const size_t pin_bs = al64(sizeof(double) * (size_t)(kLstatsWords + row * nblk));
    if ((rc = ensure_pin(h, pin_pts + pin_beg + pin_bs)) != WOST_OK) return rc;
    if (pin_pts + pin_beg > h->stage_cap) {
        if (h->d_stage) (void)hipFree(h->d_stage);
        h->d_stage = nullptr;
        h->stage_cap = 0;
        const hipError_t e = hipMalloc(&h->d_stage, pin_pts + pin_beg);
        if (e != hipSuccess)
            return fail(WOST_ERR_OOM, "hipMalloc(%zu bytes): %s", pin_pts + pin_beg, hipGetErrorString(e));
        h->stage_cap = pin_pts + pin_beg;
    }
    h->d_points = reinterpret_cast<float2*>(h->d_stage);
    h->d_begin = reinterpret_cast<int64_t*>(h->d_stage + pin_pts);
    float* const pin_points = reinterpret_cast<float*>(h->h_pin);
    int64_t* const pin_begin = reinterpret_cast<int64_t*>(h->h_pin + pin_pts);
    double* const pin_bstats = reinterpret_cast<double*>(h->h_pin + pin_pts + pin_beg);
    std::memcpy(pin_points, points, sizeof(float2) * (size_t)n_points);
    // the points go with the first batch's block ranges, unless the query points' alpha
    // (delta tracking) needs them first
    bool points_pending = true;
    if (mode_delta(mode) && n_points > 0) {
        HIP_TRY(hipMemcpyAsync(h->d_points, pin_points, sizeof(float2) * n_points, hipMemcpyHostToDevice, h->stream));
        points_pending = false;
    }
    if ((rc = ensure_workspace(h, std::min<int64_t>(walks_total, batch_limit), ns)) != WOST_OK) return rc;
    if ((rc = ensure_cap(h->d_bstats, h->bstats_cap, kLstatsWords + nblk * row)) != WOST_OK) return rc;
    // (the launch statistics in front of the block sums: one copy brings both)
    unsigned long long* const d_lstats = reinterpret_cast<unsigned long long*>(h->d_bstats);
    double* const d_rows = h->d_bstats + kLstatsWords;
    float* d_rec = nullptr;
    struct RecFree {
        float*& p;
        ~RecFree() { if (p) (void)hipFree(p); }
    } rec_free{d_rec};
    if (records) HIP_TRY(hipMalloc(&d_rec, (size_t)std::min<int64_t>(walks_total, batch_limit) * rec_walk_bytes));

    KernelShape ks;
    if ((rc = first_kernel_shape(h, mode, n_points, &ks)) != WOST_OK) return rc;
    int block = ks.block, tree_verts = ks.tree_verts, tree_level = ks.tree_level, tree_lds = ks.tree_lds;
    bool gpoly = ks.gpoly;
    const int nd_ = (int)(h->dverts.size() / 2), nn_ = (int)(h->nverts.size() / 2);
    const Options& O = h->opt;
    double jit_ms = 0.0;
    auto stage_of = [](int recs, int verts) { return recs > 0 ? (verts > 0 ? 2 : 1) : 0; };
    hipFunction_t jfn = jit_kernel(h, mode, records != nullptr, ns, block, gpoly, stage_of(tree_lds, tree_verts),
                                   &jit_ms);
    if (!jfn && block != kWalkBlock) {   // the precompiled kernels run 256-thread workgroups, no staged tree
        block = kWalkBlock;
        tree_lds = 0;
        tree_verts = 0;
    }
    if (ns > 1 && !jfn)
        return fail(WOST_ERR_UNSUPPORTED, "multi-source solves need the field-specialised kernel%s%s",
                    h->jit_enabled ? ": " : " (disabled by wost_set_jit)", h->jit_error.c_str());
    size_t lds = walk_lds_bytes(mode, nd_, nn_, (int)n_points, tree_lds, jfn && jit_const_dirichlet(O, nd_),
                                jfn && jit_const_neumann(O, mode, nn_), jfn && gpoly, block, tree_verts);
    // option lds_pad_bytes (occupancy studies): extra bytes of LDS per workgroup
    lds += (size_t)O.lds_pad_bytes;
    int blocks_per_cu = 0;
    // a workgroup whose LDS exceeds the CU's never fits: checked here, not left to the
    // occupancy query
    int lds_cap = 0;
    HIP_TRY(hipDeviceGetAttribute(&lds_cap, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device));
    auto occupancy = [&]() -> hipError_t {
        blocks_per_cu = 0;
        if (lds > (size_t)lds_cap) return hipSuccess;
        return hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&blocks_per_cu, jfn, block, lds);
    };
    if (jfn) HIP_TRY(occupancy());
    while (jfn && tree_lds > 0 && blocks_per_cu * (block / 64) < 16) {
        // what the tree stages leaves fewer than 16 waves per CU (or does not fit at all):
        // stage less (the vertices, then the records), down to reading both through L1/L2
        // from 256-thread workgroups
        tree_level = tree_verts > 0 ? 1 : 0;
        tree_lds = tree_lds_records(h, mode, tree_level, &block, &tree_verts);
        if (!(jfn = jit_kernel(h, mode, records != nullptr, ns, block, gpoly, stage_of(tree_lds, tree_verts),
                               &jit_ms))) {
            // the precompiled kernels then (256-thread workgroups, nothing of the tree staged)
            block = kWalkBlock;
            tree_lds = tree_verts = 0;
            if (ns > 1)
                return fail(WOST_ERR_UNSUPPORTED, "multi-source solves need the field-specialised kernel: %s",
                            h->jit_error.c_str());
            break;
        }
        lds = walk_lds_bytes(mode, nd_, nn_, (int)n_points, tree_lds, jit_const_dirichlet(O, nd_),
                             jit_const_neumann(O, mode, nn_), gpoly, block, tree_verts) + (size_t)O.lds_pad_bytes;
        HIP_TRY(occupancy());
    }
    if (!jfn)
        HIP_TRY(walk_occupancy(mode, (int)(h->dverts.size() / 2), (int)(h->nverts.size() / 2), (int)n_points,
                               &blocks_per_cu));
    if (blocks_per_cu < 1)
        return fail(WOST_ERR_UNSUPPORTED, "walk kernel does not fit on a CU (polylines too large for LDS: %zu bytes)",
                    lds);

    WalkArgs a{};
    a.points = h->d_points;
    a.dverts = h->d_dverts;
    a.nverts = h->d_nverts;
    a.seg_phi = h->d_seg_phi;
    a.table = h->d_table;
    a.prog = h->d_prog;
    a.counter = h->d_counter;
    a.walks_per_point = W;
    a.nd = (int)(h->dverts.size() / 2);
    a.nn = (int)(h->nverts.size() / 2);
    a.max_steps = max_steps;
    a.eps = eps;
    a.rmin = eps / 2.0f;
    a.key0 = (uint32_t)seed;
    a.key1 = (uint32_t)(seed >> 32);
    a.n_points = (int32_t)std::min<int64_t>(n_points, INT32_MAX);
    a.inv_walks_per_point = 1.0 / (double)W;
    a.rec = d_rec;
    a.rec_stride = (int32_t)rec_stride;
    a.exact_trig = exact_trig_of(h) ? 1 : 0;
    if (mode_tree(mode)) {
        a.tree = reinterpret_cast<const float4*>(h->d_tree);
        a.tree_first_leaf = h->tree.first_leaf;
        a.tree_leaf = h->tree.leaf;
        a.tree_tol = h->tree.tol;
        a.tree_stop2 = silhouette_stop2(a.rmin);
        a.tree_kmax = h->tree.kmax;
        a.tree_lds_records = tree_lds;
        a.tree_lds_verts = tree_verts;
        a.tree_depth = h->tree.depth;
        // walk pools (wost_walk.h): near = within pool_near (default 0.1) of the Neumann
        // polyline's largest extent from its bounding box; tree_pool = 0 turns them off,
        // pool_slots (default 128) walks per class and workgroup
        if (O.tree_pool != 0 && h->nverts.size() >= 4) {
            float x0 = h->nverts[0], x1 = x0, y0 = h->nverts[1], y1 = y0;
            for (size_t i = 2; i + 1 < h->nverts.size(); i += 2) {
                x0 = std::min(x0, h->nverts[i]); x1 = std::max(x1, h->nverts[i]);
                y0 = std::min(y0, h->nverts[i + 1]); y1 = std::max(y1, h->nverts[i + 1]);
            }
            const float frac = (float)O.pool_near;
            const int slots = O.pool_slots;
            const float m = frac * std::max(x1 - x0, y1 - y0);
            // (study builds, tree_iter_stats: 16 counter words after each workgroup's pools)
            const int64_t words = (int64_t)pool_wg_words(ns, slots) + (O.tree_iter_stats ? 16 : 0);
            if ((rc = ensure_cap(h->d_pool, h->pool_cap, words * (int64_t)blocks_per_cu * h->num_cus)) != WOST_OK)
                return rc;
            a.pool = h->d_pool;
            a.pool_slots = slots;
            a.pool_wg_words = (int32_t)words;
            a.pool_box = make_float4(x0 - m, y0 - m, x1 + m, y1 + m);
            if (O.tree_iter_stats)
                HIP_TRY(hipMemsetAsync(h->d_pool, 0, sizeof(uint32_t) * (size_t)(words * blocks_per_cu * h->num_cus),
                                       h->stream));
            a.pool_near_waves = O.pool_near_waves;   // (0: by majority)
        }
    }

    if (mode_delta(mode) && n_points > 0) {   // alpha at the query points, with the walk kernel's fields
        if ((rc = ensure_cap(h->d_point_alpha, h->point_alpha_cap, n_points)) != WOST_OK) return rc;
        if (jfn) {
            const float2* pts = h->d_points;
            long long n = (long long)n_points;
            float* out = h->d_point_alpha;
            const char* prog = h->d_prog;
            void* args[] = {&prog, &pts, &n, &out};
            const int grid = (int)std::min<int64_t>((n_points + 255) / 256, 4096);
            HIP_TRY(hipModuleLaunchKernel(h->jit_alpha_fn, grid, 1, 1, 256, 1, 1, 0, h->stream, args, nullptr));
        } else {
            HIP_TRY(launch_point_alpha(h->d_prog, h->d_points, n_points, h->d_point_alpha, h->stream));
        }
        a.point_alpha = h->d_point_alpha;
    }

    std::vector<int64_t> begins;
    std::vector<float> ms_walk, ms_red;
    HIP_TRY(hipEventRecord(h->ev[4], h->stream));
    int64_t j = block_begin;
    int64_t walks_done = 0;
    int launches = 0;
    double walk_ms = 0.0, red_ms = 0.0;
    while (j < block_end) {
        int64_t j2 = j, count = 0;
        begins.clear();
        if (range) {
            // whole points' ranges: local walk l is walk walk_begin + l % Wr of point p0 + l / Wr
            const int64_t p0 = j / nbr;
            const int64_t p1 = std::min<int64_t>(n_points, p0 + std::max<int64_t>(1, batch_limit / Wr));
            for (int64_t p = p0; p < p1; ++p)
                for (int64_t b = 0; b < nbr; ++b) begins.push_back((p - p0) * Wr + b * WOST_BLOCK_WALKS);
            count = (p1 - p0) * Wr;
            j2 = p1 * nbr;
            a.wid_begin = 0;
            a.range_walks = Wr;
            a.range_offset = walk_begin;
            a.range_point0 = p0;
            a.inv_range_walks = 1.0 / (double)Wr;
        } else {
            // gather whole blocks into a batch of at most kMaxBatchWalks walks
            const int64_t wb = blk_begin(j);
            while (j2 < block_end && blk_end(j2) - wb <= batch_limit) {
                begins.push_back(blk_begin(j2) - wb);
                ++j2;
            }
            if (j2 == j) return fail(WOST_ERR_INVALID_ARG, "internal: block larger than a batch");
            count = blk_end(j2 - 1) - wb;
            a.wid_begin = wb;
            a.base_pid = wb / W;
            const int64_t off = wb - a.base_pid * W;
            a.base_off = (uint32_t)std::min<int64_t>(off, INT32_MAX);
            a.small32 = (W < (int64_t(1) << 31) && off + count < (int64_t(1) << 31)) ? 1 : 0;
            a.range_walks = 0;
        }
        begins.push_back(count);
        const int64_t nb = j2 - j;

        // (the previous batch's copy from the staging has completed: its events were waited on)
        std::memcpy(pin_begin, begins.data(), sizeof(int64_t) * (size_t)(nb + 1));
        if (points_pending) {   // points and block ranges in one copy
            HIP_TRY(hipMemcpyAsync(h->d_stage, h->h_pin, pin_pts + sizeof(int64_t) * (size_t)(nb + 1),
                                   hipMemcpyHostToDevice, h->stream));
            points_pending = false;
        } else {
            HIP_TRY(hipMemcpyAsync(h->d_begin, pin_begin, sizeof(int64_t) * (nb + 1), hipMemcpyHostToDevice, h->stream));
        }
        // the queue head: zeroed by the previous launch's block reduce, or here after a
        // solve that stopped between a walk launch and its reduce
        if (!h->counter_zero)
            HIP_TRY(hipMemsetAsync(h->d_counter, 0, sizeof(unsigned long long) * kCtlWords, h->stream));
        h->counter_zero = false;

        a.out_val = h->d_val;
        a.out_steps = h->d_steps;
        a.count = count;
        // The launch's shape is a function of this call alone (never of an earlier solve:
        // the reference calls solve() once per script, so the first call is the one that
        // counts). Walks without a Neumann boundary (Laplace, Poisson, delta tracking on a
        // Dirichlet-only domain) are short (13-17 steps); those with one (C3's circle, the
        // DCR scenarios, C5) run 17-208.
        const bool short_walks = !mode_neu(mode);
        // Resident workgroups: few short walks per lane (C2: 640k walks, ~1.2 per lane at
        // full occupancy) leave the launch as long as its longest walk chains, whose steps
        // run faster with fewer waves per SIMD: ~2 walks per lane, at least 2 workgroups per
        // CU (C2: 8 -> 2 per CU took 0.21 -> 0.18 ms, profiles/r05_ab/grid_c2/; with the
        // all-static first chunk below 4 per CU beat 2: 0.127 -> 0.110 ms, and 8 stays best
        // at 4x C2's walks, profiles/r06_ab/r06s37/)
        int64_t bpc = blocks_per_cu;
        if (short_walks && bpc > 2)
            bpc = std::max<int64_t>(2, std::min<int64_t>(bpc, count / ((int64_t)h->num_cus * block * 2)));
        if (O.grid_blocks_per_cu > 0) bpc = std::max<int64_t>(1, std::min<int64_t>(blocks_per_cu, O.grid_blocks_per_cu));
        const int64_t max_grid = bpc * h->num_cus;
        const int64_t want = (count + block - 1) / block;
        const int grid = (int)std::max<int64_t>(1, std::min(max_grid, want));
        const int64_t waves = (int64_t)grid * (block / 64);
        // The work queue (wost_walk.h): a static chunk of walks per wave (below), then
        // chunks of the rest from one global counter. Every dequeue of that
        // counter serialises at its address (~11-16 ns): C2's 640k walks took 34k dequeues of
        // 19 walks, all waves hitting the counter at the launch's start, 0.60 ms for 47 us of
        // work (profiles/r05_ab/queue_chunk/, queue_static/).
        // - static chunks except for the segment-tree kernels: their long walks lose by them
        //   when launches run concurrently (the C5 survey's handle pairs: a late-starting
        //   wave still owns its 64 walks; 1.38e10 -> 1.34e10, profiles/r05_ab/queue_c5/);
        // - the dequeue's size: max(floor, min(cap, count / (waves * 4))), floor 64 for short
        //   walks and 1 otherwise; cap 64 walks (one per lane), 16 for the segment-tree
        //   kernels' long walks (C5: 208 steps; a wave's last chunk is work no other wave can
        //   take: the survey 1.42e10 -> 1.46e10, profiles/r05_ab/chunk_cap/); each wave then
        //   raises it to the floor its measured walk rate needs (WalkArgs::adaptive).
        // - the static first chunk: at most one walk per lane (64) for long walks; for short
        //   ones every walk of the launch when that is at most 6 per lane (no wave dequeues at
        //   all), else 4 per lane (256). C2's 640k walks: 313 per wave, kernel 0.176 ->
        //   0.129 ms; 12.8M walks of Laplace / Poisson: 256, +12% / +6% (64 took one walk
        //   per lane and left ~8k dequeues serialised at the counter; profiles/r06_ab/r06s3[12]/)
        const int64_t per_wave = (count + waves - 1) / waves;
        int64_t chunk0 = mode_tree(mode)  ? 0
                         : !short_walks   ? std::min<int64_t>(64, per_wave)
                         : per_wave <= 384 ? per_wave
                                           : 256;
        if (O.chunk0 >= 0) chunk0 = O.chunk0;
        const int64_t share = std::max<int64_t>(1, std::min<int64_t>(1 << 20, count / (waves * 4)));
        int64_t chunk_min = short_walks ? 64 : 1;
        if (O.chunk_min >= 1) chunk_min = O.chunk_min;
        int64_t chunk_max = mode_tree(mode) ? 16 : 64;
        if (O.chunk_max >= 1) chunk_max = O.chunk_max;
        a.chunk0 = (int32_t)chunk0;
        a.queue_base = waves * chunk0;
        a.chunk = (int)std::max<int64_t>(chunk_min, std::min<int64_t>(chunk_max, share));
        // (a guided queue -- the last ~4 walks per lane in chunks of 64 -- measured no faster
        // on C4 and 10-14% slower on the short-walk scenarios: profiles/r02_ab/guided_queue.log)
        // (the waves' rate floor assumes the 100 MHz wall clock of gfx950; the segment-tree
        // kernels keep their host-sized dequeues)
        const bool adaptive = !mode_tree(mode) && O.adaptive_chunk != 0 && O.chunk_min < 1 && O.chunk_max < 1 && h->tick_khz == 100000.0;
        a.chunk_share = adaptive ? (uint32_t)std::max<int64_t>(share, a.chunk) : 0u;
        a.waves = (uint32_t)std::min<int64_t>(waves, INT32_MAX);
        if ((int64_t)ctl_words(waves) > h->ctl_cap) {   // more waves than the control block holds
            HIP_TRY(hipStreamSynchronize(h->stream));
            (void)hipFree(h->d_counter);
            h->d_counter = nullptr;
            h->ctl_cap = 0;
            HIP_TRY(hipMalloc(&h->d_counter, sizeof(unsigned long long) * ctl_words(waves)));
            HIP_TRY(hipMemset(h->d_counter, 0, sizeof(unsigned long long) * ctl_words(waves)));
            h->ctl_cap = (int64_t)ctl_words(waves);
            a.counter = h->d_counter;
        }
        h->timing.blocks_per_cu = (int32_t)bpc;
        h->timing.block_threads = block;
        h->timing.chunk0 = (int32_t)chunk0;
        h->timing.chunk = a.chunk;
        h->timing.adaptive = adaptive ? 1 : 0;
        h->timing.grid_blocks = grid;

        HIP_TRY(hipEventRecord(h->ev[0], h->stream));
        if (jfn) {
            void* args[] = {&a};
            HIP_TRY(hipModuleLaunchKernel(jfn, grid, 1, 1, block, 1, 1, (unsigned)lds, h->stream, args, nullptr));
        } else {
            HIP_TRY(launch_walk(mode, a, grid, h->stream));
        }
        HIP_TRY(hipEventRecord(h->ev[1], h->stream));
        HIP_TRY(launch_block_reduce(h->d_val, h->d_steps, h->d_begin, nb, ns, d_rows + row * (j - block_begin),
                                    h->d_counter, h->stream, mode_tree(mode) ? 0 : waves, d_lstats,
                                    launches == 0 ? 1 : 0));   // (the tree kernels keep no wave records)
        h->counter_zero = true;
        HIP_TRY(hipEventRecord(h->ev[2], h->stream));
        if (walk_values)
            HIP_TRY(hipMemcpyAsync(walk_values + walks_done * ns, h->d_val, sizeof(float) * count * ns,
                                   hipMemcpyDeviceToHost, h->stream));
        if (walk_steps)
            HIP_TRY(hipMemcpyAsync(walk_steps + walks_done, h->d_steps, sizeof(uint32_t) * count, hipMemcpyDeviceToHost, h->stream));
        if (records)
            HIP_TRY(hipMemcpyAsync(records + walks_done * rec_stride * kRecFloats, d_rec, (size_t)count * rec_walk_bytes,
                                   hipMemcpyDeviceToHost, h->stream));
        const bool last = j2 >= block_end;
        if (last) {   // the block sums ride the same wait
            HIP_TRY(hipMemcpyAsync(pin_bstats, h->d_bstats, sizeof(double) * (kLstatsWords + row * nblk),
                                   hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipEventRecord(h->ev[5], h->stream));
            HIP_TRY(hipEventSynchronize(h->ev[5]));
        } else {
            HIP_TRY(hipEventSynchronize(h->ev[2]));
        }
        float t0 = 0.f, t1 = 0.f;
        HIP_TRY(hipEventElapsedTime(&t0, h->ev[0], h->ev[1]));
        HIP_TRY(hipEventElapsedTime(&t1, h->ev[1], h->ev[2]));
        walk_ms += t0;
        red_ms += t1;
        ++launches;
        walks_done += count;
        j = j2;
    }
    if (O.tree_iter_stats && a.pool != nullptr) {   // study builds: the tree queries' loop counters
        const int64_t nwg = (int64_t)blocks_per_cu * h->num_cus;
        std::vector<uint32_t> pw((size_t)(a.pool_wg_words * nwg));
        HIP_TRY(hipMemcpy(pw.data(), a.pool, sizeof(uint32_t) * pw.size(), hipMemcpyDeviceToHost));
        const int64_t off = a.pool_wg_words - 16;
        double c[16] = {};
        for (int64_t g = 0; g < nwg; ++g)
            for (int i = 0; i < 16; ++i) c[i] += pw[(size_t)(g * a.pool_wg_words + off + i)];
        std::fprintf(stderr, "tree_iter_stats:");
        for (int i = 0; i < 16; ++i) std::fprintf(stderr, " %.0f", c[i]);
        std::fprintf(stderr, "\n");
    }
    const double* bs = pin_bstats + kLstatsWords;   // (copied and waited for with the last batch)
    {   // the launch statistics (wost_kernels.hip reduce_wave_stats), wall-clock ticks
        unsigned long long ls[kLstatsWords];
        std::memcpy(ls, pin_bstats, sizeof(ls));
        const double ms_per_tick = 1.0 / h->tick_khz;
        h->timing.max_walk_steps = (uint32_t)std::min<unsigned long long>(ls[3], 0xFFFFFFFFull);
        h->timing.span_ms = ls[2] > ls[0] ? (double)(ls[2] - ls[0]) * ms_per_tick : 0.0;
        h->timing.tail_ms = ls[2] > ls[1] ? (double)(ls[2] - ls[1]) * ms_per_tick : 0.0;
        h->timing.last_wave_ms = (double)ls[5] * ms_per_tick;
        h->timing.last_wave_iters = (uint32_t)ls[4];
        h->timing.max_wave_iters = (uint32_t)ls[6];
    }
    float tt = 0.f;
    HIP_TRY(hipEventElapsedTime(&tt, h->ev[4], h->ev[5]));

    uint64_t steps_sum = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        steps_sum += (uint64_t)bs[row * b + row - 1];
        if (point_stats) {
            const int64_t p = (block_begin + b) / (range ? nbr : nbpp);
            for (int c = 0; c < row; ++c) point_stats[row * p + c] += bs[row * b + c];
        }
    }
    if (block_stats) std::memcpy(block_stats, bs, sizeof(double) * row * nblk);
    h->timing.walk_kernel_ms = walk_ms;
    h->timing.reduce_kernel_ms = red_ms;
    h->timing.total_ms = tt;
    h->timing.n_launches = launches;
    h->timing.total_steps = steps_sum;
    h->timing.total_walks = (uint64_t)walks_total;
    h->timing.jit_ms = jit_ms;
    h->timing.jit = jfn ? 1 : 0;
    h->timing.tree = mode_tree(mode) ? 1 : 0;
    return WOST_OK;
}

// Accumulates a piece's timing into a multi-launch solve's (wost_solve_range, solve_race).
void add_timing(wost_timing& acc, const wost_timing& t) {
    acc.walk_kernel_ms += t.walk_kernel_ms;
    acc.reduce_kernel_ms += t.reduce_kernel_ms;
    acc.total_ms += t.total_ms;
    acc.n_launches += t.n_launches;
    acc.total_steps += t.total_steps;
    acc.total_walks += t.total_walks;
    acc.grid_blocks = t.grid_blocks;
    acc.jit = t.jit;
    acc.tree = t.tree;
    acc.blocks_per_cu = t.blocks_per_cu;
    acc.block_threads = t.block_threads;
    acc.chunk0 = t.chunk0;
    acc.chunk = t.chunk;
    acc.adaptive = t.adaptive;
    acc.max_walk_steps = std::max(acc.max_walk_steps, t.max_walk_steps);
    acc.jit_ms += t.jit_ms;
    acc.span_ms += t.span_ms;
    acc.tail_ms = t.tail_ms;
    acc.last_wave_ms = t.last_wave_ms;
    acc.last_wave_iters = t.last_wave_iters;
    acc.max_wave_iters = std::max(acc.max_wave_iters, t.max_wave_iters);
    acc.precompiled_walks += t.precompiled_walks;
}

// A whole single-source solve whose field-specialised kernel is in no cache (option
// jit_race; the reference calls solve() once per script): its compile starts in a helper
// process, and meanwhile the precompiled kernel -- the same bits walk for walk
// (test_jit_kernel_matches_interpreted_kernel) but 2-5x slower -- runs the walks in ranges
// of every point (the first ~2^19 walks, then ~16 ms of work each); once the compile is
// done the specialised kernel runs the rest. Ranges of walks are whole blocks, so the
// block sums, their order and every output are those of one launch (as wost_solve_range's).
// A solve that finds the compile already running waits for it instead (jit_get_kernel).
constexpr double kCompileExpectMs = 300.0;   // a specialised kernel's compile (MI355X box: 180-600 ms)

int solve_race(wost_handle* h, const float* points, int64_t n_points, int64_t W, int32_t max_steps, float eps,
               uint64_t seed, double* block_stats, double* point_stats, float* walk_values, uint32_t* walk_steps) {
    const int64_t nb = wost_num_blocks(n_points, W);
    auto plain = [&]() {
        return solve_impl(h, points, n_points, W, 0, nb, max_steps, eps, seed, block_stats, point_stats, walk_values,
                          walk_steps, nullptr);
    };
    if (!points) return plain();
    for (int64_t i = 0; i < 2 * n_points; ++i)
        if (!std::isfinite(points[i])) return plain();   // (its error message)
    const int mode = walk_mode(h);
    if (mode_delta(mode) && !h->fields[SLOT_F].present) return plain();
    HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = upload_program(h)) != WOST_OK) return rc;
    if (mode_tree(mode) && (rc = ensure_tree(h)) != WOST_OK) return rc;
    KernelShape ks;
    if ((rc = first_kernel_shape(h, mode, n_points, &ks)) != WOST_OK) return rc;
    JitTicket ticket;
    const int stage = ks.tree_lds > 0 ? (ks.tree_verts > 0 ? 2 : 1) : 0;
    if (jit_kernel_try(h, mode, ks.block, ks.gpoly, stage, &ticket) != JitTry::kStarted) return plain();

    const int row = 3;
    const int64_t nbpp = (W + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    const int64_t max_piece = kMaxBatchWalks / WOST_BLOCK_WALKS * WOST_BLOCK_WALKS;   // walks of a point per launch
    auto blocks_up = [](double walks) {
        const double b = std::ceil(std::max(walks, 1.0) / WOST_BLOCK_WALKS);
        return (int64_t)std::min(b, 1e15) * WOST_BLOCK_WALKS;
    };
    int64_t piece = std::min(max_piece, blocks_up((double)(1 << 19) / (double)n_points));
    const auto race_t0 = std::chrono::steady_clock::now();
    std::vector<double> all((size_t)n_points * nbpp * row), part;
    std::vector<float> pv;
    std::vector<uint32_t> ps;
    wost_timing acc{};
    bool jit_now = false;
    const bool saved = h->jit_enabled;
    for (int64_t w0 = 0; w0 < W;) {
        if (!jit_now && ticket.done()) jit_now = true;
        const int64_t w1 = std::min(W, w0 + (jit_now ? max_piece : piece));
        const int64_t wc = w1 - w0, nbc = (wc + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
        part.resize((size_t)n_points * nbc * row);
        if (walk_values) pv.resize((size_t)n_points * wc);
        if (walk_steps) ps.resize((size_t)n_points * wc);
        h->jit_enabled = jit_now;
        const auto t0 = std::chrono::steady_clock::now();
        // (the whole range is an ordinary solve: solve_impl takes [0, W) as no range)
        const bool whole = w0 == 0 && w1 == W;
        rc = solve_impl(h, points, n_points, W, 0, whole ? nb : 0, max_steps, eps, seed, part.data(), nullptr,
                        walk_values ? pv.data() : nullptr, walk_steps ? ps.data() : nullptr, nullptr, false, w0,
                        whole ? -1 : w1);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        h->jit_enabled = saved;
        if (rc == WOST_ERR_UNSUPPORTED && !jit_now) {   // (a shape only the specialised kernel runs)
            jit_now = true;
            continue;
        }
        if (rc != WOST_OK) return rc;
        const int64_t boff = w0 / WOST_BLOCK_WALKS;
        for (int64_t p = 0; p < n_points; ++p) {
            std::memcpy(&all[((size_t)p * nbpp + boff) * row], &part[(size_t)p * nbc * row], sizeof(double) * nbc * row);
            if (walk_values) std::memcpy(walk_values + (size_t)p * W + w0, &pv[(size_t)p * wc], sizeof(float) * wc);
            if (walk_steps) std::memcpy(walk_steps + (size_t)p * W + w0, &ps[(size_t)p * wc], sizeof(uint32_t) * wc);
        }
        if (!jit_now) {
            h->timing.precompiled_walks = (uint64_t)(n_points * wc);
            // the next range, from this one's rate: all the rest when the precompiled kernel
            // finishes it before the compile is likely done (every range ends in a tail of
            // the longest walks: one launch, not many); else about half the compile's
            // expected remaining time, at least 16 ms of work, at most 8x this range
            const double rate = (double)wc / std::max(ms, 0.05);   // walks per point per ms
            const double since = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                                            race_t0).count();
            const double compile_left = std::max(0.0, kCompileExpectMs - since);
            if ((double)(W - w1) / rate <= compile_left) {
                piece = std::min(max_piece, W - w1);
            } else {
                const double target = std::max(16.0, 0.5 * compile_left);
                piece = std::min(max_piece, std::max(piece, std::min(8 * piece, blocks_up(rate * target))));
            }
        }
        add_timing(acc, h->timing);
        w0 = w1;
    }
    if (block_stats) std::memcpy(block_stats, all.data(), sizeof(double) * all.size());
    if (point_stats) {
        std::fill(point_stats, point_stats + (size_t)row * n_points, 0.0);
        for (int64_t p = 0; p < n_points; ++p)
            for (int64_t b = 0; b < nbpp; ++b)
                for (int c = 0; c < row; ++c) point_stats[(size_t)row * p + c] += all[((size_t)p * nbpp + b) * row + c];
    }
    acc.jit = jit_now ? 1 : 0;
    h->timing = acc;
    return WOST_OK;
}

// The handle's fields with sources[0..n) in the source slots (wost_set_sources' conversion).
int fields_with_sources(const wost_handle* h, const wost_field* const* sources, int32_t n, HostField* out) {
    if (n < 1 || n > WOST_MAX_SOURCES || !sources)
        return fail(WOST_ERR_INVALID_ARG, "need 1..%d sources (got %d)", WOST_MAX_SOURCES, n);
    std::vector<HostField> conv(n);
    int64_t grid = 0;
    for (int s = 0; s < n; ++s) {
        if (!sources[s]) return fail(WOST_ERR_INVALID_ARG, "source %d is NULL", s);
        char name[32];
        std::snprintf(name, sizeof(name), "source[%d]", s);
        int rc = convert_field(sources[s], conv[s], name);
        if (rc != WOST_OK) return rc;
        grid += (int64_t)conv[s].grid.size();
    }
    for (int s = 0; s < N_SLOTS; ++s)
        if (s != SLOT_F) grid += (int64_t)h->fields[s].grid.size();
    if (grid >= (int64_t(1) << 24))
        return fail(WOST_ERR_INVALID_ARG, "tabulated fields hold %lld values together (limit 2^24)", (long long)grid);
    for (int s = 0; s < N_FIELDS; ++s) out[s] = h->fields[s];
    out[SLOT_F] = conv[0];
    for (int s = 1; s < WOST_MAX_SOURCES; ++s) out[SLOT_EXTRA + s - 1] = s < n ? conv[s] : HostField();
    return WOST_OK;
}

std::mutex g_prepare_mu;   // wost_prepare_sources: one segment-tree build per handle

}  // namespace

extern "C" {

int wost_solve(wost_handle* h, const float* points, int64_t n_points, int64_t W,
               int64_t block_begin, int64_t block_end, int32_t max_steps, float eps, uint64_t seed,
               double* block_stats, double* point_stats, float* walk_values, uint32_t* walk_steps) {
    // a whole single-source solve may start on the precompiled kernel while its specialised
    // one compiles (solve_race)
    if (h && h->jit_enabled && h->opt.jit_race && h->n_sources == 1 && n_points > 0 && W > 0 && block_begin == 0 &&
        block_end == wost_num_blocks(n_points, W) && max_steps >= 0 && eps == eps)
        return solve_race(h, points, n_points, W, max_steps, eps, seed, block_stats, point_stats, walk_values,
                          walk_steps);
    return solve_impl(h, points, n_points, W, block_begin, block_end, max_steps, eps, seed, block_stats,
                      point_stats, walk_values, walk_steps, nullptr);
}

int wost_solve_range(wost_handle* h, const float* points, int64_t n_points, int64_t W, int64_t walk_begin,
                     int64_t walk_end, int32_t max_steps, float eps, uint64_t seed, double* block_stats,
                     double* point_stats, float* walk_values, uint32_t* walk_steps) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    if (walk_begin == 0 && walk_end == W) {   // the whole range: an ordinary solve
        const int64_t nb = wost_num_blocks(n_points, W);
        return solve_impl(h, points, n_points, W, 0, nb, max_steps, eps, seed, block_stats, point_stats,
                          walk_values, walk_steps, nullptr, true);
    }
    const int ns = h->n_sources;
    const int64_t chunk = (kMaxBatchWalks / ns) / WOST_BLOCK_WALKS * WOST_BLOCK_WALKS;   // walks of a point per launch
    if (walk_end - walk_begin <= chunk || walk_begin < 0 || walk_end <= walk_begin || n_points <= 0)
        return solve_impl(h, points, n_points, W, 0, 0, max_steps, eps, seed, block_stats, point_stats, walk_values,
                          walk_steps, nullptr, true, walk_begin, walk_end);
    // a range longer than one launch holds per point: block-aligned sub-ranges, one solve
    // each, scattered into the range's layout; point sums in the range's block order
    const int row = 2 * ns + 1;
    const int64_t Wr = walk_end - walk_begin;
    const int64_t nbr = (Wr + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    std::vector<double> all((size_t)n_points * nbr * row);
    std::vector<double> part;
    std::vector<float> pv;
    std::vector<uint32_t> ps;
    wost_timing acc{};
    for (int64_t c0 = walk_begin; c0 < walk_end; c0 += chunk) {
        const int64_t c1 = std::min(walk_end, c0 + chunk);
        const int64_t wc = c1 - c0, nbc = (wc + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
        const int64_t boff = (c0 - walk_begin) / WOST_BLOCK_WALKS, woff = c0 - walk_begin;
        part.resize((size_t)n_points * nbc * row);
        if (walk_values) pv.resize((size_t)n_points * wc * ns);
        if (walk_steps) ps.resize((size_t)n_points * wc);
        int rc = solve_impl(h, points, n_points, W, 0, 0, max_steps, eps, seed, part.data(), nullptr,
                            walk_values ? pv.data() : nullptr, walk_steps ? ps.data() : nullptr, nullptr, true, c0, c1);
        if (rc != WOST_OK) return rc;
        for (int64_t p = 0; p < n_points; ++p) {
            std::memcpy(&all[((size_t)p * nbr + boff) * row], &part[(size_t)p * nbc * row], sizeof(double) * nbc * row);
            if (walk_values)
                std::memcpy(walk_values + ((size_t)p * Wr + woff) * ns, &pv[(size_t)p * wc * ns], sizeof(float) * wc * ns);
            if (walk_steps) std::memcpy(walk_steps + (size_t)p * Wr + woff, &ps[(size_t)p * wc], sizeof(uint32_t) * wc);
        }
        add_timing(acc, h->timing);
    }
    if (block_stats) std::memcpy(block_stats, all.data(), sizeof(double) * all.size());
    if (point_stats) {
        std::fill(point_stats, point_stats + (size_t)row * n_points, 0.0);
        for (int64_t p = 0; p < n_points; ++p)
            for (int64_t b = 0; b < nbr; ++b)
                for (int c = 0; c < row; ++c) point_stats[(size_t)row * p + c] += all[((size_t)p * nbr + b) * row + c];
    }
    h->timing = acc;
    return WOST_OK;
}

int wost_solve_history(wost_handle* h, const float* points, int64_t n_points, int64_t W, int32_t max_steps,
                       float eps, uint64_t seed, double* point_stats, float* walk_values, uint32_t* walk_steps,
                       float* records) {
    if (!records) return fail(WOST_ERR_INVALID_ARG, "NULL records");
    const int64_t nb = wost_num_blocks(n_points, W);
    return solve_impl(h, points, n_points, W, 0, nb, max_steps, eps, seed, nullptr, point_stats, walk_values,
                      walk_steps, records);
}

int wost_solve_multi(wost_handle* h, const float* points, int64_t n_points, int64_t W, int64_t block_begin,
                     int64_t block_end, int32_t max_steps, float eps, uint64_t seed, double* block_stats,
                     double* point_stats, float* walk_values, uint32_t* walk_steps) {
    return solve_impl(h, points, n_points, W, block_begin, block_end, max_steps, eps, seed, block_stats, point_stats,
                      walk_values, walk_steps, nullptr, true);
}

int wost_set_sources(wost_handle* h, const wost_field* const* sources, int32_t n) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    std::vector<HostField> f(N_FIELDS);
    int rc = fields_with_sources(h, sources, n, f.data());
    if (rc != WOST_OK) return rc;
    for (int s = 0; s < N_FIELDS; ++s) h->fields[s] = std::move(f[s]);
    h->n_sources = n;
    h->prog_dirty = true;
    HIP_TRY(hipSetDevice(h->device));
    return upload_program(h);
}

int wost_prepare_sources(wost_handle* h, const wost_field* const* sources, int32_t n, int64_t n_points) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    if (n_points < 1) return fail(WOST_ERR_INVALID_ARG, "n_points must be >= 1 (got %lld)", (long long)n_points);
    std::vector<HostField> f(N_FIELDS);
    int rc = fields_with_sources(h, sources, n, f.data());
    if (rc != WOST_OK) return rc;
    if (!h->jit_enabled)
        return fail(WOST_ERR_UNSUPPORTED, "multi-source solves need the field-specialised kernel (disabled by wost_set_jit)");
    Program prog;
    build_program(f.data(), h->sigma_bar, prog);
    const int mode = walk_mode_src(h, f[SLOT_F].present);
    HIP_TRY(hipSetDevice(h->device));
    if (mode_tree(mode)) {   // the staging choice depends on the tree's size
        std::lock_guard<std::mutex> lock(g_prepare_mu);
        if ((rc = ensure_tree(h)) != WOST_OK) return rc;
    }
    KernelShape ks;
    if ((rc = first_kernel_shape(h, mode, n_points, &ks)) != WOST_OK) return rc;
    const int stage = ks.tree_lds > 0 ? (ks.tree_verts > 0 ? 2 : 1) : 0;
    std::string src, err;
    if ((rc = jit_source(h, prog, mode, false, n, ks.block, ks.gpoly, stage, &src)) != WOST_OK) return rc;
    hipFunction_t fn = nullptr;
    if (!jit_get_kernel(h->opt, h->device, src, &fn, &err, nullptr, nullptr))
        return fail(WOST_ERR_UNSUPPORTED, "field-specialised kernel unavailable: %s", err.c_str());
    return WOST_OK;
}

int wost_kernel_source_sources(const wost_problem* pb, const wost_field* const* sources, int32_t n_sources,
                               char* out, int64_t capacity, int64_t* length) {
    if (!pb || !length) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    if (n_sources < 0 || n_sources > WOST_MAX_SOURCES || (n_sources > 0 && !sources))
        return fail(WOST_ERR_INVALID_ARG, "need 0..%d sources", WOST_MAX_SOURCES);
    wost_handle* h = nullptr;
    int rc = create_host(pb, &h);
    if (rc != WOST_OK) return rc;
    int ns = 1;
    if (n_sources >= 1) {   // wost_set_sources' fields, without a device
        for (int k = 0; k < n_sources; ++k) {
            HostField hf;
            if (!sources[k] || (rc = convert_field(sources[k], hf, "source")) != WOST_OK) {
                delete h;
                return rc != WOST_OK ? rc : fail(WOST_ERR_INVALID_ARG, "source %d is NULL", k);
            }
            h->fields[k == 0 ? SLOT_F : SLOT_EXTRA + k - 1] = hf;
        }
        ns = n_sources;
    }
    build_program(h->fields, h->sigma_bar, h->prog);
    const int mode = walk_mode(h);
    // no device here: the segment angles of a compiled-in Neumann polyline come from the
    // host's atan2f (the kernels use the device's bits; this source is for offline study)
    const int nn = (int)(h->nverts.size() / 2);
    std::vector<float> phi(nn > 1 ? nn - 1 : 0);
    for (int i = 0; i + 1 < nn; ++i) {
        const float2 a{h->nverts[2 * i], h->nverts[2 * i + 1]}, b{h->nverts[2 * i + 2], h->nverts[2 * i + 3]};
        const float2 n = segment_left_normal(a, b);
        phi[i] = std::atan2(n.y, n.x);
    }
    // study builds: offline study of the tree kernels' LDS staging (tools/jit_isa.py --stage):
    // the source of staging level WOST_KERNEL_SOURCE_STAGE (2: records and vertices, 1:
    // records, with the tree_lds_block workgroup) instead of the 256-thread unstaged kernel
    int stage = 0, block = kWalkBlock;
#if defined(WOST_STUDY)
    if (const char* e = std::getenv("WOST_KERNEL_SOURCE_STAGE"); e && mode_tree(mode)) {
        stage = std::max(0, std::min(2, std::atoi(e)));
        block = stage == 2 ? kTreeStageVertsBlock : stage == 1 ? h->opt.tree_lds_block : kWalkBlock;
    }
#endif
    const std::string src = jit_generate(h->opt, mode, *h->prog.hdr(), h->prog.terms(), h->prog.factors(), h->dverts.data(),
                                         (int)(h->dverts.size() / 2), h->nverts.data(), nn, false, ns, block,
                                         phi.empty() ? nullptr : phi.data(), false, stage, exact_trig_of(h));
    delete h;
    *length = (int64_t)src.size();
    if (out && capacity > 0) {
        const size_t n = std::min<size_t>(src.size(), (size_t)capacity - 1);
        std::memcpy(out, src.data(), n);
        out[n] = '\0';
    }
    return WOST_OK;
}

int wost_kernel_source(const wost_problem* pb, char* out, int64_t capacity, int64_t* length) {
    return wost_kernel_source_sources(pb, nullptr, 0, out, capacity, length);
}

int wost_jit_compile(const char* source, const char* arch, int32_t in_process, uint8_t* out, int64_t capacity,
                     int64_t* length, int32_t* used_helper) {
    if (!source || !arch || !*arch || !length) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    Options opt;   // a new handle's compile options
    opt.jit_process = in_process ? 0 : 1;
    std::vector<char> code;
    std::string err;
    bool helper = false;
    if (!jit_compile_host(opt, source, arch, &code, &err, &helper))
        return fail(WOST_ERR_UNSUPPORTED, "%s", err.c_str());
    if (used_helper) *used_helper = helper ? 1 : 0;
    *length = (int64_t)code.size();
    if (out && capacity < (int64_t)code.size())
        return fail(WOST_ERR_INVALID_ARG, "capacity %lld < the code object's %lld bytes", (long long)capacity,
                    (long long)code.size());
    if (out) std::memcpy(out, code.data(), code.size());
    return WOST_OK;
}

int wost_set_segment_tree(wost_handle* h, int32_t min_segments, int32_t leaf_segments) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    if (leaf_segments < 0 || leaf_segments > 32) return fail(WOST_ERR_INVALID_ARG, "leaf_segments must be in [0, 32]");
    h->tree_min_segments = min_segments;
    if (leaf_segments > 0 && leaf_segments != h->tree_leaf) {
        h->tree_leaf = leaf_segments;
        h->tree_ready = false;
    }
    return WOST_OK;
}

int wost_set_trig(wost_handle* h, int32_t mode) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    if (mode != WOST_TRIG_AUTO && mode != WOST_TRIG_EXACT && mode != WOST_TRIG_FAST)
        return fail(WOST_ERR_INVALID_ARG, "trig mode must be WOST_TRIG_AUTO, _EXACT or _FAST");
    h->trig_mode = mode;
    h->jit_fn = nullptr;
    h->jit_mode = -1;
    return WOST_OK;
}

int wost_set_fixed_step_check(wost_handle* h, int32_t enable) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    h->fixed_step_check = enable != 0;
    return WOST_OK;
}

int wost_set_jit(wost_handle* h, int32_t enable) {
    if (!h) return fail(WOST_ERR_INVALID_ARG, "NULL handle");
    h->jit_enabled = enable != 0;
    h->jit_fn = nullptr;
    h->jit_mode = -1;
    return WOST_OK;
}

int wost_set_option(wost_handle* h, const char* name, double value) {
    if (!h || !name) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    bool kernel = false;
    const int rc = options_set(h->opt, name, value, &kernel);
    if (rc == -1) return fail(WOST_ERR_INVALID_ARG, "unknown option \"%s\" (wost_options.h)", name);
    if (rc == -2) return fail(WOST_ERR_INVALID_ARG, "option \"%s\": value %g out of range", name, value);
    if (rc == -3)
        return fail(WOST_ERR_UNSUPPORTED, "option \"%s\" exists in study builds only (make study)", name);
    if (kernel) {   // the generated source changes: rebuild the handle's kernel
        h->jit_fn = nullptr;
        h->jit_mode = -1;
    }
    return WOST_OK;
}

int wost_get_option(const wost_handle* h, const char* name, double* value) {
    if (!h || !name || !value) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    if (options_get(h->opt, name, value) != 0) return fail(WOST_ERR_INVALID_ARG, "unknown option \"%s\"", name);
    return WOST_OK;
}

int wost_options_report(const wost_handle* h, char* out, int64_t capacity, int64_t* length) {
    if (!length) return fail(WOST_ERR_INVALID_ARG, "NULL length");
    Options fresh;   // without a handle: what a new handle gets (study builds: from the environment)
    options_from_study_env(fresh);
    const std::string r = options_report(h ? h->opt : fresh);
    *length = (int64_t)r.size();
    if (out && capacity > 0) {
        const size_t n = std::min<size_t>(r.size(), (size_t)capacity - 1);
        std::memcpy(out, r.data(), n);
        out[n] = '\0';
    }
    return WOST_OK;
}

int wost_eval_field(wost_handle* h, int32_t which, const float* points, int64_t n, float* out) {
    if (!h || (n > 0 && (!points || !out))) return fail(WOST_ERR_INVALID_ARG, "NULL argument");
    if (which < 0 || which > 4) return fail(WOST_ERR_INVALID_ARG, "which must be 0..4");
    if (n == 0) return WOST_OK;
    HIP_TRY(hipSetDevice(h->device));
    int rc = upload_program(h);
    if (rc != WOST_OK) return rc;
    float2* dp = nullptr;
    float4* dout = nullptr;
    HIP_TRY(hipMalloc(&dp, sizeof(float2) * n));
    hipError_t e = hipMalloc(&dout, sizeof(float4) * n);
    if (e == hipSuccess) e = hipMemcpyAsync(dp, points, sizeof(float2) * n, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = launch_eval_field(h->d_prog, which, dp, n, dout, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(float4) * n, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(dp);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return fail(WOST_ERR_HIP, "wost_eval_field: %s", hipGetErrorString(e));
    return WOST_OK;
}

int wost_geometry_query(int32_t device, int32_t op, const wost_polyline* poly, const float* points,
                        const float* dirs, const float* radii, int64_t n, float* out_f, uint8_t* out_mask) {
    if (!poly || !poly->xy || poly->n_vertices < 1) return fail(WOST_ERR_INVALID_ARG, "bad polyline");
    const bool tree = (op & WOST_GEOM_TREE) != 0;
    op &= ~WOST_GEOM_TREE;
    if (op < WOST_GEOM_DISTANCE || op > WOST_GEOM_INTERSECT_POLYLINES) return fail(WOST_ERR_INVALID_ARG, "unknown op %d", op);
    if (tree && op != WOST_GEOM_SILHOUETTE_DISTANCE && op != WOST_GEOM_INTERSECT_POLYLINES)
        return fail(WOST_ERR_INVALID_ARG, "the segment tree answers silhouetteDistance and intersectPolylines only");
    const int nv = poly->n_vertices;
    if (tree && nv < 3) return fail(WOST_ERR_INVALID_ARG, "the segment tree needs >= 2 segments");
    if ((op == WOST_GEOM_DISTANCE || op == WOST_GEOM_RAY_INTERSECTION || op == WOST_GEOM_INTERSECT_POLYLINES) && nv < 2)
        return fail(WOST_ERR_INVALID_ARG, "op %d needs a polyline with >= 2 vertices", op);
    if (n < 0 || (n > 0 && !points)) return fail(WOST_ERR_INVALID_ARG, "bad points");
    const bool need_dirs = op == WOST_GEOM_RAY_INTERSECTION || op == WOST_GEOM_INTERSECT_POLYLINES;
    if (need_dirs && n > 0 && !dirs) return fail(WOST_ERR_INVALID_ARG, "directions required");
    if (op == WOST_GEOM_INTERSECT_POLYLINES && n > 0 && !radii) return fail(WOST_ERR_INVALID_ARG, "radii required");
    const int64_t nf_out = op == WOST_GEOM_RAY_INTERSECTION ? n * (nv - 1)
                         : op == WOST_GEOM_INTERSECT_POLYLINES ? 5 * n
                         : op == WOST_GEOM_IS_SILHOUETTE ? 0 : n;
    const int64_t nm_out = op == WOST_GEOM_IS_SILHOUETTE ? n * std::max(0, nv - 2) : 0;
    if ((nf_out > 0 && !out_f) || (nm_out > 0 && !out_mask)) return fail(WOST_ERR_INVALID_ARG, "output buffer missing");
    if (n == 0) return WOST_OK;
    SegmentTreeHost th;
    if (tree && !build_segment_tree(poly->xy, nv, WOST_TREE_LEAF_DEFAULT, &th) &&
        !build_segment_tree(poly->xy, nv, 32, &th))
        return fail(WOST_ERR_INVALID_ARG, "no segment tree for this polyline (degenerate or too long)");
    HIP_TRY(hipSetDevice(device));
    float4* drec = nullptr;
    if (tree) {
        HIP_TRY(hipMalloc(&drec, sizeof(float) * std::max<size_t>(th.rec.size(), 4)));
        const hipError_t e0 = hipMemcpy(drec, th.rec.data(), sizeof(float) * th.rec.size(), hipMemcpyHostToDevice);
        if (e0 != hipSuccess) {
            (void)hipFree(drec);
            return fail(WOST_ERR_HIP, "wost_geometry_query: %s", hipGetErrorString(e0));
        }
    }
    float2 *dv = nullptr, *dp = nullptr, *dd = nullptr;
    float *dr = nullptr, *df = nullptr;
    uint8_t* dm = nullptr;
    hipError_t e = hipMalloc(&dv, sizeof(float2) * nv);
    if (e == hipSuccess) e = hipMalloc(&dp, sizeof(float2) * n);
    if (e == hipSuccess && need_dirs) e = hipMalloc(&dd, sizeof(float2) * n);
    if (e == hipSuccess && op == WOST_GEOM_INTERSECT_POLYLINES) e = hipMalloc(&dr, sizeof(float) * n);
    if (e == hipSuccess && nf_out > 0) e = hipMalloc(&df, sizeof(float) * nf_out);
    if (e == hipSuccess && nm_out > 0) e = hipMalloc(&dm, nm_out);
    if (e == hipSuccess) e = hipMemcpy(dv, poly->xy, sizeof(float2) * nv, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dp, points, sizeof(float2) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && dd) e = hipMemcpy(dd, dirs, sizeof(float2) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && dr) e = hipMemcpy(dr, radii, sizeof(float) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = tree ? launch_geometry_tree_query(op, dv, nv, drec, th.first_leaf, th.depth, th.leaf, th.tol, th.kmax, dp,
                                              dd, dr, n, df, nullptr)
                 : launch_geometry_query(op, dv, nv, dp, dd, dr, n, df, dm, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess && df) e = hipMemcpy(out_f, df, sizeof(float) * nf_out, hipMemcpyDeviceToHost);
    if (e == hipSuccess && dm) e = hipMemcpy(out_mask, dm, nm_out, hipMemcpyDeviceToHost);
    void* all[] = {dv, dp, dd, dr, df, dm, drec};
    for (void* p : all)
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return fail(WOST_ERR_HIP, "wost_geometry_query: %s", hipGetErrorString(e));
    return WOST_OK;
}

}  // extern "C"
