// wost_jit.cpp -- see wost_jit.h.
#include "wost_jit.h"
#include "wost_internal.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hiprtc.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <condition_variable>
#include <cstddef>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>
#include <vector>

#include "wost_rtc.h"

extern char** environ;

// Header sources embedded at build time (Makefile: wost_embedded.cpp).
extern const char wost_embedded_wost_h[];
extern const char wost_embedded_wost_device_h[];
extern const char wost_embedded_wost_walk_h[];

namespace wost {
namespace {

// Exact float32 literal (hex float), or a builtin for non-finite values.
// y = RN(1/duu) for the segment a->b when the Markstein step q + (duv - q duu) y
// (q = RN(duv y)) equals RN(duv / duu) for every duv mantissa (checked
// exhaustively, once per mantissa of duu, cached), else 0 (wost_device.h
// poly_distance_rcp). duu is formed exactly like the kernel forms it.
// A/B switches for tools/ab_bench.sh (Options::exp_flags, a bit mask: study builds
// only, from WOST_EXP_FLAGS; always 0 in the product library): 1 generic poly_distance for compiled-in polylines, 2 IEEE
// unit_direction. Ablations (timing studies only: the results are WRONG, the
// walks merely stay statistically alike): 4 a cheap hash instead of Philox, 8 no
// alpha(z) evaluation, 16 no sigma' at collisions, 32 no Neumann ray query;
// 64 compiled-in silhouette scans unrolled by 4 only, 128 the device library's sinf/cosf
// instead of v_sin/v_cos when the handle's directions use the hardware trig
// (wost_set_trig); 512 no
// whole-field saturation shortcut in the alpha jet (jet_body); 1024 compiled-in
// Neumann ray scans unrolled by 2 instead of fully; 2048 sqrtf instead of
// sqrt_rn for the distances; 4096 the tree's ray query
// without its behind-the-origin pruning; 8192 the per-segment reciprocal filter
// (intersect_polylines_compact) instead of the per-vertex line filter
// (intersect_polylines_lines); 16384 the per-segment exact tests instead of either
// two-pass scan for 8+ compiled-in segments; 32768 the one-pass compiled-in
// silhouette scan instead of silhouette_distance_compact; ablation 65536 no
// silhouette query (dn = +inf).
// Each bit only selects one fixed code path.

// the squared segment length exactly as the kernel forms it
float segment_duu(float ax, float ay, float bx, float by) {
#pragma clang fp contract(off)
    volatile float ux = bx - ax, uy = by - ay;
    volatile float duu = ux * ux + uy * uy;
    return duu;
}

float markstein_reciprocal(float ax, float ay, float bx, float by) {
    const float d = segment_duu(ax, ay, bx, by);
    if (!(d >= 0x1p-40f && d <= 0x1p40f)) return 0.0f;
    uint32_t db;
    std::memcpy(&db, &d, 4);
    const uint32_t mant = db & 0x7FFFFFu;
    if (mant == 0) return 0.0f;   // a power of two: the compiler folds the division into an exact multiply
    static std::mutex mu;
    static std::map<uint32_t, bool> ok_cache;
    bool ok;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = ok_cache.find(mant);
        if (it != ok_cache.end()) {
            ok = it->second;
        } else {
            if (ok_cache.size() >= 64) return 0.0f;   // bound the host time (~25 ms per length)
            const uint32_t bb = 0x3F800000u | mant;
            float b;
            std::memcpy(&b, &bb, 4);
            volatile float one = 1.0f, vb = b;
            const float y = one / vb;
            ok = true;
            for (uint32_t m = 0; m < (1u << 23) && ok; ++m) {
                const uint32_t ab = 0x3F800000u | m;
                float a;
                std::memcpy(&a, &ab, 4);
                const float q = a * y;
                const float got = std::fma(std::fma(-q, b, a), y, q);
                volatile float va = a;
                const float want = va / vb;
                ok = std::memcmp(&got, &want, 4) == 0;
            }
            ok_cache[mant] = ok;
        }
    }
    if (!ok) return 0.0f;
    volatile float one = 1.0f;
    return one / d;
}

std::string lit(float v) {
    if (v != v) return "__builtin_nanf(\"\")";
    if (v == __builtin_inff()) return "__builtin_inff()";
    if (v == -__builtin_inff()) return "(-__builtin_inff())";
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%af", (double)v);
    return buf;
}

std::string factor_call(const DFactor& f, bool jet) {
    const float* p = f.p;
    std::ostringstream o;
    const char* pre = jet ? "wost::fj_" : "wost::fv_";
    switch (f.kind) {
    case WOST_FK_MONO:
        o << pre << "mono(x, y, " << (int)p[0] << ", " << (int)p[1] << ")";
        break;
    case WOST_FK_EXP_QUAD: {
        const bool diag = exp_quad_is_diag(p);   // the interpreter makes the same choice
        o << pre << (diag ? "exp_quad_diag(x, y" : "exp_quad(x, y");
        for (int k = 0; k < (diag ? 4 : 8); ++k) o << ", " << lit(p[k]);
        o << ")";
        break;
    }
    case WOST_FK_SIN_LIN:
        o << pre << "sin_lin(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ")";
        break;
    case WOST_FK_COS_LIN:
        o << pre << "cos_lin(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ")";
        break;
    case WOST_FK_SIGMOID_LIN:
        o << pre << "sigmoid_lin(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ")";
        break;
    case WOST_FK_SIGMOID_RADIAL:
        o << pre << "sigmoid_radial(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ", "
          << lit(p[3]) << ")";
        break;
    case WOST_FK_IND_BOX:
        o << pre << "ind_box(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ", " << lit(p[3])
          << ")";
        break;
    case WOST_FK_IND_DISK:
        o << pre << "ind_disk(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ")";
        break;
    case WOST_FK_GRID:   // values stay in the program buffer (grid = its tabulated part)
        o << pre << "grid(grid + " << (int)p[6] << ", x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2])
          << ", " << lit(p[3]) << ", " << (int)p[4] << ", " << (int)p[5] << ")";
        break;
    default:
        o << (jet ? "wost::Jet{__builtin_nanf(\"\"), 0.f, 0.f, 0.f}" : "__builtin_nanf(\"\")");
    }
    return o.str();
}

// Same operation sequence as wost::field_value.
std::string value_body(const DField& fd, const DTerm* terms, const DFactor* factors) {
    std::ostringstream o;
    o << "        float acc = 0.0f;\n";
    for (int t = 0; t < fd.n_terms; ++t) {
        const DTerm& tm = terms[fd.first_term + t];
        o << "        { float t = " << lit(tm.coef) << ";";
        for (int k = 0; k < tm.nf; ++k) o << " t = t * " << factor_call(factors[tm.first + k], false) << ";";
        o << " acc = acc + t; }\n";
    }
    o << "        return acc;\n";
    return o.str();
}

// Multi-source kernels with Options::param_sources: the source fields' coefficients and
// factor parameters are read from the program buffer (uniform loads through the constant
// address space) instead of compiled in as literals, so that the kernel's source -- and its
// hiprtc compile -- depends on the sources' structure (factor kinds, term counts, monomial
// exponents, grid shapes) and not on where the electrodes are. The C5 Wenner survey
// launches every electrode group with other transmitters: with literals its first survey
// compiles 36 kernels (~22 s of hiprtc one after another, profiles/r06_ab/r06s8), with
// parameters 2 (4.6 s) -- but its warm survey runs 5% slower on the loads
// (profiles/r06_ab/r06s9, r06s11), so literals stay the default (the survey's threads
// request their compiles at once, jit_get_kernel, but ROCm's compiler library runs one
// in-process compile at a time). The same float values enter the same operations: the bits
// of a single-source solve (tests/test_gpu_multisource.py).
std::string pv(size_t off) {
    std::ostringstream o;
    o << "pv(pb, " << off << "u)";
    return o.str();
}

std::string factor_call_param(const DFactor& f, size_t foff) {
    const float* p = f.p;
    const size_t p0 = foff + offsetof(DFactor, p);
    auto P = [&](int k) { return pv(p0 + 4 * (size_t)k); };
    std::ostringstream o;
    switch (f.kind) {
    case WOST_FK_MONO:
        o << "wost::fv_mono(x, y, " << (int)p[0] << ", " << (int)p[1] << ")";
        break;
    case WOST_FK_EXP_QUAD: {
        const bool diag = exp_quad_is_diag(p);   // structure: the interpreter makes the same choice
        o << (diag ? "wost::fv_exp_quad_diag(x, y" : "wost::fv_exp_quad(x, y");
        for (int k = 0; k < (diag ? 4 : 8); ++k) o << ", " << P(k);
        o << ")";
        break;
    }
    case WOST_FK_SIN_LIN:
    case WOST_FK_COS_LIN:
    case WOST_FK_SIGMOID_LIN:
        o << (f.kind == WOST_FK_SIN_LIN ? "wost::fv_sin_lin" : f.kind == WOST_FK_COS_LIN ? "wost::fv_cos_lin"
                                                                                         : "wost::fv_sigmoid_lin")
          << "(x, y, " << P(0) << ", " << P(1) << ", " << P(2) << ")";
        break;
    case WOST_FK_SIGMOID_RADIAL:
        o << "wost::fv_sigmoid_radial(x, y, " << P(0) << ", " << P(1) << ", " << P(2) << ", " << P(3) << ")";
        break;
    case WOST_FK_IND_BOX:
        o << "wost::fv_ind_box(x, y, " << P(0) << ", " << P(1) << ", " << P(2) << ", " << P(3) << ")";
        break;
    case WOST_FK_IND_DISK:
        o << "wost::fv_ind_disk(x, y, " << P(0) << ", " << P(1) << ", " << P(2) << ")";
        break;
    case WOST_FK_GRID:   // the shape and the offset stay literals (structure)
        o << "wost::fv_grid(grid + " << (int)p[6] << ", x, y, " << P(0) << ", " << P(1) << ", " << P(2) << ", " << P(3)
          << ", " << (int)p[4] << ", " << (int)p[5] << ")";
        break;
    default:
        o << "__builtin_nanf(\"\")";
    }
    return o.str();
}

// value_body with the coefficients and factor parameters read from the program buffer.
// canon[j]: the factor whose parameters factor j reads -- the first one with the same kind
// and parameters (a Wenner group's transmitters share electrodes: the same Gaussian then
// reads the same words, and the compiler evaluates it once, as it does with literals).
std::string value_body_param(const DField& fd, const DTerm* terms, const DFactor* factors, int n_terms_total,
                             const std::vector<int>& canon) {
    std::ostringstream o;
    const size_t toff = sizeof(DProgram), foff = sizeof(DProgram) + sizeof(DTerm) * (size_t)n_terms_total;
    o << "        float acc = 0.0f;\n";
    for (int t = 0; t < fd.n_terms; ++t) {
        const int ti = fd.first_term + t;
        const DTerm& tm = terms[ti];
        o << "        { float t = " << pv(toff + sizeof(DTerm) * (size_t)ti + offsetof(DTerm, coef)) << ";";
        for (int k = 0; k < tm.nf; ++k)
            o << " t = t * "
              << factor_call_param(factors[tm.first + k], foff + sizeof(DFactor) * (size_t)canon[tm.first + k]) << ";";
        o << " acc = acc + t; }\n";
    }
    o << "        return acc;\n";
    return o.str();
}

// The saturation predicate of a factor (wost_device.h sat_*), "true" for the
// indicators (zero derivatives everywhere), "" for a kind without one.
std::string sat_call(const DFactor& f) {
    const float* p = f.p;
    std::ostringstream o;
    switch (f.kind) {
    case WOST_FK_SIGMOID_RADIAL:
        o << "wost::sat_sigmoid_radial(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ", "
          << lit(p[3]) << ", centre)";
        break;
    case WOST_FK_SIGMOID_LIN:
        o << "wost::sat_sigmoid_lin(x, y, " << lit(p[0]) << ", " << lit(p[1]) << ", " << lit(p[2]) << ")";
        break;
    case WOST_FK_EXP_QUAD: {
        const bool diag = exp_quad_is_diag(p);
        o << (diag ? "wost::sat_exp_quad_diag(x, y" : "wost::sat_exp_quad(x, y");
        for (int k = 0; k < (diag ? 4 : 8); ++k) o << ", " << lit(p[k]);
        o << ")";
        break;
    }
    case WOST_FK_IND_BOX:
    case WOST_FK_IND_DISK:
        return "true";
    default:
        return "";
    }
    return o.str();
}

// Same operation sequence as wost::field_jet. When every factor has a saturation
// predicate and the coefficients are finite, a wave whose lanes are all saturated
// returns {value, z, z, z} (wost_device.h, whole-field saturation): the value from
// `value_fn` (the field's value body, the same bits as the jet's value there).
std::string jet_body(const DField& fd, const DTerm* terms, const DFactor* factors, const char* value_fn, int xflags) {
    std::ostringstream o;
    if (value_fn != nullptr && !(xflags & 512)) {
        std::ostringstream s;
        bool ok = fd.n_terms > 0, radial = false;
        for (int t = 0; t < fd.n_terms && ok; ++t) {
            const DTerm& tm = terms[fd.first_term + t];
            ok = std::isfinite(tm.coef);
            for (int k = 0; k < tm.nf && ok; ++k) {
                const DFactor& f = factors[tm.first + k];
                const std::string c = sat_call(f);
                ok = !c.empty();
                radial |= f.kind == WOST_FK_SIGMOID_RADIAL;
                if (ok && c != "true") s << (s.tellp() > 0 ? " & " : "") << c;
            }
        }
        if (ok && s.tellp() > 0) {
            o << "        {\n"
              << "            bool centre = false;\n"
              << "            const bool sat = " << s.str() << ";\n"
              << "            if (WOST_SAT_ALL(sat)) {\n"
              << "                const float z = " << (radial ? "centre ? __builtin_nanf(\"\") : 0.0f" : "0.0f")
              << ";\n"
              << "                return wost::Jet{" << value_fn << "(x, y), z, z, z};\n"
              << "            }\n"
              << "        }\n";
        }
    }
    o << "        wost::Jet acc = wost::jet_const(0.0f);\n";
    for (int t = 0; t < fd.n_terms; ++t) {
        const DTerm& tm = terms[fd.first_term + t];
        if (tm.nf == 0) {
            o << "        acc = wost::jet_add(acc, wost::jet_const(" << lit(tm.coef) << "));\n";
            continue;
        }
        o << "        { wost::Jet t = wost::jet_scale(" << lit(tm.coef) << ", " << factor_call(factors[tm.first], true)
          << ");";
        for (int k = 1; k < tm.nf; ++k) o << " t = wost::jet_mul(t, " << factor_call(factors[tm.first + k], true) << ");";
        o << " acc = wost::jet_add(acc, t); }\n";
    }
    o << "        return acc;\n";
    return o.str();
}

uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

std::string cache_dir() {
    if (const char* d = std::getenv("WOST_JIT_CACHE")) return d;
    if (const char* x = std::getenv("XDG_CACHE_HOME")) return std::string(x) + "/wost";
    if (const char* h = std::getenv("HOME")) return std::string(h) + "/.cache/wost";
    return "";
}

// File I/O by system calls only: a background compile's thread (jit_try_kernel) may still
// run while the process exits and its C++ runtime's statics are torn down.
bool read_file(const std::string& path, std::vector<char>& out) {
    const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    out.clear();
    char buf[1 << 16];
    for (;;) {
        const ssize_t n = read(fd, buf, sizeof(buf));
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) break;
        out.insert(out.end(), buf, buf + n);
    }
    close(fd);
    return !out.empty();
}

bool write_file(const std::string& path, const char* data, size_t size) {
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return false;
    size_t done = 0;
    while (done < size) {
        const ssize_t n = write(fd, data + done, size - done);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) break;
        done += (size_t)n;
    }
    return close(fd) == 0 && done == size;
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::vector<char>& data) {
    if (dir.empty()) return;
    std::string cur;
    for (size_t i = 0; i <= dir.size(); ++i) {   // mkdir -p
        if (i == dir.size() || dir[i] == '/') {
            cur = dir.substr(0, i);
            if (!cur.empty()) mkdir(cur.c_str(), 0755);
        }
    }
    // (the thread too: two threads of one process may compile the same kernel at once)
    std::string tmp = dir + "/" + name + ".tmp." + std::to_string(getpid()) + "." +
                      std::to_string(std::hash<std::thread::id>{}(std::this_thread::get_id()));
    if (write_file(tmp, data.data(), data.size())) std::rename(tmp.c_str(), (dir + "/" + name).c_str());
    else unlink(tmp.c_str());
}

struct Entry {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    hipFunction_t alpha_fn = nullptr;   // wost_point_alpha_jit, when the source has it
};

std::mutex g_mu;
std::map<std::string, Entry> g_modules;   // key: device:arch:hash

// hiprtc options besides --offload-arch. They change the code's FP semantics, so they
// are part of the cache key (cache_identity), as are the compiler and runtime versions.
const char* const kCompileOptions[] = {"-O3", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt",
                                       "-ffp-contract=fast-honor-pragmas"};
constexpr int kCacheFormat = 2;   // bump when the generator or the cached file layout changes

// Study builds only: Options::jit_sched (WOST_JIT_SCHED=<strategy>) adds -mllvm
// -amdgpu-sched-strategy=<strategy> (max-ilp, max-memory-clause, iterative-ilp, ...).
std::string sched_option(const Options& opt) {
    return !opt.jit_sched.empty() ? std::string("-amdgpu-sched-strategy=") + opt.jit_sched : std::string();
}

// -fno-slp-vectorize: no packed FP32 (v_pk_*) from the SLP vectoriser. On gfx950 a
// v_pk_{add,mul,fma}_f32 issues in the time of two scalar ones, and the pairs of
// constants it wants in SGPRs pushed the long unrolled scans (C3's 32-segment ray
// query, the tree traversal) past the SGPR budget into v_writelane/v_readlane
// spills. Options::jit_slp = 1 keeps the vectoriser (A/B).
bool slp_off(const Options& opt) { return opt.jit_slp == 0; }

std::vector<std::string> compile_options(const Options& opt, const std::string& arch) {
    std::vector<std::string> opts = {"--offload-arch=" + arch};
    for (const char* o : kCompileOptions) opts.push_back(o);
    if (slp_off(opt)) opts.push_back("-fno-slp-vectorize");
    const std::string sched = sched_option(opt);
    if (!sched.empty()) {
        opts.push_back("-mllvm");
        opts.push_back(sched);
    }
    return opts;
}

// A private scratch directory for one helper run, removed with its files.
struct Scratch {
    std::string dir;
    std::vector<std::string> files;
    bool ok = false;
    Scratch() {
        const char* tmp = std::getenv("TMPDIR");
        dir = std::string(tmp && *tmp ? tmp : "/tmp") + "/wost_jitc.XXXXXX";
        ok = mkdtemp(&dir[0]) != nullptr;
    }
    std::string file(const char* name) {
        files.push_back(dir + "/" + name);
        return files.back();
    }
    ~Scratch() {
        for (const std::string& f : files) unlink(f.c_str());
        if (ok) rmdir(dir.c_str());
    }
};

// Runs `args` (args[0] the program) as a child process with stdin from /dev/null and
// stdout / stderr into the given files, and waits for it. true when it exited 0; else
// false and *err says how it ended.
bool run_child(std::vector<std::string> args, const std::string& out_path, const std::string& err_path,
               std::string* err) {
    std::vector<char*> argv;
    for (std::string& a : args) argv.push_back(&a[0]);
    argv.push_back(nullptr);
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
    posix_spawn_file_actions_addopen(&fa, 1, out_path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
    posix_spawn_file_actions_addopen(&fa, 2, err_path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
    pid_t pid = -1;
    const int rc = posix_spawn(&pid, args[0].c_str(), &fa, nullptr, argv.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    if (rc != 0) {
        *err = "posix_spawn(" + args[0] + "): " + std::strerror(rc);
        return false;
    }
    int status = 0;
    while (waitpid(pid, &status, 0) < 0) {
        if (errno != EINTR) {
            *err = std::string("waitpid: ") + std::strerror(errno);
            return false;
        }
    }
    if (WIFEXITED(status) && WEXITSTATUS(status) == 0) return true;
    *err = WIFEXITED(status) ? "exit status " + std::to_string(WEXITSTATUS(status))
                             : "signal " + std::to_string(WTERMSIG(status));
    return false;
}

// The compile helper next to this library (dcrmontecarlo_amd/wost_jitc), or "" when it is
// not there (then every compile runs in this process).
const std::string& helper_path() {
    static const std::string path = [] {
        Dl_info info;
        if (!dladdr(reinterpret_cast<void*>(&helper_path), &info) || !info.dli_fname) return std::string();
        std::string lib = info.dli_fname;
        const size_t slash = lib.rfind('/');
        std::string p = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/wost_jitc";
        return access(p.c_str(), X_OK) == 0 ? p : std::string();
    }();
    return path;
}

// The hiprtc library the helper compiles with (wost_jitc --identity, run once per
// process), or "" when there is no helper or it cannot run: compiles stay in this process.
// wost_create starts the probe in the background (jit_start_identity_probe: ~13 ms of the
// child's start that then overlaps building the handle); the first compile waits for it.
std::string run_identity_probe(const std::string& helper) {
    if (helper.empty()) return std::string();
    Scratch sc;
    if (!sc.ok) return std::string();
    const std::string out = sc.file("identity.txt"), log = sc.file("log.txt");
    std::string err;
    std::vector<char> text;
    if (!run_child({helper, "--identity"}, out, log, &err) || !read_file(out, text)) {
        std::fprintf(stderr, "libwost: compile helper %s unusable (%s); compiling in this process\n", helper.c_str(),
                     err.c_str());
        return std::string();
    }
    std::string s(text.begin(), text.end());
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    return s;
}

struct IdentityProbe {   // (never destroyed: its thread may outlive the process's statics)
    std::mutex mu;
    std::condition_variable cv;
    bool started = false, done = false;
    std::string id;
};
IdentityProbe& identity_probe() {
    static IdentityProbe* p = new IdentityProbe;
    return *p;
}

void finish_identity_probe(const std::string& id) {
    IdentityProbe& p = identity_probe();
    std::lock_guard<std::mutex> lock(p.mu);
    p.id = id;
    p.done = true;
    p.cv.notify_all();
}

const std::string& helper_identity() {
    IdentityProbe& p = identity_probe();
    std::unique_lock<std::mutex> lock(p.mu);
    if (!p.started) {   // no handle started it: probe here
        p.started = true;
        lock.unlock();
        finish_identity_probe(run_identity_probe(helper_path()));
        lock.lock();
    }
    p.cv.wait(lock, [&p] { return p.done; });
    return p.id;
}

bool use_helper(const Options& opt) { return opt.jit_process != 0 && !helper_identity().empty(); }

const std::string& rtc_library_once() {
    static const std::string lib = rtc_library();
    return lib;
}

enum class Route { kAuto, kHelper, kInProcess };

// The compiler a handle's compile uses: its option jit_process with a usable helper
// routes through the helper's compiler, else this process's.
const std::string& route_compiler(const Options& opt) {
    return use_helper(opt) ? helper_identity() : rtc_library_once();
}


// The cache key's compile identity: the format, the compile options, the compiler -- the
// hiprtc library that compiles (the helper's, or the one this process bound: a process that
// imported PyTorch-ROCm first binds PyTorch's own copy, another ROCm release's compiler) --
// and the HIP runtime that loads the code.
std::string cache_identity(const Options& opt) {
    std::string id = "fmt" + std::to_string(kCacheFormat);
    for (const char* o : kCompileOptions) id += std::string("|") + o;
    if (!sched_option(opt).empty()) id += "|-mllvm " + sched_option(opt);
    if (slp_off(opt)) id += "|-fno-slp-vectorize";
    int maj = 0, min = 0, rt = 0;
    if (hiprtcVersion(&maj, &min) == HIPRTC_SUCCESS) id += "|hiprtc" + std::to_string(maj) + "." + std::to_string(min);
    id += "|rtc=" + route_compiler(opt);
    if (hipRuntimeGetVersion(&rt) == hipSuccess) id += "|hip" + std::to_string(rt);
    return id;
}

// At most this many helpers run at once (survey.prepare_survey_kernels: 16 threads): the
// compiles are CPU work, and the GPU box's share of the host is 16 cores.
// (never destroyed: a background compile's thread may outlive the process's statics)
constexpr int kMaxHelpers = 16;
std::mutex& g_helper_mu = *new std::mutex;
std::condition_variable& g_helper_cv = *new std::condition_variable;
int g_helpers = 0;

// One compile in a child process (wost_jitc): source, code object and the compiler's
// log pass through files of a private scratch directory. false (and *err) when the helper
// could not be started or did not produce a code object; the caller then compiles here.
bool compile_in_helper(const std::string& helper, const std::vector<std::string>& opts, const std::string& src,
                       std::vector<char>& code, std::string* err) {
    {
        std::unique_lock<std::mutex> lock(g_helper_mu);
        g_helper_cv.wait(lock, [] { return g_helpers < kMaxHelpers; });
        ++g_helpers;
    }
    struct Slot {
        ~Slot() {
            { std::lock_guard<std::mutex> lock(g_helper_mu); --g_helpers; }
            g_helper_cv.notify_one();
        }
    } slot;
    Scratch sc;
    if (!sc.ok) {
        *err = std::string("mkdtemp: ") + std::strerror(errno);
        return false;
    }
    const std::string src_path = sc.file("kernel.hip"), out_path = sc.file("kernel.hsaco"),
                      log_path = sc.file("log.txt"), stdout_path = sc.file("stdout.txt");
    if (!write_file(src_path, src.data(), src.size())) {
        *err = "cannot write " + src_path;
        return false;
    }
    // (--parent: a helper whose parent has exited removes its scratch directory itself)
    std::vector<std::string> args = {helper, "--parent=" + std::to_string(getpid()), src_path, out_path};
    args.insert(args.end(), opts.begin(), opts.end());
    std::string how;
    if (run_child(args, stdout_path, log_path, &how) && read_file(out_path, code)) return true;
    std::vector<char> log;
    read_file(log_path, log);
    *err = "wost_jitc " + (how.empty() ? std::string("wrote no code object") : how) + ": " +
           std::string(log.begin(), log.end());
    return false;
}

std::mutex g_inproc_mu;   // at most one compile in this process (comgr serialises them anyway)

// A compile for `arch`: in a helper (kAuto: handles with jit_process; kHelper), so that
// concurrent compiles overlap, or here (kInProcess). A helper that fails falls back to
// this process. (Routing a lone compile here instead saved its child's start, ~25 ms, but
// made a survey's 34 concurrent compiles 0.6-1.2 s slower: profiles/r06_cold/s23_*.)
// *compiler: the hiprtc library that compiled (the disk cache only takes code of the
// compiler its key names).
bool compile(const Options& opt, Route route, const std::string& src, const std::string& arch,
             std::vector<char>& code, std::string* err, std::string* compiler, bool* in_helper) {
    const std::vector<std::string> opts = compile_options(opt, arch);
    *in_helper = false;
    const bool helper = route != Route::kInProcess && !helper_identity().empty();
    if (helper) {
        std::string herr;
        if (compile_in_helper(helper_path(), opts, src, code, &herr)) {
            *compiler = helper_identity();
            *in_helper = true;
            return true;
        }
        std::fprintf(stderr, "libwost: compile helper failed, compiling in this process: %s\n", herr.c_str());
    }
    std::lock_guard<std::mutex> lock(g_inproc_mu);
    *compiler = rtc_library_once();
    return rtc_compile(src, opts, &code, err);
}

}  // namespace

bool jit_compile_host(const Options& opt, const std::string& source, const std::string& arch,
                      std::vector<char>* code, std::string* err, bool* in_helper) {
    std::string compiler;
    return compile(opt, opt.jit_process ? Route::kHelper : Route::kInProcess, source, arch, *code, err, &compiler,
                   in_helper);
}

bool jit_helper_available() { return !helper_identity().empty(); }

void jit_start_identity_probe() {
    IdentityProbe& p = identity_probe();
    {
        std::lock_guard<std::mutex> lock(p.mu);
        if (p.started) return;
        p.started = true;
    }
    const std::string helper = helper_path();
    try {
        std::thread([helper]() { finish_identity_probe(run_identity_probe(helper)); }).detach();
    } catch (...) {
        finish_identity_probe(run_identity_probe(helper));
    }
}

bool jit_const_dirichlet(const Options& o, int nd) { return nd <= o.const_vertices; }

bool jit_const_neumann(const Options& o, int mode, int nn) {
    return mode_neu(mode) && !mode_tree(mode) && nn >= 1 && nn <= o.const_vertices;
}

bool jit_fused_neumann_scan(const Options& o, int mode, int nn) {
    // (Options::fused_scan = 0: the two separate scans, the round-4 kernel; same bits)
    return mode_neu(mode) && !mode_tree(mode) && !mode_fix(mode) && !jit_const_neumann(o, mode, nn) && nn >= 66 &&
           o.fused_scan != 0;
}

std::string jit_generate(const Options& opt, int mode, const DProgram& hdr, const DTerm* terms, const DFactor* factors,
                         const float* dverts, int nd, const float* nverts, int nn, bool record, int n_sources,
                         int block, const float* seg_phi, bool global_polylines, int tree_stage,
                         bool exact_trig) {
    const bool neu = mode_neu(mode);
    const bool src = mode_src(mode);
    const bool delta = mode_delta(mode);
    const bool tree = mode_tree(mode);
    const DField& fG = hdr.field[SLOT_G];
    const DField& fF = hdr.field[SLOT_F];
    const DField& fS = hdr.field[SLOT_SIGMA];
    const DField& fA = hdr.field[SLOT_ALPHA];
    std::ostringstream o;
    const int xf = opt.exp_flags;   // study builds only (0 in the product library)
    if (xf & 2) o << "#define WOST_EXP_IEEE_DIRECTION 1\n";
    if (xf & 4096) o << "#define WOST_NO_TREE_BEHIND 1\n";   // A/B: line pruning only
    if (xf & 4) o << "#define WOST_ABL_NO_PHILOX 1\n";
    if (xf & 8) o << "#define WOST_ABL_NO_ALPHA_Z 1\n";
    if (xf & 16) o << "#define WOST_ABL_NO_SIGMA_PRIME 1\n";
    if (xf & 32) o << "#define WOST_ABL_NO_RAY 1\n";
    if (xf & 65536) o << "#define WOST_ABL_NO_SILHOUETTE 1\n";
    if (xf & 64) o << "#define WOST_EXP_PARTIAL_UNROLL 1\n";
    if (xf & 128) o << "#define WOST_EXP_LIBM_SINCOS 1\n";
    if (xf & (1 << 29)) o << "#define WOST_EXP_UNIT_TAB 1\n";   // A/B: unit_direction's (n, y) table
    if (xf & 131072) o << "#define WOST_EXP_SCAN_BITS 1\n";   // A/B: neumann_scan_both's per-vertex bits
    if ((xf >> 18) & 1023) o << "#define WOST_ABL_DUP " << ((xf >> 18) & 1023) << "\n";   // phase_dup.sh
    o << "#define WOST_JIT_TRIG_EXACT " << (exact_trig ? 1 : 0) << "\n";   // wost_set_trig
    if (xf & 2048) o << "#define WOST_EXP_IEEE_SQRT 1\n";
    // the handle's bit-preserving kernel options (wost_set_option; -1: the kernel's default)
    if (opt.philox_ahead >= 0) o << "#define WOST_PHILOX_AHEAD " << opt.philox_ahead << "\n";
    if (opt.refill_min >= 1) o << "#define WOST_REFILL_MIN " << opt.refill_min << "\n";
    if (opt.tree_share >= 0) o << "#define WOST_TREE_SHARE " << opt.tree_share << "\n";
    if (opt.tree_share_descent >= 0) o << "#define WOST_TREE_SHARE_DESCENT " << opt.tree_share_descent << "\n";
    if (opt.pool_min_push != 1) o << "#define WOST_POOL_MIN_PUSH " << opt.pool_min_push << "\n";
    if (opt.tree_iter_stats && tree) o << "#define WOST_TREE_ITER_STATS 1\n";   // study builds: loop counters
    if (tree && tree_stage >= 1) o << "#define WOST_TREE_STAGED 1\n";    // every record in LDS
    if (tree && tree_stage >= 2) o << "#define WOST_TREE_VSTAGED 1\n";   // and the Neumann vertices
    if (opt.tree_qmargin >= 0) o << "#define WOST_TREE_QMARGIN " << opt.tree_qmargin << "\n";
    if (opt.tree_share_min >= 1) o << "#define WOST_TREE_SHARE_MIN " << opt.tree_share_min << "\n";
    if (opt.tree_batch >= 1) o << "#define WOST_TREE_BATCH " << (opt.tree_batch >= 4 ? 4 : opt.tree_batch >= 2 ? 2 : 1) << "\n";
    o << "// generated by libwost (wost_jit.cpp): walk kernel, mode " << mode << "\n"
      << "#include \"wost_walk.h\"\n\nnamespace {\nstruct GenFields {\n"
      << "    const float* grid;   // tabulated field values (WOST_FK_GRID) in the program buffer\n"
      << "    const char* pb;      // the program buffer (multi-source kernels read the sources' parameters)\n"
      << "    __device__ __forceinline__ static float pv(const char* p, unsigned off) {\n"
      << "        return *(const __attribute__((address_space(4))) float*)(p + off);\n    }\n";
    o << "    __device__ __forceinline__ bool has_g() const { return " << (fG.present ? "true" : "false") << "; }\n";
    o << "    __device__ __forceinline__ float g(float x, float y) const {\n"
      << (fG.present ? value_body(fG, terms, factors) : "        return 0.0f;\n") << "    }\n";
    // (a multi-source kernel never calls f(): its walks score the sources through f_multi)
    o << "    __device__ __forceinline__ float f(float x, float y) const {\n"
      << (fF.present && n_sources == 1 ? value_body(fF, terms, factors) : "        return 0.0f;\n") << "    }\n";
    if (n_sources > 1) {   // multi-source: every source's value, each with f()'s operation sequence
        o << "    __device__ __forceinline__ void f_multi(float x, float y, float* out) const {\n";
        std::vector<int> canon(hdr.n_factors_total);   // (value_body_param)
        for (int j = 0; j < hdr.n_factors_total; ++j) {
            canon[j] = j;
            for (int i = 0; i < j; ++i)
                if (factors[i].kind == factors[j].kind && std::memcmp(factors[i].p, factors[j].p, sizeof(factors[j].p)) == 0) {
                    canon[j] = i;
                    break;
                }
        }
        for (int s = 0; s < n_sources; ++s) {
            const DField& fs = hdr.field[s == 0 ? SLOT_F : SLOT_EXTRA + s - 1];
            o << "        out[" << s << "] = [&]() {\n"
              << (!fs.present          ? std::string("        return 0.0f;\n")
                  : opt.param_sources ? value_body_param(fs, terms, factors, hdr.n_terms_total, canon)
                                      : value_body(fs, terms, factors))
              << "        }();\n";
        }
        o << "    }\n";
    }
    o << "    __device__ __forceinline__ float sigma(float x, float y) const {\n"
      << (fS.present ? value_body(fS, terms, factors) : "        return 0.0f;\n") << "    }\n";
    o << "    __device__ __forceinline__ float alpha(float x, float y) const {\n"
      << (fA.present ? value_body(fA, terms, factors) : "        return 1.0f;\n") << "    }\n";
    o << "    __device__ __forceinline__ wost::Jet alpha_jet(float x, float y) const {\n"
      << (fA.present ? jet_body(fA, terms, factors, (fA.flags & WOST_FIELD_DETACHED) ? nullptr : "alpha", xf) : "        return wost::jet_const(1.0f);\n") << "    }\n";
    o << "    __device__ __forceinline__ bool detached() const { return "
      << ((fA.flags & WOST_FIELD_DETACHED) ? "true" : "false") << "; }\n";
    o << "    __device__ __forceinline__ float sigma_bar() const { return " << lit(hdr.sigma_bar) << "; }\n";
    o << "    __device__ __forceinline__ float sqrt_sigma_bar() const { return " << lit(hdr.sqrt_sigma_bar) << "; }\n";
    o << "    __device__ __forceinline__ float inv_sigma_bar() const { return " << lit(hdr.inv_sigma_bar) << "; }\n";
    // a short Dirichlet polyline is compiled in: the scan unrolls, the segment
    // vectors and squared lengths fold to constants (the same IEEE operations)
    const bool dconst = jit_const_dirichlet(opt, nd);
    // a compiled-in Neumann polyline also needs its segment angles as constants
    const bool nconst = jit_const_neumann(opt, mode, nn) && (seg_phi != nullptr || nn < 2);
    o << "    static constexpr bool kConstDirichlet = " << (dconst ? "true" : "false") << ";\n";
    o << "    static constexpr bool kConstNeumann = " << (nconst ? "true" : "false") << ";\n";
    // a long Neumann polyline scanned (no segment tree: the brute-force kernel): both
    // queries in one pass with the per-vertex line filter (neumann_scan_both);
    // Options::fused_scan = 0: the two separate scans instead (A/B)
    const bool fused = !nconst && jit_fused_neumann_scan(opt, mode, nn);
    o << "    static constexpr bool kFusedNeumann = " << (fused ? "true" : "false") << ";\n";
    if (fused) {
        float c1 = 0.0f;
        for (int i = 0; i < nn; ++i) c1 = std::max(c1, std::fabs(nverts[2 * i]) + std::fabs(nverts[2 * i + 1]));
        o << "    __device__ __forceinline__ wost::ScanBoth neumann_scan_both(const float2* sN, int nn, float x, float y,"
             " float dx, float dy) const {\n"
          << "        return wost::neumann_scan_both<" << (global_polylines ? "true" : "false") << ">(sN, nn, "
          << lit(c1 * 1.0001f) << ", x, y, dx, dy);\n    }\n";
    } else {
        o << "    __device__ __forceinline__ wost::ScanBoth neumann_scan_both(const float2*, int, float, float, float,"
             " float) const { return wost::ScanBoth{}; }\n";
    }
    o << "    __device__ __forceinline__ float dirichlet_distance(const float2* sD, int nd, float x, float y) const {\n";
    if (dconst) {
        o << "        const float2 v[" << nd << "] = {";
        for (int i = 0; i < nd; ++i) o << (i ? ", " : "") << "{" << lit(dverts[2 * i]) << ", " << lit(dverts[2 * i + 1]) << "}";
        o << "};\n";
        // poly_distance_const when every segment has 0 < duu and the coordinates are
        // below 2^60, with the reciprocal squared lengths for the Markstein division
        bool ok = nd >= 2 && !(xf & 1);
        std::ostringstream r;
        for (int i = 0; i < nd && ok; ++i) ok = std::fabs(dverts[2 * i]) <= 0x1p60f && std::fabs(dverts[2 * i + 1]) <= 0x1p60f;
        for (int i = 0; ok && i + 1 < nd; ++i) {
            ok = segment_duu(dverts[2 * i], dverts[2 * i + 1], dverts[2 * i + 2], dverts[2 * i + 3]) > 0.0f;
            r << (i ? ", " : "")
              << lit(markstein_reciprocal(dverts[2 * i], dverts[2 * i + 1], dverts[2 * i + 2], dverts[2 * i + 3]));
        }
        if (ok)
            o << "        const float rcp[" << nd - 1 << "] = {" << r.str() << "};\n"
              << "        return wost::poly_distance_const(v, rcp, " << nd << ", x, y);\n";
        else
            o << "        return wost::poly_distance(v, " << nd << ", x, y);\n";
    } else {
        o << "        return wost::poly_distance(sD, nd, x, y);\n";
    }
    o << "    }\n";
    auto nverts_decl = [&]() {
        std::ostringstream v;
        v << "        const float2 v[" << nn << "] = {";
        for (int i = 0; i < nn; ++i) v << (i ? ", " : "") << "{" << lit(nverts[2 * i]) << ", " << lit(nverts[2 * i + 1]) << "}";
        v << "};\n";
        return v.str();
    };
    o << "    __device__ __forceinline__ float neumann_silhouette_distance(const float2* sN, int nn, float x, float y) const {\n";
    // 9+ compiled-in vertices: the two-pass scan (squared distances only for each
    // lane's own silhouette vertices, from the staged copy)
    if (nconst && nn >= 9 && nn <= 66 && !(xf & 32768))
        o << nverts_decl() << "        return wost::silhouette_distance_compact<" << nn << ">(v, sN, x, y);\n";
    else if (nconst) o << nverts_decl() << "        return wost::silhouette_distance<" << nn << ">(v, " << nn << ", x, y);\n";
    else o << "        return wost::silhouette_distance(sN, nn, x, y);\n";
    o << "    }\n";
    o << "    __device__ __forceinline__ wost::Hit neumann_intersect(const float2* sN, int nn, float x, float y, float dx,"
         " float dy, float r) const {\n";
    // (a two-pass variant with one exact division per lane and a rescan on near ties
    // measured slower on C3's 32-segment circle: 1.24e10 vs 1.94e10 walk-steps/s)
    // 8+ compiled-in segments: the two-pass scan (C3's 32-segment circle +11%; with one or
    // two segments its loop costs more than it saves: C4 -9%, profiles/r02_ab/ray_scan_two_pass.log)
    if (nconst && nn >= 9 && nn <= 65 && !(xf & (16384 | 8192))) {   // the per-vertex line filter
        float c1 = 0.0f;
        for (int i = 0; i < nn; ++i) c1 = std::max(c1, std::fabs(nverts[2 * i]) + std::fabs(nverts[2 * i + 1]));
        o << nverts_decl() << "        return wost::intersect_polylines_lines<" << nn << ">(v, sN, x, y, dx, dy, r, "
          << lit(c1 * 1.0001f) << ");\n";
    } else if (nconst && nn >= 9 && nn <= 65 && !(xf & 16384))   // (16384: per-segment exact tests, A/B)
        o << nverts_decl() << "        return wost::intersect_polylines_compact<" << nn << ">(v, sN, x, y, dx, dy, r);\n";
    else if (nconst && !(xf & 1024))   // (1024: the generic unroll-by-2 scan, A/B)
        o << nverts_decl() << "        return wost::intersect_polylines<false, " << nn << ">(v, " << nn
          << ", x, y, dx, dy, r);\n";
    else if (nconst) o << nverts_decl() << "        return wost::intersect_polylines<false>(v, " << nn << ", x, y, dx, dy, r);\n";
    else o << "        return wost::intersect_polylines<false>(sN, nn, x, y, dx, dy, r);\n";
    o << "    }\n";
    o << "    __device__ __forceinline__ wost::Hit neumann_intersect_nearest(const float2* sN, int nn, float x, float y,"
         " float dx, float dy, float r) const {\n";
    // (the staged copy: fully unrolled over compiled-in vertices it measured no faster,
    // profiles/r02_ab/ray_scan_full_unroll.log)
    o << "        return wost::intersect_polylines_ray(sN, nn, x, y, dx, dy, r);\n";
    o << "    }\n";
    o << "    __device__ __forceinline__ float neumann_phi(const float* sPhi, int seg) const {\n";
    if (nconst && nn >= 2) {
        o << "        const float phi[" << nn - 1 << "] = {";
        for (int i = 0; i + 1 < nn; ++i) o << (i ? ", " : "") << lit(seg_phi[i]);
        o << "};\n        return phi[seg];\n";
    } else {
        o << "        return sPhi[seg];\n";
    }
    o << "    }\n};\n}  // namespace\n\n";
    // waves per SIMD the register budget is sized for: 7 for the scan kernels (their
    // 256-thread workgroups are LDS-bound at 7 per CU either way; the 7-wave budget
    // schedules C4 1.3% faster than 6: profiles/r04_ab/scan_waves_6_vs_7_ab.log), 5 for
    // the cooperative tree kernels, whose record visits load four children's words at
    // once (profiles/r03_tree/tree_batch_waves_ab.log), 4 when the tree's records are
    // staged (one 16-wave or two 8-wave workgroups per CU)
    int waves = tree ? (block != kWalkBlock ? 4 : 5) : 7;
    if (opt.jit_waves > 0) waves = opt.jit_waves;
    o << "extern \"C\" __global__ void __launch_bounds__(" << block << ", " << waves << ")\n"
      << "wost_walk_jit(const wost::WalkArgs A) {\n"
      << "    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];\n"
      << "    const GenFields fld{reinterpret_cast<const float*>(A.prog + "
      << program_grid_offset(hdr.n_terms_total, hdr.n_factors_total) << "ull), A.prog};\n"
      << "    wost::walk_body<" << (neu ? "true" : "false") << ", " << (src ? "true" : "false") << ", "
      << (delta ? "true" : "false") << ", " << (tree ? "true" : "false") << ", " << (record ? "true" : "false")
      << ", " << n_sources << ", " << (mode_fix(mode) ? "true" : "false") << ", "
      << (global_polylines ? "true" : "false") << ">(A, fld, smem);\n}\n";
    if (delta)   // alpha at the query points, with these fields (WalkArgs::point_alpha)
        o << "extern \"C\" __global__ void __launch_bounds__(256)\n"
          << "wost_point_alpha_jit(const char* prog, const float2* pts, long long n, float* out) {\n"
          << "    const GenFields fld{reinterpret_cast<const float*>(prog + "
          << program_grid_offset(hdr.n_terms_total, hdr.n_factors_total) << "ull), prog};\n"
          << "    wost::point_alpha_body(pts, (int64_t)n, out, fld);\n}\n";
    return o.str();
}

namespace {

// Background compiles (jit_try_kernel): one record per kernel key, written by a detached
// thread that waits for the compile helper. The records and their lock are never freed:
// the thread may still run while the process exits.
struct Pending {
    int state = 0;   // 0 compiling, 1 done (code), 2 failed
    std::vector<char> code;
};
std::mutex& g_pend_mu = *new std::mutex;
std::condition_variable& g_pend_cv = *new std::condition_variable;
std::map<std::string, Pending*>& g_pending = *new std::map<std::string, Pending*>;

struct KeyInfo {
    std::string arch, key, name, dir;
};

bool key_of(const Options& opt, int device, const std::string& source, KeyInfo* k, std::string* err) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        *err = "hipGetDeviceProperties failed";
        return false;
    }
    k->arch = prop.gcnArchName;
    k->arch = k->arch.substr(0, k->arch.find(':'));
    // the embedded headers, compile options and compiler/runtime versions are part of the
    // key: a rebuilt library, other options or a ROCm upgrade never reuse stale code
    const std::string ident = cache_identity(opt);
    const uint64_t h = fnv1a(source + "|" + k->arch + "|" + ident + "|" + wost_embedded_wost_h +
                             wost_embedded_wost_device_h + wost_embedded_wost_walk_h);
    char hex[32];
    std::snprintf(hex, sizeof(hex), "%016llx", (unsigned long long)h);
    k->key = std::to_string(device) + ":" + k->arch + ":" + hex;
    k->name = std::string("walk_") + k->arch + "_" + hex + ".hsaco";
    k->dir = cache_dir();
#if defined(WOST_STUDY)
    if (const char* dump = std::getenv("WOST_JIT_DUMP")) {   // generated source, for offline ISA study
        const std::string s(source);
        write_file_atomic(dump, std::string("walk_") + hex + ".hip", std::vector<char>(s.begin(), s.end()));
    }
#endif
    return true;
}

bool memory_lookup(const std::string& key, hipFunction_t* fn, hipFunction_t* alpha_fn) {
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_modules.find(key);
    if (it == g_modules.end()) return false;
    *fn = it->second.fn;
    if (alpha_fn) *alpha_fn = it->second.alpha_fn;
    return true;
}

bool load_module(const std::string& key, const std::vector<char>& code, hipFunction_t* fn, hipFunction_t* alpha_fn,
                 std::string* err) {
    Entry e;
    if (hipModuleLoadData(&e.mod, code.data()) != hipSuccess) {
        *err = "hipModuleLoadData failed";
        return false;
    }
    if (hipModuleGetFunction(&e.fn, e.mod, "wost_walk_jit") != hipSuccess) {
        *err = "hipModuleGetFunction(wost_walk_jit) failed";
        return false;
    }
    if (hipModuleGetFunction(&e.alpha_fn, e.mod, "wost_point_alpha_jit") != hipSuccess) e.alpha_fn = nullptr;
    (void)hipGetLastError();   // a source without the alpha kernel leaves a lookup error behind
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_modules.find(key);
    if (it != g_modules.end()) {   // another thread loaded the same kernel meanwhile: use its module
        (void)hipModuleUnload(e.mod);
        e = it->second;
    } else {
        g_modules[key] = e;
    }
    *fn = e.fn;
    if (alpha_fn) *alpha_fn = e.alpha_fn;
    return true;
}

// A finished background compile's code object (state 1), copied out; blocks while one
// runs when `wait`. Returns its state (-1: none).
int pending_code(const std::string& key, bool wait, std::vector<char>* code) {
    std::unique_lock<std::mutex> lock(g_pend_mu);
    auto it = g_pending.find(key);
    if (it == g_pending.end()) return -1;
    Pending* p = it->second;
    if (wait) g_pend_cv.wait(lock, [p] { return p->state != 0; });
    if (p->state == 1) *code = p->code;
    return p->state;
}

}  // namespace

bool JitTicket::done() const {
    if (!p) return true;
    std::lock_guard<std::mutex> lock(g_pend_mu);
    return static_cast<const Pending*>(p)->state != 0;
}

bool jit_get_kernel(const Options& opt, int device, const std::string& source, hipFunction_t* fn, std::string* err,
                    hipFunction_t* alpha_fn, double* compile_ms) {
    if (compile_ms) *compile_ms = 0.0;
    KeyInfo k;
    if (!key_of(opt, device, source, &k, err)) return false;
    // the in-memory cache (the lock is not held during a compile: the handles of a survey's
    // concurrent threads compile their kernels at once)
    if (memory_lookup(k.key, fn, alpha_fn)) return true;
    std::vector<char> code;
    const auto t0 = std::chrono::steady_clock::now();
    // a background compile of it (jit_try_kernel): wait for its code object
    if (pending_code(k.key, true, &code) == 1) {
        if (compile_ms)
            *compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return load_module(k.key, code, fn, alpha_fn, err);
    }
    if (k.dir.empty() || !read_file(k.dir + "/" + k.name, code)) {
        bool in_helper = false;
        std::string compiler;
        if (!compile(opt, opt.jit_process ? Route::kAuto : Route::kInProcess, source, k.arch, code, err, &compiler,
                     &in_helper))
            return false;
        if (compile_ms)
            *compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        // (a helper route that fell back to another compiler does not fill the disk cache
        // under the key of the helper's)
        if (compiler == route_compiler(opt)) write_file_atomic(k.dir, k.name, code);
    }
    return load_module(k.key, code, fn, alpha_fn, err);
}

JitTry jit_try_kernel(const Options& opt, int device, const std::string& source, hipFunction_t* fn,
                      hipFunction_t* alpha_fn, JitTicket* ticket, std::string* err) {
    KeyInfo k;
    if (!key_of(opt, device, source, &k, err)) return JitTry::kWait;
    if (memory_lookup(k.key, fn, alpha_fn)) return JitTry::kReady;
    std::vector<char> code;
    const int st = pending_code(k.key, false, &code);
    if (st == 1) return load_module(k.key, code, fn, alpha_fn, err) ? JitTry::kReady : JitTry::kWait;
    if (st >= 0) return JitTry::kWait;   // compiling (another solve started it), or failed
    if (!k.dir.empty() && read_file(k.dir + "/" + k.name, code))
        return load_module(k.key, code, fn, alpha_fn, err) ? JitTry::kReady : JitTry::kWait;
    if (!use_helper(opt)) return JitTry::kWait;
    Pending* p = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_pend_mu);
        if (g_pending.count(k.key)) return JitTry::kWait;   // (another thread started it meanwhile)
        p = new Pending;
        g_pending[k.key] = p;
    }
    const std::string helper = helper_path(), dir = k.dir, name = k.name;
    std::vector<std::string> opts = compile_options(opt, k.arch);
    try {
        std::thread([p, helper, opts, source, dir, name]() {
            std::vector<char> out;
            std::string e;
            const bool ok = compile_in_helper(helper, opts, source, out, &e);
            if (ok) write_file_atomic(dir, name, out);
            std::lock_guard<std::mutex> lock(g_pend_mu);
            if (ok) p->code.swap(out);
            p->state = ok ? 1 : 2;
            g_pend_cv.notify_all();
        }).detach();
    } catch (...) {   // no thread: mark it failed (a blocking compile then)
        std::lock_guard<std::mutex> lock(g_pend_mu);
        p->state = 2;
        g_pend_cv.notify_all();
        return JitTry::kWait;
    }
    if (ticket) ticket->p = p;
    return JitTry::kStarted;
}

}  // namespace wost
