// wost_comm.cpp -- the multi-GPU path of libwost: one process per GPU, RCCL over xGMI
// (include/wost.h, "Multi-GPU"). SURVEY 8(e): walks shard trivially; the only exchange
// is one all-gather of the per-block partial sums, after which every rank sums them
// per point in global block order, so the result is bitwise that of one GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "wost.h"

namespace {

thread_local std::string g_comm_err;
// wall-clock phases of this thread's last wost_distributed_run (wost_dist_last_phases)
thread_local double g_phases[4] = {0.0, 0.0, 0.0, 0.0};

struct PhaseClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    double lap() {   // ms since the last lap
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
        return ms;
    }
};

int cfail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_comm_err = buf;
    return code;
}

}  // namespace

struct wost_comm {
    int n_ranks = 0;
    int rank = 0;
    int device = 0;
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;
    double* d_send = nullptr;
    double* d_recv = nullptr;
    int64_t cap = 0;   // doubles per rank in d_send / d_recv
};

namespace {

#define NCCL_TRY(expr)                                                                             \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess) return cfail(WOST_ERR_COMM, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)
#define CHIP_TRY(expr)                                                                             \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return cfail(WOST_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_));  \
    } while (0)

int ensure_comm_buffers(wost_comm* c, int64_t per_rank) {
    if (per_rank <= c->cap) return WOST_OK;
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_recv) (void)hipFree(c->d_recv);
    c->d_send = c->d_recv = nullptr;
    c->cap = 0;
    CHIP_TRY(hipMalloc(&c->d_send, sizeof(double) * (size_t)per_rank));
    CHIP_TRY(hipMalloc(&c->d_recv, sizeof(double) * (size_t)per_rank * (size_t)c->n_ranks));
    c->cap = per_rank;
    return WOST_OK;
}

}  // namespace

extern "C" {

const char* wost_comm_last_error(void) { return g_comm_err.c_str(); }

int wost_comm_unique_id(uint8_t* id) {
    if (!id) return cfail(WOST_ERR_INVALID_ARG, "NULL id buffer");
    static_assert(sizeof(ncclUniqueId) == WOST_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, WOST_COMM_ID_BYTES);
    return WOST_OK;
}

int wost_comm_create(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, wost_comm** out) {
    if (!id || !out) return cfail(WOST_ERR_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return cfail(WOST_ERR_INVALID_ARG, "rank %d of %d ranks", rank, n_ranks);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return cfail(WOST_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return cfail(WOST_ERR_INVALID_ARG, "device %d out of range [0,%d)", device, ndev);
    wost_comm* c = new wost_comm();
    c->n_ranks = n_ranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, WOST_COMM_ID_BYTES);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return cfail(WOST_ERR_HIP, "communicator stream: %s", hipGetErrorString(e));
    }
    const ncclResult_t r = ncclCommInitRank(&c->nccl, n_ranks, u, rank);
    if (r != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return cfail(WOST_ERR_COMM, "ncclCommInitRank(%d of %d): %s", rank, n_ranks, ncclGetErrorString(r));
    }
    *out = c;
    return WOST_OK;
}

void wost_comm_destroy(wost_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_recv) (void)hipFree(c->d_recv);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int wost_comm_info(const wost_comm* c, int32_t* n_ranks, int32_t* rank, int32_t* device) {
    if (!c) return cfail(WOST_ERR_INVALID_ARG, "NULL communicator");
    if (n_ranks) *n_ranks = c->n_ranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return WOST_OK;
}

int wost_comm_allgather(wost_comm* c, const double* send, int64_t count, double* recv) {
    if (!c || count < 0 || (count > 0 && (!send || !recv))) return cfail(WOST_ERR_INVALID_ARG, "bad arguments");
    if (count == 0) return WOST_OK;
    CHIP_TRY(hipSetDevice(c->device));
    int rc = ensure_comm_buffers(c, count);
    if (rc != WOST_OK) return rc;
    CHIP_TRY(hipMemcpyAsync(c->d_send, send, sizeof(double) * (size_t)count, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclAllGather(c->d_send, c->d_recv, (size_t)count, ncclDouble, c->nccl, c->stream));
    CHIP_TRY(hipMemcpyAsync(recv, c->d_recv, sizeof(double) * (size_t)count * (size_t)c->n_ranks,
                            hipMemcpyDeviceToHost, c->stream));
    CHIP_TRY(hipStreamSynchronize(c->stream));
    return WOST_OK;
}

int wost_comm_allreduce(wost_comm* c, double* inout, int64_t count, int32_t op) {
    if (!c || count < 0 || (count > 0 && !inout)) return cfail(WOST_ERR_INVALID_ARG, "bad arguments");
    if (op != WOST_COMM_SUM && op != WOST_COMM_MAX) return cfail(WOST_ERR_INVALID_ARG, "unknown reduction %d", op);
    if (count == 0) return WOST_OK;
    CHIP_TRY(hipSetDevice(c->device));
    int rc = ensure_comm_buffers(c, count);
    if (rc != WOST_OK) return rc;
    CHIP_TRY(hipMemcpyAsync(c->d_send, inout, sizeof(double) * (size_t)count, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclAllReduce(c->d_send, c->d_recv, (size_t)count, ncclDouble, op == WOST_COMM_SUM ? ncclSum : ncclMax,
                           c->nccl, c->stream));
    CHIP_TRY(hipMemcpyAsync(inout, c->d_recv, sizeof(double) * (size_t)count, hipMemcpyDeviceToHost, c->stream));
    CHIP_TRY(hipStreamSynchronize(c->stream));
    return WOST_OK;
}

int wost_comm_barrier(wost_comm* c) {
    double x = 0.0;
    return wost_comm_allreduce(c, &x, 1, WOST_COMM_SUM);
}

int wost_shard_walk_range(int64_t walks_per_point, int32_t n_ranks, int32_t rank, int64_t* walk_begin,
                          int64_t* walk_end) {
    if (walks_per_point < 1 || n_ranks < 1 || rank < 0 || rank >= n_ranks || !walk_begin || !walk_end)
        return cfail(WOST_ERR_INVALID_ARG, "bad arguments");
    const int64_t nb = (walks_per_point + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    const int64_t b0 = nb * rank / n_ranks, b1 = nb * (rank + 1) / n_ranks;
    *walk_begin = std::min<int64_t>(b0 * WOST_BLOCK_WALKS, walks_per_point);
    *walk_end = std::min<int64_t>(b1 * WOST_BLOCK_WALKS, walks_per_point);
    return WOST_OK;
}

int64_t wost_shard_blocks_max(int64_t walks_per_point, int32_t n_ranks) {
    if (walks_per_point < 1 || n_ranks < 1) return -1;
    const int64_t nbpp = (walks_per_point + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    return (nbpp + n_ranks - 1) / n_ranks;   // blocks per point of the largest shard
}

int wost_shard_pack(const double* blocks, int64_t n_points, int64_t walks_per_point, int32_t n_ranks, int32_t rank,
                    int32_t row, double* packed) {
    int64_t w0 = 0, w1 = 0;
    if (n_points < 0 || row < 1 || !packed || (n_points > 0 && !blocks && walks_per_point > 0) ||
        wost_shard_walk_range(walks_per_point, n_ranks, rank, &w0, &w1) != WOST_OK)
        return cfail(WOST_ERR_INVALID_ARG, "wost_shard_pack: bad arguments");
    const int64_t nb_max = wost_shard_blocks_max(walks_per_point, n_ranks);
    const int64_t nbr = w1 > w0 ? (w1 - w0 + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS : 0;
    std::fill(packed, packed + (size_t)n_points * (size_t)nb_max * (size_t)row, 0.0);
    for (int64_t p = 0; p < n_points; ++p)
        if (nbr) std::memcpy(&packed[(size_t)p * nb_max * row], &blocks[(size_t)p * nbr * row], sizeof(double) * nbr * row);
    return WOST_OK;
}

int wost_shard_merge(const double* gathered, int64_t n_points, int64_t walks_per_point, int32_t n_ranks, int32_t row,
                     double* point_stats) {
    const int64_t nb_max = wost_shard_blocks_max(walks_per_point, n_ranks);
    if (nb_max < 0 || n_points < 0 || row < 1 || !point_stats || (n_points > 0 && !gathered))
        return cfail(WOST_ERR_INVALID_ARG, "wost_shard_merge: bad arguments");
    const size_t per_rank = (size_t)n_points * (size_t)nb_max * (size_t)row;
    std::fill(point_stats, point_stats + (size_t)n_points * (size_t)row, 0.0);
    // per point, every rank's blocks in rank order = the global block order of one GPU
    for (int r = 0; r < n_ranks; ++r) {
        int64_t a0 = 0, a1 = 0;
        (void)wost_shard_walk_range(walks_per_point, n_ranks, r, &a0, &a1);
        const int64_t nbr = a1 > a0 ? (a1 - a0 + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS : 0;
        const double* part = gathered + (size_t)r * per_rank;
        for (int64_t p = 0; p < n_points; ++p)
            for (int64_t b = 0; b < nbr; ++b)
                for (int k = 0; k < row; ++k) point_stats[(size_t)p * row + k] += part[((size_t)p * nb_max + b) * row + k];
    }
    return WOST_OK;
}

int wost_dist_solve_key(uint64_t seed, float eps, int32_t max_steps, const float* points, int64_t n_points,
                        double* key) {
    if (!key || n_points < 0 || (n_points > 0 && !points)) return cfail(WOST_ERR_INVALID_ARG, "bad arguments");
    uint64_t hsh = 1469598103934665603ull;   // FNV-1a 64 over the points' bytes
    const auto* b = reinterpret_cast<const unsigned char*>(points);
    for (int64_t i = 0; i < 8 * n_points; ++i) hsh = (hsh ^ b[i]) * 1099511628211ull;
    key[0] = (double)(uint32_t)seed;
    key[1] = (double)(uint32_t)(seed >> 32);
    key[2] = (double)eps;
    key[3] = (double)max_steps;
    key[4] = (double)(uint32_t)hsh;
    key[5] = (double)(uint32_t)(hsh >> 32);
    return WOST_OK;
}

int wost_dist_last_phases(double* ms) {
    if (!ms) return cfail(WOST_ERR_INVALID_ARG, "NULL argument");
    for (int i = 0; i < 4; ++i) ms[i] = g_phases[i];
    return WOST_OK;
}

int wost_distributed_run(const wost_dist_ops* ops, int32_t n_ranks, int32_t rank, int64_t n_points,
                         int64_t walks_per_point, int32_t row, double* point_stats, int64_t* walk_begin,
                         int64_t* walk_end, uint64_t* total_steps) {
    for (double& v : g_phases) v = 0.0;
    PhaseClock clk;
    if (!ops || !ops->allreduce || !ops->allgather || n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return cfail(WOST_ERR_INVALID_ARG, "wost_distributed_run: no transport or bad rank %d of %d", rank, n_ranks);
    // Every rank reaches the same two collectives, whatever fails locally: the
    // agreement all-reduce (MAX) carries a failure flag and the call's shape, and
    // only when no rank failed and all agree does the all-gather of the blocks run.
    int local = WOST_OK;
    std::string local_msg;
    int64_t w0 = 0, w1 = 0;
    const bool args_ok = point_stats && n_points >= 0 && walks_per_point >= 1 && row >= 1 && ops->solve_range;
    if (!args_ok) {
        local = WOST_ERR_INVALID_ARG;
        local_msg = "bad arguments";
    } else {
        (void)wost_shard_walk_range(walks_per_point, n_ranks, rank, &w0, &w1);
    }
    const int64_t nb_max = args_ok ? wost_shard_blocks_max(walks_per_point, n_ranks) : 0;
    const int64_t nbr = w1 > w0 ? (w1 - w0 + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS : 0;
    const size_t per_rank = args_ok ? (size_t)n_points * (size_t)nb_max * (size_t)row : 0;
    std::vector<double> mine, all;
    if (local == WOST_OK) {
        try {
            mine.assign(per_rank, 0.0);
            all.assign(per_rank * (size_t)n_ranks, 0.0);
        } catch (const std::bad_alloc&) {
            local = WOST_ERR_OOM;
            local_msg = "host buffers of the gather";
        }
    }
    if (local == WOST_OK && ops->prepare) {
        local = ops->prepare(ops->ctx, (int64_t)per_rank);
        if (local != WOST_OK) local_msg = "transport buffers: " + g_comm_err;
    }
    if (local == WOST_OK && n_points > 0 && nbr > 0) {
        std::vector<double> bs;
        try {
            bs.assign((size_t)n_points * (size_t)nbr * (size_t)row, 0.0);
        } catch (const std::bad_alloc&) {
            local = WOST_ERR_OOM;
            local_msg = "host block buffer";
        }
        if (local == WOST_OK) {
            local = ops->solve_range(ops->ctx, w0, w1, bs.data());
            if (local != WOST_OK) local_msg = "local solve: " + g_comm_err;
        }
        if (local == WOST_OK) (void)wost_shard_pack(bs.data(), n_points, walks_per_point, n_ranks, rank, row, mine.data());
    }
    // agreement: max of (failed, n_points, -n_points, row, -row, W, -W, key[k], -key[k] ...);
    // the key's length is part of what must agree (a rank with another n_key fails it)
    const int nk = (ops->key && ops->n_key > 0) ? std::min<int>(ops->n_key, WOST_DIST_MAX_KEY) : 0;
    if (ops->n_key < 0 || ops->n_key > WOST_DIST_MAX_KEY || (ops->n_key > 0 && !ops->key)) {
        local = WOST_ERR_INVALID_ARG;
        local_msg = "bad agreement key";
    }
    // a NaN key entry (e.g. eps) fails this rank, and through the failure flag every rank:
    // NaN compares unequal to itself, so it cannot be agreed on
    for (int k = 0; k < nk && local == WOST_OK; ++k)
        if (!(ops->key[k] == ops->key[k])) {
            local = WOST_ERR_INVALID_ARG;
            local_msg = "NaN in the solve's arguments (agreement key)";
        }
    double agree[9 + 2 * WOST_DIST_MAX_KEY] = {local != WOST_OK ? 1.0 : 0.0, (double)n_points, -(double)n_points,
                                               (double)row, -(double)row, (double)walks_per_point,
                                               -(double)walks_per_point, (double)nk, -(double)nk};
    for (int k = 0; k < nk; ++k) {
        // (a NaN entry already failed this rank above; 0 keeps the reduction finite)
        const double v = ops->key[k] == ops->key[k] ? ops->key[k] : 0.0;
        agree[9 + 2 * k] = v;
        agree[10 + 2 * k] = -v;
    }
    const int na = 9 + 2 * WOST_DIST_MAX_KEY;   // fixed length: every rank reduces the same count
    g_phases[0] = clk.lap();
    int rc = ops->allreduce(ops->ctx, agree, na, WOST_COMM_MAX);
    g_phases[1] = clk.lap();
    if (rc != WOST_OK) return cfail(rc, "agreement all-reduce: %s", g_comm_err.c_str());
    if (local != WOST_OK) return cfail(local, "rank %d: %s", rank, local_msg.c_str());
    if (agree[0] > 0.0) return cfail(WOST_ERR_COMM, "rank %d: another rank failed; no result", rank);
    if (agree[1] != -agree[2] || agree[3] != -agree[4] || agree[5] != -agree[6])
        return cfail(WOST_ERR_INVALID_ARG, "ranks disagree on the solve (n_points %g..%g, row %g..%g, walks %g..%g)",
                     -agree[2], agree[1], -agree[4], agree[3], -agree[6], agree[5]);
    for (int k = 0; k < 1 + WOST_DIST_MAX_KEY; ++k)
        if (agree[7 + 2 * k] != -agree[8 + 2 * k])
            return cfail(WOST_ERR_INVALID_ARG,
                         "ranks disagree on the solve's arguments (%s %d: %.17g..%.17g; seed, eps, maxSteps, points)",
                         k == 0 ? "key length" : "key entry", k == 0 ? 0 : k - 1, -agree[8 + 2 * k], agree[7 + 2 * k]);
    if (per_rank > 0) {
        rc = ops->allgather(ops->ctx, mine.data(), (int64_t)per_rank, all.data());
        if (rc != WOST_OK) return cfail(rc, "block all-gather: %s", g_comm_err.c_str());
    }
    g_phases[2] = clk.lap();
    rc = wost_shard_merge(all.data(), n_points, walks_per_point, n_ranks, row, point_stats);
    g_phases[3] = clk.lap();
    if (rc != WOST_OK) return rc;
    if (walk_begin) *walk_begin = w0;
    if (walk_end) *walk_end = w1;
    if (total_steps) {
        double s = 0.0;
        for (int64_t p = 0; p < n_points; ++p) s += point_stats[(size_t)p * row + row - 1];
        *total_steps = (uint64_t)s;
    }
    return WOST_OK;
}

}  // extern "C"

namespace {

// wost_solve_distributed's transport: RCCL on the communicator's stream, and the
// handle's wost_solve_range as the local solve
struct RcclRun {
    wost_handle* h;
    wost_comm* c;
    const float* points;
    int64_t n_points, walks_per_point;
    int32_t max_steps;
    float eps;
    uint64_t seed;
    wost_timing t{};
};

int32_t rccl_prepare(void* ctx, int64_t per_rank) {
    auto* r = static_cast<RcclRun*>(ctx);
    CHIP_TRY(hipSetDevice(r->c->device));
    return ensure_comm_buffers(r->c, std::max<int64_t>(per_rank, 8));
}

int32_t rccl_solve_range(void* ctx, int64_t w0, int64_t w1, double* blocks) {
    auto* r = static_cast<RcclRun*>(ctx);
    const int rc = wost_solve_range(r->h, r->points, r->n_points, r->walks_per_point, w0, w1, r->max_steps, r->eps,
                                    r->seed, blocks, nullptr, nullptr, nullptr);
    if (rc != WOST_OK) return cfail(rc, "%s", wost_last_error());
    (void)wost_last_timing(r->h, &r->t);
    return WOST_OK;
}

int32_t rccl_allreduce(void* ctx, double* inout, int64_t count, int32_t op) {
    return wost_comm_allreduce(static_cast<RcclRun*>(ctx)->c, inout, count, op);
}

int32_t rccl_allgather(void* ctx, const double* send, int64_t count, double* recv) {
    return wost_comm_allgather(static_cast<RcclRun*>(ctx)->c, send, count, recv);
}

}  // namespace

extern "C" {

int wost_solve_distributed(wost_handle* h, wost_comm* c, const float* points, int64_t n_points,
                           int64_t walks_per_point, int32_t max_steps, float eps, uint64_t seed, double* point_stats,
                           wost_dist_timing* timing) {
    if (!c) return cfail(WOST_ERR_INVALID_ARG, "NULL communicator");
    // local argument and handle problems go through the agreement collective
    // (wost_distributed_run), so that no rank is left waiting in the gather
    int32_t ns = 1;
    int32_t row = 3;
    if (!h || wost_num_sources(h, &ns) != WOST_OK) row = 0;
    else row = 2 * ns + 1;
    if (n_points > 0 && !points) row = 0;
    RcclRun run{h, c, points, n_points, walks_per_point, max_steps, eps, seed};
    double key[6] = {0, 0, 0, 0, 0, 0};
    if (n_points >= 0 && (points || n_points == 0)) (void)wost_dist_solve_key(seed, eps, max_steps, points, n_points, key);
    wost_dist_ops ops{&run, rccl_prepare, rccl_solve_range, rccl_allreduce, rccl_allgather, key, 6};
    int64_t w0 = 0, w1 = 0;
    uint64_t steps = 0;
    const int rc = wost_distributed_run(&ops, c->n_ranks, c->rank, n_points, walks_per_point, row, point_stats, &w0,
                                        &w1, &steps);
    if (rc != WOST_OK) return rc;
    if (timing) {
        timing->local = run.t;
        timing->walk_begin = w0;
        timing->walk_end = w1;
        timing->total_steps = steps;
        timing->local_ms = g_phases[0];
        timing->agree_ms = g_phases[1];
        timing->gather_ms = g_phases[2];
        timing->merge_ms = g_phases[3];
    }
    return WOST_OK;
}

}  // extern "C"
