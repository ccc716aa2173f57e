// wost_comm.cpp -- the multi-GPU path of libwost: one process per GPU, RCCL over xGMI
// (include/wost.h, "Multi-GPU"). SURVEY 8(e): walks shard trivially; the only exchange
// is one all-gather of the per-block partial sums, after which every rank sums them
// per point in global block order, so the result is bitwise that of one GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "wost.h"

namespace {

thread_local std::string g_comm_err;

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

int wost_solve_distributed(wost_handle* h, wost_comm* c, const float* points, int64_t n_points,
                           int64_t walks_per_point, int32_t max_steps, float eps, uint64_t seed, double* point_stats,
                           wost_dist_timing* timing) {
    if (!h || !c || !point_stats || n_points < 0 || (n_points > 0 && !points) || walks_per_point < 1)
        return cfail(WOST_ERR_INVALID_ARG, "bad arguments");
    double sb = 0.0;
    int32_t delta = 0;
    (void)wost_get_info(h, &sb, &delta);
    int32_t ns = 1;
    if (wost_num_sources(h, &ns) != WOST_OK) return cfail(WOST_ERR_INVALID_ARG, "%s", wost_last_error());
    const int row = 2 * ns + 1;
    const int R = c->n_ranks;
    const int64_t nbpp = (walks_per_point + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
    const int64_t nb_max = (nbpp + R - 1) / R;   // blocks per point of the largest shard
    std::fill(point_stats, point_stats + (size_t)row * (size_t)n_points, 0.0);
    if (n_points == 0) return WOST_OK;
    int64_t w0 = 0, w1 = 0;
    int rc = wost_shard_walk_range(walks_per_point, R, c->rank, &w0, &w1);
    if (rc != WOST_OK) return rc;
    // this rank's blocks, padded to nb_max per point for the all-gather
    std::vector<double> mine((size_t)n_points * (size_t)nb_max * (size_t)row, 0.0);
    wost_timing t{};
    if (w1 > w0) {
        const int64_t nbr = (w1 - w0 + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS;
        std::vector<double> bs((size_t)n_points * (size_t)nbr * (size_t)row);
        rc = wost_solve_range(h, points, n_points, walks_per_point, w0, w1, max_steps, eps, seed, bs.data(), nullptr,
                              nullptr, nullptr);
        if (rc != WOST_OK) return cfail(rc, "%s", wost_last_error());
        (void)wost_last_timing(h, &t);
        for (int64_t p = 0; p < n_points; ++p)
            std::memcpy(&mine[((size_t)p * nb_max) * row], &bs[((size_t)p * nbr) * row], sizeof(double) * nbr * row);
    }
    std::vector<double> all((size_t)R * mine.size());
    rc = wost_comm_allgather(c, mine.data(), (int64_t)mine.size(), all.data());
    if (rc != WOST_OK) return rc;
    // per point, every rank's blocks in rank order = the global block order of one GPU
    for (int r = 0; r < R; ++r) {
        int64_t a0 = 0, a1 = 0;
        (void)wost_shard_walk_range(walks_per_point, R, r, &a0, &a1);
        const int64_t nbr = a1 > a0 ? (a1 - a0 + WOST_BLOCK_WALKS - 1) / WOST_BLOCK_WALKS : 0;
        const double* part = &all[(size_t)r * mine.size()];
        for (int64_t p = 0; p < n_points; ++p)
            for (int64_t b = 0; b < nbr; ++b)
                for (int k = 0; k < row; ++k) point_stats[(size_t)p * row + k] += part[((size_t)p * nb_max + b) * row + k];
    }
    if (timing) {
        timing->local = t;
        timing->walk_begin = w0;
        timing->walk_end = w1;
        double steps = (double)t.total_steps;
        rc = wost_comm_allreduce(c, &steps, 1, WOST_COMM_SUM);
        if (rc != WOST_OK) return rc;
        timing->total_steps = (uint64_t)steps;
    }
    return WOST_OK;
}

}  // extern "C"
