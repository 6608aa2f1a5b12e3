// multi.cpp -- the multi-GPU context of the C ABI (include/sparsematrix.h, sm_multi_*).
//
// the rows of B (the outputs) are split across the GPUs of one node,
// one process per GPU; every rank holds its rows with GLOBAL column indices; x is
// split in equal slices.  Per product the only exchange is one ncclAllGather of x
// (or of the X panel for SpMM) over xGMI, then the rank's local SpMV / SpMM -- the
// reference's panels already write disjoint output columns (sparse-matrix.cc:164-190),
// so no reduction is ever needed.
//
// RCCL is opened at run time (dlopen) rather than linked: a process that already has
// an RCCL loaded (PyTorch-ROCm ships one) shares it, so there is one RCCL per process,
// and the library itself loads on machines without RCCL (single-GPU use).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "sm_internal.h"

namespace {

struct Rccl {
    void *handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string why;
};

// RCCL, loaded once: the copy already in the process if any, else the system's.
const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *names[] = {"librccl.so.1", "librccl.so"};
        for (const char *n : names)
            if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        for (const char *n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
            if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (!r.handle) {
            r.why = std::string("cannot load librccl: ") + (dlerror() ? dlerror() : "?");
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.handle, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.handle, "ncclCommInitRank");
        r.all_gather = (decltype(r.all_gather))dlsym(r.handle, "ncclAllGather");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.handle, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(r.handle, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy ||
            !r.error_string)
            r.why = "librccl lacks ncclGetUniqueId/CommInitRank/AllGather/CommDestroy";
    });
    return r;
}

bool rccl_ok() { return rccl().why.empty(); }

}  // namespace

struct sm_multi {
    int32_t nranks = 0, rank = 0, device = 0;
    const sm_matrix *local = nullptr;
    int64_t n_cols = 0, x_local_len = 0;
    ncclComm_t comm = nullptr;
    hipStream_t comm_stream = nullptr;        // the pipelined batch's all-gathers
    float *xbuf[2] = {nullptr, nullptr};       // gathered x (or X panel), two for the pipeline
    size_t xbuf_floats = 0;
    hipEvent_t gathered[2] = {nullptr, nullptr}, consumed[2] = {nullptr, nullptr};
    hipEvent_t start = nullptr, joined = nullptr;
    // Optional device timing of the last sm_multi_spmv / _spmm (sm_multi_set_timing).
    bool timing = false;
    hipEvent_t t0 = nullptr, t1 = nullptr, t2 = nullptr;
    std::mutex mu;                             // one product at a time per context
};

namespace {

thread_local std::string g_merr;

sm_status mfail(sm_status s, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_merr = buf;
    return s;
}

sm_status hip_mfail(hipError_t e, const char *what) {
    return mfail(e == hipErrorOutOfMemory ? SM_ERR_OUT_OF_MEMORY : SM_ERR_HIP, "%s: %s (%d)", what,
                 hipGetErrorString(e), (int)e);
}

sm_status nccl_fail(ncclResult_t r, const char *what) {
    return mfail(SM_ERR_HIP, "%s: %s (%d)", what, rccl().error_string ? rccl().error_string(r) : "?",
                 (int)r);
}

struct DevScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DevScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DevScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

void release(sm_multi *mc) {
    DevScope g(mc->device);
    if (mc->comm && rccl_ok()) (void)rccl().comm_destroy(mc->comm);
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(mc->xbuf[i]);
        if (mc->gathered[i]) (void)hipEventDestroy(mc->gathered[i]);
        if (mc->consumed[i]) (void)hipEventDestroy(mc->consumed[i]);
    }
    for (hipEvent_t ev : {mc->start, mc->joined, mc->t0, mc->t1, mc->t2})
        if (ev) (void)hipEventDestroy(ev);
    if (mc->comm_stream) (void)hipStreamDestroy(mc->comm_stream);
}

// The gather buffers hold `floats` each (grown on demand, after the device is idle
// with respect to them: callers pass through sm_multi's mutex and sync on growth).
sm_status ensure_buffers(sm_multi *mc, size_t floats) {
    if (mc->xbuf_floats >= floats) return SM_OK;
    hipError_t e = hipDeviceSynchronize();
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
        (void)hipFree(mc->xbuf[i]);
        mc->xbuf[i] = nullptr;
        e = hipMalloc((void **)&mc->xbuf[i], floats * sizeof(float));
    }
    if (e != hipSuccess) {
        mc->xbuf_floats = 0;
        return hip_mfail(e, "sm_multi gather buffers");
    }
    mc->xbuf_floats = floats;
    return SM_OK;
}

}  // namespace

extern "C" {

const char *sm_multi_last_error(void) { return g_merr.c_str(); }

sm_status sm_multi_partition(int64_t n, int32_t nranks, int32_t rank, int64_t *r0, int64_t *r1) {
    if (n < 0 || nranks < 1 || rank < 0 || rank >= nranks || !r0 || !r1)
        return mfail(SM_ERR_INVALID_ARG, "bad partition arguments n=%lld nranks=%d rank=%d",
                     (long long)n, nranks, rank);
    const int64_t q = n / nranks, rem = n % nranks;
    *r0 = rank * q + std::min<int64_t>(rank, rem);
    *r1 = *r0 + q + (rank < rem ? 1 : 0);
    return SM_OK;
}

sm_status sm_multi_unique_id(sm_unique_id *id) {
    static_assert(sizeof(sm_unique_id) == sizeof(ncclUniqueId), "unique id size");
    if (!id) return mfail(SM_ERR_INVALID_ARG, "id is null");
    if (!rccl_ok()) return mfail(SM_ERR_NOT_SUPPORTED, "%s", rccl().why.c_str());
    ncclUniqueId u;
    const ncclResult_t r = rccl().get_unique_id(&u);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
    return SM_OK;
}

sm_status sm_multi_create(const sm_unique_id *id, int32_t nranks, int32_t rank,
                          const sm_matrix *local, sm_multi **out) {
    if (!out) return mfail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (!id || !local) return mfail(SM_ERR_INVALID_ARG, "null id or local matrix");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return mfail(SM_ERR_INVALID_ARG, "rank %d not in [0, %d)", rank, nranks);
    sm_info info;
    if (sm_get_info(local, &info) != SM_OK) return mfail(SM_ERR_INVALID_ARG, "bad local matrix");
    // ncclAllGather moves equal counts: x splits in nranks equal slices.
    if (info.n_cols % nranks != 0)
        return mfail(SM_ERR_INVALID_ARG, "global columns %lld not a multiple of nranks %d",
                     (long long)info.n_cols, nranks);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return mfail(SM_ERR_NO_DEVICE, "no HIP device visible");
    if (!rccl_ok()) return mfail(SM_ERR_NOT_SUPPORTED, "%s", rccl().why.c_str());
    auto *mc = new sm_multi();
    mc->nranks = nranks;
    mc->rank = rank;
    mc->device = info.device;
    mc->local = local;
    mc->n_cols = info.n_cols;
    mc->x_local_len = info.n_cols / nranks;
    DevScope g(mc->device);
    hipError_t e = g.err;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&mc->comm_stream, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
        e = hipEventCreateWithFlags(&mc->gathered[i], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&mc->consumed[i], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&mc->start, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&mc->joined, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&mc->t0);
    if (e == hipSuccess) e = hipEventCreate(&mc->t1);
    if (e == hipSuccess) e = hipEventCreate(&mc->t2);
    if (e != hipSuccess) {
        release(mc);
        delete mc;
        return hip_mfail(e, "sm_multi_create");
    }
    sm_status st = ensure_buffers(mc, (size_t)std::max<int64_t>(mc->n_cols, 1));
    if (st != SM_OK) {
        release(mc);
        delete mc;
        return st;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    const ncclResult_t r = rccl().comm_init_rank(&mc->comm, nranks, u, rank);   // collective
    if (r != ncclSuccess) {
        mc->comm = nullptr;
        release(mc);
        delete mc;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = mc;
    return SM_OK;
}

void sm_multi_destroy(sm_multi *mc) {
    if (!mc) return;
    release(mc);
    delete mc;
}

sm_status sm_multi_set_timing(sm_multi *mc, int32_t on) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    mc->timing = on != 0;
    return SM_OK;
}

sm_status sm_multi_last_times(sm_multi *mc, float *allgather_ms, float *compute_ms) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (!mc->timing) return mfail(SM_ERR_NOT_SUPPORTED, "timing is off (sm_multi_set_timing)");
    DevScope g(mc->device);
    hipError_t e = hipEventSynchronize(mc->t2);
    float a = 0.f, b = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&a, mc->t0, mc->t1);
    if (e == hipSuccess) e = hipEventElapsedTime(&b, mc->t1, mc->t2);
    if (e != hipSuccess) return hip_mfail(e, "sm_multi_last_times");
    if (allgather_ms) *allgather_ms = a;
    if (compute_ms) *compute_ms = b;
    return SM_OK;
}

sm_status sm_multi_allgather(sm_multi *mc, const float *x_local, int32_t n_rhs, sm_stream stream,
                             const float **x_full) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (n_rhs < 1 || (!x_local && mc->x_local_len > 0))
        return mfail(SM_ERR_INVALID_ARG, "bad x_local / n_rhs");
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    sm_status st = ensure_buffers(mc, (size_t)mc->n_cols * n_rhs);
    if (st != SM_OK) return st;
    const ncclResult_t r = rccl().all_gather(x_local, mc->xbuf[0], (size_t)mc->x_local_len * n_rhs,
                                             ncclFloat32, mc->comm, (hipStream_t)stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
    if (x_full) *x_full = mc->xbuf[0];
    return SM_OK;
}

sm_status sm_multi_spmv(sm_multi *mc, float alpha, const float *x_local, float beta, float *y_local,
                        sm_algo algo, sm_stream stream) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (!y_local || (!x_local && mc->x_local_len > 0)) return mfail(SM_ERR_INVALID_ARG, "null x/y");
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = mc->timing ? hipEventRecord(mc->t0, s) : hipSuccess;
    if (e != hipSuccess) return hip_mfail(e, "sm_multi_spmv");
    // The one collective of the product: x slices -> the full x, on the caller's stream.
    const ncclResult_t r = rccl().all_gather(x_local, mc->xbuf[0], (size_t)mc->x_local_len,
                                             ncclFloat32, mc->comm, s);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
    if (mc->timing && (e = hipEventRecord(mc->t1, s)) != hipSuccess) return hip_mfail(e, "sm_multi_spmv");
    const sm_status st = sm_spmv(mc->local, alpha, mc->xbuf[0], beta, y_local, algo, stream);
    if (st != SM_OK) return mfail(st, "local SpMV: %s", sm_last_error());
    if (mc->timing && (e = hipEventRecord(mc->t2, s)) != hipSuccess) return hip_mfail(e, "sm_multi_spmv");
    return SM_OK;
}

sm_status sm_multi_spmm(sm_multi *mc, int32_t n_rhs, float alpha, const float *X_local, float beta,
                        float *Y_local, int64_t ldy, sm_algo algo, sm_stream stream) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (n_rhs < 1 || ldy < n_rhs || !Y_local || (!X_local && mc->x_local_len > 0))
        return mfail(SM_ERR_INVALID_ARG, "bad SpMM arguments");
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    hipStream_t s = (hipStream_t)stream;
    sm_status st = ensure_buffers(mc, (size_t)mc->n_cols * n_rhs);
    if (st != SM_OK) return st;
    hipError_t e = mc->timing ? hipEventRecord(mc->t0, s) : hipSuccess;
    if (e != hipSuccess) return hip_mfail(e, "sm_multi_spmm");
    // Row-major X: rank r's rows [r*len, (r+1)*len) are contiguous, so gathering the
    // slices in rank order yields the full row-major X panel.
    const ncclResult_t r = rccl().all_gather(X_local, mc->xbuf[0], (size_t)mc->x_local_len * n_rhs,
                                             ncclFloat32, mc->comm, s);
    if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
    if (mc->timing && (e = hipEventRecord(mc->t1, s)) != hipSuccess) return hip_mfail(e, "sm_multi_spmm");
    st = sm_spmm(mc->local, n_rhs, alpha, mc->xbuf[0], n_rhs, beta, Y_local, ldy, algo, stream);
    if (st != SM_OK) return mfail(st, "local SpMM: %s", sm_last_error());
    if (mc->timing && (e = hipEventRecord(mc->t2, s)) != hipSuccess) return hip_mfail(e, "sm_multi_spmm");
    return SM_OK;
}

sm_status sm_multi_spmv_batch(sm_multi *mc, int32_t count, const sm_matrix *const *locals,
                              float alpha, const float *const *x_local, float beta,
                              float *const *y_local, sm_algo algo, sm_stream stream) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (count < 0 || (count > 0 && (!x_local || !y_local)))
        return mfail(SM_ERR_INVALID_ARG, "bad batch arguments");
    for (int32_t i = 0; locals && i < count; ++i) {   // other matrices: same rank, same columns
        sm_info li;
        if (!locals[i] || sm_get_info(locals[i], &li) != SM_OK || li.n_cols != mc->n_cols ||
            li.device != mc->device)
            return mfail(SM_ERR_INVALID_ARG, "batch matrix %d: needs %lld global columns on device %d",
                         i, (long long)mc->n_cols, mc->device);
    }
    if (count == 0) return SM_OK;
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    hipStream_t s = (hipStream_t)stream, c = mc->comm_stream;
    // The x slices were written on the caller's stream: the gathers start after them.
    hipError_t e = hipEventRecord(mc->start, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(c, mc->start, 0);
    if (e != hipSuccess) return hip_mfail(e, "sm_multi_spmv_batch");
    auto gather = [&](int32_t i) -> sm_status {
        const int b = i & 1;
        // Buffer b was last read by product i-2's SpMV.
        if (i >= 2 && (e = hipStreamWaitEvent(c, mc->consumed[b], 0)) != hipSuccess)
            return hip_mfail(e, "sm_multi_spmv_batch");
        const ncclResult_t r = rccl().all_gather(x_local[i], mc->xbuf[b], (size_t)mc->x_local_len,
                                                 ncclFloat32, mc->comm, c);
        if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
        if ((e = hipEventRecord(mc->gathered[b], c)) != hipSuccess) return hip_mfail(e, "sm_multi_spmv_batch");
        return SM_OK;
    };
    sm_status st = gather(0);
    for (int32_t i = 0; i < count && st == SM_OK; ++i) {
        // Product i+1's all-gather runs on the context's stream beside product i's SpMV.
        if (i + 1 < count) st = gather(i + 1);
        if (st != SM_OK) break;
        const int b = i & 1;
        if ((e = hipStreamWaitEvent(s, mc->gathered[b], 0)) != hipSuccess) {
            st = hip_mfail(e, "sm_multi_spmv_batch");
            break;
        }
        st = sm_spmv(locals ? locals[i] : mc->local, alpha, mc->xbuf[b], beta, y_local[i], algo,
                     stream);
        if (st != SM_OK) {
            st = mfail(st, "local SpMV: %s", sm_last_error());
            break;
        }
        if ((e = hipEventRecord(mc->consumed[b], s)) != hipSuccess) st = hip_mfail(e, "sm_multi_spmv_batch");
    }
    // Join: nothing of this batch stays on the context's stream behind the caller's.
    if ((e = hipEventRecord(mc->joined, c)) == hipSuccess) e = hipStreamWaitEvent(s, mc->joined, 0);
    if (st == SM_OK && e != hipSuccess) st = hip_mfail(e, "sm_multi_spmv_batch");
    return st;
}

}  // extern "C"
