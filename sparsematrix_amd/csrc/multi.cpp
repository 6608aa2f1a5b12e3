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
// SM_RCCL_LIB names the one library to load instead (an installation whose RCCL lives
// elsewhere; the tests point it at a missing file to exercise SM_ERR_NOT_SUPPORTED).
//
// The collective is pluggable (sm_multi_create_with): the context keeps the partition,
// the two gather buffers and their stream ordering, and calls either RCCL's
// ncclAllGather or a caller-supplied all-gather -- e.g. a host-staged gloo gather, so
// that two ranks on one GPU (or a CPU-only control plane) drive the same C-ABI path.
//
// Stream ordering of the gather buffers: every product records `consumed[b]` on the
// stream that read xbuf[b]; every all-gather into xbuf[b] first waits for it, whatever
// stream either runs on (the same contract as the matrix's scratch, capi.cpp).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
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
        const char *forced = getenv("SM_RCCL_LIB");
        if (forced && *forced) {
            r.handle = dlopen(forced, RTLD_NOW | RTLD_GLOBAL);
        } else {
            for (const char *n : {"librccl.so.1", "librccl.so"})
                if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
            for (const char *n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
                if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        }
        if (!r.handle) {
            const char *de = dlerror();   // once: a second call returns NULL
            r.why = std::string("cannot load librccl: ") + (de ? de : "?");
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
    ncclComm_t comm = nullptr;                 // RCCL's communicator (RCCL collective)
    sm_collective coll = {nullptr, nullptr};   // or the caller's all-gather
    hipStream_t comm_stream = nullptr;        // the pipelined batch's all-gathers
    float *xbuf[2] = {nullptr, nullptr};       // gathered x (or X panel), two for the pipeline
    size_t xbuf_floats = 0;
    hipEvent_t gathered[2] = {nullptr, nullptr};
    // consumed[b]: recorded after the last product that read xbuf[b] (on its stream);
    // every later all-gather into xbuf[b] waits for it.  Valid once recorded outside a
    // stream capture (a captured record is a graph node, not an event to wait on).
    hipEvent_t consumed[2] = {nullptr, nullptr};
    bool consumed_valid[2] = {false, false};
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
    (void)hipDeviceSynchronize();   // no product may still use the buffers or events
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

// The gather buffers hold `floats` each, grown on demand: the new pair is allocated
// first (on failure the old pair stays in place and the call fails), then the old pair
// is released once the device is idle with respect to it.
bool capturing(hipStream_t s);

// Growing the gather buffers frees the old pair after a device-wide sync, which a stream
// capture cannot contain (it would invalidate the capture): under capture the buffers must
// already be large enough -- run one eager product of the largest n_rhs first.
sm_status ensure_buffers(sm_multi *mc, size_t floats, hipStream_t s) {
    if (mc->xbuf_floats >= floats && mc->xbuf[0] && mc->xbuf[1]) return SM_OK;
    if (s && capturing(s))
        return mfail(SM_ERR_NOT_SUPPORTED, "gather buffers of %zu floats needed inside a stream capture "
                     "(held: %zu): run one product of this size eagerly before capturing", floats,
                     mc->xbuf_floats);
    float *nb[2] = {nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipMalloc((void **)&nb[i], floats * sizeof(float));
    if (e != hipSuccess) {
        for (float *p : nb) (void)hipFree(p);
        return hip_mfail(e, "sm_multi gather buffers");
    }
    e = hipDeviceSynchronize();   // nothing may still read or fill the old pair
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(mc->xbuf[i]);
        mc->xbuf[i] = nb[i];
        mc->consumed_valid[i] = false;
    }
    mc->xbuf_floats = floats;
    return e == hipSuccess ? SM_OK : hip_mfail(e, "sm_multi gather buffers");
}

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) return false;
    return cs != hipStreamCaptureStatusNone;
}

// Before an all-gather into xbuf[b] on stream w: wait for the last product that read it.
sm_status order_write(sm_multi *mc, int b, hipStream_t w) {
    if (!mc->consumed_valid[b] || capturing(w)) return SM_OK;
    const hipError_t e = hipStreamWaitEvent(w, mc->consumed[b], 0);
    return e == hipSuccess ? SM_OK : hip_mfail(e, "sm_multi buffer ordering");
}

// After a product (or a bare all-gather) that used xbuf[b] on stream s.  Under a
// stream capture the record is a graph node: later calls inside the same capture (the
// batch's own products) may wait on it, calls outside it may not.
sm_status mark_read(sm_multi *mc, int b, hipStream_t s) {
    const bool cap = capturing(s);
    const hipError_t e = hipEventRecord(mc->consumed[b], s);
    mc->consumed_valid[b] = e == hipSuccess && !cap;
    return e == hipSuccess ? SM_OK : hip_mfail(e, "sm_multi buffer ordering");
}

// The product's one collective: x slices (count floats per rank) -> recv, on stream s.
sm_status gather(sm_multi *mc, const float *send, float *recv, size_t count, hipStream_t s) {
    if (mc->coll.allgather) {
        const int32_t rc = mc->coll.allgather(send, recv, (int64_t)count, (sm_stream)s, mc->coll.user);
        return rc == 0 ? SM_OK : mfail(SM_ERR_HIP, "caller's all-gather returned %d", rc);
    }
    const ncclResult_t r = rccl().all_gather(send, recv, count, ncclFloat32, mc->comm, s);
    return r == ncclSuccess ? SM_OK : nccl_fail(r, "ncclAllGather");
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

namespace {

// Shared by sm_multi_create (RCCL) and sm_multi_create_with (the caller's all-gather):
// the context, its streams, events and gather buffers; the communicator comes after.
sm_status create_common(int32_t nranks, int32_t rank, const sm_matrix *local, sm_multi **out,
                        sm_multi **made) {
    if (!out) return mfail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (!local) return mfail(SM_ERR_INVALID_ARG, "null local matrix");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return mfail(SM_ERR_INVALID_ARG, "rank %d not in [0, %d)", rank, nranks);
    sm_info info;
    if (sm_get_info(local, &info) != SM_OK) return mfail(SM_ERR_INVALID_ARG, "bad local matrix");
    // An all-gather moves equal counts: x splits in nranks equal slices.
    if (info.n_cols % nranks != 0)
        return mfail(SM_ERR_INVALID_ARG, "global columns %lld not a multiple of nranks %d",
                     (long long)info.n_cols, nranks);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return mfail(SM_ERR_NO_DEVICE, "no HIP device visible");
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
    sm_status st = e == hipSuccess ? SM_OK : hip_mfail(e, "sm_multi_create");
    if (st == SM_OK) st = ensure_buffers(mc, (size_t)std::max<int64_t>(mc->n_cols, 1), nullptr);
    if (st != SM_OK) {
        release(mc);
        delete mc;
        return st;
    }
    *made = mc;
    return SM_OK;
}

}  // namespace

sm_status sm_multi_create(const sm_unique_id *id, int32_t nranks, int32_t rank,
                          const sm_matrix *local, sm_multi **out) {
    if (out) *out = nullptr;
    if (!id) return mfail(SM_ERR_INVALID_ARG, "null id");
    if (out && local && !rccl_ok()) return mfail(SM_ERR_NOT_SUPPORTED, "%s", rccl().why.c_str());
    sm_multi *mc = nullptr;
    sm_status st = create_common(nranks, rank, local, out, &mc);
    if (st != SM_OK) return st;
    if (!rccl_ok()) {
        release(mc);
        delete mc;
        return mfail(SM_ERR_NOT_SUPPORTED, "%s", rccl().why.c_str());
    }
    DevScope g(mc->device);
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

sm_status sm_multi_create_with(const sm_collective *coll, int32_t nranks, int32_t rank,
                               const sm_matrix *local, sm_multi **out) {
    if (out) *out = nullptr;
    if (!coll || !coll->allgather) return mfail(SM_ERR_INVALID_ARG, "null collective");
    sm_multi *mc = nullptr;
    sm_status st = create_common(nranks, rank, local, out, &mc);
    if (st != SM_OK) return st;
    mc->coll = *coll;
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
    hipStream_t s = (hipStream_t)stream;
    sm_status st = ensure_buffers(mc, (size_t)mc->n_cols * n_rhs, s);
    if (st == SM_OK) st = order_write(mc, 0, s);
    if (st == SM_OK) st = gather(mc, x_local, mc->xbuf[0], (size_t)mc->x_local_len * n_rhs, s);
    if (st == SM_OK) st = mark_read(mc, 0, s);   // later writers wait for the gather at least
    if (st != SM_OK) return st;
    if (x_full) *x_full = mc->xbuf[0];
    return SM_OK;
}

namespace {

// One product on stream s: all-gather into xbuf[0] (after its last reader), the local
// SpMV (n_rhs == 0) or SpMM, then xbuf[0]'s consumed event.
sm_status one_product(sm_multi *mc, int32_t n_rhs, float alpha, const float *x_local, float beta,
                      float *y_local, int64_t ldy, sm_algo algo, hipStream_t s) {
    const size_t per = (size_t)std::max<int32_t>(n_rhs, 1);
    sm_status st = ensure_buffers(mc, (size_t)mc->n_cols * per, s);
    if (st == SM_OK) st = order_write(mc, 0, s);
    if (st != SM_OK) return st;
    hipError_t e = mc->timing ? hipEventRecord(mc->t0, s) : hipSuccess;
    if (e != hipSuccess) return hip_mfail(e, "sm_multi product");
    // The one collective of the product: x slices (or X row slices) -> the full x.
    // Row-major X: rank r's rows [r*L, (r+1)*L) are contiguous, so gathering the slices
    // in rank order yields the full row-major X panel.
    st = gather(mc, x_local, mc->xbuf[0], (size_t)mc->x_local_len * per, s);
    if (st != SM_OK) return st;
    if (mc->timing && (e = hipEventRecord(mc->t1, s)) != hipSuccess) return hip_mfail(e, "sm_multi product");
    st = n_rhs == 0 ? sm_spmv(mc->local, alpha, mc->xbuf[0], beta, y_local, algo, (sm_stream)s)
                    : sm_spmm(mc->local, n_rhs, alpha, mc->xbuf[0], n_rhs, beta, y_local, ldy, algo,
                              (sm_stream)s);
    // Recorded on the error path too: a failed launch may still have queued kernels.
    const sm_status mr = mark_read(mc, 0, s);
    if (st != SM_OK) return mfail(st, "local product: %s", sm_last_error());
    if (mr != SM_OK) return mr;
    if (mc->timing && (e = hipEventRecord(mc->t2, s)) != hipSuccess) return hip_mfail(e, "sm_multi product");
    return SM_OK;
}

}  // namespace

sm_status sm_multi_spmv(sm_multi *mc, float alpha, const float *x_local, float beta, float *y_local,
                        sm_algo algo, sm_stream stream) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (!y_local || (!x_local && mc->x_local_len > 0)) return mfail(SM_ERR_INVALID_ARG, "null x/y");
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    return one_product(mc, 0, alpha, x_local, beta, y_local, 1, algo, (hipStream_t)stream);
}

sm_status sm_multi_spmm(sm_multi *mc, int32_t n_rhs, float alpha, const float *X_local, float beta,
                        float *Y_local, int64_t ldy, sm_algo algo, sm_stream stream) {
    if (!mc) return mfail(SM_ERR_INVALID_ARG, "null context");
    if (n_rhs < 1 || ldy < n_rhs || !Y_local || (!X_local && mc->x_local_len > 0))
        return mfail(SM_ERR_INVALID_ARG, "bad SpMM arguments");
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    return one_product(mc, n_rhs, alpha, X_local, beta, Y_local, ldy, algo, (hipStream_t)stream);
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
    for (int32_t i = 0; i < count; ++i)
        if (!y_local[i] || (!x_local[i] && mc->x_local_len > 0))
            return mfail(SM_ERR_INVALID_ARG, "batch product %d: null x/y", i);
    if (count == 0) return SM_OK;
    std::lock_guard<std::mutex> lk(mc->mu);
    DevScope g(mc->device);
    hipStream_t s = (hipStream_t)stream, c = mc->comm_stream;
    sm_status st = ensure_buffers(mc, (size_t)mc->n_cols, s);
    if (st != SM_OK) return st;
    // The x slices were written on the caller's stream: the gathers start after them.
    hipError_t e = hipEventRecord(mc->start, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(c, mc->start, 0);
    if (e != hipSuccess) return hip_mfail(e, "sm_multi_spmv_batch");
    auto gather_into = [&](int32_t i) -> sm_status {
        const int b = i & 1;
        // Buffer b was last read by product i-2's SpMV (recorded in this batch), or for
        // the first two by an earlier call's product on any stream (consumed[b]).
        sm_status r = SM_OK;
        if (i >= 2) {
            if ((e = hipStreamWaitEvent(c, mc->consumed[b], 0)) != hipSuccess)
                return hip_mfail(e, "sm_multi_spmv_batch");
        } else {
            r = order_write(mc, b, c);
        }
        if (r == SM_OK) r = gather(mc, x_local[i], mc->xbuf[b], (size_t)mc->x_local_len, c);
        if (r != SM_OK) return r;
        if ((e = hipEventRecord(mc->gathered[b], c)) != hipSuccess) return hip_mfail(e, "sm_multi_spmv_batch");
        return SM_OK;
    };
    st = gather_into(0);
    for (int32_t i = 0; i < count && st == SM_OK; ++i) {
        // Product i+1's all-gather runs on the context's stream beside product i's SpMV.
        if (i + 1 < count) st = gather_into(i + 1);
        if (st != SM_OK) break;
        const int b = i & 1;
        if ((e = hipStreamWaitEvent(s, mc->gathered[b], 0)) != hipSuccess) {
            st = hip_mfail(e, "sm_multi_spmv_batch");
            break;
        }
        st = sm_spmv(locals ? locals[i] : mc->local, alpha, mc->xbuf[b], beta, y_local[i], algo,
                     stream);
        const sm_status mr = mark_read(mc, b, s);
        if (st != SM_OK) {
            st = mfail(st, "local SpMV: %s", sm_last_error());
            break;
        }
        st = mr;
    }
    // Join: nothing of this batch stays on the context's stream behind the caller's.
    if ((e = hipEventRecord(mc->joined, c)) == hipSuccess) e = hipStreamWaitEvent(s, mc->joined, 0);
    if (st == SM_OK && e != hipSuccess) st = hip_mfail(e, "sm_multi_spmv_batch");
    return st;
}

}  // extern "C"
