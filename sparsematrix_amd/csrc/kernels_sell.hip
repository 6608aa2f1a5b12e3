// kernels_sell.hip -- SpMV over the sorted sliced-ELL layout (sell.h, sell.cpp).
//
// One wavefront per slice of 64 rows, four slices per 256-thread workgroup, no LDS
// and no barrier: lane l owns row row[s*64 + l] and walks term slots j = 0, 1, ...
// of its slice; slot j of the 64 lanes is one coalesced 256-byte load of columns and
// one of values, then 64 x gathers.  Each lane adds x * (v * alpha) to beta * y in
// its row's stored order (kernel.cc:791, 580-582: separate rounding of every
// product and sum), so every row of up to kSellMaxLen terms is bit-identical to the
// reference.  Slots past a lane's own length are padding (column 0, value 0) and are
// not added.  Longer rows are cut in kSellMaxLen-term segments that sit in the slices
// like rows; each segment's sum (from -0.0) goes to a partial, and the finalize adds
// beta * y and the partials in segment order (deterministic, within the Sum|terms|
// bound).  The codebook form (spmv_csell_kernel) reads one 4-byte word per slot.
#include "sm_internal.h"
#include "sell.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace smamd {
namespace {

constexpr int kSellThreads = 64 * kSellGroup;

// ABL (development only, SM_SELL_ABLATE; results wrong): 1 replaces the x gathers by
// one broadcast address.
template <int U, int ABL = 0>
__global__ __launch_bounds__(kSellThreads) void spmv_sell_kernel(
    int64_t n_slices, const int64_t *__restrict__ off, const int32_t *__restrict__ len,
    const int32_t *__restrict__ row, const int32_t *__restrict__ row_len,
    const int32_t *__restrict__ col, const float *__restrict__ val, const float *__restrict__ x,
    float *__restrict__ y, float *__restrict__ partials, float alpha, float beta) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * (kSellThreads / 64) + (threadIdx.x >> 6);
    if (s >= n_slices) return;   // wave-uniform
    const int64_t base = off[s];
    const int32_t L = len[s];
    const int32_t r = row[s * kSellLanes + lane];
    const int32_t n = row_len[s * kSellLanes + lane];
    // A row starts from beta * y; a long row's segment from -0.0 (the identity of fp32
    // addition), its sum going to the segment's partial.
    float acc = r >= 0 ? y[r] : -0.0f;
    if (r >= 0 && beta != 1.0f) acc = __fmul_rn(acc, beta);
    const int32_t *c = col + base + lane;
    const float *v = val + base + lane;
    for (int32_t j = 0; j < L; j += U) {
        int32_t cc[U];
        float vv[U], xg[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            cc[u] = __builtin_nontemporal_load(c + (int64_t)(j + u) * kSellLanes);
            vv[u] = __builtin_nontemporal_load(v + (int64_t)(j + u) * kSellLanes);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xg[u] = x[(ABL & 1) ? (cc[u] & 0) : cc[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float t = __fmul_rn(xg[u], __fmul_rn(vv[u], alpha));
            if (j + u < n) acc = __fadd_rn(acc, t);
        }
    }
    if (r >= 0) y[r] = acc;
    else if (r < -1) partials[-2 - r] = acc;
}

// Codebook form (sell.h, SM_SELL_CB): slot = column | id << 24, one coalesced 256-byte
// load per slot of 64 lanes instead of two.  The workgroup first puts fl(table[id] *
// alpha) in LDS (kTabCopies copies, lane l reads copy l % kTabCopies: fewer bank
// conflicts), so each term is x * fl(v * alpha) -- the same bits as the plain form.
constexpr int kCsellTabCopies = 4;
#ifdef SM_DEV
// TS (development builds, SM_SELL_TS=1): lane 0 of every slice's wave stores the wall clock
// (s_memrealtime, 100 MHz) at its start and end here (slices < kSellTsMax).
constexpr int64_t kSellTsMax = 1 << 18;
__device__ unsigned long long g_sell_ts[2 * kSellTsMax];
#endif
// XAUX (development A/B, SM_SELL_XAUX): cache-policy bits of the x gathers (buffer loads).
template <int U, bool TS = false, int ABL = 0, int XAUX = -1>
__global__ __launch_bounds__(kSellThreads) void spmv_csell_kernel(
    int64_t n_slices, const int64_t *__restrict__ off, const int32_t *__restrict__ len,
    const int32_t *__restrict__ row, const int32_t *__restrict__ row_len,
    const uint32_t *__restrict__ word, const float *__restrict__ table, int32_t table_size,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials, float alpha,
    float beta) {
    static_assert(256 * kCsellTabCopies == 4 * kSellThreads, "one float4 of copies per thread");
    __shared__ __attribute__((aligned(16))) float tab[256 * kCsellTabCopies];
    {
        const int id = threadIdx.x;   // 256 threads: one id each, all its copies
        const float t = id < table_size ? __fmul_rn(table[id], alpha) : 0.0f;
        *reinterpret_cast<float4 *>(&tab[kCsellTabCopies * id]) = make_float4(t, t, t, t);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * (kSellThreads / 64) + (threadIdx.x >> 6);
    if (s >= n_slices) return;   // wave-uniform, after the only barrier
#ifdef SM_DEV
    if constexpr (TS) {
        if (lane == 0 && s < kSellTsMax) g_sell_ts[2 * s] = wall_clock64();
    }
#endif
    const int64_t base = off[s];
    const int32_t L = len[s];
    const int32_t r = row[s * kSellLanes + lane];
    const int32_t n = row_len[s * kSellLanes + lane];
    float acc = r >= 0 ? y[r] : -0.0f;
    if (r >= 0 && beta != 1.0f) acc = __fmul_rn(acc, beta);
    const uint32_t *w = word + base + lane;
    const int cp = lane & (kCsellTabCopies - 1);
    constexpr uint32_t kColMask = (1u << kSellCbColBits) - 1u;
    for (int32_t j = 0; j < L; j += U) {
        uint32_t ww[U];
        float xg[U], tv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) ww[u] = __builtin_nontemporal_load(w + (int64_t)(j + u) * kSellLanes);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t xi = (ABL & 1) ? 0u : (ww[u] & kColMask);
            if constexpr (XAUX < 0)
                xg[u] = x[xi];
            else
                xg[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), (short)0, (int)0x7FFFFFFF, 0x00020000),
                    4u * xi, 0, XAUX));
            tv[u] = tab[(ww[u] >> kSellCbColBits) * kCsellTabCopies + cp];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float t = __fmul_rn(xg[u], tv[u]);
            if (j + u < n) acc = __fadd_rn(acc, t);
        }
    }
    if (r >= 0) y[r] = acc;
    else if (r < -1) partials[-2 - r] = acc;
#ifdef SM_DEV
    if constexpr (TS) {
        if (lane == 0 && s < kSellTsMax) g_sell_ts[2 * s + 1] = wall_clock64();
    }
#endif
}

#ifdef SM_DEV
// Timeline of the last TS launch (SM_SELL_TS): per slice length class, how many slices,
// their mean duration and latest end; when 50 / 90 / 99 / 100 % of the slices had ended;
// and the kernel's span -- where the time of the slice kernel goes.
void sell_ts_report(const SellDev &sd, hipStream_t s) {
    const int64_t ns = std::min<int64_t>(sd.n_slices, kSellTsMax);
    std::vector<unsigned long long> h((size_t)(2 * ns));
    std::vector<int32_t> len((size_t)ns);
    void *sym = nullptr;
    if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_sell_ts)) != hipSuccess) return;
    (void)hipMemcpyAsync(h.data(), sym, h.size() * 8, hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(len.data(), sd.d_len, (size_t)ns * 4, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int64_t i = 0; i < ns; i++) {
        t0 = std::min(t0, h[(size_t)(2 * i)]);
        t1 = std::max(t1, h[(size_t)(2 * i + 1)]);
    }
    std::vector<double> ends((size_t)ns);
    struct Cls { int64_t n = 0; double dur = 0, last = 0, first = 1e30, slots = 0; };
    Cls cls[13];
    for (int64_t i = 0; i < ns; i++) {
        const double a = (h[(size_t)(2 * i)] - t0) * 0.01, b = (h[(size_t)(2 * i + 1)] - t0) * 0.01;
        ends[(size_t)i] = b;
        int k = 0;
        while (k < 12 && (1 << (k + 1)) <= len[(size_t)i]) k++;
        cls[k].n++;
        cls[k].dur += b - a;
        cls[k].last = std::max(cls[k].last, b);
        cls[k].first = std::min(cls[k].first, a);
        cls[k].slots += len[(size_t)i];
    }
    std::vector<double> se = ends;
    std::sort(se.begin(), se.end());
    fprintf(stderr, "sell timeline: %lld slices, span %.1f us; 50/90/99/100 %% of the slices ended by "
            "%.1f / %.1f / %.1f / %.1f us\n", (long long)ns, (t1 - t0) * 0.01, se[(size_t)(ns / 2)],
            se[(size_t)(9 * ns / 10)], se[(size_t)(99 * ns / 100)], se.back());
    for (int k = 0; k < 13; k++)
        if (cls[k].n)
            fprintf(stderr, "  len [%5d, %5d): %7lld slices, %9.0f slot rows, mean %7.2f us, first start %7.1f, "
                    "last end %7.1f us\n", 1 << k, 2 << k, (long long)cls[k].n, cls[k].slots,
                    cls[k].dur / cls[k].n, cls[k].first, cls[k].last);
}
#endif

}  // namespace

hipError_t launch_spmv_sell(const SellDev &sd, const float *x, float *y, float alpha, float beta,
                            hipStream_t s) {
    if (sd.n_slices <= 0) return hipSuccess;
    if (!sd.d_off || !sd.d_len || !sd.d_row || !sd.d_row_len || !sd.d_col || (!sd.d_val && !sd.d_table))
        return hipErrorInvalidValue;
    if (sd.d_table && (sd.table_size < 0 || sd.table_size > 256)) return hipErrorInvalidValue;
    const int64_t grid = (sd.n_slices + kSellThreads / 64 - 1) / (kSellThreads / 64);
    if (grid > 0x7FFFFFFF) return hipErrorInvalidValue;
    static_assert(kSellUnroll % 8 == 0, "slice lengths are multiples of the unroll");
    // Unrolls past kSellUnroll read slots past a slice's padded length: those lanes'
    // row lengths stop the adds, and the reads stay inside the arrays' zero tail.
#define SM_SELL_K(U, A)                                                                        \
    hipLaunchKernelGGL((spmv_sell_kernel<U, A>), dim3((unsigned)grid), dim3(kSellThreads), 0, s, \
                       sd.n_slices, sd.d_off, sd.d_len, sd.d_row, sd.d_row_len, sd.d_col,       \
                       sd.d_val, x, y, sd.d_partials, alpha, beta)
#define SM_CSELL_K(U)                                                                          \
    hipLaunchKernelGGL((spmv_csell_kernel<U>), dim3((unsigned)grid), dim3(kSellThreads), 0, s,      \
                       sd.n_slices, sd.d_off, sd.d_len, sd.d_row, sd.d_row_len,                     \
                       reinterpret_cast<const uint32_t *>(sd.d_col), sd.d_table, sd.table_size,    \
                       x, y, sd.d_partials, alpha, beta)
#ifdef SM_DEV
    // Development builds: the gather ablation (SM_SELL_ABLATE=1, results wrong) and the
    // unroll A/B (SM_SELL_UNROLL).
    static const int abl = [] {
        const char *e = dev_env("SM_SELL_ABLATE");
        return e ? atoi(e) : 0;
    }();
    static const int unroll = [] {
        const char *e = dev_env("SM_SELL_UNROLL");
        return e ? atoi(e) : 8;
    }();
    static const bool ts = dev_env("SM_SELL_TS") != nullptr;
    static const int xaux = [] {
        const char *e = dev_env("SM_SELL_XAUX");
        return e ? atoi(e) : -1;
    }();
    if (sd.d_table && xaux >= 0 && abl == 0 && !ts) {
#define SM_CSELLX(A)                                                                                      \
    hipLaunchKernelGGL((spmv_csell_kernel<8, false, 0, A>), dim3((unsigned)grid), dim3(kSellThreads), 0, s,   \
                       sd.n_slices, sd.d_off, sd.d_len, sd.d_row, sd.d_row_len,                               \
                       reinterpret_cast<const uint32_t *>(sd.d_col), sd.d_table, sd.table_size, x, y,          \
                       sd.d_partials, alpha, beta)
        switch (xaux) {
        case 1: SM_CSELLX(1); break;
        case 2: SM_CSELLX(2); break;
        case 16: SM_CSELLX(16); break;
        case 17: SM_CSELLX(17); break;
        default: SM_CSELLX(0); break;
        }
#undef SM_CSELLX
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return launch_long_finalize(sd.n_long, sd.d_long_rows, sd.d_long_ptr, sd.d_partials, y, beta, s);
    }
    if (sd.d_table && abl == 1) {   // the gathers ablated (one broadcast address), with the timeline
        hipLaunchKernelGGL((spmv_csell_kernel<8, true, 1>), dim3((unsigned)grid), dim3(kSellThreads), 0, s,
                           sd.n_slices, sd.d_off, sd.d_len, sd.d_row, sd.d_row_len,
                           reinterpret_cast<const uint32_t *>(sd.d_col), sd.d_table, sd.table_size, x, y,
                           sd.d_partials, alpha, beta);
        if (ts) sell_ts_report(sd, s);
    } else if (sd.d_table && ts) {
        hipLaunchKernelGGL((spmv_csell_kernel<8, true>), dim3((unsigned)grid), dim3(kSellThreads), 0, s,
                           sd.n_slices, sd.d_off, sd.d_len, sd.d_row, sd.d_row_len,
                           reinterpret_cast<const uint32_t *>(sd.d_col), sd.d_table, sd.table_size, x, y,
                           sd.d_partials, alpha, beta);
        sell_ts_report(sd, s);
    } else if (sd.d_table) {
        if (unroll == 16) SM_CSELL_K(16);
        else SM_CSELL_K(8);
    } else if (abl == 1) SM_SELL_K(8, 1);
    else if (unroll == 16) SM_SELL_K(16, 0);
    else if (unroll == 32) SM_SELL_K(32, 0);
    else SM_SELL_K(8, 0);
#else
    if (sd.d_table) SM_CSELL_K(8);
    else SM_SELL_K(8, 0);
#endif
#undef SM_SELL_K
#undef SM_CSELL_K
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // Long rows: beta * y + their segment partials, in segment order.
    return launch_long_finalize(sd.n_long, sd.d_long_rows, sd.d_long_ptr, sd.d_partials, y, beta, s);
}

}  // namespace smamd
