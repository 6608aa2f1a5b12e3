// kernels_ccsell.hip -- SpMV over the column-chunked sorted sliced-ELL layout
// (ccsell.h, ccsell.cpp): one launch per column chunk, in chunk order.
//
// Why: with x far larger than an XCD's 4 MiB L2 (config 5: a rank's x is 256 MiB),
// a row-ordered sliced ELL gathers every term's x from the Infinity Cache or HBM --
// one 64-128-byte line per 4-byte term.  Cut by column chunks of 4 MiB instead, a
// launch's gathers all fall in the chunk the XCDs have just pulled into their L2s;
// the price is that y is read and written once per (row, chunk) pair -- sequential,
// coalesced-by-slice traffic that the cache hierarchy absorbs far better than
// random line gathers.
//
// Per launch: one wavefront per slice of 64 units (a unit = one row's terms inside
// the chunk), four slices per 256-thread workgroup, no LDS except the codebook table,
// no barrier after it.  Lane l loads y[row] (applying beta when the unit is the row's
// first), adds x * fl(v * alpha) for its terms in stored order (kernel.cc:791,
// 580-582) and stores y[row].  A row's units sit in ascending chunks and the launches
// run in chunk order on one stream, so every row is summed in the reference's order
// (ascending column), bit for bit; within a launch no two lanes share a row.
#include "sm_internal.h"
#include "ccsell.h"
#include "sell.h"

namespace smamd {
namespace {

constexpr int kCcThreads = 256;
constexpr int kCcTabCopies = 4;

template <int U, bool CB>
__global__ __launch_bounds__(kCcThreads) void spmv_ccsell_kernel(
    int64_t s0, int64_t s1, const int64_t *__restrict__ off, const int32_t *__restrict__ len,
    const int32_t *__restrict__ row, const uint16_t *__restrict__ row_len,
    const uint32_t *__restrict__ word, const float *__restrict__ val,
    const float *__restrict__ table, int32_t table_size, const float *__restrict__ xc,
    uint32_t cmask, int32_t chunk_log2, float *__restrict__ y, float alpha, float beta) {
    __shared__ __attribute__((aligned(16))) float tab[CB ? 256 * kCcTabCopies : 4];
    if constexpr (CB) {
        static_assert(256 * kCcTabCopies == 4 * kCcThreads, "one float4 of copies per thread");
        const int id = threadIdx.x;
        const float t = id < table_size ? __fmul_rn(table[id], alpha) : 0.0f;
        *reinterpret_cast<float4 *>(&tab[kCcTabCopies * id]) = make_float4(t, t, t, t);
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t s = s0 + (int64_t)blockIdx.x * (kCcThreads / 64) + (threadIdx.x >> 6);
    if (s >= s1) return;   // wave-uniform, after the only barrier
    const int32_t rw = row[s * kSellLanes + lane];
    if (rw == -1) return;  // a lane past the chunk's last unit
    const int32_t r = rw & 0x7FFFFFFF;
    const int32_t n = row_len[s * kSellLanes + lane];
    const int64_t base = off[s];
    const int32_t L = len[s];
    float acc = y[r];
    if ((rw & (int32_t)kCcFirst) && beta != 1.0f) acc = __fmul_rn(acc, beta);   // kernel.cc:10-29
    const uint32_t *w = word + base + lane;
    const float *v = CB ? nullptr : val + base + lane;
    const int cp = lane & (kCcTabCopies - 1);
    int32_t j = 0;
    for (; j + U <= L; j += U) {   // slices are not padded: whole groups of U slots, then the rest
        uint32_t ww[U];
        float xg[U], tv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) ww[u] = __builtin_nontemporal_load(w + (int64_t)(j + u) * kSellLanes);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            xg[u] = xc[ww[u] & cmask];
            if constexpr (CB)
                tv[u] = tab[(ww[u] >> chunk_log2) * kCcTabCopies + cp];
            else
                tv[u] = __fmul_rn(__builtin_nontemporal_load(v + (int64_t)(j + u) * kSellLanes), alpha);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float t = __fmul_rn(xg[u], tv[u]);
            if (j + u < n) acc = __fadd_rn(acc, t);
        }
    }
    for (; j < L; ++j) {
        const uint32_t ww = __builtin_nontemporal_load(w + (int64_t)j * kSellLanes);
        const float xg = xc[ww & cmask];
        float tv;
        if constexpr (CB)
            tv = tab[(ww >> chunk_log2) * kCcTabCopies + cp];
        else
            tv = __fmul_rn(__builtin_nontemporal_load(v + (int64_t)j * kSellLanes), alpha);
        const float t = __fmul_rn(xg, tv);
        if (j < n) acc = __fadd_rn(acc, t);
    }
    y[r] = acc;
}

}  // namespace

hipError_t launch_spmv_ccsell(const CcsellDev &cd, const float *x, float *y, float alpha,
                              float beta, hipStream_t s) {
    if (cd.n_slices <= 0) return hipSuccess;
    if (!cd.d_off || !cd.d_len || !cd.d_row || !cd.d_row_len || !cd.d_word ||
        (!cd.d_table && !cd.d_val) || (int64_t)cd.chunk_slice.size() != cd.n_chunks + 1 ||
        cd.chunk_log2 < 8 || cd.chunk_log2 > 30 || (cd.d_table && cd.chunk_log2 > 24))
        return hipErrorInvalidValue;
    if (cd.d_table && (cd.table_size < 0 || cd.table_size > 256)) return hipErrorInvalidValue;
    const uint32_t cmask = (uint32_t)((1ull << cd.chunk_log2) - 1);
    for (int32_t c = 0; c < cd.n_chunks; ++c) {
        const int64_t a = cd.chunk_slice[(size_t)c], b = cd.chunk_slice[(size_t)c + 1];
        if (a == b) continue;
        const int64_t grid = (b - a + kCcThreads / 64 - 1) / (kCcThreads / 64);
        if (grid > 0x7FFFFFFF) return hipErrorInvalidValue;
        const float *xc = x + ((int64_t)c << cd.chunk_log2);
        if (cd.d_table)
            hipLaunchKernelGGL((spmv_ccsell_kernel<8, true>), dim3((unsigned)grid), dim3(kCcThreads),
                               0, s, a, b, cd.d_off, cd.d_len, cd.d_row, cd.d_row_len, cd.d_word,
                               nullptr, cd.d_table, cd.table_size, xc, cmask, cd.chunk_log2, y,
                               alpha, beta);
        else
            hipLaunchKernelGGL((spmv_ccsell_kernel<8, false>), dim3((unsigned)grid), dim3(kCcThreads),
                               0, s, a, b, cd.d_off, cd.d_len, cd.d_row, cd.d_row_len, cd.d_word,
                               cd.d_val, nullptr, 0, xc, cmask, cd.chunk_log2, y, alpha, beta);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace smamd
