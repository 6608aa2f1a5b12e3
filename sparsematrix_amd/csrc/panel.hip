// panel.hip -- the reference's own storage format on the device: one panel of
// uint8 delta positions + uint8 codebook ids (kernel.h:42-62, kernel.cc:213-369,
// 771-800), decoded and applied by gfx950 kernels.
//
//   1. scan      single workgroup: running prefix sum of the delta bytes
//                (kernel.cc:780-782), ids >= T skipped, survivors compacted in
//                stream order as (row = off>>8, col = off&255, table[id]*alpha).
//   2. bucket    stable per-column lists (panel columns <= 256): each of 256
//                threads owns one column and appends its entries in stream
//                order, i.e. ascending row -- the per-output order the
//                reference accumulates in.
//   3. apply     one thread per output (i, col): c += a[i][row] * v over the
//                column's list, separate round-to-nearest mul/add: bit-identical
//                to all four reference variants (they agree bit for bit).
// Not a hot path (the hot path is CSR, kernels.hip); sized for panels of up to a
// few million entries.
#include "sm_internal.h"

namespace smamd {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kPanelCols = 256;   // 1 << SBLAS_BLOCK_COL_SHIFT

struct PanelEntry {
    int32_t row, col;
    float v;
    int32_t pad;
};

__global__ __launch_bounds__(kScanThreads) void panel_scan_kernel(
    const uint8_t *__restrict__ ppos, const uint8_t *__restrict__ pval, int32_t pos_len,
    const float *__restrict__ table, int32_t T, float alpha, PanelEntry *__restrict__ out,
    int32_t *__restrict__ n_out) {
    __shared__ int32_t s_off[kScanThreads];
    __shared__ int32_t s_cnt[kScanThreads];
    __shared__ int32_t carry_off, carry_cnt;
    const int tid = threadIdx.x;
    if (tid == 0) { carry_off = 0; carry_cnt = 0; }
    __syncthreads();
    for (int32_t base = 0; base < pos_len; base += kScanThreads) {
        const int32_t e = base + tid;
        const int32_t d = e < pos_len ? (int32_t)ppos[e] : 0;
        const int32_t id = e < pos_len ? (int32_t)pval[e] : T;
        const int32_t live = (e < pos_len && id < T) ? 1 : 0;
        s_off[tid] = d;
        s_cnt[tid] = live;
        __syncthreads();
        for (int s = 1; s < kScanThreads; s <<= 1) {   // Hillis-Steele inclusive scan
            const int32_t a = tid >= s ? s_off[tid - s] : 0;
            const int32_t c = tid >= s ? s_cnt[tid - s] : 0;
            __syncthreads();
            s_off[tid] += a;
            s_cnt[tid] += c;
            __syncthreads();
        }
        const int32_t off = carry_off + s_off[tid];
        const int32_t slot = carry_cnt + s_cnt[tid] - live;
        if (live) {
            const float v = __fmul_rn(table[id], alpha);
            out[slot] = PanelEntry{off >> 8, off & (kPanelCols - 1), v, 0};
        }
        __syncthreads();
        if (tid == kScanThreads - 1) {
            carry_off = off;
            carry_cnt = carry_cnt + s_cnt[tid];
        }
        __syncthreads();
    }
    if (tid == 0) *n_out = carry_cnt;
}

// Stable bucketing by column: thread c collects its column's entries in order.
__global__ __launch_bounds__(kPanelCols) void panel_bucket_kernel(
    const PanelEntry *__restrict__ in, const int32_t *__restrict__ n_in,
    int32_t *__restrict__ col_ptr, int32_t *__restrict__ rows, float *__restrict__ vals) {
    __shared__ int32_t cnt[kPanelCols + 1];
    const int c = threadIdx.x;
    const int32_t n = *n_in;
    int32_t k = 0;
    for (int32_t e = 0; e < n; ++e) k += in[e].col == c;
    cnt[c + 1] = k;
    if (c == 0) cnt[0] = 0;
    __syncthreads();
    if (c == 0)
        for (int i = 0; i < kPanelCols; ++i) cnt[i + 1] += cnt[i];
    __syncthreads();
    col_ptr[c] = cnt[c];
    if (c == kPanelCols - 1) col_ptr[kPanelCols] = cnt[kPanelCols];
    int32_t o = cnt[c];
    for (int32_t e = 0; e < n; ++e) {
        const PanelEntry pe = in[e];
        if (pe.col == c) {
            rows[o] = pe.row;
            vals[o] = pe.v;
            ++o;
        }
    }
}

// transposed: a[row*lda + i], c[col*ldc + i]; else a[i*lda + row], c[i*ldc + col]
template <bool TRANSPOSED>
__global__ __launch_bounds__(256) void panel_apply_kernel(int32_t m, int32_t n,
                                                          const float *__restrict__ a, int32_t lda,
                                                          float *__restrict__ c, int32_t ldc,
                                                          const int32_t *__restrict__ col_ptr,
                                                          const int32_t *__restrict__ rows,
                                                          const float *__restrict__ vals) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)m * n) return;
    int32_t i, j;
    if (TRANSPOSED) { j = (int32_t)(gid / m); i = (int32_t)(gid % m); }
    else { i = (int32_t)(gid / n); j = (int32_t)(gid % n); }
    float *cp = TRANSPOSED ? c + (int64_t)j * ldc + i : c + (int64_t)i * ldc + j;
    float acc = *cp;
    for (int32_t e = col_ptr[j]; e < col_ptr[j + 1]; ++e) {
        const int64_t r = rows[e];
        const float av = TRANSPOSED ? a[r * lda + i] : a[(int64_t)i * lda + r];
        acc = __fadd_rn(acc, __fmul_rn(av, vals[e]));
    }
    *cp = acc;
}

}  // namespace

size_t panel_kernel_workspace_bytes(int32_t pos_len, int32_t) {
    const size_t n = (size_t)std::max(pos_len, 1);
    return n * sizeof(PanelEntry) + 16 + (kPanelCols + 1) * 4 + n * 8 + 64;
}

hipError_t launch_panel_kernel(int variant, int32_t m, int32_t n, int32_t k, const float *a,
                               int32_t lda, float *c, int32_t ldc, float alpha,
                               const uint8_t *ppos, const uint8_t *pval, int32_t pos_len,
                               const float *table, int32_t valid_table_size, void *ws,
                               hipStream_t s) {
    (void)k;
    if (m <= 0 || n <= 0 || pos_len <= 0) return hipSuccess;
    char *p = static_cast<char *>(ws);
    PanelEntry *ent = reinterpret_cast<PanelEntry *>(p);
    p += (size_t)pos_len * sizeof(PanelEntry);
    int32_t *n_ent = reinterpret_cast<int32_t *>(p);
    p += 16;
    int32_t *col_ptr = reinterpret_cast<int32_t *>(p);
    p += (kPanelCols + 1) * 4;
    int32_t *rows = reinterpret_cast<int32_t *>(p);
    p += (size_t)pos_len * 4;
    float *vals = reinterpret_cast<float *>(p);
    hipLaunchKernelGGL(panel_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, ppos, pval, pos_len,
                       table, valid_table_size, alpha, ent, n_ent);
    hipLaunchKernelGGL(panel_bucket_kernel, dim3(1), dim3(kPanelCols), 0, s, ent, n_ent, col_ptr,
                       rows, vals);
    const unsigned grid = (unsigned)(((int64_t)m * n + 255) / 256);
    if (variant >= 2)
        hipLaunchKernelGGL(panel_apply_kernel<true>, dim3(grid), dim3(256), 0, s, m, n, a, lda, c,
                           ldc, col_ptr, rows, vals);
    else
        hipLaunchKernelGGL(panel_apply_kernel<false>, dim3(grid), dim3(256), 0, s, m, n, a, lda, c,
                           ldc, col_ptr, rows, vals);
    return hipGetLastError();
}

}  // namespace smamd
