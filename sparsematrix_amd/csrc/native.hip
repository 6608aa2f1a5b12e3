// native.hip -- AddMatMat straight from the reference's own storage format on the
// device (kernel.cc:771-800, sparse-matrix.cc:139-194): the
// uint8 delta positions and uint8 codebook ids of every 256-column panel (2 bytes per
// entry, fillers included) are decoded in parallel and applied, bit-identical to the
// reference for every output.
//
// Grid: one workgroup per (panel, group of 64 output columns, group of 4 rows of A);
// 256 threads, thread (cl, il) owns output C[i][col] (col = panel col_off + 64 g + cl,
// i = 4 ig + il) and keeps it in a register for the whole kernel.  The workgroup walks
// its panel's stream in chunks of 4096 entries, in order:
//   1. decode   each thread loads 16 consecutive delta bytes and ids (one 16-byte load
//               each), sums its deltas, and a wave prefix scan (DPP row shifts through
//               __shfl_up) plus a 4-wave carry in LDS turns them into in-panel offsets
//               off = running sum (kernel.cc:780-782), continued from the previous chunk;
//   2. bucket   entries with id < T and a column in the group go to per-column lists in
//               LDS (count, prefix over 64 columns, place); a column's entries in one
//               chunk lie in distinct S-rows, so sorting each short list by row restores
//               the stream order;
//   3. apply    thread (cl, il) adds a[i][row] * fl(table[id] * alpha) for its column's
//               entries in ascending row, separate roundings (kernel.cc:791, 568-582).
// Across chunks the entries of a column keep ascending rows, so each output receives
// its terms in exactly the reference's order after beta (kernel.cc:10-29).
#include "sm_internal.h"

namespace smamd {
namespace {

constexpr int kNatThreads = 256;
constexpr int kNatPer = 16;                         // entries per thread per chunk
constexpr int kNatChunk = kNatThreads * kNatPer;    // 4096
constexpr int kNatCols = 64;                        // output columns per workgroup
constexpr int kNatRows = kNatThreads / kNatCols;    // rows of A per workgroup

__global__ __launch_bounds__(kNatThreads) void native_addmatmat_kernel(
    const uint8_t *__restrict__ pos, const uint8_t *__restrict__ val,
    const int64_t *__restrict__ pbeg, const int64_t *__restrict__ pend,
    const int32_t *__restrict__ pcol, const float *__restrict__ table, int32_t T, int32_t n,
    int32_t m, const float *__restrict__ a, int32_t lda, float *__restrict__ c, int32_t ldc,
    float alpha, float beta) {
    __shared__ float tab[256];
    __shared__ int32_t wsum[kNatThreads / 64];
    __shared__ int32_t cnt[kNatCols], base[kNatCols + 1], cur[kNatCols];
    __shared__ int32_t lrow[kNatChunk];
    __shared__ uint8_t lid[kNatChunk];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int32_t p = blockIdx.x, g = blockIdx.y, ig = blockIdx.z;
    const int cl = t & (kNatCols - 1), il = t / kNatCols;
    const int32_t col = pcol[p] + g * kNatCols + cl;
    const int32_t i = ig * kNatRows + il;
    const bool own = col < n && g * kNatCols + cl < 256 && i < m;
    tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
    float acc = 0.0f;
    if (own) {
        acc = c[(int64_t)i * ldc + col];
        if (beta != 1.0f) acc = __fmul_rn(acc, beta);
    }
    const int64_t e_beg = pbeg[p], e_end = pend[p];
    int32_t carry = 0;
    for (int64_t e0 = e_beg; e0 < e_end; e0 += kNatChunk) {
        // 1. decode: 16 entries per thread, in-panel offsets by a workgroup prefix sum.
        const int64_t e = e0 + (int64_t)t * kNatPer;
        uint8_t d[kNatPer], id[kNatPer];
        if (e + kNatPer <= e_end && ((e & 15) == 0)) {
            const uint4 dv = *reinterpret_cast<const uint4 *>(pos + e);
            const uint4 iv = *reinterpret_cast<const uint4 *>(val + e);
            __builtin_memcpy(d, &dv, 16);
            __builtin_memcpy(id, &iv, 16);
        } else {
#pragma unroll
            for (int k = 0; k < kNatPer; ++k) {
                const bool in = e + k < e_end;
                d[k] = in ? pos[e + k] : 0;
                id[k] = in ? val[e + k] : 255;
            }
        }
        int32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) tot += d[k];
        int32_t incl = tot;   // inclusive scan of the thread totals across the wave
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const int32_t v = __shfl_up(incl, s, 64);
            if (lane >= s) incl += v;
        }
        if (lane == 63) wsum[wave] = incl;
        if (t < kNatCols) cnt[t] = 0;
        __syncthreads();
        int32_t before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        int32_t chunk_total = 0;
#pragma unroll
        for (int w = 0; w < kNatThreads / 64; ++w) chunk_total += wsum[w];
        int32_t off = before + incl - tot;
        int32_t offs[kNatPer];
        bool live[kNatPer];
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            off += d[k];
            offs[k] = off;
            const int32_t pc = off & 255;
            live[k] = id[k] < T && (pc >> 6) == g;   // fillers carry id T
            if (live[k]) atomicAdd(&cnt[pc & (kNatCols - 1)], 1);
        }
        carry += chunk_total;
        __syncthreads();
        // 2. bucket: column lists in LDS (placement order arbitrary, sorted by row below).
        if (t == 0) {
            int32_t s = 0;
            for (int q = 0; q < kNatCols; ++q) { base[q] = s; cur[q] = s; s += cnt[q]; }
            base[kNatCols] = s;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            if (!live[k]) continue;
            const int32_t slot = atomicAdd(&cur[offs[k] & (kNatCols - 1)], 1);
            lrow[slot] = offs[k] >> 8;
            lid[slot] = id[k];
        }
        __syncthreads();
        if (il == 0) {   // insertion sort of the column's list by S-row (rows are distinct)
            for (int32_t s = base[cl] + 1; s < base[cl + 1]; ++s) {
                const int32_t r = lrow[s];
                const uint8_t q = lid[s];
                int32_t u = s - 1;
                while (u >= base[cl] && lrow[u] > r) {
                    lrow[u + 1] = lrow[u];
                    lid[u + 1] = lid[u];
                    --u;
                }
                lrow[u + 1] = r;
                lid[u + 1] = q;
            }
        }
        __syncthreads();
        // 3. apply, in ascending row.
        if (own && alpha != 0.0f) {
            const float *ai = a + (int64_t)i * lda;
            for (int32_t s = base[cl]; s < base[cl + 1]; ++s)
                acc = __fadd_rn(acc, __fmul_rn(ai[lrow[s]], tab[lid[s]]));
        }
        __syncthreads();
    }
    if (own) c[(int64_t)i * ldc + col] = acc;
}

}  // namespace

hipError_t launch_native_addmatmat(const NativeDev &nd, int32_t m, const float *a, int32_t lda,
                                   float *c, int32_t ldc, float alpha, float beta, hipStream_t s) {
    const int32_t P = beta != 1.0f ? nd.n_all : nd.n_panels;   // empty blocks only scale
    if (P <= 0 || m <= 0) return hipSuccess;
    if (!nd.d_pos || !nd.d_val || !nd.d_beg || !nd.d_end || !nd.d_col || !nd.d_table ||
        nd.table_size < 0 || nd.table_size > 255)
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)P, 256 / kNatCols, (unsigned)((m + kNatRows - 1) / kNatRows));
    hipLaunchKernelGGL(native_addmatmat_kernel, grid, dim3(kNatThreads), 0, s, nd.d_pos, nd.d_val,
                       nd.d_beg, nd.d_end, nd.d_col, nd.d_table, nd.table_size,
                       (int32_t)nd.s_cols, m, a, lda, c, ldc, alpha, beta);
    return hipGetLastError();
}

}  // namespace smamd
