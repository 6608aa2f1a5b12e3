// encode_dev.hip -- CopyForm's dense codebook-index scan on the device
// (sparse-matrix.cc:20-99): CSR of B = S^T straight from a
// device-resident rows x stride uint8 index, the same CSR the host encoder
// (encode.cpp) builds -- B row j lists, in ascending S-row order, the S-row index
// and table[id] of every id < table_size of S column j.
//   NoTrans (S = index):   B row j = column j of the index (strided bytes);
//   Trans   (S = index^T): B row j = row j of the index (contiguous bytes).
// The fill pass can also keep each term's id (ids != null) for the reference stream
// (refenc_dev.hip).  Two passes (count, fill) around a host prefix sum of the counts: the count
// arrays are small (one int per B row, or per (row chunk, B row)), and the
// matrix constructor copies row_ptr to the host for its plans anyway.
#include "sm_internal.h"

#include <algorithm>

namespace smamd {
namespace {

// NoTrans.  Thread = (B row j, chunk of index rows): counts, then fills at its
// chunk's offset; chunks ascend in index row, so each B row stays in order.  A
// wave reads 64 consecutive bytes of one index row per step (coalesced).
__global__ __launch_bounds__(256) void encode_cols_kernel(const uint8_t *__restrict__ dm,
                                                          int32_t rows, int32_t cols, int32_t stride,
                                                          int32_t chunk_rows, uint8_t T,
                                                          int32_t *__restrict__ cnt,
                                                          const int32_t *__restrict__ offs,
                                                          const float *__restrict__ table,
                                                          int32_t *__restrict__ col,
                                                          float *__restrict__ val,
                                                          uint8_t *__restrict__ ids) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t ch = blockIdx.y;
    if (j >= cols) return;
    const int32_t r0 = ch * chunk_rows;
    const int32_t r1 = min(rows, r0 + chunk_rows);
    const uint8_t *p = dm + (int64_t)r0 * stride + j;
    if (!offs) {
        int32_t c = 0;
        for (int32_t r = r0; r < r1; ++r, p += stride) c += *p < T;
        cnt[(int64_t)ch * cols + j] = c;
        return;
    }
    int32_t o = offs[(int64_t)ch * cols + j];
    for (int32_t r = r0; r < r1; ++r, p += stride) {
        const uint8_t id = *p;
        if (id < T) {
            col[o] = r;
            val[o] = table[id];
            if (ids) ids[o] = id;
            ++o;
        }
    }
}

// Trans.  Wave = B row j (grid-stride): 64 bytes per step, ballot + mbcnt give
// each kept lane its slot, in ascending index-column order.
__global__ __launch_bounds__(256) void encode_rows_kernel(const uint8_t *__restrict__ dm,
                                                          int32_t rows, int32_t cols, int32_t stride,
                                                          uint8_t T, int32_t *__restrict__ cnt,
                                                          const int32_t *__restrict__ row_ptr,
                                                          const float *__restrict__ table,
                                                          int32_t *__restrict__ col,
                                                          float *__restrict__ val,
                                                          uint8_t *__restrict__ ids) {
    const int lane = threadIdx.x & 63;
    const int32_t waves = gridDim.x * (blockDim.x / 64);
    for (int32_t j = (blockIdx.x * blockDim.x + threadIdx.x) / 64; j < rows; j += waves) {
        const uint8_t *p = dm + (int64_t)j * stride;
        int32_t o = row_ptr ? row_ptr[j] : 0;
        for (int32_t i0 = 0; i0 < cols; i0 += 64) {
            const int32_t i = i0 + lane;
            const uint8_t id = i < cols ? p[i] : T;
            const bool keep = id < T;
            const uint64_t m = __ballot(keep);
            if (row_ptr && keep) {
                const int32_t slot = o + (int32_t)__builtin_amdgcn_mbcnt_hi(
                                             (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                col[slot] = i;
                val[slot] = table[id];
                if (ids) ids[slot] = id;
            }
            o += __popcll(m);
        }
        if (!row_ptr && lane == 0) cnt[j] = o;
    }
}

}  // namespace

hipError_t launch_encode_count(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                               bool trans, int32_t chunk_rows, int32_t n_chunks, uint8_t T,
                               int32_t *cnt, hipStream_t s) {
    if (trans) {
        const int64_t blocks = std::min<int64_t>(((int64_t)rows + 3) / 4, 65535);
        if (blocks > 0)
            hipLaunchKernelGGL(encode_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dm, rows,
                               cols, stride, T, cnt, nullptr, nullptr, nullptr, nullptr, nullptr);
    } else if (cols > 0 && n_chunks > 0) {
        hipLaunchKernelGGL(encode_cols_kernel, dim3((unsigned)((cols + 255) / 256), (unsigned)n_chunks),
                           dim3(256), 0, s, dm, rows, cols, stride, chunk_rows, T, cnt, nullptr,
                           nullptr, nullptr, nullptr, nullptr);
    }
    return hipGetLastError();
}

hipError_t launch_encode_fill(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                              bool trans, int32_t chunk_rows, int32_t n_chunks, uint8_t T,
                              const int32_t *offs, const float *table, int32_t *col, float *val,
                              uint8_t *ids, hipStream_t s) {
    if (trans) {
        const int64_t blocks = std::min<int64_t>(((int64_t)rows + 3) / 4, 65535);
        if (blocks > 0)
            hipLaunchKernelGGL(encode_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dm, rows,
                               cols, stride, T, nullptr, offs, table, col, val, ids);
    } else if (cols > 0 && n_chunks > 0) {
        hipLaunchKernelGGL(encode_cols_kernel, dim3((unsigned)((cols + 255) / 256), (unsigned)n_chunks),
                           dim3(256), 0, s, dm, rows, cols, stride, chunk_rows, T, nullptr, offs,
                           table, col, val, ids);
    }
    return hipGetLastError();
}

}  // namespace smamd
