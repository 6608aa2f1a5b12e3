// refenc_dev.hip -- the reference's encoding (sparse-matrix.cc:32-97) built on the device
// from a device-resident CSR of B = S^T: what sm_build_ref_stream and the device CopyForm
// constructor keep, the same bytes encode_csr_ref (encode.cpp) produces on the host.
//
// The stream's order is per panel of 256 S columns (= 256 CSR rows), entries row-major in
// S: by (S row = CSR column, S column in the panel).  Each CSR row is sorted already, so a
// panel's entries are the merge of its 256 rows -- done here as one device radix sort of
// 64-bit keys (panel, column, row in panel), the panel in the high bits so each panel's
// entries keep the CSR's [row_ptr[256 p], row_ptr[256 p + 256]) span.  Then per entry the
// gap to the previous one in its panel gives its bytes (gap > 255: (gap - 1) / 255 filler
// steps of (255, T), sparse-matrix.cc:49-56), an exclusive scan places them, and one pass
// writes the stream.  The codebook (when none is given): the values' distinct fp32 bit
// patterns in first-occurrence order (a stable sort of (bits, index) and the run heads).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "encode.h"
#include "sm_internal.h"

namespace smamd {
namespace {

constexpr int kPanelShift = 8;   // SBLAS_BLOCK_COL_SHIFT (kernel.h:26)
constexpr int64_t kMaxStep = 255;

// Value -> id: binary search over the codebook's distinct bit patterns (sorted, <= 255).
__device__ __forceinline__ int lookup_id(uint32_t u, const uint32_t *tb, const uint8_t *tid, int K) {
    int lo = 0, hi = K;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tb[mid] < u) lo = mid + 1;
        else hi = mid;
    }
    return lo < K && tb[lo] == u ? (int)tid[lo] : -1;
}

// Wave per CSR row (grid-stride): the sort keys and ids of its terms.  ids given (the
// dense-index constructor's own) or looked up from the values; a value outside the
// codebook sets *bad.
__global__ __launch_bounds__(256) void refenc_keys_kernel(
    int64_t n_rows, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, const uint8_t *__restrict__ ids_in, const uint32_t *__restrict__ tb,
    const uint8_t *__restrict__ tid, int K, int lin_bits, uint64_t *__restrict__ key,
    uint8_t *__restrict__ ids, int32_t *__restrict__ bad) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; r < n_rows; r += waves) {
        const uint64_t hi = ((uint64_t)(r >> kPanelShift) << lin_bits) | (uint64_t)(r & 255);
        for (int64_t e = rp[r] + lane; e < rp[r + 1]; e += 64) {
            key[e] = hi | ((uint64_t)(uint32_t)col[e] << kPanelShift);
            int id;
            if (ids_in) {
                id = ids_in[e];
            } else {
                id = lookup_id(__float_as_uint(val[e]), tb, tid, K);
                if (id < 0) {
                    atomicOr(bad, 1);
                    id = 0;
                }
            }
            ids[e] = (uint8_t)id;
        }
    }
}

// Codebook discovery: after a stable sort of (bits, index), the head of each run of equal
// bits carries the value's first index; heads go to slots (at most 256 kept, all counted).
__global__ __launch_bounds__(256) void refenc_heads_kernel(int64_t n, const uint32_t *__restrict__ bits,
                                                           const int32_t *__restrict__ idx,
                                                           int32_t *__restrict__ n_heads,
                                                           uint32_t *__restrict__ head_bits,
                                                           int32_t *__restrict__ head_idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i > 0 && bits[i] == bits[i - 1]) continue;
        const int32_t slot = atomicAdd(n_heads, 1);
        if (slot < 256) {
            head_bits[slot] = bits[i];
            head_idx[slot] = idx[i];
        }
    }
}

__global__ __launch_bounds__(256) void refenc_bits_kernel(int64_t n, const float *__restrict__ val,
                                                          uint32_t *__restrict__ bits, int32_t *__restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bits[i] = __float_as_uint(val[i]);
        idx[i] = (int32_t)i;
    }
}

__device__ __forceinline__ int64_t entry_gap(const uint64_t *key, int64_t i, int lin_bits) {
    const uint64_t mask = ((uint64_t)1 << lin_bits) - 1;
    const uint64_t k = key[i];
    uint64_t prev = 0;
    if (i > 0 && (key[i - 1] >> lin_bits) == (k >> lin_bits)) prev = key[i - 1] & mask;
    return (int64_t)((k & mask) - prev);
}

// Bytes of each sorted entry: its filler steps + itself.
__global__ __launch_bounds__(256) void refenc_bytes_kernel(int64_t n, const uint64_t *__restrict__ key,
                                                           int lin_bits, int64_t *__restrict__ bytes) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t gap = entry_gap(key, i, lin_bits);
        bytes[i] = (gap > kMaxStep ? (gap - 1) / kMaxStep : 0) + 1;
    }
}

__global__ __launch_bounds__(256) void refenc_emit_kernel(int64_t n, const uint64_t *__restrict__ key,
                                                          const uint8_t *__restrict__ ids, int lin_bits,
                                                          const int64_t *__restrict__ off, uint8_t T,
                                                          uint8_t *__restrict__ pos, uint8_t *__restrict__ vid) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t gap = entry_gap(key, i, lin_bits);
        int64_t o = off[i];
        while (gap > kMaxStep) {   // sparse-matrix.cc:49-56
            pos[o] = (uint8_t)kMaxStep;
            vid[o] = T;
            ++o;
            gap -= kMaxStep;
        }
        pos[o] = (uint8_t)gap;
        vid[o] = ids[i];
    }
}

// Per panel of 256 CSR rows: its span of the stream (begin == end: no entries).
__global__ __launch_bounds__(256) void refenc_panels_kernel(int64_t n_panels, int64_t n_rows,
                                                            const int32_t *__restrict__ rp,
                                                            const int64_t *__restrict__ off, int64_t total,
                                                            int64_t *__restrict__ pb, int64_t *__restrict__ pe) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_panels; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = rp[std::min<int64_t>(p << kPanelShift, n_rows)];
        const int64_t e1 = rp[std::min<int64_t>((p + 1) << kPanelShift, n_rows)];
        const int64_t nnz = rp[n_rows];
        pb[p] = e0 < nnz ? off[e0] : total;
        pe[p] = e1 < nnz ? off[e1] : total;
    }
}

unsigned grid_for(int64_t n) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 16));
}

struct DevBufs {
    std::vector<void *> p;
    template <class T>
    hipError_t alloc(T **out, int64_t n) {
        *out = nullptr;
        const hipError_t e = hipMalloc((void **)out, (size_t)std::max<int64_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(*out);
        return e;
    }
    ~DevBufs() {
        for (void *q : p) (void)hipFree(q);
    }
};

#define RE_TRY(x)                   \
    do {                            \
        const hipError_t e_ = (x);  \
        if (e_ != hipSuccess) {     \
            err = e_;               \
            return -5;              \
        }                           \
    } while (0)

}  // namespace

int encode_csr_ref_device(const int32_t *d_rp, const int32_t *d_col, const float *d_val, const uint8_t *d_ids,
                          int64_t n_rows, int64_t n_cols, int64_t nnz, const float *table,
                          int32_t table_size, EncodeResult &out, hipStream_t s, hipError_t &err) {
    out = EncodeResult();
    err = hipSuccess;
    if (n_cols >= ((int64_t)1 << (31 - kPanelShift))) return -4;
    if (table && (table_size < 0 || table_size > (int32_t)kMaxStep)) return -1;
    if (d_ids && !table) return -1;
    DevBufs b;
    const unsigned g_rows = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_rows + 3) / 4, 1 << 16));
    // ---- the codebook: value bits -> id (the first entry with those bits) ----------------
    std::vector<std::pair<uint32_t, uint8_t>> book;   // sorted by bits
    auto bits_of = [](float v) {
        uint32_t u;
        memcpy(&u, &v, 4);
        return u;
    };
    if (table) {
        out.table.assign(table, table + table_size);
        for (int32_t i = 0; i < table_size; i++) book.push_back({bits_of(table[i]), (uint8_t)i});
    } else if (nnz > 0) {
        uint32_t *bits = nullptr, *bits_s = nullptr, *hb = nullptr;
        int32_t *idx = nullptr, *idx_s = nullptr, *nh = nullptr, *hi = nullptr;
        RE_TRY(b.alloc(&bits, nnz));
        RE_TRY(b.alloc(&bits_s, nnz));
        RE_TRY(b.alloc(&idx, nnz));
        RE_TRY(b.alloc(&idx_s, nnz));
        RE_TRY(b.alloc(&nh, 1));
        RE_TRY(b.alloc(&hb, 256));
        RE_TRY(b.alloc(&hi, 256));
        hipLaunchKernelGGL(refenc_bits_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, nnz, d_val, bits, idx);
        RE_TRY(hipGetLastError());
        size_t tmp_bytes = 0;
        RE_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, bits, bits_s, idx, idx_s, (int)nnz, 0, 32, s));
        uint8_t *tmp = nullptr;
        RE_TRY(b.alloc(&tmp, (int64_t)tmp_bytes));
        RE_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, bits, bits_s, idx, idx_s, (int)nnz, 0, 32, s));
        RE_TRY(hipMemsetAsync(nh, 0, 4, s));
        hipLaunchKernelGGL(refenc_heads_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, nnz, bits_s, idx_s, nh, hb, hi);
        RE_TRY(hipGetLastError());
        int32_t n_heads = 0;
        RE_TRY(hipMemcpyAsync(&n_heads, nh, 4, hipMemcpyDeviceToHost, s));
        RE_TRY(hipStreamSynchronize(s));
        if (n_heads > (int32_t)kMaxStep) return -3;
        std::vector<uint32_t> hbits((size_t)n_heads);
        std::vector<int32_t> hidx((size_t)n_heads);
        if (n_heads) {
            RE_TRY(hipMemcpy(hbits.data(), hb, (size_t)n_heads * 4, hipMemcpyDeviceToHost));
            RE_TRY(hipMemcpy(hidx.data(), hi, (size_t)n_heads * 4, hipMemcpyDeviceToHost));
        }
        std::vector<int32_t> order((size_t)n_heads);
        for (int32_t i = 0; i < n_heads; i++) order[(size_t)i] = i;
        std::sort(order.begin(), order.end(), [&](int32_t a, int32_t c) { return hidx[(size_t)a] < hidx[(size_t)c]; });
        for (int32_t i = 0; i < n_heads; i++) {   // ids in first-occurrence order
            const uint32_t u = hbits[(size_t)order[(size_t)i]];
            float f;
            memcpy(&f, &u, 4);
            out.table.push_back(f);
            book.push_back({u, (uint8_t)i});
        }
        table_size = n_heads;
    } else {
        table_size = 0;
    }
    out.table.push_back(0.0f);
    out.table_size = table_size;
    out.s_rows = n_cols;
    out.s_cols = n_rows;
    if (nnz == 0) return 0;
    if (table_size == 0) return -2;
    // First table entry per bit pattern (a dense index naming either of two equal entries
    // decodes to the same value), sorted by bits for the device search.
    std::stable_sort(book.begin(), book.end(),
                     [](const std::pair<uint32_t, uint8_t> &a, const std::pair<uint32_t, uint8_t> &c) {
                         return a.first < c.first;
                     });
    book.erase(std::unique(book.begin(), book.end(),
                           [](const std::pair<uint32_t, uint8_t> &a, const std::pair<uint32_t, uint8_t> &c) {
                               return a.first == c.first;
                           }),
               book.end());
    const int K = (int)book.size();
    std::vector<uint32_t> tbits((size_t)K);
    std::vector<uint8_t> tids((size_t)K);
    for (int i = 0; i < K; i++) tbits[(size_t)i] = book[(size_t)i].first, tids[(size_t)i] = book[(size_t)i].second;
    const uint8_t T = (uint8_t)table_size;
    // ---- keys, sort, bytes, scan, emit --------------------------------------------------
    int lin_bits = kPanelShift;
    while (((int64_t)1 << (lin_bits - kPanelShift)) < n_cols) lin_bits++;
    const int64_t n_panels = (n_rows + 255) >> kPanelShift;
    int panel_bits = 0;
    while (((int64_t)1 << panel_bits) < n_panels) panel_bits++;
    uint32_t *d_tb = nullptr;
    uint8_t *d_tid = nullptr, *ids = nullptr, *ids_s = nullptr;
    uint64_t *key = nullptr, *key_s = nullptr;
    int32_t *bad = nullptr;
    int64_t *bytes = nullptr, *off = nullptr, *pb = nullptr, *pe = nullptr;
    RE_TRY(b.alloc(&d_tb, K));
    RE_TRY(b.alloc(&d_tid, K));
    RE_TRY(b.alloc(&ids, nnz));
    RE_TRY(b.alloc(&ids_s, nnz));
    RE_TRY(b.alloc(&key, nnz));
    RE_TRY(b.alloc(&key_s, nnz));
    RE_TRY(b.alloc(&bad, 1));
    RE_TRY(hipMemcpyAsync(d_tb, tbits.data(), (size_t)K * 4, hipMemcpyHostToDevice, s));
    RE_TRY(hipMemcpyAsync(d_tid, tids.data(), (size_t)K, hipMemcpyHostToDevice, s));
    RE_TRY(hipMemsetAsync(bad, 0, 4, s));
    hipLaunchKernelGGL(refenc_keys_kernel, dim3(g_rows), dim3(256), 0, s, n_rows, d_rp, d_col, d_val, d_ids, d_tb,
                       d_tid, K, lin_bits, key, ids, bad);
    RE_TRY(hipGetLastError());
    int32_t h_bad = 0;
    RE_TRY(hipMemcpyAsync(&h_bad, bad, 4, hipMemcpyDeviceToHost, s));
    RE_TRY(hipStreamSynchronize(s));
    if (h_bad) return -2;
    {
        size_t tmp_bytes = 0;
        const int end_bit = lin_bits + panel_bits;
        RE_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, key, key_s, ids, ids_s, (int)nnz, 0, end_bit, s));
        uint8_t *tmp = nullptr;
        RE_TRY(b.alloc(&tmp, (int64_t)tmp_bytes));
        RE_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key, key_s, ids, ids_s, (int)nnz, 0, end_bit, s));
    }
    RE_TRY(b.alloc(&bytes, nnz));
    RE_TRY(b.alloc(&off, nnz));
    hipLaunchKernelGGL(refenc_bytes_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, nnz, key_s, lin_bits, bytes);
    RE_TRY(hipGetLastError());
    {
        size_t tmp_bytes = 0;
        RE_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, bytes, off, (int)nnz, s));
        uint8_t *tmp = nullptr;
        RE_TRY(b.alloc(&tmp, (int64_t)tmp_bytes));
        RE_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, bytes, off, (int)nnz, s));
    }
    int64_t last[2] = {0, 0};
    RE_TRY(hipMemcpyAsync(&last[0], off + nnz - 1, 8, hipMemcpyDeviceToHost, s));
    RE_TRY(hipMemcpyAsync(&last[1], bytes + nnz - 1, 8, hipMemcpyDeviceToHost, s));
    RE_TRY(hipStreamSynchronize(s));
    const int64_t total = last[0] + last[1];
    uint8_t *pos = nullptr, *vid = nullptr;
    RE_TRY(b.alloc(&pos, total));
    RE_TRY(b.alloc(&vid, total));
    RE_TRY(b.alloc(&pb, n_panels));
    RE_TRY(b.alloc(&pe, n_panels));
    hipLaunchKernelGGL(refenc_emit_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, nnz, key_s, ids_s, lin_bits, off, T,
                       pos, vid);
    RE_TRY(hipGetLastError());
    hipLaunchKernelGGL(refenc_panels_kernel, dim3(grid_for(n_panels)), dim3(256), 0, s, n_panels, n_rows, d_rp, off,
                       total, pb, pe);
    RE_TRY(hipGetLastError());
    out.pos.resize((size_t)total);
    out.val_id.resize((size_t)total);
    std::vector<int64_t> hb((size_t)n_panels), he((size_t)n_panels);
    RE_TRY(hipMemcpyAsync(out.pos.data(), pos, (size_t)total, hipMemcpyDeviceToHost, s));
    RE_TRY(hipMemcpyAsync(out.val_id.data(), vid, (size_t)total, hipMemcpyDeviceToHost, s));
    RE_TRY(hipMemcpyAsync(hb.data(), pb, (size_t)n_panels * 8, hipMemcpyDeviceToHost, s));
    RE_TRY(hipMemcpyAsync(he.data(), pe, (size_t)n_panels * 8, hipMemcpyDeviceToHost, s));
    RE_TRY(hipStreamSynchronize(s));
    for (int64_t p = 0; p < n_panels; p++) {   // panels with entries only (sparse-matrix.cc:57-61)
        if (he[(size_t)p] == hb[(size_t)p]) continue;
        out.panel_row_off.push_back(0);
        out.panel_col_off.push_back((int32_t)(p << kPanelShift));
        out.panel_begin.push_back(hb[(size_t)p]);
        out.panel_end.push_back(he[(size_t)p]);
    }
    return 0;
}

#undef RE_TRY

}  // namespace smamd
