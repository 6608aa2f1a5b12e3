// builddev.hip -- the column relabeling and the sorted sliced ELL built on the device from a
// device CSR: the same bytes the host builders produce (capi.cpp
// upload_relabel, sell.cpp sell_build, xband.h codebook_ids), without copying the terms to the
// host and back.  R-MAT scale 24 (config 4, 263 M terms) took 5.4 s on the host path.
//
//   relabel   degree histogram (atomics), a stable radix sort of the columns by descending
//             degree (ties in column order = the host's counting sort), rank = the inverse
//             permutation, the skew check (the top 1/16 of the columns hold >= 40 % of the
//             terms) and rcol = rank[col];
//   codebook  the values' distinct bit patterns in first-occurrence order (a stable sort of
//             (bits, index); the run heads), ids by binary search (<= 255 patterns);
//   sell      units (rows of <= max_len terms, max_len-term segments of longer rows, in row
//             order), a stable radix sort by descending length, 64 units per slice, slice
//             lengths rounded up to kSellUnroll, offsets by an exclusive scan, and one wave per
//             slice writing its lanes' terms column-interleaved (zero padding);
//   merge     the merge path's column-sorted staging stream (merge.cpp merge_stage_build): a
//             stable radix sort of every slice's terms by (slice, column), then column << 8 |
//             id and the term's offset in its slice.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "merge.h"
#include "sell.h"
#include "sm_internal.h"

namespace smamd {
namespace {

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 16)); }

#define GS_LOOP(i, n) for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

__global__ __launch_bounds__(256) void bd_degree_kernel(int64_t nnz, const int32_t *__restrict__ col,
                                                        int32_t *__restrict__ deg) {
    GS_LOOP(e, nnz) atomicAdd(&deg[col[e]], 1);
}

__global__ __launch_bounds__(256) void bd_max_kernel(int64_t n, const int32_t *__restrict__ v, int32_t *__restrict__ out) {
    int32_t mx = 0;
    GS_LOOP(i, n) mx = max(mx, v[i]);
    for (int d = 32; d >= 1; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(out, mx);
}

// key = dmax - degree (ascending key = descending degree), value = the column.
__global__ __launch_bounds__(256) void bd_colkey_kernel(int64_t nc, const int32_t *__restrict__ deg, int32_t dmax,
                                                        uint32_t *__restrict__ key, int32_t *__restrict__ idx) {
    GS_LOOP(c, nc) {
        key[c] = (uint32_t)(dmax - deg[c]);
        idx[c] = (int32_t)c;
    }
}

// rank[perm[j]] = j; and the degree sum of the first `top` columns of the new order.
__global__ __launch_bounds__(256) void bd_rank_kernel(int64_t nc, const int32_t *__restrict__ perm,
                                                      const uint32_t *__restrict__ skey, int32_t dmax, int64_t top,
                                                      int32_t *__restrict__ rank, unsigned long long *__restrict__ hot) {
    unsigned long long h = 0;
    GS_LOOP(j, nc) {
        rank[perm[j]] = (int32_t)j;
        if (j < top) h += (unsigned long long)(dmax - (int32_t)skey[j]);
    }
    for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
    if ((threadIdx.x & 63) == 0 && h) atomicAdd(hot, h);
}

__global__ __launch_bounds__(256) void bd_remap_kernel(int64_t nnz, const int32_t *__restrict__ col,
                                                       const int32_t *__restrict__ rank, int32_t *__restrict__ rcol) {
    GS_LOOP(e, nnz) rcol[e] = rank[col[e]];
}

__global__ __launch_bounds__(256) void bd_bits_kernel(int64_t n, const float *__restrict__ val,
                                                      uint32_t *__restrict__ bits, int32_t *__restrict__ idx) {
    GS_LOOP(i, n) {
        bits[i] = __float_as_uint(val[i]);
        idx[i] = (int32_t)i;
    }
}

// After a stable sort of (bits, index): the head of every run of equal bits carries the
// pattern's first index (at most 256 kept, all counted).
__global__ __launch_bounds__(256) void bd_heads_kernel(int64_t n, const uint32_t *__restrict__ bits,
                                                       const int32_t *__restrict__ idx, int32_t *__restrict__ n_heads,
                                                       uint32_t *__restrict__ hb, int32_t *__restrict__ hi) {
    GS_LOOP(i, n) {
        if (i > 0 && bits[i] == bits[i - 1]) continue;
        const int32_t k = atomicAdd(n_heads, 1);
        if (k < 256) {
            hb[k] = bits[i];
            hi[k] = idx[i];
        }
    }
}

// id of every term: binary search of its bits over the (sorted) distinct patterns.
__global__ __launch_bounds__(256) void bd_ids_kernel(int64_t n, const float *__restrict__ val,
                                                     const uint32_t *__restrict__ tb, const uint8_t *__restrict__ tid,
                                                     int32_t K, uint8_t *__restrict__ ids) {
    __shared__ uint32_t s_b[256];
    __shared__ uint8_t s_i[256];
    if (threadIdx.x < K) {
        s_b[threadIdx.x] = tb[threadIdx.x];
        s_i[threadIdx.x] = tid[threadIdx.x];
    }
    __syncthreads();
    GS_LOOP(e, n) {
        const uint32_t u = __float_as_uint(val[e]);
        int lo = 0, hi = K;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_b[mid] < u) lo = mid + 1;
            else hi = mid;
        }
        ids[e] = s_i[lo < K ? lo : 0];   // every pattern is in the table (it came from these values)
    }
}

// Per row: units (1, or ceil(len / max_len) segments), segment partials, long-row flag.
__global__ __launch_bounds__(256) void bd_units_count_kernel(int64_t n_rows, const int32_t *__restrict__ rp,
                                                             int32_t max_len, int32_t *__restrict__ nu,
                                                             int32_t *__restrict__ np, int32_t *__restrict__ lf) {
    GS_LOOP(r, n_rows) {
        const int32_t l = rp[r + 1] - rp[r];
        const bool lng = l > max_len;
        const int32_t k = lng ? (l + max_len - 1) / max_len : 1;
        nu[r] = k;
        np[r] = lng ? k : 0;
        lf[r] = lng ? 1 : 0;
    }
}

// The units in row order: row, first term, length, partial (-1: a whole row); sort key
// max_len - length; the long rows' list and partial offsets (sell.h SellHost).
__global__ __launch_bounds__(256) void bd_units_emit_kernel(
    int64_t n_rows, const int32_t *__restrict__ rp, int32_t max_len, const int32_t *__restrict__ ubase,
    const int32_t *__restrict__ pbase, const int32_t *__restrict__ lbase, int32_t *__restrict__ urow,
    int32_t *__restrict__ ustart, int32_t *__restrict__ un, int32_t *__restrict__ upart,
    uint32_t *__restrict__ ukey, int32_t *__restrict__ uidx, int32_t *__restrict__ long_rows,
    int32_t *__restrict__ long_ptr) {
    GS_LOOP(r, n_rows) {
        const int32_t a = rp[r], l = rp[r + 1] - a;
        int32_t u = ubase[r];
        if (l <= max_len) {
            urow[u] = (int32_t)r;
            ustart[u] = a;
            un[u] = l;
            upart[u] = -1;
            ukey[u] = (uint32_t)(max_len - l);
            uidx[u] = u;
            continue;
        }
        int32_t p = pbase[r];
        for (int32_t b = 0; b < l; b += max_len, ++u, ++p) {
            const int32_t n = min(max_len, l - b);
            urow[u] = (int32_t)r;
            ustart[u] = a + b;
            un[u] = n;
            upart[u] = p;
            ukey[u] = (uint32_t)(max_len - n);
            uidx[u] = u;
        }
        long_rows[lbase[r]] = (int32_t)r;
        long_ptr[lbase[r] + 1] = p;
    }
}

// Slice s = units order[64 s, 64 s + 64): its padded length (the longest = the first).
__global__ __launch_bounds__(256) void bd_slice_len_kernel(int64_t n_slices, int64_t n_units,
                                                           const int32_t *__restrict__ order,
                                                           const int32_t *__restrict__ un, int32_t *__restrict__ len,
                                                           int64_t *__restrict__ slots) {
    GS_LOOP(s, n_slices) {
        const int32_t L = 64 * s < n_units ? un[order[64 * s]] : 0;
        const int32_t pl = (L + kSellUnroll - 1) / kSellUnroll * kSellUnroll;
        len[s] = pl;
        slots[s] = (int64_t)pl * kSellLanes;
    }
}

// One wave per slice (grid-stride): lane l's row / length and its terms, column-interleaved.
template <bool CB>
__global__ __launch_bounds__(256) void bd_fill_kernel(int64_t n_slices, int64_t n_units,
                                                      const int32_t *__restrict__ order, const int32_t *__restrict__ urow,
                                                      const int32_t *__restrict__ ustart, const int32_t *__restrict__ un,
                                                      const int32_t *__restrict__ upart, const int64_t *__restrict__ off,
                                                      const int32_t *__restrict__ col, const float *__restrict__ val,
                                                      const uint8_t *__restrict__ ids, int32_t *__restrict__ row,
                                                      int32_t *__restrict__ row_len, int32_t *__restrict__ ocol,
                                                      float *__restrict__ oval) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; s < n_slices; s += waves) {
        const int64_t i = 64 * s + lane;
        if (i >= n_units) continue;   // row -1, length 0 (set by the memsets)
        const int32_t u = order[i];
        const int32_t n = un[u], a = ustart[u];
        row[i] = upart[u] >= 0 ? -2 - upart[u] : urow[u];
        row_len[i] = n;
        int32_t *c = ocol + off[s] + lane;
        for (int32_t j = 0; j < n; ++j) {
            if constexpr (CB) {
                c[(int64_t)j * kSellLanes] = (int32_t)((uint32_t)col[a + j] | (uint32_t)ids[a + j] << kSellCbColBits);
            } else {
                c[(int64_t)j * kSellLanes] = col[a + j];
                oval[off[s] + lane + (int64_t)j * kSellLanes] = val[a + j];
            }
        }
    }
}

// Merge staging (merge.cpp merge_stage_build): per merge slice b, its terms [z0, z1) keyed by
// (b, column) -- a stable sort then orders each slice's terms by column, ties in term order.
__global__ __launch_bounds__(256) void bd_mkey_kernel(int64_t nb, const int32_t *__restrict__ corner,
                                                      const int32_t *__restrict__ col,
                                                      unsigned long long *__restrict__ key, int32_t *__restrict__ idx) {
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const int32_t z0 = corner[2 * b + 1], z1 = corner[2 * b + 3];
        for (int32_t e = z0 + (int32_t)threadIdx.x; e < z1; e += (int32_t)blockDim.x) {
            key[e] = ((unsigned long long)b << 24) | (unsigned)col[e];
            idx[e] = e;
        }
    }
}

// w = column << 8 | id, z = the term's offset in its slice (its original order there).
__global__ __launch_bounds__(256) void bd_mstage_kernel(int64_t n, const unsigned long long *__restrict__ skey,
                                                        const int32_t *__restrict__ sidx,
                                                        const int32_t *__restrict__ corner,
                                                        const int32_t *__restrict__ col, const uint8_t *__restrict__ ids,
                                                        uint32_t *__restrict__ w, uint16_t *__restrict__ z) {
    GS_LOOP(i, n) {
        const int32_t e = sidx[i];
        const int64_t b = (int64_t)(skey[i] >> 24);
        w[i] = ((uint32_t)col[e] << 8) | ids[e];
        z[i] = (uint16_t)(e - corner[2 * b + 1]);
    }
}

struct Tmp {
    std::vector<void *> p;
    template <class T>
    hipError_t alloc(T **out, int64_t n) {
        *out = nullptr;
        const hipError_t e = hipMalloc((void **)out, (size_t)std::max<int64_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(*out);
        return e;
    }
    ~Tmp() {
        for (void *q : p) (void)hipFree(q);
    }
};

template <class T>
hipError_t keep_alloc(T **out, int64_t n, int64_t &acct) {
    const size_t bytes = (size_t)std::max<int64_t>(n, 1) * sizeof(T);
    const hipError_t e = hipMalloc((void **)out, bytes);
    if (e == hipSuccess) acct += (int64_t)bytes;
    return e;
}

#define BD_TRY(x)                  \
    do {                           \
        const hipError_t e_ = (x); \
        if (e_ != hipSuccess) {    \
            err = e_;              \
            return -5;             \
        }                          \
    } while (0)

template <class K, class V>
hipError_t sort_pairs(Tmp &t, const K *k, K *ks, const V *v, V *vs, int64_t n, int end_bit, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k, ks, v, vs, (int)n, 0, end_bit, s);
    if (e != hipSuccess) return e;
    uint8_t *tmp = nullptr;
    if ((e = t.alloc(&tmp, (int64_t)bytes)) != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k, ks, v, vs, (int)n, 0, end_bit, s);
}

template <class T, class O>
hipError_t excl_sum(Tmp &t, const T *in, O *out, int64_t n, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, s);
    if (e != hipSuccess) return e;
    uint8_t *tmp = nullptr;
    if ((e = t.alloc(&tmp, (int64_t)bytes)) != hipSuccess) return e;
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, (int)n, s);
}

int bits_for(uint32_t v) {
    int b = 1;
    while (b < 32 && (v >> b) != 0) ++b;
    return b;
}

}  // namespace

int devbuild_relabel(sm_matrix *m, bool check_skew, hipStream_t s, hipError_t &err) {
    err = hipSuccess;
    Plan &p = m->plan;
    const int64_t nc = m->n_cols, nnz = m->nnz;
    Tmp t;
    int32_t *deg = nullptr, *dmx = nullptr, *idx = nullptr, *perm = nullptr;
    uint32_t *key = nullptr, *skey = nullptr;
    unsigned long long *hot = nullptr;
    BD_TRY(t.alloc(&deg, nc));
    BD_TRY(t.alloc(&dmx, 1));
    BD_TRY(t.alloc(&hot, 1));
    BD_TRY(hipMemsetAsync(deg, 0, (size_t)nc * 4, s));
    BD_TRY(hipMemsetAsync(dmx, 0, 4, s));
    BD_TRY(hipMemsetAsync(hot, 0, 8, s));
    hipLaunchKernelGGL(bd_degree_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, nnz, m->d_col, deg);
    hipLaunchKernelGGL(bd_max_kernel, dim3(grid_of(nc)), dim3(256), 0, s, nc, deg, dmx);
    BD_TRY(hipGetLastError());
    int32_t dmax = 0;
    BD_TRY(hipMemcpyAsync(&dmax, dmx, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    BD_TRY(t.alloc(&key, nc));
    BD_TRY(t.alloc(&skey, nc));
    BD_TRY(t.alloc(&idx, nc));
    BD_TRY(t.alloc(&perm, nc));
    hipLaunchKernelGGL(bd_colkey_kernel, dim3(grid_of(nc)), dim3(256), 0, s, nc, deg, dmax, key, idx);
    BD_TRY(hipGetLastError());
    BD_TRY(sort_pairs(t, key, skey, idx, perm, nc, bits_for((uint32_t)dmax), s));
    int32_t *rank = nullptr;
    BD_TRY(keep_alloc(&p.d_perm, nc + 4, m->device_bytes));
    rank = p.d_perm;
    hipLaunchKernelGGL(bd_rank_kernel, dim3(grid_of(nc)), dim3(256), 0, s, nc, perm, skey, dmax, nc / 16, rank, hot);
    BD_TRY(hipGetLastError());
    unsigned long long hot_h = 0;
    BD_TRY(hipMemcpyAsync(&hot_h, hot, 8, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    if (check_skew && (double)hot_h < 0.4 * (double)nnz) {   // not skewed: no gain (upload_relabel)
        (void)hipFree(p.d_perm);
        m->device_bytes -= (int64_t)(nc + 4) * 4;
        p.d_perm = nullptr;
        return 0;
    }
    BD_TRY(keep_alloc(&p.d_rcol, nnz + kPadElems, m->device_bytes));
    BD_TRY(keep_alloc(&p.d_xperm, nc + 4, m->device_bytes));
    hipLaunchKernelGGL(bd_remap_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, nnz, m->d_col, rank, p.d_rcol);
    BD_TRY(hipGetLastError());
    BD_TRY(hipMemsetAsync(p.d_rcol + nnz, 0, kPadElems * sizeof(int32_t), s));
    BD_TRY(hipStreamSynchronize(s));
    p.n_relabel = nc;
    return 0;
}

int devbuild_codebook(const float *d_val, int64_t n, std::vector<float> &table, uint8_t *d_ids, hipStream_t s,
                      hipError_t &err) {
    err = hipSuccess;
    table.clear();
    if (n <= 0) return 0;
    Tmp t;
    uint32_t *bits = nullptr, *bits_s = nullptr, *hb = nullptr;
    int32_t *idx = nullptr, *idx_s = nullptr, *nh = nullptr, *hi = nullptr;
    BD_TRY(t.alloc(&bits, n));
    BD_TRY(t.alloc(&bits_s, n));
    BD_TRY(t.alloc(&idx, n));
    BD_TRY(t.alloc(&idx_s, n));
    BD_TRY(t.alloc(&nh, 1));
    BD_TRY(t.alloc(&hb, 256));
    BD_TRY(t.alloc(&hi, 256));
    hipLaunchKernelGGL(bd_bits_kernel, dim3(grid_of(n)), dim3(256), 0, s, n, d_val, bits, idx);
    BD_TRY(hipGetLastError());
    BD_TRY(sort_pairs(t, bits, bits_s, idx, idx_s, n, 32, s));
    BD_TRY(hipMemsetAsync(nh, 0, 4, s));
    hipLaunchKernelGGL(bd_heads_kernel, dim3(grid_of(n)), dim3(256), 0, s, n, bits_s, idx_s, nh, hb, hi);
    BD_TRY(hipGetLastError());
    int32_t K = 0;
    BD_TRY(hipMemcpyAsync(&K, nh, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    if (K > 255) return 1;   // codebook_ids: at most kCbDummyId = 255 ids
    std::vector<uint32_t> hbits((size_t)K);
    std::vector<int32_t> hidx((size_t)K);
    BD_TRY(hipMemcpy(hbits.data(), hb, (size_t)K * 4, hipMemcpyDeviceToHost));
    BD_TRY(hipMemcpy(hidx.data(), hi, (size_t)K * 4, hipMemcpyDeviceToHost));
    std::vector<int32_t> ord((size_t)K);
    for (int32_t i = 0; i < K; i++) ord[(size_t)i] = i;
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t c) { return hidx[(size_t)a] < hidx[(size_t)c]; });
    // ids in first-occurrence order; the search table sorted by bits
    std::vector<std::pair<uint32_t, uint8_t>> book((size_t)K);
    table.resize((size_t)K);
    for (int32_t i = 0; i < K; i++) {
        const uint32_t u = hbits[(size_t)ord[(size_t)i]];
        memcpy(&table[(size_t)i], &u, 4);
        book[(size_t)i] = {u, (uint8_t)i};
    }
    std::sort(book.begin(), book.end());
    std::vector<uint32_t> tb((size_t)K);
    std::vector<uint8_t> tid((size_t)K);
    for (int32_t i = 0; i < K; i++) tb[(size_t)i] = book[(size_t)i].first, tid[(size_t)i] = book[(size_t)i].second;
    uint32_t *d_tb = nullptr;
    uint8_t *d_tid = nullptr;
    BD_TRY(t.alloc(&d_tb, 256));
    BD_TRY(t.alloc(&d_tid, 256));
    BD_TRY(hipMemcpy(d_tb, tb.data(), (size_t)K * 4, hipMemcpyHostToDevice));
    BD_TRY(hipMemcpy(d_tid, tid.data(), (size_t)K, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(bd_ids_kernel, dim3(grid_of(n)), dim3(256), 0, s, n, d_val, d_tb, d_tid, K, d_ids);
    BD_TRY(hipGetLastError());
    BD_TRY(hipStreamSynchronize(s));
    return 0;
}

int devbuild_merge_stage(sm_matrix *m, hipStream_t s, hipError_t &err) {
    err = hipSuccess;
    Plan &p = m->plan;
    const int64_t nnz = m->nnz;
    if (nnz <= 0 || m->n_cols > (1 << 24) || !p.d_merge_corner) return 1;   // merge_stage_build declines
    const int32_t *col = p.n_relabel > 0 ? p.d_rcol : m->d_col;
    const int32_t *corner = reinterpret_cast<const int32_t *>(p.d_merge_corner);
    Tmp t;
    uint8_t *ids = nullptr;
    BD_TRY(t.alloc(&ids, nnz));
    std::vector<float> table;
    const int rc = devbuild_codebook(m->d_val, nnz, table, ids, s, err);
    if (rc != 0) return rc;   // > 255 distinct values: declined (as codebook_ids)
    const int64_t nb = merge_blocks(m->n_rows, nnz);
    unsigned long long *key = nullptr, *skey = nullptr;
    int32_t *idx = nullptr, *sidx = nullptr;
    BD_TRY(t.alloc(&key, nnz));
    BD_TRY(t.alloc(&skey, nnz));
    BD_TRY(t.alloc(&idx, nnz));
    BD_TRY(t.alloc(&sidx, nnz));
    hipLaunchKernelGGL(bd_mkey_kernel, dim3((unsigned)std::min<int64_t>(nb, 1 << 16)), dim3(256), 0, s, nb, corner, col,
                       key, idx);
    BD_TRY(hipGetLastError());
    BD_TRY(sort_pairs(t, key, skey, idx, sidx, nnz, 24 + bits_for((uint32_t)std::max<int64_t>(nb - 1, 1)), s));
    BD_TRY(keep_alloc(&p.d_mstage_w, nnz, m->device_bytes));
    BD_TRY(keep_alloc(&p.d_mstage_z, nnz, m->device_bytes));
    BD_TRY(keep_alloc(&p.d_mstage_tab, 256, m->device_bytes));
    table.resize(256, 0.0f);
    BD_TRY(hipMemcpy(p.d_mstage_tab, table.data(), 256 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(bd_mstage_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, nnz, skey, sidx, corner, col, ids,
                       p.d_mstage_w, p.d_mstage_z);
    BD_TRY(hipGetLastError());
    BD_TRY(hipStreamSynchronize(s));
    return 0;
}

int devbuild_sell(sm_matrix *m, int32_t max_len, bool codebook, hipStream_t s, hipError_t &err) {
    err = hipSuccess;
    Plan &p = m->plan;
    const int64_t nr = m->n_rows, nnz = m->nnz;
    const int32_t *col = p.n_relabel > 0 ? p.d_rcol : m->d_col;
    Tmp t;
    // codebook ids (sell_upload: columns < 2^24 and <= 255 distinct patterns)
    std::vector<float> table;
    uint8_t *ids = nullptr;
    bool cb = codebook && m->n_cols <= ((int64_t)1 << kSellCbColBits);
    if (cb) {
        BD_TRY(t.alloc(&ids, nnz));
        const int rc = devbuild_codebook(m->d_val, nnz, table, ids, s, err);
        if (rc < 0) return rc;
        cb = rc == 0;
    }
    // units
    int32_t *nu = nullptr, *np = nullptr, *lf = nullptr, *ubase = nullptr, *pbase = nullptr, *lbase = nullptr;
    BD_TRY(t.alloc(&nu, nr + 1));
    BD_TRY(t.alloc(&np, nr + 1));
    BD_TRY(t.alloc(&lf, nr + 1));
    BD_TRY(t.alloc(&ubase, nr + 1));
    BD_TRY(t.alloc(&pbase, nr + 1));
    BD_TRY(t.alloc(&lbase, nr + 1));
    BD_TRY(hipMemsetAsync(nu + nr, 0, 4, s));
    BD_TRY(hipMemsetAsync(np + nr, 0, 4, s));
    BD_TRY(hipMemsetAsync(lf + nr, 0, 4, s));
    hipLaunchKernelGGL(bd_units_count_kernel, dim3(grid_of(nr)), dim3(256), 0, s, nr, m->d_row_ptr, max_len, nu, np, lf);
    BD_TRY(hipGetLastError());
    BD_TRY(excl_sum(t, nu, ubase, nr + 1, s));
    BD_TRY(excl_sum(t, np, pbase, nr + 1, s));
    BD_TRY(excl_sum(t, lf, lbase, nr + 1, s));
    int32_t tot[3] = {0, 0, 0};
    BD_TRY(hipMemcpyAsync(&tot[0], ubase + nr, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipMemcpyAsync(&tot[1], pbase + nr, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipMemcpyAsync(&tot[2], lbase + nr, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    const int64_t U = tot[0];
    const int32_t n_parts = tot[1], n_long = tot[2];
    SellDev &d = p.sell;
    d.max_len = max_len;
    d.n_long = n_long;
    BD_TRY(keep_alloc(&d.d_long_rows, n_long, m->device_bytes));
    BD_TRY(keep_alloc(&d.d_long_ptr, n_long + 1, m->device_bytes));
    BD_TRY(keep_alloc(&d.d_partials, n_parts, m->device_bytes));
    BD_TRY(hipMemsetAsync(d.d_long_ptr, 0, 4, s));
    int32_t *urow = nullptr, *ustart = nullptr, *un = nullptr, *upart = nullptr, *uidx = nullptr, *order = nullptr;
    uint32_t *ukey = nullptr, *ukey_s = nullptr;
    BD_TRY(t.alloc(&urow, U));
    BD_TRY(t.alloc(&ustart, U));
    BD_TRY(t.alloc(&un, U));
    BD_TRY(t.alloc(&upart, U));
    BD_TRY(t.alloc(&uidx, U));
    BD_TRY(t.alloc(&order, U));
    BD_TRY(t.alloc(&ukey, U));
    BD_TRY(t.alloc(&ukey_s, U));
    hipLaunchKernelGGL(bd_units_emit_kernel, dim3(grid_of(nr)), dim3(256), 0, s, nr, m->d_row_ptr, max_len, ubase,
                       pbase, lbase, urow, ustart, un, upart, ukey, uidx, d.d_long_rows, d.d_long_ptr);
    BD_TRY(hipGetLastError());
    BD_TRY(sort_pairs(t, ukey, ukey_s, uidx, order, U, bits_for((uint32_t)max_len), s));
    // slices
    const int64_t ns = (U + kSellLanes - 1) / kSellLanes;
    int64_t *slots = nullptr;
    BD_TRY(t.alloc(&slots, ns + 1));
    BD_TRY(keep_alloc(&d.d_off, ns, m->device_bytes));
    BD_TRY(keep_alloc(&d.d_len, ns, m->device_bytes));
    BD_TRY(hipMemsetAsync(slots + ns, 0, 8, s));
    hipLaunchKernelGGL(bd_slice_len_kernel, dim3(grid_of(ns)), dim3(256), 0, s, ns, U, order, un, d.d_len, slots);
    BD_TRY(hipGetLastError());
    int64_t *offs = nullptr;
    BD_TRY(t.alloc(&offs, ns + 1));
    BD_TRY(excl_sum(t, slots, offs, ns + 1, s));
    int64_t padded = 0;
    BD_TRY(hipMemcpyAsync(&padded, offs + ns, 8, hipMemcpyDeviceToHost, s));
    BD_TRY(hipMemcpyAsync(d.d_off, offs, (size_t)ns * 8, hipMemcpyDeviceToDevice, s));
    BD_TRY(hipStreamSynchronize(s));
    if (ns == 0 || padded >= ((int64_t)1 << 31) - kSellLanes * kSellUnroll) {   // upload_sell declines
        (void)hipFree(d.d_long_rows), (void)hipFree(d.d_long_ptr), (void)hipFree(d.d_partials);
        (void)hipFree(d.d_off), (void)hipFree(d.d_len);
        d = SellDev();
        return 0;
    }
    BD_TRY(keep_alloc(&d.d_row, ns * kSellLanes, m->device_bytes));
    BD_TRY(keep_alloc(&d.d_row_len, ns * kSellLanes, m->device_bytes));
    BD_TRY(hipMemsetAsync(d.d_row, 0xFF, (size_t)ns * kSellLanes * 4, s));   // -1: no row
    BD_TRY(hipMemsetAsync(d.d_row_len, 0, (size_t)ns * kSellLanes * 4, s));
    const int64_t tail = 32 * kSellLanes;
    BD_TRY(keep_alloc(&d.d_col, padded + tail, m->device_bytes));
    BD_TRY(hipMemsetAsync(d.d_col, 0, (size_t)(padded + tail) * 4, s));
    if (cb) {
        BD_TRY(keep_alloc(&d.d_table, std::max<int64_t>((int64_t)table.size(), 1), m->device_bytes));
        if (!table.empty()) BD_TRY(hipMemcpy(d.d_table, table.data(), table.size() * 4, hipMemcpyHostToDevice));
        d.table_size = (int32_t)table.size();
    } else {
        BD_TRY(keep_alloc(&d.d_val, padded + tail, m->device_bytes));
        BD_TRY(hipMemsetAsync(d.d_val, 0, (size_t)(padded + tail) * 4, s));
    }
    const unsigned gf = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ns + 3) / 4, 1 << 16));
    if (cb)
        hipLaunchKernelGGL(bd_fill_kernel<true>, dim3(gf), dim3(256), 0, s, ns, U, order, urow, ustart, un, upart,
                           d.d_off, col, m->d_val, ids, d.d_row, d.d_row_len, d.d_col, d.d_val);
    else
        hipLaunchKernelGGL(bd_fill_kernel<false>, dim3(gf), dim3(256), 0, s, ns, U, order, urow, ustart, un, upart,
                           d.d_off, col, m->d_val, ids, d.d_row, d.d_row_len, d.d_col, d.d_val);
    BD_TRY(hipGetLastError());
    BD_TRY(hipStreamSynchronize(s));
    d.n_slices = ns;
    return 0;
}

}  // namespace smamd
