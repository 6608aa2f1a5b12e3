// kernels_merge.hip -- merge-path CSR SpMV (SM_ALGO_MERGE; north_star's "merge-path row
// balancing").
//
// The work of y = alpha * B x + beta * y is the merge of two lists: the n row ends (rp[1..n])
// and the nnz term indices 0..nnz-1.  Every workgroup takes an equal slice of kMgTile merge
// items and every thread kMgIpt of them, wherever rows start and end -- a row of 10^5 terms
// and 10^5 empty rows cost the same (Merrill & Garland's merge-based SpMV):
//   1. the slices' (row, term) corners depend only on the row pointers: the plan holds them
//      (merge_corners, binary searches on the host at creation), so a workgroup starts with
//      two loads instead of a chain of dependent ones;
//   2. it stages the slice's terms fl(x[col] * fl(v * alpha)) (coalesced col / val loads, the
//      x gathers back to back) and row ends in LDS;
//   3. each thread finds its own corner in LDS and walks its items: a term adds to the running
//      sum, a row end finishes the row.  A row whose first term the thread saw started from
//      beta*y and is written at once, in the reference's order (kernel.cc:780-796) -- bit-exact;
//   4. rows cut between threads: each thread leaves the open row's partial (a "tail") and the
//      partial of a row it finished but did not start (a "head"); a segmented scan over the
//      tails joins the cut rows inside the workgroup -- per wavefront by __shfl_up
//      (ds_bpermute; Hillis-Steele, six rounds, no barrier), then one cross-wave step that adds
//      the earlier waves' ends to the lanes whose row began before their wave -- y = (start
//      part + middle parts) + end part: within 1e-6 * sum|terms| of the reference,
//      deterministic (a fixed tree);
//   5. rows cut between workgroups leave one record per workgroup (its first row's end part,
//      its last row's open part); spmv_merge_fixup_kernel joins them from the row's start
//      workgroup (found from the row pointer): in order by one thread, or -- rows over more
//      than 64 workgroups -- by the whole wavefront in a fixed tree.
#include "sm_internal.h"
#include "xband_dev.h"

#include "merge.h"

namespace smamd {
namespace {

// Corner of merge diagonal d: the number of row ends (row) and terms (nz) before it.
// rend[i] = end of row i; a row end is taken before a term with the same index.
template <typename RendT>
__device__ __forceinline__ void merge_corner(int64_t d, RendT rend, int64_t n, int64_t nnz, int64_t &row,
                                             int64_t &nz) {
    int64_t lo = d - nnz > 0 ? d - nnz : 0, hi = d < n ? d : n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)rend(mid) <= d - mid - 1) lo = mid + 1;
        else hi = mid;
    }
    row = lo;
    nz = d - lo;
}

// STAGE: the slice's terms come from the column-sorted staging stream (MergeStage) instead of
// the CSR order -- the same terms, the same products, placed at the same LDS slots.
template <bool STAGE>
__global__ __launch_bounds__(kMgThreads) void spmv_merge_kernel(
    int32_t n, int32_t nnz, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ x, float *__restrict__ y, float alpha, float beta,
    const int2 *__restrict__ corner, MergeRec *__restrict__ rec, const uint32_t *__restrict__ sw,
    const uint16_t *__restrict__ sz, const float *__restrict__ stab) {
    __shared__ float s_term[kMgTile];
    __shared__ int32_t s_rend[kMgTile];
    __shared__ int32_t s_first;   // the workgroup's first row, when it began in an earlier one
    __shared__ float s_first_val;
    __shared__ float s_tab[STAGE ? 256 : 1];   // fl(table[id] * alpha)
    constexpr int kWaves = kMgThreads / 64;
    __shared__ int32_t t_row[kMgThreads], t_sf[kMgThreads];
    __shared__ float t_val[kMgThreads];
    __shared__ float w_val[kWaves];   // each wave's last lane after the wave scan
    __shared__ int32_t w_fs[kWaves];
    const int tid = threadIdx.x;
    const int2 c0 = corner[blockIdx.x], c1 = corner[blockIdx.x + 1];
    const int32_t r0 = c0.x, z0 = c0.y, r1 = c1.x, z1 = c1.y;
    const int32_t tile_rows = r1 - r0, tile_nnz = z1 - z0;
    // Stage: the slice's terms (every load issued before the first is used) and row ends.
    if constexpr (STAGE) {
        static_assert(kMgThreads == 256, "one scaled codebook entry per thread");
        s_tab[tid] = __fmul_rn(stab[tid], alpha);
        uint32_t w[kMgIpt];
        uint32_t zz[kMgIpt];
#pragma unroll
        for (int k = 0; k < kMgIpt; ++k) {
            const int32_t z = k * kMgThreads + tid;
            const int32_t gz = z < tile_nnz ? z0 + z : 0;   // nnz > 0 here
            w[k] = sw[gz];
            zz[k] = sz[gz];
        }
        __syncthreads();   // s_tab
#pragma unroll
        for (int k = 0; k < kMgIpt; ++k) {
            const int32_t z = k * kMgThreads + tid;
            const float xv = x[w[k] >> 8];
            if (z < tile_nnz) s_term[zz[k]] = __fmul_rn(xv, s_tab[w[k] & 255u]);
        }
    } else {
        int32_t c[kMgIpt];
        float v[kMgIpt];
#pragma unroll
        for (int k = 0; k < kMgIpt; ++k) {
            const int32_t z = k * kMgThreads + tid;
            const int32_t gz = z < tile_nnz ? z0 + z : 0;   // nnz > 0 here
            c[k] = col[gz];
            v[k] = val[gz];
        }
#pragma unroll
        for (int k = 0; k < kMgIpt; ++k) {
            const int32_t z = k * kMgThreads + tid;
            const float xv = x[c[k]];
            if (z < tile_nnz) s_term[z] = __fmul_rn(xv, __fmul_rn(v[k], alpha));
        }
    }
#pragma unroll
    for (int k = 0; k < kMgIpt; ++k) {
        const int32_t r = k * kMgThreads + tid;
        if (r < tile_rows) s_rend[r] = rp[r0 + 1 + r] - z0;
    }
    const int32_t rstart0 = rp[r0] - z0;   // the slice's first row's start (<= 0)
    __syncthreads();

    // This thread's items [dt, de) of the slice and its corner (ri, zi) in it.
    const int32_t items = tile_rows + tile_nnz;
    const int32_t dt = min(tid * kMgIpt, items), de = min(dt + kMgIpt, items);
    int64_t ri64, zi64;
    merge_corner(dt, [&](int64_t i) { return s_rend[i]; }, tile_rows, tile_nnz, ri64, zi64);
    int32_t ri = (int32_t)ri64, zi = (int32_t)zi64;
    auto y_init = [&](int32_t row) -> float {   // beta * y (multiplied iff beta != 1, kernel.cc:10-29)
        if (row >= n) return 0.0f;
        const float yv = y[row];
        return beta != 1.0f ? __fmul_rn(yv, beta) : yv;
    };
    const int32_t first_row = r0 + ri;
    bool fresh = dt < de && (ri == 0 ? rstart0 : s_rend[ri - 1]) == zi;   // the thread sees the row's start
    float acc = fresh ? y_init(first_row) : -0.0f;
    bool open = false, has_head = false;
    float head = 0.0f;
#pragma unroll
    for (int k = 0; k < kMgIpt; ++k) {
        if (dt + k < de) {
            if (ri < tile_rows && s_rend[ri] <= zi) {   // row r0 + ri ends
                if (fresh) {
                    y[r0 + ri] = acc;
                } else {   // the thread's first row, started before it
                    has_head = true;
                    head = acc;
                }
                ++ri;
                fresh = true;
                open = false;
                acc = y_init(r0 + ri);
            } else {
                acc = __fadd_rn(acc, s_term[zi]);
                ++zi;
                open = true;
            }
        }
    }
    // Tails: a segmented inclusive scan over threads (segments = runs of one cut row; a run
    // starts at a thread that saw the row's start or follows a thread without that row).
    // fs bit 0: the segment's start is at or before this lane; bit 1: that start was fresh.
    t_row[tid] = open ? r0 + ri : -1;
    __syncthreads();
    const bool seg_start = !open || tid == 0 || t_row[tid - 1] != t_row[tid] || fresh;
    float tv = open ? acc : 0.0f;
    int32_t fs = (seg_start ? 1 : 0) | (open && fresh ? 2 : 0);
    const int32_t lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {   // every lane shifts before any updates: lockstep wave
        const float pv = __shfl_up(tv, d, 64);
        const int32_t pfs = __shfl_up(fs, d, 64);
        if (lane >= d && !(fs & 1)) {
            tv = __fadd_rn(pv, tv);
            fs = pfs;
        }
    }
    if (lane == 63) {
        w_val[wid] = tv;
        w_fs[wid] = fs;
    }
    __syncthreads();
    if (wid > 0 && !(fs & 1)) {   // the segment began in an earlier wave: add those waves' parts
        float c = w_val[wid - 1];
        int32_t cfs = w_fs[wid - 1];
        for (int32_t k = wid - 2; k >= 0 && !(cfs & 1); --k) {
            c = __fadd_rn(w_val[k], c);
            cfs = w_fs[k];
        }
        tv = __fadd_rn(c, tv);
        fs = cfs;
    }
    t_val[tid] = tv;
    t_sf[tid] = (fs >> 1) & 1;
    // Heads: the thread finished a row started before it -- join it with the tails before.
    // Only the workgroup's first row can have started in an earlier workgroup; its end part
    // goes to the workgroup's record.
    if (tid == 0) s_first = -1;
    __syncthreads();
    if (has_head) {
        float tot = head;
        bool started_here = false;
        if (tid > 0 && t_row[tid - 1] == first_row) {
            tot = __fadd_rn(t_val[tid - 1], head);
            started_here = t_sf[tid - 1] != 0;
        }
        if (started_here) {
            y[first_row] = tot;
        } else {
            s_first = first_row;
            s_first_val = tot;
        }
    }
    // The workgroup's last open row (the thread holding the slice's last item).
    const int32_t t_last = items > 0 ? (items - 1) / kMgIpt : 0;
    if (tid == t_last) {
        rec[blockIdx.x].last_row = open ? r0 + ri : -1;
        rec[blockIdx.x].last_val = t_val[tid];
        rec[blockIdx.x].last_fresh = t_sf[tid];
    }
    __syncthreads();
    if (tid == 0) {
        rec[blockIdx.x].first_row = s_first;
        rec[blockIdx.x].first_val = s_first >= 0 ? s_first_val : 0.0f;
    }
}

// Rows cut between workgroups: workgroup m finished row R (first_row) that began in an earlier
// one, the workgroup j holding R's first merge item (diagonal rp[R] + R), whose record's open
// row is R; the workgroups in between lie inside R.  y[R] = (parts j .. m-1) + end part.  One
// thread per record: a row over at most kMgLongSpan workgroups (almost every cut row) is joined
// by its thread in workgroup order; a longer one by the whole wavefront -- lane l adds the
// parts j + l, j + l + 64, ... in order, then a fixed butterfly joins the lanes -- so a row of
// 10^8 terms (~5 * 10^4 workgroups) costs ~800 loads per lane instead of 5 * 10^4 in a chain.
// Which form a row takes depends on the matrix only: deterministic.
constexpr int64_t kMgLongSpan = 64;
__global__ __launch_bounds__(256) void spmv_merge_fixup_kernel(int32_t n_blocks, const int32_t *__restrict__ rp,
                                                                const MergeRec *__restrict__ rec,
                                                                float *__restrict__ y) {
    const int32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t lane = threadIdx.x & 63;
    const int32_t R = m < n_blocks ? rec[m].first_row : -1;
    const int64_t j = R >= 0 ? ((int64_t)rp[R] + R) / kMgTile : 0;
    const bool wide = R >= 0 && m - j > kMgLongSpan;
    if (R >= 0 && !wide) {
        float tot = rec[j].last_val;
        for (int64_t i = j + 1; i < m; ++i) tot = __fadd_rn(tot, rec[i].last_val);
        y[R] = __fadd_rn(tot, rec[m].first_val);
    }
    for (uint64_t pend = __ballot(wide); pend != 0; pend &= pend - 1) {   // wave-uniform
        const int src = __builtin_ctzll(pend);
        const int32_t mm = __shfl(m, src, 64), RR = __shfl(R, src, 64);
        const int64_t jj = ((int64_t)rp[RR] + RR) / kMgTile;
        float part = 0.0f;
        bool any = false;
        for (int64_t i = jj + lane; i < mm; i += 64) {
            const float v = rec[i].last_val;
            part = any ? __fadd_rn(part, v) : v;
            any = true;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {   // lane l joins lane l ^ d, the lower lane's part first
            const float o = __shfl_xor(part, d, 64);
            const bool oany = __shfl_xor((int)any, d, 64) != 0;
            if (oany) part = !any ? o : ((lane & d) ? __fadd_rn(o, part) : __fadd_rn(part, o));
            any = any || oany;
        }
        if (lane == 0) y[RR] = __fadd_rn(part, rec[mm].first_val);
    }
}

}  // namespace

hipError_t launch_spmv_merge(int32_t n, int32_t nnz, const int32_t *rp, const int32_t *col, const float *val,
                             const float *x, float *y, float alpha, float beta, const int2 *corner, MergeRec *rec,
                             hipStream_t s, const MergeStage *stage) {
    if (n <= 0) return hipSuccess;
    if (nnz == 0) return launch_beta(y, 1, n, n, beta, s);
    const int64_t nb = merge_blocks(n, nnz);
    if (nb > INT32_MAX || !rec || !corner) return hipErrorInvalidValue;
    if (stage && stage->w && stage->z && stage->table)
        hipLaunchKernelGGL(spmv_merge_kernel<true>, dim3((unsigned)nb), dim3(kMgThreads), 0, s, n, nnz, rp, col, val,
                           x, y, alpha, beta, corner, rec, stage->w, stage->z, stage->table);
    else
        hipLaunchKernelGGL(spmv_merge_kernel<false>, dim3((unsigned)nb), dim3(kMgThreads), 0, s, n, nnz, rp, col,
                           val, x, y, alpha, beta, corner, rec, nullptr, nullptr, nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(spmv_merge_fixup_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, (int32_t)nb,
                       rp, rec, y);
    return hipGetLastError();
}

}  // namespace smamd
