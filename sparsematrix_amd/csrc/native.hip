// native.hip -- AddMatMat straight from the reference's own storage format on the
// device (kernel.cc:771-800, sparse-matrix.cc:139-194): the
// uint8 delta positions and uint8 codebook ids of every 256-column panel (2 bytes per
// entry, fillers included) are decoded in parallel and applied, bit-identical to the
// reference for every output.
//
// Grid: (panel, group of 64 output columns, group of R rows of A), 256 threads.  Output
// C[i][col] (col = panel col_off + 64 g + c, i = i0 + il) lives in a register of thread
// c + 64 il for the whole kernel.  The workgroup walks its panel's stream in batches of
// 4096 entries (16 per thread: one 16-byte load of deltas, one of ids; the next batch's
// loads fly while this one is processed):
//   1. decode  each thread sums its 16 deltas; a wave prefix scan, the wave totals and
//              the carry of earlier batches give every entry its in-panel offset
//              (kernel.cc:780-782): row = off >> 8, column = off & 255.  m = 1: the x
//              value of every live entry is loaded now, so its latency hides behind 2-3;
//   2. mark    live entries (id < T, kernel.cc:782; column in the group) set bit
//              (row - row of the carry) in their column's bitmap -- a batch spans at most
//              4082 rows (deltas <= 255), 128 words per column;
//   3. rank    4 threads per column prefix-sum the popcounts of a quarter of its words
//              each; one wave turns the quarter totals into list bases (a scan over the
//              64 columns); an entry's slot is its column's base + the popcount of the
//              bits below its own = its rank by row, so every list is in stream order;
//   4. apply   thread (c, il) adds a[i][row] * fl(table[id] * alpha) over column c's
//              list in order, separate roundings (kernel.cc:791, 568-582): m = 1 from the
//              x values placed in LDS, m > 1 loading 8 entries' A values at a time.
// Across batches a column's rows keep ascending, so each output receives its terms in
// exactly the reference's order after beta (kernel.cc:10-29, sparse-matrix.cc:149-151).
#include "sm_internal.h"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace smamd {
namespace {

constexpr int kNatThreads = 256;
constexpr int kNatPer = 16;                          // entries per thread per batch
constexpr int kNatBatch = kNatThreads * kNatPer;     // 4096
constexpr int kNatCols = 64;                         // output columns per workgroup
constexpr int kNs1MaxBatches = 4;                    // native_spmv_kernel: panels up to this long (r4: 1.2x faster on config 1, 1.1x slower at 9 batches)
constexpr int kNatWords = 128;                       // bitmap words per column (4096 rows)
constexpr int kNatStride = kNatWords + 4;            // word w of column c at c*132 + w + w/32:
                                                     // the 4 quarter readers of one column,
                                                     // and adjacent columns, on distinct banks
__device__ __forceinline__ int32_t bit_index(int32_t c, int32_t w) { return c * kNatStride + w + (w >> 5); }

__device__ __forceinline__ int32_t wave_incl_scan(int32_t v, int lane) {
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const int32_t u = __shfl_up(v, s, 64);
        if (lane >= s) v += u;
    }
    return v;
}

// PROF (development builds, SM_NAT_PROF): thread 0 of every workgroup adds the cycles
// (s_memtime) of each phase into prof[0..7].
// RT: rows of A per thread (rows i0 + il + 4 j, j < RT); X1: m = 1, the x values are
// loaded at decode and placed in the lists (only the first wave applies).
template <int RT, bool X1, bool PROF>
__global__ __launch_bounds__(kNatThreads) void native_addmatmat_kernel(
    const uint8_t *__restrict__ pos, const uint8_t *__restrict__ val,
    const int64_t *__restrict__ pbeg, const int64_t *__restrict__ pend,
    const int32_t *__restrict__ pcol, const float *__restrict__ table, int32_t T, int32_t n,
    int32_t m, const float *__restrict__ a, int32_t lda, float *__restrict__ c, int32_t ldc,
    float alpha, float beta, unsigned long long *__restrict__ prof) {
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tk = PROF ? clock64() : 0;
    auto mark_phase = [&](int k) {
        if constexpr (PROF) {
            const unsigned long long now = clock64();
            ph[k] += now - tk;
            tk = now;
        }
    };
    constexpr int kDummyWord = kNatCols * kNatStride;   // dead entries OR 0 into it
    __shared__ float tab[256];
    __shared__ uint32_t bits[kNatCols * kNatStride + 1];
    __shared__ uint16_t wbase[kNatCols * kNatStride + 1];
    __shared__ int32_t qbase[kNatCols * 4];          // quarter counts, then list bases
    __shared__ int32_t cend[kNatCols];
    __shared__ int32_t wsum[kNatThreads / 64];
    __shared__ uint32_t lent[kNatBatch + 1];         // X1: x value bits; else the row
    __shared__ uint8_t lid[kNatBatch + 4];           // (+1: the dead entries' slot)
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int32_t p = blockIdx.x, g = blockIdx.y;
    const int32_t i0 = blockIdx.z * 4 * RT;
    const int cl = t & (kNatCols - 1), il = t >> 6;  // apply role: column, first row of A
    const int qc = t >> 2, qq = t & 3;               // rank role: column, quarter of its words
    const int32_t col = pcol[p] + g * kNatCols + cl;
    const bool own = col < n && (!X1 || il == 0);
    tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
    for (int w = t; w <= kDummyWord; w += kNatThreads) bits[w] = 0u;
    float acc[RT];
#pragma unroll
    for (int j = 0; j < RT; ++j) {
        const int32_t i = i0 + il + 4 * j;
        acc[j] = 0.0f;
        if (own && i < m) {
            acc[j] = c[(int64_t)i * ldc + col];
            if (beta != 1.0f) acc[j] = __fmul_rn(acc[j], beta);
        }
    }
    const int64_t e_beg = pbeg[p], e_end = pend[p];
    auto load = [&](int64_t e0, uint4 &dv, uint4 &iv) {
        const int64_t e = e0 + (int64_t)t * kNatPer;
        if (e + kNatPer <= e_end) {   // panel runs start 16-byte aligned (upload_native)
            dv = *reinterpret_cast<const uint4 *>(pos + e);
            iv = *reinterpret_cast<const uint4 *>(val + e);
        } else {
            uint8_t d[kNatPer], id[kNatPer];
#pragma unroll
            for (int k = 0; k < kNatPer; ++k) {
                const bool in = e + k < e_end;
                d[k] = in ? pos[e + k] : 0;
                id[k] = in ? val[e + k] : 255;   // >= T: skipped
            }
            __builtin_memcpy(&dv, d, 16);
            __builtin_memcpy(&iv, id, 16);
        }
    };
    uint4 dv_n = {0, 0, 0, 0}, iv_n = {0, 0, 0, 0};
    if (e_beg < e_end) load(e_beg, dv_n, iv_n);
    int32_t carry = 0;
    __syncthreads();
    mark_phase(0);
    for (int64_t e0 = e_beg; e0 < e_end; e0 += kNatBatch) {
        uint8_t d[kNatPer], id[kNatPer];
        __builtin_memcpy(d, &dv_n, 16);
        __builtin_memcpy(id, &iv_n, 16);
        if (e0 + kNatBatch < e_end) load(e0 + kNatBatch, dv_n, iv_n);   // next batch in flight
        // 1. decode
        int32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) tot += d[k];
        const int32_t incl = wave_incl_scan(tot, lane);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        mark_phase(1);
        int32_t off = carry + incl - tot;
        int32_t batch_total = 0;
#pragma unroll
        for (int w = 0; w < kNatThreads / 64; ++w) {
            if (w < wave) off += wsum[w];
            batch_total += wsum[w];
        }
        const int32_t row_lo = carry >> 8;
        carry += batch_total;
        const int32_t span_words = (((carry >> 8) - row_lo) >> 5) + 1;   // <= 128
        // 2. mark (branch-free: dead entries OR 0 into the dummy word); rr = column << 16
        // | row - row_lo, or -1 for a dead entry
        int32_t rr[kNatPer];
        float xv[kNatPer];
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            off += d[k];
            const int32_t pc = off & 255, r = (off >> 8) - row_lo;
            const bool live = id[k] < T && (pc >> 6) == g;
            if constexpr (X1) {   // m = 1: row 0 of A, live entries only
                xv[k] = 0.0f;
                if (live) xv[k] = a[off >> 8];
            }
            // Dead lanes (fillers, other column groups: most of a sparse panel's entries) issue
            // no atomic: an OR of 0 into one dummy word from every dead lane serialised them on
            // one address (r05 PMC: 70 % of the LDS cycles were address/bank conflicts).
            if (live) atomicOr(&bits[bit_index(pc & 63, r >> 5)], 1u << (r & 31));
            rr[k] = live ? ((pc & 63) << 16) | r : -1;
        }
        __syncthreads();
        mark_phase(2);
        // 3. rank: quarter-local word prefix sums (thread (qc, qq): words 32 qq .. 32 qq + 31)
        {
            int32_t cnt = 0;
            const int32_t w_hi = min(32 * qq + 32, span_words);
            for (int32_t w0 = 32 * qq; w0 < w_hi; w0 += 8) {
                uint32_t b[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) b[j] = w0 + j < w_hi ? bits[bit_index(qc, w0 + j)] : 0u;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (w0 + j < w_hi) wbase[bit_index(qc, w0 + j)] = (uint16_t)cnt;
                    cnt += __popc(b[j]);
                }
            }
            qbase[t] = cnt;   // t = 4 qc + qq
        }
        __syncthreads();
        mark_phase(3);
        if (wave == 0) {   // lane = column: quarter bases, then a scan over the columns
            int32_t q4[4], ctot = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                q4[q] = qbase[4 * lane + q];
                ctot += q4[q];
            }
            int32_t b = wave_incl_scan(ctot, lane) - ctot;
            cend[lane] = b + ctot;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                qbase[4 * lane + q] = b;
                b += q4[q];
            }
        }
        __syncthreads();
        mark_phase(4);
        // place (branch-free: dead entries write the spare slot)
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            const bool live = rr[k] >= 0;
            const int32_t q = live ? rr[k] >> 16 : 0, r = live ? rr[k] & 0xFFFF : 0;
            const int32_t bi = live ? bit_index(q, r >> 5) : kDummyWord;
            const int32_t rank = qbase[4 * q + (r >> 10)] + wbase[bi] +
                                 __popc(bits[bi] & ((1u << (r & 31)) - 1u));
            const int32_t slot = live ? rank : kNatBatch;
            lent[slot] = X1 ? __float_as_uint(xv[k]) : (uint32_t)(r + row_lo);
            lid[slot] = id[k];
        }
        __syncthreads();
        mark_phase(5);
        // 4. apply, in ascending row, 8 entries' reads ahead of their additions; the
        // quarter readers clear their words meanwhile
        if (X1 && own) {   // x values already in the list
            const int32_t s0 = qbase[4 * cl], s1 = cend[cl];
            for (int32_t s = s0; s < s1; ++s)
                acc[0] = __fadd_rn(acc[0], __fmul_rn(__uint_as_float(lent[s]), tab[lid[s]]));
        } else if (own) {
            const int32_t s0 = qbase[4 * cl], s1 = cend[cl];
            for (int32_t s = s0; s < s1; s += 8) {
                float tv[8], av[8][RT];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int32_t sj = s + j < s1 ? s + j : kNatBatch;
                    const uint32_t e = lent[sj];
                    tv[j] = tab[lid[sj]];
#pragma unroll
                    for (int q = 0; q < RT; ++q) {
                        const int32_t i = i0 + il + 4 * q;
                        if constexpr (X1) av[j][q] = __uint_as_float(e);
                        else av[j][q] = s + j < s1 && i < m ? a[(int64_t)i * lda + e] : 0.0f;
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool in = s + j < s1;
#pragma unroll
                    for (int q = 0; q < RT; ++q) {
                        const float sum = __fadd_rn(acc[q], __fmul_rn(av[j][q], tv[j]));
                        acc[q] = in ? sum : acc[q];
                    }
                }
            }
        }
        {
            const int32_t w_hi = min(32 * qq + 32, span_words);
            for (int32_t w = 32 * qq; w < w_hi; ++w) bits[bit_index(qc, w)] = 0u;
        }
        __syncthreads();
        mark_phase(6);
    }
#pragma unroll
    for (int j = 0; j < RT; ++j) {
        const int32_t i = i0 + il + 4 * j;
        if (own && i < m) c[(int64_t)i * ldc + col] = acc[j];
    }
    if constexpr (PROF) {
        if (t == 0) {
            ph[7] = 1;
            for (int k = 0; k < 8; ++k) atomicAdd(prof + k, ph[k]);
        }
    }
}

// ---- two-kernel form (panels of more than kNatFusedBatches batches) --------------------
// The fused kernel walks a panel's batches one after the other, so a long panel is one
// workgroup's serial chain.  Here every (batch, column group) decodes at once -- its carry
// (the offset before the batch) comes from the upload -- and writes each column's list,
// in stream order, to d_lists; then one thread per output walks its column's lists batch
// after batch.  m = 1: the list holds the term fl(x[row] * fl(table[id] * alpha))
// itself (the same two roundings, kernel.cc:791 / 580-582); m > 1: row | id << 23.
template <bool X1, bool PROF = false>
__global__ __launch_bounds__(kNatThreads) void native_decode_kernel(
    const uint8_t *__restrict__ pos, const uint8_t *__restrict__ val,
    const NatBatch *__restrict__ bmeta, const int32_t *__restrict__ boff,
    const float *__restrict__ table, int32_t T, const float *__restrict__ x, float alpha,
    uint32_t *__restrict__ lists, uint32_t *__restrict__ hdr, unsigned long long *__restrict__ prof = nullptr) {
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tk = PROF ? clock64() : 0;
    auto mark_phase = [&](int k) {
        if constexpr (PROF) {
            const unsigned long long now = clock64();
            ph[k] += now - tk;
            tk = now;
        }
    };
    constexpr int kDummyWord = kNatCols * kNatStride;
    __shared__ float tab[256];
    __shared__ uint32_t bits[kNatCols * kNatStride + 1];
    __shared__ uint16_t wbase[kNatCols * kNatStride + 1];
    __shared__ int32_t qbase[kNatCols * 4];
    __shared__ int32_t wsum[kNatThreads / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int qc = t >> 2, qq = t & 3;
    const int32_t b = blockIdx.x, g = blockIdx.y;
    const NatBatch bm = bmeta[b];
    const int64_t e0 = bm.start, e_end = bm.start + bm.len;
    const int32_t list_off = boff[b * 4 + g];
    if (X1) tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
    for (int w = t; w <= kDummyWord; w += kNatThreads) bits[w] = 0u;
    uint8_t d[kNatPer], id[kNatPer];
    {
        const int64_t e = e0 + (int64_t)t * kNatPer;
        if (e + kNatPer <= e_end) {   // 16-byte aligned (upload_native)
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
    }
    const int32_t carry = bm.carry;
    mark_phase(0);
    int32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kNatPer; ++k) tot += d[k];
    const int32_t incl = wave_incl_scan(tot, lane);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    mark_phase(1);
    int32_t off = carry + incl - tot, batch_total = 0;
#pragma unroll
    for (int w = 0; w < kNatThreads / 64; ++w) {
        if (w < wave) off += wsum[w];
        batch_total += wsum[w];
    }
    const int32_t row_lo = carry >> 8;
    const int32_t span_words = ((((carry + batch_total) >> 8) - row_lo) >> 5) + 1;   // <= 128
    int32_t rr[kNatPer];
    float xv[kNatPer];
#pragma unroll
    for (int k = 0; k < kNatPer; ++k) {
        off += d[k];
        const int32_t pc = off & 255, r = (off >> 8) - row_lo;
        const bool live = id[k] < T && (pc >> 6) == g;
        if constexpr (X1) {
            xv[k] = 0.0f;
            if (live) xv[k] = x[off >> 8];
        }
        if (live) atomicOr(&bits[bit_index(pc & 63, r >> 5)], 1u << (r & 31));   // dead lanes: none (above)
        rr[k] = live ? ((pc & 63) << 16) | r : -1;
    }
    __syncthreads();
    mark_phase(2);
    {
        int32_t cnt = 0;
        const int32_t w_hi = min(32 * qq + 32, span_words);
        for (int32_t w0 = 32 * qq; w0 < w_hi; w0 += 8) {
            uint32_t bw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) bw[j] = w0 + j < w_hi ? bits[bit_index(qc, w0 + j)] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (w0 + j < w_hi) wbase[bit_index(qc, w0 + j)] = (uint16_t)cnt;
                cnt += __popc(bw[j]);
            }
        }
        qbase[t] = cnt;
    }
    __syncthreads();
    mark_phase(3);
    if (wave == 0) {   // lane = column: quarter bases, the column scan, the list header
        int32_t q4[4], ctot = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            q4[q] = qbase[4 * lane + q];
            ctot += q4[q];
        }
        const int32_t cincl = wave_incl_scan(ctot, lane);
        int32_t cb = cincl - ctot;
        hdr[((int64_t)b * 4 + g) * kNatCols + lane] = (uint32_t)cb | ((uint32_t)cincl << 16);
        if (lane == 63) wsum[0] = cincl;   // the group's live entries
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            qbase[4 * lane + q] = cb;
            cb += q4[q];
        }
    }
    __syncthreads();
    mark_phase(4);
    // Slots and values in registers, then staged in LDS over the bitmap (no longer read)
    // and written out with coalesced stores.
    int32_t slot[kNatPer];
    uint32_t v[kNatPer];
#pragma unroll
    for (int k = 0; k < kNatPer; ++k) {
        const bool live = rr[k] >= 0;
        const int32_t q = live ? rr[k] >> 16 : 0, r = live ? rr[k] & 0xFFFF : 0;
        const int32_t bi = live ? bit_index(q, r >> 5) : kDummyWord;
        slot[k] = live ? qbase[4 * q + (r >> 10)] + wbase[bi] + __popc(bits[bi] & ((1u << (r & 31)) - 1u)) : -1;
        v[k] = X1 ? __float_as_uint(__fmul_rn(xv[k], tab[id[k]])) : (uint32_t)(r + row_lo) | ((uint32_t)id[k] << 23);
    }
    const int32_t n_live = wsum[0];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kNatPer; ++k)
        if (slot[k] >= 0) bits[slot[k]] = v[k];
    __syncthreads();
    uint32_t *out = lists + list_off;
    for (int32_t i = t; i < n_live; i += kNatThreads) out[i] = bits[i];
    if constexpr (PROF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        mark_phase(5);
        if (t == 0) {
            ph[7] = 1;
            for (int k = 0; k < 8; ++k) atomicAdd(prof + k, ph[k]);
        }
    }
}

// TS (development builds, SM_NAT_TS): thread 0 stamps s_memrealtime (100 MHz) at the start,
// after the stream load, after the rank steps and at the end into ts[4 * workgroup + k].
[[maybe_unused]] __device__ __forceinline__ unsigned long long nat_rt() {
    unsigned long long v;
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(v));
    return v;
}

// The same lists by a stable counting sort, one 1024-thread workgroup per batch for all four
// column groups (round 6; the default).  The bitmap kernel above decodes every batch four times
// (once per group) and its 53 KB of LDS allow ~2 workgroups per CU.  A per-(batch, group)
// counting sort with 22 KB (one generation, all workgroups resident from the start) still took
// 10.7 us per workgroup by per-workgroup stamps (SM_NAT_TS): VALU issue -- ≈ 2000 instructions
// per wave, 5 waves per SIMD, 4 cycles per wave64 instruction -- not latency, bounded it.  Here
// each entry is decoded and ranked once:
//   decode   thread t: entries 4 t .. 4 t + 3 (one 4-byte load each of deltas and ids), a wave
//            scan and the 16 wave totals give the offsets; word (row | id << 23) and column
//            (0x100: dead) to LDS in stream order;
//   rank     wave w: entries 256 w .. 256 w + 255, 64 consecutive per step, eight ballots of
//            the column bits, a per-wave running count per column (as above);
//   offsets  waves 0-3 take columns 64 g .. 64 g + 63 (group g): each column's 16 wave counts,
//            a wave scan (the group's header) and the group totals;
//   place    staged in LDS and stored coalesced: the batch's groups are contiguous in the
//            lists (upload_native: boff[4 b + g] = boff[4 b] + the live entries of groups < g).
template <bool X1, bool TS = false>
__global__ __launch_bounds__(1024) void native_decode_batch_kernel(
    const uint8_t *__restrict__ pos, const uint8_t *__restrict__ val,
    const NatBatch *__restrict__ bmeta, const int32_t *__restrict__ boff,
    const float *__restrict__ table, int32_t T, const float *__restrict__ x, float alpha,
    uint32_t *__restrict__ lists, uint32_t *__restrict__ hdr, unsigned long long *__restrict__ ts = nullptr) {
    constexpr int kThr = 1024, kWaves = kThr / 64, kPer = kNatBatch / kThr;   // 4 entries per thread
    static_assert(kPer == 4, "one 4-byte load of deltas and ids per thread");
    __shared__ float tab[X1 ? 256 : 1];
    __shared__ uint32_t lw[kNatBatch];               // row | id << 23, then the staged values
    __shared__ uint16_t lc[kNatBatch];               // column, 0x100: dead
    __shared__ int32_t wcnt[kWaves][256];            // running counts, then run starts
    __shared__ int32_t wsum[kWaves];
    __shared__ int32_t gtot[4];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int32_t b = blockIdx.x;
    if constexpr (TS) {
        if (t == 0) ts[4 * b] = nat_rt();
    }
    const NatBatch bm = bmeta[b];
    const int64_t e0 = bm.start, e_end = bm.start + bm.len;
    const int32_t list_off = boff[b * 4];
    if (X1 && t < 256) tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
#pragma unroll
    for (int k = 0; k < kWaves * 256 / kThr; ++k) (&wcnt[0][0])[t + k * kThr] = 0;
    uint8_t d[kPer], id[kPer];
    {
        const int64_t e = e0 + (int64_t)t * kPer;
        if (e + kPer <= e_end) {   // batch starts are 16-byte aligned (upload_native)
            const uint32_t dv = *reinterpret_cast<const uint32_t *>(pos + e);
            const uint32_t iv = *reinterpret_cast<const uint32_t *>(val + e);
            __builtin_memcpy(d, &dv, 4);
            __builtin_memcpy(id, &iv, 4);
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const bool in = e + k < e_end;
                d[k] = in ? pos[e + k] : 0;
                id[k] = in ? val[e + k] : 255;
            }
        }
    }
    const int32_t tot = (int32_t)d[0] + d[1] + d[2] + d[3];
    if constexpr (TS) {
        if (t == 0) ts[4 * b + 1] = nat_rt() + (unsigned long long)(tot & 0);
    }
    const int32_t incl = wave_incl_scan(tot, lane);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int32_t off = bm.carry + incl - tot;
#pragma unroll
    for (int w = 0; w < kWaves; ++w)
        if (w < wave) off += wsum[w];
    {
        uint32_t wv[kPer];
        uint16_t cv[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            off += d[k];
            wv[k] = (uint32_t)(off >> 8) | ((uint32_t)id[k] << 23);
            cv[k] = id[k] < T ? (uint16_t)(off & 255) : (uint16_t)0x100;
        }
        *reinterpret_cast<uint4 *>(lw + t * kPer) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        uint2 c2;
        __builtin_memcpy(&c2, cv, 8);
        *reinterpret_cast<uint2 *>(lc + t * kPer) = c2;
    }
    __syncthreads();
    uint32_t rc[kPer];   // live: column << 24 | id << 16 | rank in the wave's run; dead: ~0
    uint32_t wr[kPer];   // X1: x bits; else the word
#pragma unroll
    for (int s = 0; s < kPer; ++s) {
        const int e = 256 * wave + 64 * s + lane;
        const int32_t c = lc[e];
        const uint32_t w = lw[e];
        const bool live = c < 256;
        if constexpr (X1) wr[s] = live ? __float_as_uint(x[w & 0x7FFFFFu]) : 0u;
        else wr[s] = w;
        uint64_t same = __ballot(live);
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            const uint64_t mb = __ballot((c >> bb) & 1);
            same &= ((c >> bb) & 1) ? mb : ~mb;
        }
        const int32_t cl = c & 255;
        const int32_t base = wcnt[wave][cl];
        const uint32_t rank = (uint32_t)base + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        rc[s] = live ? ((uint32_t)cl << 24) | ((w >> 23) << 16) | rank : ~0u;
        if (live && (same >> lane) == 1ull) wcnt[wave][cl] = base + (int32_t)__popcll(same);
    }
    __syncthreads();
    if constexpr (TS) {
        if (t == 0) ts[4 * b + 2] = nat_rt();
    }
    int32_t cn[kWaves], ctot = 0, cincl = 0;
    if (wave < 4) {   // column 64 wave + lane of group `wave`
        const int c = t;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            cn[w] = wcnt[w][c];
            ctot += cn[w];
        }
        cincl = wave_incl_scan(ctot, lane);
        hdr[((int64_t)b * 4 + wave) * kNatCols + lane] = (uint32_t)(cincl - ctot) | ((uint32_t)cincl << 16);
        if (lane == 63) gtot[wave] = cincl;
    }
    __syncthreads();
    const int32_t n_live = gtot[0] + gtot[1] + gtot[2] + gtot[3];
    if (wave < 4) {
        int32_t cb = cincl - ctot;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            if (g < wave) cb += gtot[g];
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            wcnt[w][t] = cb;
            cb += cn[w];
        }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kPer; ++s) {
        if (rc[s] == ~0u) continue;
        const int32_t cl = (int32_t)(rc[s] >> 24), idv = (int32_t)((rc[s] >> 16) & 255), rank = (int32_t)(rc[s] & 0xFFFF);
        lw[wcnt[wave][cl] + rank] = X1 ? __float_as_uint(__fmul_rn(__uint_as_float(wr[s]), tab[idv])) : wr[s];
    }
    __syncthreads();
    uint32_t *out = lists + list_off;
    for (int32_t i = t; i < n_live; i += kThr) out[i] = lw[i];
    if constexpr (TS) {
        __syncthreads();
        if (t == 0) ts[4 * b + 3] = nat_rt();
    }
}

// One thread per (column, RT rows of A); X1: one wave per (panel, group), the terms added.
template <int RT, bool X1>
__global__ __launch_bounds__(X1 ? 64 : kNatThreads) void native_apply_kernel(
    const int32_t *__restrict__ pcol, const int32_t *__restrict__ pbatch,
    const int32_t *__restrict__ boff, const uint32_t *__restrict__ lists,
    const uint32_t *__restrict__ hdr, const float *__restrict__ table, int32_t T, int32_t n,
    int32_t m, const float *__restrict__ a, int32_t lda, float *__restrict__ c, int32_t ldc,
    float alpha, float beta) {
    __shared__ float tab[X1 ? 1 : 256];
    const int t = threadIdx.x, cl = t & 63, il = t >> 6;
    const int32_t p = blockIdx.x, g = blockIdx.y;
    const int32_t i0 = blockIdx.z * 4 * RT;
    const int32_t col = pcol[p] + g * kNatCols + cl;
    const bool own = col < n;
    if constexpr (!X1) {
        tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
        __syncthreads();
    }
    float acc[RT];
#pragma unroll
    for (int j = 0; j < RT; ++j) {
        const int32_t i = i0 + il + 4 * j;
        acc[j] = 0.0f;
        if (own && i < m) {
            acc[j] = c[(int64_t)i * ldc + col];
            if (beta != 1.0f) acc[j] = __fmul_rn(acc[j], beta);
        }
    }
    const int32_t b0 = pbatch[p], b1 = pbatch[p + 1];
    if (own && b0 < b1) {
        uint32_t h = hdr[((int64_t)b0 * 4 + g) * kNatCols + cl];
        int32_t o = boff[b0 * 4 + g];
        for (int32_t b = b0; b < b1; ++b) {
            const int32_t s0 = o + (int32_t)(h & 0xFFFF), s1 = o + (int32_t)(h >> 16);
            if (b + 1 < b1) {   // the next batch's header, in flight meanwhile
                h = hdr[((int64_t)(b + 1) * 4 + g) * kNatCols + cl];
                o = boff[(b + 1) * 4 + g];
            }
            for (int32_t s = s0; s < s1; s += 8) {
                uint32_t e[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) e[j] = lists[s + j < s1 ? s + j : s0];
                if constexpr (X1) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float sum = __fadd_rn(acc[0], __uint_as_float(e[j]));
                        acc[0] = s + j < s1 ? sum : acc[0];
                    }
                } else {
                    float av[8][RT], tv[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int32_t row = (int32_t)(e[j] & 0x7FFFFFu);
                        tv[j] = tab[e[j] >> 23];
#pragma unroll
                        for (int q = 0; q < RT; ++q) {
                            const int32_t i = i0 + il + 4 * q;
                            av[j][q] = s + j < s1 && i < m ? a[(int64_t)i * lda + row] : 0.0f;
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const bool in = s + j < s1;
#pragma unroll
                        for (int q = 0; q < RT; ++q) {
                            const float sum = __fadd_rn(acc[q], __fmul_rn(av[j][q], tv[j]));
                            acc[q] = in ? sum : acc[q];
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < RT; ++j) {
        const int32_t i = i0 + il + 4 * j;
        if (own && i < m) c[(int64_t)i * ldc + col] = acc[j];
    }
}

// ---- m = 1: one workgroup per panel, a stable counting sort per batch ----------------
// Thread t owns output column t of the panel (its running sum lives in a register for the
// whole panel).  Per batch of 4096 entries (16 contiguous entries per thread):
//   decode   the thread's delta sum, a wave scan, the wave totals (LDS) and the carry give
//            every entry its in-panel offset (kernel.cc:780-782); live entries (id < T) load
//            x[row] -- the NEXT batch is decoded and its x gathers issued while this batch is
//            sorted and applied, so their latency hides behind it;
//   rank     each wave takes its 1024 entries in stream order, 64 at a time: eight ballots
//            of the column bits give every lane the lanes holding the same column, so its
//            rank among them and the group's count; a per-wave running count per column
//            (LDS, the wave's own row of it) adds the earlier steps -- a stable rank by
//            column without atomics;
//   offsets  thread t sums column t's four wave counts, a block scan over the columns gives
//            each (wave, column) its list start;
//   scatter  every live entry stores its term fl(x * fl(table[id] * alpha)) (kernel.cc:791)
//            at list start + rank: per column, the batch's terms in stream (= row) order;
//   apply    thread t adds column t's terms in that order (separate roundings).
// So each output receives its terms exactly in the reference's order after beta.  About
// 2-3 K cycles of LDS and ballot work per batch, against the bitmap kernel's 14-17 K.
constexpr int kNs1Waves = kNatThreads / 64;

__device__ __forceinline__ int32_t block_excl_scan256(int32_t v, int32_t *wtot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int32_t base = 0;
#pragma unroll
    for (int w = 0; w < kNs1Waves; ++w)
        if (w < wave) base += wtot[w];
    return base + incl - v;
}

__global__ __launch_bounds__(kNatThreads) void native_spmv_kernel(
    const uint8_t *__restrict__ pos, const uint8_t *__restrict__ val,
    const int64_t *__restrict__ pbeg, const int64_t *__restrict__ pend,
    const int32_t *__restrict__ pcol, const float *__restrict__ table, int32_t T, int32_t n,
    const float *__restrict__ x, float *__restrict__ y, float alpha, float beta) {
    __shared__ float tab[256];
    __shared__ uint16_t lc[kNatBatch];                 // column of entry e (0x100: dead)
    __shared__ float lt[kNatBatch];                    // its term
    __shared__ float ls[kNatBatch + 1];                // terms by column (+ the dead entries' slot)
    __shared__ int32_t wcnt[kNs1Waves][256];           // running counts, then list starts
    __shared__ int32_t wsum[2][kNs1Waves];
    __shared__ int32_t wtot[kNs1Waves];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int32_t p = blockIdx.x;
    const int32_t col = pcol[p] + t;
    const bool own = col < n;
    tab[t] = t < T ? __fmul_rn(table[t], alpha) : 0.0f;
#pragma unroll
    for (int w = 0; w < kNs1Waves; ++w) wcnt[w][t] = 0;
    float acc = 0.0f;
    if (own) {
        acc = y[col];
        if (beta != 1.0f) acc = __fmul_rn(acc, beta);
    }
    const int64_t e_beg = pbeg[p], e_end = pend[p];
    auto load = [&](int64_t e0, uint4 &dv, uint4 &iv) {
        const int64_t e = e0 + (int64_t)t * kNatPer;
        if (e + kNatPer <= e_end) {   // panel runs start 16-byte aligned (upload_native)
            dv = *reinterpret_cast<const uint4 *>(pos + e);
            iv = *reinterpret_cast<const uint4 *>(val + e);
        } else {
            uint8_t d[kNatPer], id[kNatPer];
#pragma unroll
            for (int k = 0; k < kNatPer; ++k) {
                const bool in = e + k < e_end;
                d[k] = in ? pos[e + k] : 0;
                id[k] = in ? val[e + k] : 255;   // >= T: dead
            }
            __builtin_memcpy(&dv, d, 16);
            __builtin_memcpy(&iv, id, 16);
        }
    };
    // Decode, part 1 (before a barrier): the thread's delta sum and its wave's inclusive scan.
    // Part 2 (after it): offsets, live flags and the x gathers of live entries.
    int32_t carry = 0;
    uint4 dv_c = {0, 0, 0, 0}, iv_c = {0, 0, 0, 0}, dv_n = {0, 0, 0, 0}, iv_n = {0, 0, 0, 0};
    int32_t cpos[kNatPer];      // current batch: offset (dead: -1)
    float cx[kNatPer];          // current batch: x of live entries
    uint8_t cid[kNatPer];
    auto decode1 = [&](const uint4 &dv, int buf) -> int32_t {   // returns the thread's exclusive prefix
        uint8_t d[kNatPer];
        __builtin_memcpy(d, &dv, 16);
        int32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) tot += d[k];
        const int32_t incl = wave_incl_scan(tot, lane);
        if (lane == 63) wsum[buf][wave] = incl;
        return incl - tot;
    };
    auto decode2 = [&](const uint4 &dv, const uint4 &iv, int buf, int32_t excl) {
        uint8_t d[kNatPer];
        __builtin_memcpy(d, &dv, 16);
        __builtin_memcpy(cid, &iv, 16);
        int32_t off = carry + excl, batch_total = 0;
#pragma unroll
        for (int w = 0; w < kNs1Waves; ++w) {
            if (w < wave) off += wsum[buf][w];
            batch_total += wsum[buf][w];
        }
        carry += batch_total;
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            off += d[k];
            const bool live = cid[k] < T;
            cpos[k] = live ? off : -1;
            cx[k] = live ? x[off >> 8] : 0.0f;   // gathers in flight through the sort below
        }
    };
    int64_t e0 = e_beg;
    if (e0 < e_end) load(e0, dv_c, iv_c);
    int32_t ex = decode1(dv_c, 0);
    __syncthreads();   // tab, wcnt, wsum[0]
    if (e0 < e_end) decode2(dv_c, iv_c, 0, ex);
    if (e0 + kNatBatch < e_end) load(e0 + kNatBatch, dv_n, iv_n);
    int buf = 1;
    for (; e0 < e_end; e0 += kNatBatch, buf ^= 1) {
        // The current batch's columns and terms into LDS, in batch (= stream) order.
#pragma unroll
        for (int k = 0; k < kNatPer; ++k) {
            const bool live = cpos[k] >= 0;
            lc[t * kNatPer + k] = live ? (uint16_t)(cpos[k] & 255) : (uint16_t)0x100;
            lt[t * kNatPer + k] = live ? __fmul_rn(cx[k], tab[cid[k]]) : 0.0f;
        }
        // The next batch's decode, part 1.
        const bool more = e0 + kNatBatch < e_end;
        uint4 dv_x = dv_n, iv_x = iv_n;
        ex = decode1(dv_x, buf);
        if (e0 + 2 * kNatBatch < e_end) load(e0 + 2 * kNatBatch, dv_n, iv_n);   // two ahead
        __syncthreads();
        // Rank: this wave's 1024 entries, 64 per step, in stream order.
        int32_t rk[kNatPer], cc[kNatPer];
        float tv[kNatPer];
#pragma unroll
        for (int s2 = 0; s2 < kNatPer; ++s2) {
            const int e = 1024 * wave + 64 * s2 + lane;
            const int32_t c = lc[e];
            tv[s2] = lt[e];
            const bool live = c < 256;
            uint64_t same = __ballot(live);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint64_t mb = __ballot((c >> b) & 1);
                same &= ((c >> b) & 1) ? mb : ~mb;
            }
            const uint64_t below = same & ((1ull << lane) - 1ull);
            const int32_t cl = c & 255;
            const int32_t base = wcnt[wave][cl];
            rk[s2] = base + __popcll(below);
            cc[s2] = live ? cl : -1;
            if (live && (same >> lane) == 1ull) wcnt[wave][cl] = base + __popcll(same);
        }
        __syncthreads();
        // Offsets: column t's four wave counts, a scan over the columns.
        int32_t cn[kNs1Waves], ctot = 0;
#pragma unroll
        for (int w = 0; w < kNs1Waves; ++w) {
            cn[w] = wcnt[w][t];
            ctot += cn[w];
        }
        const int32_t cbase = block_excl_scan256(ctot, wtot);   // (one barrier inside)
        {
            int32_t b = cbase;
#pragma unroll
            for (int w = 0; w < kNs1Waves; ++w) {
                wcnt[w][t] = b;
                b += cn[w];
            }
        }
        // The next batch's decode, part 2 (wsum[buf] is final): offsets and x gathers.
        if (more) decode2(dv_x, iv_x, buf, ex);
        __syncthreads();
        // Scatter (dead entries write the spare slot).
#pragma unroll
        for (int s2 = 0; s2 < kNatPer; ++s2) {
            const int32_t slot = cc[s2] >= 0 ? wcnt[wave][cc[s2]] + rk[s2] : kNatBatch;
            ls[slot] = tv[s2];
        }
        __syncthreads();
        // Apply column t's terms in order; the counts restart at zero.
        if (own) {
            int32_t s = cbase;
            const int32_t s1 = cbase + ctot;
            for (; s + 4 <= s1; s += 4) {
                const float a0 = ls[s], a1 = ls[s + 1], a2 = ls[s + 2], a3 = ls[s + 3];
                acc = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(acc, a0), a1), a2), a3);
            }
            for (; s < s1; ++s) acc = __fadd_rn(acc, ls[s]);
        }
#pragma unroll
        for (int w = 0; w < kNs1Waves; ++w) wcnt[w][t] = 0;
        __syncthreads();
    }
    if (own) y[col] = acc;
}

}  // namespace

hipError_t launch_native_addmatmat(const NativeDev &nd, int32_t m, const float *a, int32_t lda,
                                   float *c, int32_t ldc, float alpha, float beta, hipStream_t s) {
    const int32_t P = beta != 1.0f ? nd.n_all : nd.n_panels;   // empty blocks only scale
    if (P <= 0 || m <= 0) return hipSuccess;
    if (!nd.d_pos || !nd.d_val || !nd.d_beg || !nd.d_end || !nd.d_col || !nd.d_table ||
        nd.table_size < 0 || nd.table_size > 255 || nd.s_rows >= ((int64_t)1 << 23))
        return hipErrorInvalidValue;
    // m = 1 with panels of up to kNs1MaxBatches batches: one workgroup per panel, the
    // counting-sort kernel above (a longer panel is one workgroup's serial chain: the
    // two-kernel form below spreads its batches instead).
    bool ns1 = m == 1 && nd.max_panel_batches <= kNs1MaxBatches;
#ifdef SM_DEV
    if (const char *e = dev_env("SM_NAT_SORT")) ns1 = m == 1 && atoi(e) != 0;   // A/B
#endif
    if (ns1) {
        hipLaunchKernelGGL(native_spmv_kernel, dim3((unsigned)P), dim3(kNatThreads), 0, s, nd.d_pos, nd.d_val,
                           nd.d_beg, nd.d_end, nd.d_col, nd.d_table, nd.table_size, (int32_t)nd.s_cols, a, c,
                           alpha, beta);
        return hipGetLastError();
    }
    if (nd.max_panel_batches > kNatFusedBatches && nd.d_lists) {
        // Two kernels: decode every batch at once, then walk the lists.
        const int RT = m == 1 ? 1 : m <= 4 ? 1 : m <= 8 ? 2 : m <= 16 ? 4 : 8;
        if (nd.n_batches > 0) {
            const dim3 dgrid((unsigned)nd.n_batches, 256 / kNatCols);
            // One workgroup per batch (native_decode_batch_kernel); development builds keep the
            // per-(batch, group) bitmap form of rounds 3-5 for A/B (SM_NAT_DECODE=0).
            bool bitmap = false;
#ifdef SM_DEV
            if (const char *e = dev_env("SM_NAT_DECODE")) bitmap = atoi(e) == 0;
#endif
            if (!bitmap) {
                if (m == 1)
                    hipLaunchKernelGGL(native_decode_batch_kernel<true>, dim3((unsigned)nd.n_batches), dim3(1024), 0, s,
                                       nd.d_pos, nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table, nd.table_size, a,
                                       alpha, nd.d_lists, nd.d_hdr);
                else
                    hipLaunchKernelGGL(native_decode_batch_kernel<false>, dim3((unsigned)nd.n_batches), dim3(1024), 0, s,
                                       nd.d_pos, nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table, nd.table_size, a,
                                       alpha, nd.d_lists, nd.d_hdr);
            } else if (m == 1)
                hipLaunchKernelGGL(native_decode_kernel<true>, dgrid, dim3(kNatThreads), 0, s, nd.d_pos,
                                   nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table, nd.table_size, a, alpha,
                                   nd.d_lists, nd.d_hdr);
            else
                hipLaunchKernelGGL(native_decode_kernel<false>, dgrid, dim3(kNatThreads), 0, s, nd.d_pos,
                                   nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table, nd.table_size, a, alpha,
                                   nd.d_lists, nd.d_hdr);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
#ifdef SM_DEV
            if (m == 1 && !bitmap && dev_env("SM_NAT_TS")) {   // the decode again, stamped (same outputs)
                const int64_t nw = (int64_t)nd.n_batches;
                unsigned long long *d = nullptr;
                std::vector<unsigned long long> h((size_t)nw * 4);
                if (hipMalloc(&d, h.size() * 8) != hipSuccess) return hipErrorOutOfMemory;
                hipLaunchKernelGGL((native_decode_batch_kernel<true, true>), dim3((unsigned)nd.n_batches), dim3(1024), 0,
                                   s, nd.d_pos, nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table, nd.table_size, a,
                                   alpha, nd.d_lists, nd.d_hdr, d);
                (void)hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                (void)hipFree(d);
                unsigned long long t0 = ~0ull, t1 = 0;
                for (int64_t i = 0; i < nw; i++) t0 = std::min(t0, h[(size_t)(4 * i)]), t1 = std::max(t1, h[(size_t)(4 * i + 3)]);
                std::vector<double> st, life, load, rank, tail;
                for (int64_t i = 0; i < nw; i++) {
                    const unsigned long long *q = &h[(size_t)(4 * i)];
                    st.push_back((q[0] - t0) / 100.0);
                    life.push_back((q[3] - q[0]) / 100.0);
                    load.push_back((q[1] - q[0]) / 100.0);
                    rank.push_back((q[2] - q[1]) / 100.0);
                    tail.push_back((q[3] - q[2]) / 100.0);
                }
                auto pct = [](std::vector<double> v, double f) {
                    std::sort(v.begin(), v.end());
                    return v[(size_t)std::min<double>((double)v.size() - 1, f * (double)v.size())];
                };
                fprintf(stderr, "native decode ts (us, %lld wgs): span %.2f | start p50 %.2f p90 %.2f max %.2f | life p50 %.2f p90 %.2f max %.2f | "
                        "load p50 %.2f p90 %.2f | rank p50 %.2f p90 %.2f | tail p50 %.2f p90 %.2f\n", (long long)nw,
                        (t1 - t0) / 100.0, pct(st, .5), pct(st, .9), pct(st, 1), pct(life, .5), pct(life, .9), pct(life, 1),
                        pct(load, .5), pct(load, .9), pct(rank, .5), pct(rank, .9), pct(tail, .5), pct(tail, .9));
            }
            if (dev_env("SM_NAT_PROF")) {   // the decode again, profiled (same outputs)
                unsigned long long *d = nullptr, h[8] = {};
                if (hipMalloc(&d, sizeof(h)) != hipSuccess) return hipErrorOutOfMemory;
                (void)hipMemsetAsync(d, 0, sizeof(h), s);
                if (m == 1)
                    hipLaunchKernelGGL((native_decode_kernel<true, true>), dgrid, dim3(kNatThreads), 0, s,
                                       nd.d_pos, nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table,
                                       nd.table_size, a, alpha, nd.d_lists, nd.d_hdr, d);
                else
                    hipLaunchKernelGGL((native_decode_kernel<false, true>), dgrid, dim3(kNatThreads), 0, s,
                                       nd.d_pos, nd.d_val, nd.d_bmeta, nd.d_boff, nd.d_table,
                                       nd.table_size, a, alpha, nd.d_lists, nd.d_hdr, d);
                (void)hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                (void)hipFree(d);
                const double w = (double)h[7];
                fprintf(stderr, "native decode prof (kcycles per workgroup, %.0f wgs): meta+load %.2f scan %.2f "
                        "mark %.2f rank1 %.2f rank2 %.2f place+drain %.2f\n", w, h[0] / w / 1e3, h[1] / w / 1e3,
                        h[2] / w / 1e3, h[3] / w / 1e3, h[4] / w / 1e3, h[5] / w / 1e3);
            }
#endif
        }
        const dim3 agrid((unsigned)P, 256 / kNatCols, (unsigned)(m == 1 ? 1 : (m + 4 * RT - 1) / (4 * RT)));
#define SM_NAT_APPLY(RR, XX)                                                                  \
    hipLaunchKernelGGL((native_apply_kernel<RR, XX>), agrid, dim3(XX ? 64 : kNatThreads), 0, s, \
                       nd.d_col, nd.d_pbatch, nd.d_boff, nd.d_lists, nd.d_hdr, nd.d_table,    \
                       nd.table_size, (int32_t)nd.s_cols, m, a, lda, c, ldc, alpha, beta)
        if (m == 1) SM_NAT_APPLY(1, true);
        else if (RT == 1) SM_NAT_APPLY(1, false);
        else if (RT == 2) SM_NAT_APPLY(2, false);
        else if (RT == 4) SM_NAT_APPLY(4, false);
        else SM_NAT_APPLY(8, false);
#undef SM_NAT_APPLY
        return hipGetLastError();
    }
    // m = 1: x values carried in the lists; m > 1: RT rows of A per thread, 4 RT per
    // workgroup (one decode serves them all), at most 8.
    const int RT = m == 1 ? 1 : m <= 4 ? 1 : m <= 8 ? 2 : m <= 16 ? 4 : 8;
    const dim3 grid((unsigned)P, 256 / kNatCols, (unsigned)((m + 4 * RT - 1) / (4 * RT)));
#define SM_NAT(RR, XX, PP, PTR)                                                               \
    hipLaunchKernelGGL((native_addmatmat_kernel<RR, XX, PP>), grid, dim3(kNatThreads), 0, s,  \
                       nd.d_pos, nd.d_val, nd.d_beg, nd.d_end, nd.d_col, nd.d_table,          \
                       nd.table_size, (int32_t)nd.s_cols, m, a, lda, c, ldc, alpha, beta, PTR)
#define SM_NAT_ALL(PP, PTR)                                                                   \
    do {                                                                                      \
        if (m == 1) SM_NAT(1, true, PP, PTR);                                                 \
        else if (RT == 1) SM_NAT(1, false, PP, PTR);                                          \
        else if (RT == 2) SM_NAT(2, false, PP, PTR);                                          \
        else if (RT == 4) SM_NAT(4, false, PP, PTR);                                          \
        else SM_NAT(8, false, PP, PTR);                                                       \
    } while (0)
#ifdef SM_DEV
    if (dev_env("SM_NAT_PROF")) {   // per-phase cycles, summed over workgroups, to stderr
        unsigned long long *d = nullptr, h[8] = {};
        if (hipMalloc(&d, sizeof(h)) != hipSuccess) return hipErrorOutOfMemory;
        (void)hipMemsetAsync(d, 0, sizeof(h), s);
        SM_NAT_ALL(true, d);
        (void)hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipFree(d);
        const double wgs = (double)h[7];
        fprintf(stderr, "native prof (kcycles per workgroup, %.0f wgs): init %.2f scan %.2f mark %.2f "
                "rank1 %.2f rank2 %.2f place %.2f apply %.2f\n", wgs, h[0] / wgs / 1e3, h[1] / wgs / 1e3,
                h[2] / wgs / 1e3, h[3] / wgs / 1e3, h[4] / wgs / 1e3, h[5] / wgs / 1e3, h[6] / wgs / 1e3);
        return hipGetLastError();
    }
#endif
    SM_NAT_ALL(false, nullptr);
#undef SM_NAT_ALL
#undef SM_NAT
    return hipGetLastError();
}

}  // namespace smamd
