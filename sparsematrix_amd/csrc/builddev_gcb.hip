// builddev_gcb.hip -- the gathered chunk bands (gcb.h) built on the device from a device CSR
// (config 5's host build took 15 s).  The same bytes gcb.cpp's gcb_build
// produces -- every band's start, its 4096 words and the tile -> band offsets -- without copying
// the terms to the host and back.
//
//   keys    per term: key = block << cbits | column (a block's columns ascending = its slabs in
//           order, so the key order is the tile order), the row in the block, and the check that
//           every row's columns strictly ascend (gcb_build declines otherwise);
//   sort    a stable radix sort of (key, term) -- terms of one column stay in row order, so the
//           sorted sequence is gcb.cpp's per-tile (column, row) order;
//   cut     one workgroup per tile runs gcb.cpp's greedy: the longest next run within the window
//           and the capacity, shrunk by 31/32 until its by-row segments pack into 32 chunks.  A
//           band's terms are ordered by (row, position) with a bitonic sort in LDS (position
//           order = column order inside a row, gcb.cpp's stable sort by row), the segments come
//           from two block scans, and one wave replays the sequential packing with the segment
//           list in its lanes (s_ registers hold the packing state);
//   emit    after a scan of the band counts, one workgroup per band repeats the sort and the
//           packing of its (now known) run and writes the band's image -- headers, words,
//           values, zero padding -- from LDS in one coalesced pass.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "gcb.h"
#include "sm_internal.h"

namespace smamd {
namespace {

constexpr int kCutThreads = 1024;
constexpr int kCap = kGcbChunks * kGcbChunkTerms;   // 2016 terms per band at most
constexpr int kSortN = 2048;                         // bitonic width (>= kCap)
constexpr int kPosBits = 11;
constexpr uint32_t kPad = 0xFFFFFFFFu;
static_assert(kCap <= kSortN && kSortN == 2 * kCutThreads, "one compare per thread per stage");

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 16)); }

#define GS_LOOP(i, n) for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// One thread per row: keys, rows in block, term indices; flag 1 = a row's columns not strictly
// ascending.
__global__ __launch_bounds__(256) void gk_keys_kernel(int64_t n_rows, const int32_t *__restrict__ rp,
                                                      const int32_t *__restrict__ col, int rows_log2, int cbits,
                                                      unsigned long long *__restrict__ key, int32_t *__restrict__ idx,
                                                      int32_t *__restrict__ rowl, int32_t *__restrict__ flag) {
    GS_LOOP(r, n_rows) {
        const int32_t a = rp[r], z = rp[r + 1];
        const unsigned long long hi = (unsigned long long)(r >> rows_log2) << cbits;
        const int32_t rl = (int32_t)(r & ((1 << rows_log2) - 1));
        int32_t prev = -1;
        bool bad = false;
        for (int32_t e = a; e < z; ++e) {
            const int32_t c = col[e];
            bad |= c <= prev;
            prev = c;
            key[e] = hi | (unsigned)c;
            idx[e] = e;
            rowl[e] = rl;
        }
        if (bad) atomicOr(flag, 1);
    }
}

// Sorted order: column, row in block, value bits.
__global__ __launch_bounds__(256) void gk_gather_kernel(int64_t n, const unsigned long long *__restrict__ skey,
                                                        const int32_t *__restrict__ sidx, const int32_t *__restrict__ rowl,
                                                        const float *__restrict__ val, unsigned long long cmask,
                                                        int32_t *__restrict__ scol, int32_t *__restrict__ srl,
                                                        uint32_t *__restrict__ sval) {
    GS_LOOP(i, n) {
        const int32_t e = sidx[i];
        scol[i] = (int32_t)(skey[i] & cmask);
        srl[i] = rowl[e];
        sval[i] = __float_as_uint(val[e]);
    }
}

// Tile t = b * S + s starts at the first key >= b << cbits | s * slab_cols.
__global__ __launch_bounds__(256) void gk_tile_start_kernel(int64_t n_tiles, int32_t n_slabs, int64_t slab_cols,
                                                            int cbits, int64_t n, const unsigned long long *__restrict__ skey,
                                                            int32_t *__restrict__ tts) {
    GS_LOOP(t, n_tiles + 1) {
        if (t == n_tiles) {
            tts[t] = (int32_t)n;
            continue;
        }
        const unsigned long long want = ((unsigned long long)(t / n_slabs) << cbits) |
                                        (unsigned long long)((t % n_slabs) * slab_cols);
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (skey[mid] < want) lo = mid + 1;
            else hi = mid;
        }
        tts[t] = (int32_t)lo;
    }
}

// LDS of one band's packing.
struct BandLds {
    uint32_t key[kSortN];          // (row << 11 | position), sorted; kPad beyond the run
    uint16_t crl[kSortN];          // kept entries in (row, position) order: row (< 2^15)
    uint16_t cpos[kSortN];         //   position in the run
    uint16_t cseg[kSortN];         //   segment
    int32_t seg_first[kSortN + 1]; // segment -> first kept entry
    uint16_t seg_rl[kSortN];
    uint8_t seg_chunk[kSortN];
    uint16_t seg_lane[kSortN];     // lane of the segment's first term
    int32_t cbase[kGcbChunks];
    int32_t wsum[kCutThreads / 64];
    int32_t nseg, ok, len;
};

// Exclusive scan of two flags per thread (elements 2t, 2t + 1); returns the prefix of 2t and
// the total in *tot.  Ends with a barrier.
__device__ __forceinline__ int scan2(BandLds &L, int f0, int f1, int *tot) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int v = f0 + f1;
    int inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    if (lane == 63) L.wsum[w] = inc;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kCutThreads / 64; ++k) {
        const int s = L.wsum[k];
        before += k < w ? s : 0;
        all += s;
    }
    __syncthreads();   // wsum reused by the next scan
    *tot = all;
    return before + inc - v;
}

// Loads the run [a, a + n) (n <= kCap) and sorts it by (row, position).
__device__ void band_sort(BandLds &L, const int32_t *__restrict__ srl, int64_t a, int n) {
    const int t = threadIdx.x;
    for (int j = t; j < kSortN; j += kCutThreads)
        L.key[j] = j < n ? ((uint32_t)srl[a + j] << kPosBits) | (uint32_t)j : kPad;
    __syncthreads();
    for (int k = 2; k <= kSortN; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
            const int l = i | j;
            const uint32_t x = L.key[i], y = L.key[l];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
                L.key[i] = y;
                L.key[l] = x;
            }
            __syncthreads();
        }
}

// Packs the sorted run's entries of position < len (gcb.cpp segments + pack): segments by row,
// a segment never split, a chunk's rows spanning < 4096, at most 32 chunks of 63 terms.  Sets
// L.ok; on success the segment -> (chunk, lane) map and the chunk bases.  All threads return
// after a barrier.
__device__ void band_pack(BandLds &L, int len) {
    const int t = threadIdx.x;
    const int j0 = 2 * t, j1 = 2 * t + 1;
    const uint32_t k0 = L.key[j0], k1 = L.key[j1];
    const int f0 = k0 != kPad && (int)(k0 & ((1u << kPosBits) - 1)) < len;
    const int f1 = k1 != kPad && (int)(k1 & ((1u << kPosBits) - 1)) < len;
    int tot;
    const int p0 = scan2(L, f0, f1, &tot);
    if (f0) {
        L.crl[p0] = (uint16_t)(k0 >> kPosBits);
        L.cpos[p0] = (uint16_t)(k0 & ((1u << kPosBits) - 1));
    }
    if (f1) {
        L.crl[p0 + f0] = (uint16_t)(k1 >> kPosBits);
        L.cpos[p0 + f0] = (uint16_t)(k1 & ((1u << kPosBits) - 1));
    }
    __syncthreads();
    // tot == len: every position < len is in the run exactly once.
    const int s0 = j0 < len && (j0 == 0 || L.crl[j0] != L.crl[j0 - 1]);
    const int s1 = j1 < len && L.crl[j1] != L.crl[j1 - 1];
    int nseg;
    const int q0 = scan2(L, s0, s1, &nseg);
    if (s0) {
        L.seg_first[q0] = j0;
        L.seg_rl[q0] = L.crl[j0];
    }
    if (s1) {
        L.seg_first[q0 + s0] = j1;
        L.seg_rl[q0 + s0] = L.crl[j1];
    }
    if (j0 < len) L.cseg[j0] = (uint16_t)(q0 + s0 - 1);
    if (j1 < len) L.cseg[j1] = (uint16_t)(q0 + s0 + s1 - 1);
    if (t == 0) L.seg_first[nseg] = len;
    __syncthreads();
    if (t < 64) {
        const int lane = t;
        int fill = kGcbChunkTerms, chunks = 0, base = 0, my_base = 0;
        bool bad = false;
        for (int g0 = 0; g0 < nseg && !bad; g0 += 64) {
            const int g = g0 + lane;
            const int grl = g < nseg ? L.seg_rl[g] : 0;
            const int gn = g < nseg ? L.seg_first[g + 1] - L.seg_first[g] : 0;
            int my_c = 0, my_l = 0;
            const int m = min(64, nseg - g0);
            for (int u = 0; u < m; ++u) {
                const int r = __builtin_amdgcn_readlane(grl, u);
                const int n = __builtin_amdgcn_readlane(gn, u);
                if (n > kGcbChunkTerms) {   // a row's segment must fit one chunk
                    bad = true;
                    break;
                }
                if (fill + n > kGcbChunkTerms || r - base >= kGcbRowSpan) {
                    ++chunks;
                    fill = 0;
                    base = r;
                    if (chunks > kGcbChunks) {
                        bad = true;
                        break;
                    }
                    my_base = lane == chunks - 1 ? r : my_base;
                }
                my_c = lane == u ? chunks - 1 : my_c;
                my_l = lane == u ? fill + 1 : my_l;
                fill += n;
            }
            if (g < nseg) {
                L.seg_chunk[g] = (uint8_t)my_c;
                L.seg_lane[g] = (uint16_t)my_l;
            }
        }
        if (lane < kGcbChunks) L.cbase[lane] = my_base;
        if (lane == 0) {
            L.ok = bad ? 0 : 1;
            L.nseg = nseg;
        }
    }
    __syncthreads();
}

// One workgroup per tile: the band starts (gcb.cpp build_tile's loop), written at the tile's
// term offset + band index; the band count per tile.
__global__ __launch_bounds__(kCutThreads) void gk_cut_kernel(const int32_t *__restrict__ tts,
                                                             const int32_t *__restrict__ scol,
                                                             const int32_t *__restrict__ srl, int32_t window,
                                                             int32_t *__restrict__ bstart, int32_t *__restrict__ nbands) {
    __shared__ BandLds L;
    const int64_t tile = blockIdx.x;
    const int64_t t0 = tts[tile], t1 = tts[tile + 1];
    const int t = threadIdx.x;
    int32_t k = 0;
    for (int64_t a = t0; a < t1;) {
        const int64_t bmax = min(t1, a + (int64_t)kCap);
        const int32_t clo = scol[a];
        // b = the first term at or past clo + window (the run is sorted by column); at most
        // kCap < 2 * kCutThreads candidates
        const int in0 = a + t < bmax && scol[a + t] < clo + window;
        const int in1 = a + t + kCutThreads < bmax && scol[a + t + kCutThreads] < clo + window;
        const int n = __syncthreads_count(in0) + __syncthreads_count(in1);
        band_sort(L, srl, a, n);
        int len = n;
        for (;;) {
            band_pack(L, len);
            if (L.ok) break;
            len = max(1, len * 31 / 32);
            __syncthreads();   // every thread read L.ok before the next pack rewrites it
        }
        if (t == 0) bstart[t0 + k] = (int32_t)a;
        ++k;
        a += len;
        __syncthreads();
    }
    if (t == 0) nbands[tile] = k;
}

// Band starts by global band index, and each band's tile.
__global__ __launch_bounds__(256) void gk_compact_kernel(int64_t n_tiles, const int32_t *__restrict__ tts,
                                                         const int32_t *__restrict__ tbs,
                                                         const int32_t *__restrict__ bstart,
                                                         int32_t *__restrict__ gstart, int32_t *__restrict__ gtile) {
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int32_t b0 = tbs[tile], nb = tbs[tile + 1] - b0;
        for (int32_t k = threadIdx.x; k < nb; k += blockDim.x) {
            gstart[b0 + k] = bstart[tts[tile] + k];
            gtile[b0 + k] = (int32_t)tile;
        }
    }
}

// One workgroup per band: its image (gcb.cpp build_tile's emission) through LDS.
__global__ __launch_bounds__(kCutThreads) void gk_emit_kernel(int64_t n_bands, const int32_t *__restrict__ tts,
                                                              const int32_t *__restrict__ gstart,
                                                              const int32_t *__restrict__ gtile,
                                                              const int32_t *__restrict__ scol,
                                                              const int32_t *__restrict__ srl,
                                                              const uint32_t *__restrict__ sval,
                                                              int32_t *__restrict__ band_clo, uint32_t *__restrict__ word,
                                                              int32_t *__restrict__ flag) {
    __shared__ BandLds L;
    __shared__ uint32_t img[kGcbBandWords];
    const int64_t g = blockIdx.x;
    const int t = threadIdx.x;
    const int32_t tile = gtile[g];
    const int64_t a = gstart[g];
    const int64_t b = g + 1 < n_bands && gtile[g + 1] == tile ? (int64_t)gstart[g + 1] : (int64_t)tts[tile + 1];
    const int n = (int)(b - a);
    if (n < 1 || n > kCap) {   // uniform: cut and emit disagree (a builder bug)
        if (t == 0) atomicOr(flag, 2);
        return;
    }
    for (int i = t; i < kGcbBandWords; i += kCutThreads) img[i] = 0u;
    band_sort(L, srl, a, n);
    band_pack(L, n);
    if (!L.ok) {
        if (t == 0) atomicOr(flag, 2);
        return;
    }
    const int32_t clo = scol[a];
    const int nseg = L.nseg;
    for (int q = t; q < nseg; q += kCutThreads)
        if (q == 0 || L.seg_chunk[q] != L.seg_chunk[q - 1]) {   // a chunk's first segment
            const int c = L.seg_chunk[q];
            img[(c >> 1) * 64 * 4 + (c & 1)] = (uint32_t)L.cbase[c];   // header: the chunk's base row
        }
    for (int j = t; j < n; j += kCutThreads) {
        const int q = L.cseg[j];
        const int c = L.seg_chunk[q];
        const int first = L.seg_first[q];
        const int lane = L.seg_lane[q] + (j - first);
        const int p = L.cpos[j];
        const int k = c & 1;
        const uint32_t w = (uint32_t)(scol[a + p] - clo) | ((uint32_t)((int)L.crl[j] - L.cbase[c]) << kGcbColBits) |
                           kGcbLive | (j > first ? kGcbCont : 0u);
        const int slot = ((c >> 1) * 64 + lane) * 4;
        img[slot + k] = w;
        img[slot + 2 + k] = sval[a + p];
    }
    __syncthreads();
    uint4 *dst = reinterpret_cast<uint4 *>(word + g * kGcbBandWords);
    const uint4 *src = reinterpret_cast<const uint4 *>(img);
    for (int i = t; i < kGcbBandWords / 4; i += kCutThreads) dst[i] = src[i];
    if (t == 0) band_clo[g] = clo;
}

__global__ __launch_bounds__(256) void gk_max_kernel(int64_t n, const int32_t *__restrict__ v, int32_t *__restrict__ out) {
    int32_t mx = 0;
    GS_LOOP(i, n) mx = max(mx, v[i]);
    for (int d = 32; d >= 1; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(out, mx);
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
    void release(void *q) {
        for (auto &x : p)
            if (x == q) {
                (void)hipFree(x);
                x = nullptr;
            }
    }
    ~Tmp() {
        for (void *q : p)
            if (q) (void)hipFree(q);
    }
};

template <class T>
hipError_t keep_alloc_dev(T **out, int64_t n, int64_t &acct) {
    const size_t bytes = (size_t)std::max<int64_t>(n, 1) * sizeof(T);
    const hipError_t e = hipMalloc((void **)out, bytes);
    if (e == hipSuccess) acct += (int64_t)bytes;
    return e;
}

#define GK_TRY(x)                  \
    do {                           \
        const hipError_t e_ = (x); \
        if (e_ != hipSuccess) {    \
            err = e_;              \
            return -5;             \
        }                          \
    } while (0)

int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

}  // namespace

int devbuild_gcb(sm_matrix *m, int rows_log2, int32_t n_slabs, int32_t window, GcbHost &meta, hipStream_t s,
                 hipError_t &err) {
    err = hipSuccess;
    meta = GcbHost();
    const int64_t n_rows = m->n_rows, n_cols = m->n_cols, nnz = m->nnz;
    // gcb_build's limits
    if (rows_log2 < 6 || rows_log2 > 15 || window < 64 || window > kGcbMaxWindow) return 1;
    if (n_rows <= 0 || n_cols <= 0 || n_slabs < 1 || n_cols >= ((int64_t)1 << 30) || nnz <= 0) return 1;
    const int32_t br = (int32_t)std::min<int64_t>((int64_t)1 << rows_log2, n_rows);
    const int64_t nblk = (n_rows + br - 1) / br;
    const int64_t sc = ((n_cols + n_slabs - 1) / n_slabs + 255) & ~(int64_t)255;
    const int64_t ns = (n_cols + sc - 1) / sc;
    const int64_t ntile = nblk * ns;
    if (ntile >= ((int64_t)1 << 30)) return 1;
    const int cbits = bits_for((uint64_t)(n_cols - 1));
    const int end_bit = cbits + bits_for((uint64_t)std::max<int64_t>(nblk - 1, 1));
    Tmp tp;
    unsigned long long *key = nullptr, *skey = nullptr;
    int32_t *idx = nullptr, *sidx = nullptr, *rowl = nullptr, *flag = nullptr;
    GK_TRY(tp.alloc(&key, nnz));
    GK_TRY(tp.alloc(&skey, nnz));
    GK_TRY(tp.alloc(&idx, nnz));
    GK_TRY(tp.alloc(&sidx, nnz));
    GK_TRY(tp.alloc(&rowl, nnz));
    GK_TRY(tp.alloc(&flag, 1));
    GK_TRY(hipMemsetAsync(flag, 0, 4, s));
    hipLaunchKernelGGL(gk_keys_kernel, dim3(grid_of(n_rows)), dim3(256), 0, s, n_rows, m->d_row_ptr, m->d_col,
                       rows_log2, cbits, key, idx, rowl, flag);
    GK_TRY(hipGetLastError());
    {
        size_t bytes = 0;
        GK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, key, skey, idx, sidx, (int)nnz, 0, end_bit, s));
        uint8_t *tmp = nullptr;
        GK_TRY(tp.alloc(&tmp, (int64_t)bytes));
        GK_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, key, skey, idx, sidx, (int)nnz, 0, end_bit, s));
        GK_TRY(hipStreamSynchronize(s));
        tp.release(tmp);
    }
    int32_t fl = 0;
    GK_TRY(hipMemcpyAsync(&fl, flag, 4, hipMemcpyDeviceToHost, s));
    GK_TRY(hipStreamSynchronize(s));
    if (fl) return 1;   // a row's columns not strictly ascending (gcb_build declines)
    tp.release(key);
    tp.release(idx);
    int32_t *scol = nullptr, *srl = nullptr, *tts = nullptr;
    uint32_t *sval = nullptr;
    GK_TRY(tp.alloc(&scol, nnz));
    GK_TRY(tp.alloc(&srl, nnz));
    GK_TRY(tp.alloc(&sval, nnz));
    GK_TRY(tp.alloc(&tts, ntile + 1));
    const unsigned long long cmask = ((unsigned long long)1 << cbits) - 1;
    hipLaunchKernelGGL(gk_gather_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, nnz, skey, sidx, rowl, m->d_val, cmask,
                       scol, srl, sval);
    hipLaunchKernelGGL(gk_tile_start_kernel, dim3(grid_of(ntile + 1)), dim3(256), 0, s, ntile, (int32_t)ns, sc, cbits,
                       nnz, skey, tts);
    GK_TRY(hipGetLastError());
    GK_TRY(hipStreamSynchronize(s));
    tp.release(skey);
    tp.release(sidx);
    tp.release(rowl);
    // cut
    int32_t *bstart = nullptr, *nb = nullptr, *tbs = nullptr, *mx = nullptr;
    GK_TRY(tp.alloc(&bstart, nnz));
    GK_TRY(tp.alloc(&nb, ntile + 1));
    GK_TRY(tp.alloc(&mx, 1));
    GK_TRY(hipMemsetAsync(nb + ntile, 0, 4, s));
    GK_TRY(hipMemsetAsync(mx, 0, 4, s));
    hipLaunchKernelGGL(gk_cut_kernel, dim3((unsigned)ntile), dim3(kCutThreads), 0, s, tts, scol, srl, window, bstart, nb);
    GK_TRY(hipGetLastError());
    GK_TRY(keep_alloc_dev(&m->plan.xb.d_chunk_start, ntile + 1, m->device_bytes));
    tbs = m->plan.xb.d_chunk_start;
    {
        size_t bytes = 0;
        GK_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, nb, tbs, (int)(ntile + 1), s));
        uint8_t *tmp = nullptr;
        GK_TRY(tp.alloc(&tmp, (int64_t)bytes));
        GK_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, nb, tbs, (int)(ntile + 1), s));
    }
    hipLaunchKernelGGL(gk_max_kernel, dim3(grid_of(ntile)), dim3(256), 0, s, ntile, nb, mx);
    GK_TRY(hipGetLastError());
    int32_t n_bands = 0, max_bands = 0;
    GK_TRY(hipMemcpyAsync(&n_bands, tbs + ntile, 4, hipMemcpyDeviceToHost, s));
    GK_TRY(hipMemcpyAsync(&max_bands, mx, 4, hipMemcpyDeviceToHost, s));
    GK_TRY(hipStreamSynchronize(s));
    // gcb_build's output limits: a tile's bands under 4 GiB of 32-bit byte offsets.
    if ((int64_t)max_bands * kGcbBandWords * 4 >= ((int64_t)1 << 32) || n_bands <= 0 || n_bands >= INT32_MAX) {
        (void)hipFree(m->plan.xb.d_chunk_start);
        m->device_bytes -= (ntile + 1) * 4;
        m->plan.xb.d_chunk_start = nullptr;
        return 1;
    }
    int32_t *gstart = nullptr, *gtile = nullptr;
    GK_TRY(tp.alloc(&gstart, n_bands));
    GK_TRY(tp.alloc(&gtile, n_bands));
    hipLaunchKernelGGL(gk_compact_kernel, dim3((unsigned)std::min<int64_t>(ntile, 1 << 16)), dim3(256), 0, s, ntile,
                       tts, tbs, bstart, gstart, gtile);
    GK_TRY(hipGetLastError());
    XbandDev &d = m->plan.xb;
    GK_TRY(keep_alloc_dev(&d.d_band_clo, n_bands, m->device_bytes));
    GK_TRY(keep_alloc_dev(&d.d_word, (int64_t)n_bands * kGcbBandWords, m->device_bytes));
    hipLaunchKernelGGL(gk_emit_kernel, dim3((unsigned)n_bands), dim3(kCutThreads), 0, s, (int64_t)n_bands, tts, gstart,
                       gtile, scol, srl, sval, d.d_band_clo, d.d_word, flag);
    GK_TRY(hipGetLastError());
    GK_TRY(hipMemcpyAsync(&fl, flag, 4, hipMemcpyDeviceToHost, s));
    GK_TRY(hipStreamSynchronize(s));
    if (fl) {   // the emission's packing disagreed with the cut's: a builder bug, not a decline
        err = hipErrorUnknown;
        return -6;
    }
    meta.rows_log2 = rows_log2;
    meta.window = window;
    meta.block_rows = br;
    meta.n_blocks = (int32_t)nblk;
    meta.n_slabs = (int32_t)ns;
    meta.slab_cols = (int32_t)sc;
    meta.max_bands_per_tile = max_bands;
    meta.n_bands = n_bands;
    meta.real_terms = nnz;
    return 0;
}

}  // namespace smamd
