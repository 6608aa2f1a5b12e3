// kernels.hip -- gfx950 kernels of libsparsematrix_amd.so.
//
// Everything here is HBM-bound integer/fp32 streaming: no MFMA.  The design
// (DESIGN.md "Kernels") in one line per kernel:
//   spmv_parity      one thread per row, terms added in stored order with
//                    separate round-to-nearest mul/add: bit-identical to the
//                    reference's generic-C AddMatMat (kernel.cc:568-582, 791).
//   spmv_stream      nnz-balanced row tiles (<= 4096 terms): aligned 16-byte
//                    loads of col/val, x gathered, terms staged in LDS, then
//                    each short row summed by one thread in stored order
//                    (bit-exact), rows > 64 terms by a wavefront (DPP/shuffle
//                    tree), rows > 4096 terms split across workgroups with a
//                    deterministic ordered finalize.
//   spmv_vector      CSR-vector: L lanes per row (L = pow2 near the mean row
//                    length), shuffle reduction.
//   spmm_rowpanel    N right-hand sides, row-major X/Y: N/4 lanes per row own
//                    a float4 slice of the output row; the row's (col, val)
//                    pairs are loaded cooperatively and broadcast by shuffle;
//                    every output element accumulates in stored order
//                    (bit-exact).
//   spmm_generic     any N and any X/Y strides (AddMatMat layouts), one thread
//                    per output element, stored order (bit-exact).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (Makefile).
#include "sm_internal.h"

namespace smamd {
namespace {

__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
// One term of the reference: a * (table_value * alpha) (kernel.cc:791, 580-582).
__device__ __forceinline__ float term(float xv, float v, float alpha) {
    return mul_rn(xv, mul_rn(v, alpha));
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streamed (read-once) 16-byte loads of val/col.  SM_NT_LOADS selects the
// non-temporal cache policy (measured both ways).
#ifndef SM_NT_LOADS
#define SM_NT_LOADS 0
#endif
__device__ __forceinline__ float4 ld_stream(const float4 *p) {
#if SM_NT_LOADS
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
#else
    const f32x4 v = *reinterpret_cast<const f32x4 *>(p);
#endif
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 ld_stream(const int4 *p) {
#if SM_NT_LOADS
    const i32x4 v = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(p));
#else
    const i32x4 v = *reinterpret_cast<const i32x4 *>(p);
#endif
    return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s = add_rn(s, __shfl_xor(s, off, 64));
    return s;
}

// LDS slot of the l-th staged term: one pad word every 32 keeps the
// thread-per-row reads (stride = row length) off a single bank.
__device__ __forceinline__ int lds_slot(int l) { return l + (l >> 5); }

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void spmv_parity_kernel(int32_t n, const int32_t *__restrict__ rp,
                                                          const int32_t *__restrict__ col,
                                                          const float *__restrict__ val,
                                                          const float *__restrict__ x,
                                                          float *__restrict__ y, float alpha,
                                                          float beta) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    float acc = y[r];
    if (beta != 1.0f) acc = mul_rn(acc, beta);
    const int32_t e1 = rp[r + 1];
    for (int32_t e = rp[r]; e < e1; ++e) acc = add_rn(acc, term(x[col[e]], val[e], alpha));
    y[r] = acc;
}

// ---------------------------------------------------------------------------
// ABL (development only, SM_STREAM_ABLATE; results wrong): 1 replaces the x gathers
// of short-row tiles by one broadcast address.
template <int THREADS, int TILE, int ABL = 0>
__global__ __launch_bounds__(THREADS) void spmv_stream_kernel(
    const Tile *__restrict__ tiles, const Chunk *__restrict__ chunks, int32_t n_chunks,
    const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ x, float *__restrict__ y,
    float alpha, float beta, float *__restrict__ partials) {
    constexpr int kLds = TILE + TILE / 32 + 8;
    constexpr int kWaves = THREADS / 64;
    constexpr int kIt = TILE / (4 * THREADS) + 1;   // +1: unaligned tile start
    __shared__ float prod[kLds];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int32_t b = blockIdx.x;

    if (b < n_chunks) {
        // ---- one chunk of a long row: tree sum of its terms ----------------
        const Chunk ch = chunks[b];
        float s = 0.0f;
        for (int32_t i0 = (ch.begin & ~3) + 4 * tid; i0 < ch.end; i0 += 4 * THREADS * kIt) {
            float4 vv[kIt];
            int4 cc[kIt];
#pragma unroll
            for (int it = 0; it < kIt; ++it) {
                const int32_t i = i0 + 4 * THREADS * it;
                const int32_t il = i < ch.end ? i : i0;
                vv[it] = ld_stream(reinterpret_cast<const float4 *>(val + il));
                cc[it] = ld_stream(reinterpret_cast<const int4 *>(col + il));
            }
            float xg[kIt][4];
#pragma unroll
            for (int it = 0; it < kIt; ++it) {
                xg[it][0] = x[cc[it].x]; xg[it][1] = x[cc[it].y];
                xg[it][2] = x[cc[it].z]; xg[it][3] = x[cc[it].w];
            }
#pragma unroll
            for (int it = 0; it < kIt; ++it) {
                const int32_t i = i0 + 4 * THREADS * it;
                const float vq[4] = {vv[it].x, vv[it].y, vv[it].z, vv[it].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float tq = term(xg[it][q], vq[q], alpha);
                    if (i + q >= ch.begin && i + q < ch.end) s = add_rn(s, tq);
                }
            }
        }
        s = wave_sum(s);
        if (lane == 0) prod[wave] = s;
        __syncthreads();
        if (tid == 0) {
            float t = prod[0];
#pragma unroll
            for (int w = 1; w < kWaves; ++w) t = add_rn(t, prod[w]);
            partials[b] = t;
        }
        return;
    }

    // ---- a tile of short rows -----------------------------------------------
    const Tile t = tiles[b - n_chunks];
    const int32_t s0 = rp[t.r0];
    const int32_t e0 = rp[t.r1];
    // Row bounds and y of this thread's first row, fetched before the tile's
    // terms so their latency hides under the stream.
    const int32_t r_first = t.r0 + tid;
    const bool has_row = r_first < t.r1;
    int32_t ra = 0, re = 0;
    float y_first = 0.0f;
    if (has_row) {
        ra = rp[r_first];
        re = rp[r_first + 1];
        y_first = y[r_first];
    }
    if (e0 > s0) {
        // Aligned 16-byte loads over [s0 & ~3, e0): every slot loads (slots past
        // the tile re-read the first vector), so the col/val loads and then all
        // x gathers issue back to back with no branch between them.  Columns of
        // slots outside [s0, e0) belong to neighbouring rows or to the zeroed
        // pad: always valid indices.
        const int32_t base = s0 & ~3;
        float4 vv[kIt];
        int4 cc[kIt];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const int32_t i = base + 4 * (tid + it * THREADS);
            const int32_t il = i < e0 ? i : base;
            vv[it] = ld_stream(reinterpret_cast<const float4 *>(val + il));
            cc[it] = ld_stream(reinterpret_cast<const int4 *>(col + il));
        }
        float xg[kIt][4];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            if constexpr (ABL & 1) {
                const int32_t c0 = cc[it].x & 0;
                xg[it][0] = x[c0]; xg[it][1] = x[c0 + (cc[it].y & 0)];
                xg[it][2] = x[c0 + (cc[it].z & 0)]; xg[it][3] = x[c0 + (cc[it].w & 0)];
            } else {
                xg[it][0] = x[cc[it].x]; xg[it][1] = x[cc[it].y];
                xg[it][2] = x[cc[it].z]; xg[it][3] = x[cc[it].w];
            }
        }
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const int32_t i = base + 4 * (tid + it * THREADS);
            const float vq[4] = {vv[it].x, vv[it].y, vv[it].z, vv[it].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int32_t idx = i + q;
                const float tq = term(xg[it][q], vq[q], alpha);
                if (idx >= s0 && idx < e0) prod[lds_slot(idx - s0)] = tq;
            }
        }
    }
    __syncthreads();

    // Short rows: one thread each, terms in stored order (reference order).
    if (has_row && re - ra <= kSerialRowMax) {
        float acc = y_first;
        if (beta != 1.0f) acc = mul_rn(acc, beta);
        const int32_t a = ra - s0, e = re - s0;
#pragma unroll 4
        for (int32_t k = a; k < e; ++k) acc = add_rn(acc, prod[lds_slot(k)]);
        y[r_first] = acc;
    }
    for (int32_t r = r_first + THREADS; r < t.r1; r += THREADS) {
        const int32_t a = rp[r] - s0;
        const int32_t e = rp[r + 1] - s0;
        if (e - a > kSerialRowMax) continue;
        float acc = y[r];
        if (beta != 1.0f) acc = mul_rn(acc, beta);
        for (int32_t k = a; k < e; ++k) acc = add_rn(acc, prod[lds_slot(k)]);
        y[r] = acc;
    }
    // Medium rows: one wavefront each, shuffle tree.
    if (t.flags & 1) {
        for (int32_t r = t.r0 + wave; r < t.r1; r += kWaves) {
            const int32_t a = rp[r] - s0;
            const int32_t e = rp[r + 1] - s0;
            if (e - a <= kSerialRowMax) continue;
            float s = 0.0f;
            for (int32_t k = a + lane; k < e; k += 64) s = add_rn(s, prod[lds_slot(k)]);
            s = wave_sum(s);
            if (lane == 0) {
                float acc = y[r];
                if (beta != 1.0f) acc = mul_rn(acc, beta);
                y[r] = add_rn(acc, s);
            }
        }
    }
}

__global__ __launch_bounds__(256) void spmv_long_finalize_kernel(
    int32_t n_long, const int32_t *__restrict__ long_rows, const int32_t *__restrict__ long_ptr,
    const float *__restrict__ partials, float *__restrict__ y, float beta) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_long) return;
    const int32_t r = long_rows[i];
    float acc = y[r];
    if (beta != 1.0f) acc = mul_rn(acc, beta);
    for (int32_t c = long_ptr[i]; c < long_ptr[i + 1]; ++c) acc = add_rn(acc, partials[c]);
    y[r] = acc;
}

// ---------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(256) void spmv_vector_kernel(int32_t n, const int32_t *__restrict__ rp,
                                                          const int32_t *__restrict__ col,
                                                          const float *__restrict__ val,
                                                          const float *__restrict__ x,
                                                          float *__restrict__ y, float alpha,
                                                          float beta) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t r = (int32_t)(gid / L);
    const int lane = (int)(gid % L);
    if (r >= n) return;   // whole L-lane groups leave together
    const int32_t e1 = rp[r + 1];
    float s = 0.0f;
    for (int32_t e = rp[r] + lane; e < e1; e += L) s = add_rn(s, term(x[col[e]], val[e], alpha));
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1) s = add_rn(s, __shfl_xor(s, off, L));
    if (lane == 0) {
        float acc = y[r];
        if (beta != 1.0f) acc = mul_rn(acc, beta);
        y[r] = add_rn(acc, s);
    }
}

// ---------------------------------------------------------------------------
template <int G>   // lanes per row (power of two); lane g owns rhs [4g, 4g+4)
__global__ __launch_bounds__(256) void spmm_rowpanel_kernel(
    int32_t n, int32_t nrhs, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t ldx,
    float *__restrict__ Y, int64_t ldy, float alpha, float beta) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t r = (int32_t)(gid / G);
    const int g = (int)(gid % G);
    if (r >= n) return;
    const bool active = 4 * g < nrhs;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float *yp = Y + (int64_t)r * ldy + 4 * g;
    if (active) acc = *reinterpret_cast<const float4 *>(yp);
    if (beta != 1.0f) {
        acc.x = mul_rn(acc.x, beta); acc.y = mul_rn(acc.y, beta);
        acc.z = mul_rn(acc.z, beta); acc.w = mul_rn(acc.w, beta);
    }
    const int32_t a = rp[r];
    const int32_t e = rp[r + 1];
    for (int32_t b0 = a; b0 < e; b0 += G) {
        int32_t myc = 0;
        float myv = 0.0f;
        if (b0 + g < e) {
            myc = col[b0 + g];
            myv = mul_rn(val[b0 + g], alpha);
        }
        const int cnt = min(G, e - b0);
        float4 xv[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int32_t cj = __shfl(myc, j, G);
            if (j < cnt && active)
                xv[j] = *reinterpret_cast<const float4 *>(X + (int64_t)cj * ldx + 4 * g);
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const float vj = __shfl(myv, j, G);
            if (j < cnt) {
                acc.x = add_rn(acc.x, mul_rn(xv[j].x, vj));
                acc.y = add_rn(acc.y, mul_rn(xv[j].y, vj));
                acc.z = add_rn(acc.z, mul_rn(xv[j].z, vj));
                acc.w = add_rn(acc.w, mul_rn(xv[j].w, vj));
            }
        }
    }
    if (active) *reinterpret_cast<float4 *>(yp) = acc;
}

// Range-checked buffer descriptor: loads past `bytes` read 0 and make no memory
// request, so a padded slot needs no branch (a branch around a load makes hipcc
// drain vmcnt before the next one).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t panel_rsrc(const void *base, uint64_t bytes) {
    const uint32_t nb = bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)nb,
                                             0x00020000);
}

// SpMM row panel, gather-pipelined: like spmm_rowpanel_kernel (G lanes per output row,
// lane g owns Y[r, 4g:4g+4]) but a row's terms go in groups of UU: the group's
// (col, val) are loaded at once (UU/G per lane, broadcast by shuffles), then all UU
// X-row gathers are in flight together -- branch-free range-checked buffer loads,
// padded slots sent past the range -- and the terms are added in stored order
// (padded slots skipped by a select, so the sum is bit-identical).  Requires X
// (x_rows * ldx floats) under 4 GiB.
template <int G>
__global__ __launch_bounds__(256) void spmm_rowpanel2_kernel(
    int32_t n, int32_t nrhs, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, int32_t nnz, const float *__restrict__ X, int64_t ldx,
    int64_t x_rows, float *__restrict__ Y, int64_t ldy, float alpha, float beta) {
    constexpr int UU = 16 > G ? 16 : G;   // terms per group
    constexpr int T = UU / G;             // (col, val) loads per lane per group
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t r = (int32_t)(gid / G);
    const int g = (int)(gid % G);
    if (r >= n) return;   // whole groups of G lanes
    const bool active = 4 * g < nrhs;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float *yp = Y + (int64_t)r * ldy + 4 * g;
    if (active) acc = *reinterpret_cast<const float4 *>(yp);
    if (beta != 1.0f) {
        acc.x = mul_rn(acc.x, beta); acc.y = mul_rn(acc.y, beta);
        acc.z = mul_rn(acc.z, beta); acc.w = mul_rn(acc.w, beta);
    }
    const __amdgpu_buffer_rsrc_t c_src = panel_rsrc(col, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t v_src = panel_rsrc(val, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t x_src = panel_rsrc(X, (uint64_t)x_rows * ldx * 4);
    const int32_t a = rp[r];
    const int32_t e = rp[r + 1];
    for (int32_t b0 = a; b0 < e; b0 += UU) {
        int32_t ci[T];
        float vi[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int32_t i = b0 + g + G * t;
            const uint32_t off = i < e ? 4u * (uint32_t)i : kOob;
            ci[t] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(c_src, off, 0, 0);
            vi[t] = mul_rn(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_src, off, 0, 0)),
                           alpha);
        }
        const int cnt = min(UU, e - b0);
        u32x4 xv[UU];
#pragma unroll
        for (int j = 0; j < UU; ++j) {
            const int32_t cj = __shfl(ci[j / G], j % G, G);
            const uint32_t off = (j < cnt && active)
                                     ? 4u * (uint32_t)((int64_t)cj * ldx + 4 * g)
                                     : kOob;
            xv[j] = __builtin_amdgcn_raw_buffer_load_b128(x_src, off, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < UU; ++j) {
            const float vj = __shfl(vi[j / G], j % G, G);
            const float4 s4 = make_float4(add_rn(acc.x, mul_rn(__uint_as_float(xv[j].x), vj)),
                                          add_rn(acc.y, mul_rn(__uint_as_float(xv[j].y), vj)),
                                          add_rn(acc.z, mul_rn(__uint_as_float(xv[j].z), vj)),
                                          add_rn(acc.w, mul_rn(__uint_as_float(xv[j].w), vj)));
            if (j < cnt) acc = s4;
        }
    }
    if (active) *reinterpret_cast<float4 *>(yp) = acc;
}

template <bool RHS_FASTEST>
__global__ __launch_bounds__(256) void spmm_generic_kernel(
    int32_t n, int32_t nrhs, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t x_sk, int64_t x_si,
    float *__restrict__ Y, int64_t y_sj, int64_t y_si, float alpha, float beta) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)n * nrhs) return;
    int64_t j, i;
    if (RHS_FASTEST) { j = gid / nrhs; i = gid % nrhs; }
    else { i = gid / n; j = gid % n; }
    float *yp = Y + j * y_sj + i * y_si;
    float acc = *yp;
    if (beta != 1.0f) acc = mul_rn(acc, beta);
    const float *xi = X + i * x_si;
    const int32_t e1 = rp[j + 1];
    for (int32_t e = rp[j]; e < e1; ++e)
        acc = add_rn(acc, term(xi[(int64_t)col[e] * x_sk], val[e], alpha));
    *yp = acc;
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void beta_kernel(float *__restrict__ c, int32_t m, int32_t n,
                                                   int64_t ldc, float beta) {
    const int64_t total = (int64_t)m * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / n, j = t % n;
        float *p = c + i * ldc + j;
        *p = mul_rn(*p, beta);
    }
}

__global__ __launch_bounds__(256) void transpose_kernel(const float *__restrict__ a, int32_t m,
                                                        int32_t n, int64_t lda,
                                                        float *__restrict__ sa, int64_t ldsa,
                                                        int32_t tiles_n) {
    __shared__ float tile[64][65];
    const int32_t tb = blockIdx.x;
    const int32_t ti = tb / tiles_n, tj = tb % tiles_n;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int k = ty; k < 64; k += 4) {
        const int64_t i = (int64_t)ti * 64 + k, j = (int64_t)tj * 64 + tx;
        if (i < m && j < n) tile[k][tx] = a[i * lda + j];
    }
    __syncthreads();
    for (int k = ty; k < 64; k += 4) {
        const int64_t j = (int64_t)tj * 64 + k, i = (int64_t)ti * 64 + tx;
        if (i < m && j < n) sa[j * ldsa + i] = tile[tx][k];
    }
}

// Device CSR ingestion: one grid-stride pass over max(rows + 1, terms) -- row i checks its
// pointers, term i its column (a per-row loop over the terms took 12 ms on R-MAT 24, whose
// longest row has 238 K terms).
__global__ __launch_bounds__(256) void validate_kernel(int32_t n_rows, int32_t n_cols, int32_t nnz,
                                                       const int32_t *__restrict__ rp,
                                                       const int32_t *__restrict__ col,
                                                       int32_t *flag) {
    const int64_t n = max((int64_t)n_rows + 1, (int64_t)nnz);
    int32_t f = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i == 0 && rp[0] != 0) f |= 1;
        if (i == n_rows && rp[n_rows] != nnz) f |= 2;
        if (i < n_rows) {
            const int32_t a = rp[i], e = rp[i + 1];
            if (a > e || a < 0 || e > nnz) f |= 4;
        }
        if (i < nnz) {
            const int32_t c = col[i];
            if (c < 0 || c >= n_cols) f |= 8;
        }
    }
    if (f) atomicOr(flag, f);
}

__global__ __launch_bounds__(256) void scatter_dense_kernel(int32_t n, const int32_t *__restrict__ rp,
                                                            const int32_t *__restrict__ col,
                                                            const float *__restrict__ val,
                                                            float *__restrict__ out, int64_t stride,
                                                            bool b_layout) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
        const int64_t c = col[e];
        if (b_layout) out[(int64_t)r * stride + c] = val[e];
        else out[c * stride + r] = val[e];
    }
}

// xp[i] = x[perm[i]]: 4 outputs per thread (one 16-byte load of perm, four
// gathers in flight, one 16-byte store); the tail (n % 4) one by one.
// xp[rank[c]] = x[c]: coalesced reads of x and rank, scattered stores (nothing waits
// on a store; a gather xp[i] = x[perm[i]] exposed one read latency per element).
template <bool VEC>
__global__ __launch_bounds__(256) void x_relabel_kernel(int64_t n, const int32_t *__restrict__ rank,
                                                        const float *__restrict__ x,
                                                        float *__restrict__ xp) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if constexpr (VEC) {
        const int64_t i = 4 * t;
        if (i + 4 <= n) {
            const int4 r = *reinterpret_cast<const int4 *>(rank + i);
            const float4 v = *reinterpret_cast<const float4 *>(x + i);
            xp[r.x] = v.x;
            xp[r.y] = v.y;
            xp[r.z] = v.z;
            xp[r.w] = v.w;
        } else {
            for (int64_t k = i; k < n; ++k) xp[rank[k]] = x[k];
        }
    } else {
        if (t < n) xp[rank[t]] = x[t];
    }
}

inline unsigned blocks_for(int64_t work, int per = 256) {
    return (unsigned)((work + per - 1) / per);
}

}  // namespace

// ---------------------------------------------------------------------------
hipError_t launch_spmv_parity(int32_t n, const int32_t *rp, const int32_t *col, const float *val,
                              const float *x, float *y, float alpha, float beta, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(spmv_parity_kernel, dim3(blocks_for(n)), dim3(256), 0, s, n, rp, col, val,
                       x, y, alpha, beta);
    return hipGetLastError();
}

hipError_t launch_spmv_stream(const Plan &p, const int32_t *rp, const int32_t *col,
                              const float *val, const float *x, float *y, float alpha,
                              float beta, float *partials, hipStream_t s) {
    const int64_t grid = (int64_t)p.n_chunks + p.n_tiles;
    if (grid == 0) return hipSuccess;
#ifdef SM_DEV
    static const int abl = [] {
        const char *e = dev_env("SM_STREAM_ABLATE");
        return e ? atoi(e) : 0;
    }();
#define SM_STREAM_ABL(TT)                                                                     \
    if (abl == 1) {                                                                           \
        hipLaunchKernelGGL((spmv_stream_kernel<kStreamThreads, TT, 1>), dim3((unsigned)grid), \
                           dim3(kStreamThreads), 0, s, p.d_tiles, p.d_chunks, p.n_chunks, rp, \
                           col, val, x, y, alpha, beta, partials);                            \
        break;                                                                                \
    }
#else
#define SM_STREAM_ABL(TT)
#endif
#define SM_STREAM(TT)                                                                         \
    case TT:                                                                                  \
        SM_STREAM_ABL(TT)                                                                     \
        hipLaunchKernelGGL((spmv_stream_kernel<kStreamThreads, TT>), dim3((unsigned)grid),    \
                           dim3(kStreamThreads), 0, s, p.d_tiles, p.d_chunks, p.n_chunks, rp, \
                           col, val, x, y, alpha, beta, partials);                            \
        break;
    switch (p.tile_nnz) {
        SM_STREAM(1024) SM_STREAM(2048) SM_STREAM(4096) SM_STREAM(8192)
        default: return hipErrorInvalidValue;
    }
#undef SM_STREAM
#undef SM_STREAM_ABL
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.n_long == 0) return e;
    hipLaunchKernelGGL(spmv_long_finalize_kernel, dim3(blocks_for(p.n_long)), dim3(256), 0, s,
                       p.n_long, p.d_long_rows, p.d_long_ptr, partials, y, beta);
    return hipGetLastError();
}

hipError_t launch_long_finalize(int32_t n_long, const int32_t *long_rows, const int32_t *long_ptr,
                                const float *partials, float *y, float beta, hipStream_t s) {
    if (n_long <= 0) return hipSuccess;
    hipLaunchKernelGGL(spmv_long_finalize_kernel, dim3(blocks_for(n_long)), dim3(256), 0, s, n_long,
                       long_rows, long_ptr, partials, y, beta);
    return hipGetLastError();
}

hipError_t launch_spmv_vector(int32_t n, double avg_row, const int32_t *rp, const int32_t *col,
                              const float *val, const float *x, float *y, float alpha, float beta,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int L = 2;
    while (L < 64 && L < avg_row) L <<= 1;
    const unsigned grid = blocks_for((int64_t)n * L);
#define SM_VEC(LL)                                                                        \
    case LL:                                                                              \
        hipLaunchKernelGGL(spmv_vector_kernel<LL>, dim3(grid), dim3(256), 0, s, n, rp, col, \
                           val, x, y, alpha, beta);                                        \
        break;
    switch (L) { SM_VEC(2) SM_VEC(4) SM_VEC(8) SM_VEC(16) SM_VEC(32) SM_VEC(64) }
#undef SM_VEC
    return hipGetLastError();
}

hipError_t launch_spmm_generic(int32_t n, int32_t nrhs, const int32_t *rp, const int32_t *col,
                               const float *val, const float *X, int64_t x_sk, int64_t x_si,
                               float *Y, int64_t y_sj, int64_t y_si, float alpha, float beta,
                               bool rhs_fastest, hipStream_t s) {
    const int64_t total = (int64_t)n * nrhs;
    if (total <= 0) return hipSuccess;
    if (rhs_fastest)
        hipLaunchKernelGGL(spmm_generic_kernel<true>, dim3(blocks_for(total)), dim3(256), 0, s, n,
                           nrhs, rp, col, val, X, x_sk, x_si, Y, y_sj, y_si, alpha, beta);
    else
        hipLaunchKernelGGL(spmm_generic_kernel<false>, dim3(blocks_for(total)), dim3(256), 0, s, n,
                           nrhs, rp, col, val, X, x_sk, x_si, Y, y_sj, y_si, alpha, beta);
    return hipGetLastError();
}

hipError_t launch_spmm_rowpanel(int32_t n, int32_t nrhs, const int32_t *rp, const int32_t *col,
                                const float *val, int32_t nnz, const float *X, int64_t ldx,
                                int64_t x_rows, float *Y, int64_t ldy, float alpha, float beta,
                                bool allow_pipelined, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int G = 1;
    while (4 * G < nrhs) G <<= 1;
    const unsigned grid = blocks_for((int64_t)n * G);
    // The gather-pipelined kernel while its X descriptor can span X (< 4 GiB) and a
    // group's gathers fit the registers (G <= 16, i.e. N <= 64); allow_pipelined =
    // false (sm_spmm with SM_ALGO_VECTOR) keeps the one-group-at-a-time kernel.
    const bool pipelined = allow_pipelined && G <= 16 &&
                           (uint64_t)x_rows * (uint64_t)ldx * 4u < 0xFFFFFFF0ull;
#define SM_PANEL(GG)                                                                         \
    case GG:                                                                                 \
        if (pipelined)                                                                       \
            hipLaunchKernelGGL(spmm_rowpanel2_kernel<(GG <= 16 ? GG : 16)>, dim3(grid), dim3(256), 0, s, \
                               n, nrhs, rp, col, val, nnz, X, ldx, x_rows, Y, ldy, alpha, beta); \
        else                                                                                 \
            hipLaunchKernelGGL(spmm_rowpanel_kernel<GG>, dim3(grid), dim3(256), 0, s, n, nrhs, rp, \
                               col, val, X, ldx, Y, ldy, alpha, beta);                        \
        break;
    switch (G) {
        SM_PANEL(1) SM_PANEL(2) SM_PANEL(4) SM_PANEL(8) SM_PANEL(16) SM_PANEL(32)
        default: return hipErrorInvalidValue;
    }
#undef SM_PANEL
    return hipGetLastError();
}

hipError_t launch_beta(float *c, int32_t m, int32_t n, int64_t ldc, float beta, hipStream_t s) {
    const int64_t total = (int64_t)m * n;
    if (total <= 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>(blocks_for(total), 256 * 16);
    hipLaunchKernelGGL(beta_kernel, dim3((unsigned)grid), dim3(256), 0, s, c, m, n, ldc, beta);
    return hipGetLastError();
}

hipError_t launch_transpose(const float *a, int32_t m, int32_t n, int64_t lda, float *sa,
                            int64_t ldsa, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    const int32_t tm = (m + 63) / 64, tn = (n + 63) / 64;
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((int64_t)tm * tn)), dim3(256), 0, s, a, m,
                       n, lda, sa, ldsa, tn);
    return hipGetLastError();
}

hipError_t launch_validate(int32_t n_rows, int32_t n_cols, int32_t nnz, const int32_t *rp,
                           const int32_t *col, int32_t *d_flag, hipStream_t s) {
    const int64_t n = std::max<int64_t>((int64_t)n_rows + 1, nnz);
    hipLaunchKernelGGL(validate_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1 << 16)), dim3(256), 0, s,
                       n_rows, n_cols, nnz, rp, col, d_flag);
    return hipGetLastError();
}

hipError_t launch_x_relabel(int64_t n, const int32_t *rank, const float *x, float *xp,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (((uintptr_t)x & 15) == 0)
        hipLaunchKernelGGL(x_relabel_kernel<true>, dim3(blocks_for((n + 3) / 4)), dim3(256), 0, s,
                           n, rank, x, xp);
    else
        hipLaunchKernelGGL(x_relabel_kernel<false>, dim3(blocks_for(n)), dim3(256), 0, s, n, rank,
                           x, xp);
    return hipGetLastError();
}

hipError_t launch_scatter_dense(int32_t n, const int32_t *rp, const int32_t *col,
                                const float *val, float *out, int64_t stride, bool b_layout,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_dense_kernel, dim3(blocks_for(n)), dim3(256), 0, s, n, rp, col, val,
                       out, stride, b_layout);
    return hipGetLastError();
}

}  // namespace smamd
