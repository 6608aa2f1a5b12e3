// spmm_mfma.hip -- SpMM Y = alpha * B * X + beta * Y with N = 32 right-hand sides on the
// matrix cores (SM_ALGO_MFMA; north_star: "MFMA used only on the dense N-panel of SpMM").
//
// One wavefront per tile of 16 consecutive rows.  The tile's terms (its CSR span, in
// stored order) are the K dimension of a dense product: term t is k-index t, so
//   A (16 x K):  A[i][t] = fl(v_t * alpha) when term t belongs to row i, else 0
//   B (K x 32):  B[t][:] = X[col_t][:]          (the X row the term gathers)
//   Y_tile = beta * Y_tile + A * B
// and v_mfma_f32_16x16x4_f32 takes four terms per step (K / 4 steps, two MFMAs each
// for the two 16-column halves of the panel).  Lane l holds A[l & 15][4j + (l >> 4)] and
// B[4j + (l >> 4)][l & 15] (cdna_hip_programming.md, the f32 16x16x4 operand map): the 16
// lanes of one term read its X row as 16 consecutive 8-byte pairs (one 128-byte line),
// half 0 taking the even columns and half 1 the odd ones; D/C rows 4 (l >> 4) + r,
// column l & 15 (the standard map).  Two forms: spmm_mfma_kernel takes the B operand
// straight from the gather into registers; spmm_mfma_lds_kernel (the one SM_ALGO_MFMA runs)
// stages the gathered X rows through LDS by LDS-DMA and reads the B operand back from there.
//
// Arithmetic: the f32 MFMA is an exact fma chain in k order (MI355X_MICROARCH.md: "exact
// f32 (= fmaf chain, bitwise)"), so each output is beta*y followed by fma(fl(v*alpha), x,
// acc) over its terms in stored order, plus fma(0, x, acc) for the tile's other rows'
// terms.  Against the reference's round(acc + round(x * fl(v * alpha))) that is one
// rounding per term instead of two: within 1e-6 * sum|terms|, not bit-identical (the
// row-panel kernels stay the bit-exact SpMM).  The zero entries multiply the other rows'
// X values, so a non-finite X row turns the tile's other outputs into NaN: finite X only;
// and they add fma(0, x, acc), which reads an accumulator of -0.0 (beta = 0 on a negative
// y, with no term of its own yet) as +0.0 -- the one bit pattern that differs from the chain.
// The A matrix is 1/16 dense (16 rows share a step's four terms), so the matrix cores do
// 16x the useful flops -- at about 2 flop per byte the SpMM has flops to spare, and the
// question this kernel answers is whether the gather stream runs any
// faster when its arithmetic moves off the vector ALUs.
#include "sm_internal.h"
#include "xband_dev.h"

#include <cstdlib>

namespace smamd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int U>   // k-steps whose loads are in flight together
__global__ __launch_bounds__(256) void spmm_mfma_kernel(
    int32_t n, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, int32_t nnz, const float *__restrict__ X, int64_t ldx,
    int64_t x_rows, float *__restrict__ Y, int64_t ldy, float alpha, float beta) {
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    const int lane = threadIdx.x & 63;
    const int32_t r0 = (int32_t)((((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16);
    if (r0 >= n) return;   // whole wavefronts
    const int m = lane & 15, kq = lane >> 4;
    // This lane's A row (row r0 + m): its terms are [lo, hi).
    const int32_t lo = rp[min(r0 + m, n)], hi = rp[min(r0 + m + 1, n)];
    const int32_t t0 = rp[r0], t1 = rp[min(r0 + 16, n)];
    // Accumulators: D rows 4 kq + r, column m of each half (output columns 2m, 2m + 1).
    f32x4 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t row = r0 + 4 * kq + r;
        float2 yv = make_float2(0.f, 0.f);
        if (row < n) yv = *reinterpret_cast<const float2 *>(Y + (int64_t)row * ldy + 2 * m);
        if (beta != 1.0f) yv = make_float2(__fmul_rn(yv.x, beta), __fmul_rn(yv.y, beta));
        acc0[r] = yv.x;
        acc1[r] = yv.y;
    }
    const __amdgpu_buffer_rsrc_t c_src = rsrc(col, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t v_src = rsrc(val, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t x_src = rsrc(X, (uint64_t)x_rows * ldx * 4);
    for (int32_t tb = t0; tb < t1; tb += 4 * U) {
        float a[U];
        u32x2 b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {   // every load of the U steps in flight at once
            const int32_t t = tb + 4 * u + kq;
            const uint32_t off = t < t1 ? 4u * (uint32_t)t : kOob;
            const int32_t c = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(c_src, off, 0, 0);
            const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_src, off, 0, 0));
            a[u] = (t >= lo && t < hi) ? __fmul_rn(v, alpha) : 0.0f;
            const uint32_t xo = t < t1 ? 4u * (uint32_t)((int64_t)c * ldx + 2 * m) : kOob;
            b[u] = __builtin_amdgcn_raw_buffer_load_b64(x_src, xo, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], __uint_as_float(b[u].x), acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], __uint_as_float(b[u].y), acc1, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t row = r0 + 4 * kq + r;
        if (row < n)
            *reinterpret_cast<float2 *>(Y + (int64_t)row * ldy + 2 * m) = make_float2(acc0[r], acc1[r]);
    }
}

// The same product with the gathered X rows staged through LDS: per wave, the 4U X rows of a
// chunk of 4U terms go L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds: 64 lanes x 16 B =
// eight 128-byte rows per instruction, lane l taking piece l & 7 of row l >> 3), into one of
// two buffers, while the previous chunk's rows are read back as the MFMA B operand
// (ds_read_b64: lane l reads B[4u + (l >> 4)][2 (l & 15) .. + 1], 16 lanes on one row's
// consecutive 8-byte pairs -- conflict-free).  The gather needs no VGPRs and its latency
// overlaps the previous chunk's MFMAs; the operands and their order are the register form's,
// so the results are bit-identical to it.  Needs ldx % 4 == 0 and a 16-byte aligned X.
template <int U>
__global__ __launch_bounds__(256) void spmm_mfma_lds_kernel(
    int32_t n, const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
    const float *__restrict__ val, int32_t nnz, const float *__restrict__ X, int64_t ldx,
    int64_t x_rows, float *__restrict__ Y, int64_t ldy, float alpha, float beta) {
    static_assert(U % 2 == 0, "whole DMA instructions (eight rows each) per chunk");
    constexpr int kT = 4 * U;   // terms per chunk
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    __shared__ __attribute__((aligned(16))) float panel[4][2][kT][32];   // per wave: two chunks of rows
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int32_t r0 = (int32_t)((((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 16);
    if (r0 >= n) return;   // whole wavefronts
    const int m = lane & 15, kq = lane >> 4;
    const int32_t lo = rp[min(r0 + m, n)], hi = rp[min(r0 + m + 1, n)];
    const int32_t t0 = rp[r0], t1 = rp[min(r0 + 16, n)];
    f32x4 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t row = r0 + 4 * kq + r;
        float2 yv = make_float2(0.f, 0.f);
        if (row < n) yv = *reinterpret_cast<const float2 *>(Y + (int64_t)row * ldy + 2 * m);
        if (beta != 1.0f) yv = make_float2(__fmul_rn(yv.x, beta), __fmul_rn(yv.y, beta));
        acc0[r] = yv.x;
        acc1[r] = yv.y;
    }
    const __amdgpu_buffer_rsrc_t c_src = rsrc(col, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t v_src = rsrc(val, (uint64_t)nnz * 4);
    const __amdgpu_buffer_rsrc_t x_src = rsrc(X, (uint64_t)x_rows * ldx * 4);
    const uint32_t pl = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&panel[wv][0][0][0];
    // Values of step u's terms of the chunk at tb (raw: the A operand is formed at use, so
    // hipcc need not wait for these loads before the next ones go out).
    auto load_v = [&](int32_t tb, float *v) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = tb + 4 * u + kq;
            v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_src, t < t1 ? 4u * (uint32_t)t : kOob, 0, 0));
        }
    };
    // The chunk's X rows into buffer buf: instruction i moves rows 8i .. 8i + 7 (past t1: zeros).
    // Column loads first, then the chunk's value loads, then the DMAs: their wait for the
    // columns leaves the value loads in flight.
    auto gather = [&](int32_t tb, int buf, float *v) {
        int32_t c[U / 2];
#pragma unroll
        for (int i = 0; i < U / 2; ++i) {
            const int32_t t = tb + 8 * i + (lane >> 3);
            c[i] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(c_src, t < t1 ? 4u * (uint32_t)t : kOob, 0, 0);
        }
        load_v(tb, v);
#pragma unroll
        for (int i = 0; i < U / 2; ++i) {
            const int32_t t = tb + 8 * i + (lane >> 3);
            // 32-bit offsets (the launcher keeps X under 4 GiB) and a select, not a branch: a
            // branch here makes hipcc drain vmcnt inside it
            const uint32_t xc = 4u * ((uint32_t)c[i] * (uint32_t)ldx + 4u * (uint32_t)(lane & 7));
            const uint32_t xo = t < t1 ? xc : kOob;
            const uint32_t lds = __builtin_amdgcn_readfirstlane(pl + 4u * (uint32_t)((buf * kT + 8 * i) * 32));
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(xo), "s"(x_src), "s"(lds)
                : "memory");
        }
    };
    // Static two-chunk ring (buffers and value registers by step parity) and unconditional
    // gathers -- past t1 they are out-of-range loads (no memory request, zeros into a buffer
    // nobody reads): a branch around a load or a ring register makes hipcc copy registers and
    // drain vmcnt.
    float v[2][U];
    auto consume = [&](int32_t tb, int b, const float *vv) {
        const float *pb = &panel[wv][b][0][0];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = tb + 4 * u + kq;
            const float a = (t >= lo && t < hi) ? __fmul_rn(vv[u], alpha) : 0.0f;
            const float2 bv = *reinterpret_cast<const float2 *>(pb + (4 * u + kq) * 32 + 2 * m);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.y, acc1, 0, 0, 0);
        }
    };
    gather(t0, 0, v[0]);
    for (int32_t tb = t0; tb < t1; tb += 2 * kT) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int32_t tc = tb + p * kT;
            gather(tc + kT, p ^ 1, v[p ^ 1]);   // the next chunk goes out first
            // chunk tc's rows have landed (in-order retirement: the next chunk's U / 2 column
            // loads, U value loads and U / 2 DMAs may stay in flight)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * U) : "memory");
            if (tc < t1) consume(tc, p, v[p]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the wave
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t row = r0 + 4 * kq + r;
        if (row < n)
            *reinterpret_cast<float2 *>(Y + (int64_t)row * ldy + 2 * m) = make_float2(acc0[r], acc1[r]);
    }
}

}  // namespace

hipError_t launch_spmm_mfma(int32_t n, const int32_t *rp, const int32_t *col, const float *val,
                            int32_t nnz, const float *X, int64_t ldx, int64_t x_rows, float *Y,
                            int64_t ldy, float alpha, float beta, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if ((uint64_t)x_rows * (uint64_t)ldx * 4u >= 0xFFFFFFF0ull || ldx % 2 || ldy % 2 ||
        ((uintptr_t)X % 8) || ((uintptr_t)Y % 8))
        return hipErrorInvalidValue;
    const int64_t waves = ((int64_t)n + 15) / 16;
    const unsigned grid = (unsigned)((waves + 3) / 4);   // 4 wavefronts per 256-thread block
    bool lds = ldx % 4 == 0 && (uintptr_t)X % 16 == 0;
#ifdef SM_DEV
    if (const char *e = dev_env("SM_SPMM_MFMA_LDS")) lds = lds && atoi(e) != 0;   // A/B
#endif
    if (lds)
        hipLaunchKernelGGL(spmm_mfma_lds_kernel<8>, dim3(grid), dim3(256), 0, s, n, rp, col, val, nnz, X, ldx,
                           x_rows, Y, ldy, alpha, beta);
    else
        hipLaunchKernelGGL(spmm_mfma_kernel<8>, dim3(grid), dim3(256), 0, s, n, rp, col, val, nnz, X, ldx,
                           x_rows, Y, ldy, alpha, beta);
    return hipGetLastError();
}

}  // namespace smamd
