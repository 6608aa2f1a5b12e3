// kernels_sweep.hip -- SpMV over the column-swept row blocks (sweep.h, sweep.cpp).
//
// One wavefront per block of kSwRows rows, its accumulators (beta * y to start) and the
// codebook fl(table[id] * alpha) in LDS.  It walks the block's chunks in order -- they
// ascend in column, so all the grid's wavefronts move across x together and their x
// gathers hit lines the others just pulled into L2 -- four at a time: the four chunks'
// 8-byte slots were loaded during the previous group, their x values are gathered
// (range-checked buffer loads), then each chunk is applied: term = x * fl(v * alpha),
// a row's segment summed up its lanes in column order by DPP rounds on SGPR lane masks
// (as in the cband kernel), the segment's last lane writing the row's accumulator.  No
// barrier after the set-up and no other workgroup involved, so no hand-off: each row is
// summed in the reference's order (kernel.cc:780-796, 791), bit for bit.
#include "sm_internal.h"
#include "sweep.h"
#include "xband_dev.h"

namespace smamd {
namespace {

constexpr int kSwGroup = 4;   // chunks per group (their slots prefetched a group ahead)

__global__ __launch_bounds__(64) void spmv_sweep_kernel(
    int32_t n_rows, int32_t n_cols, const int64_t *__restrict__ block_chunk,
    const uint2 *__restrict__ ent, const float *__restrict__ table, int32_t table_size,
    const float *__restrict__ x, float *__restrict__ y, float alpha, float beta) {
    __shared__ float tab[256];
    __shared__ float yacc[kSwRows];
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int64_t r0 = b * kSwRows;
    const int32_t nr = (int32_t)min((int64_t)kSwRows, (int64_t)n_rows - r0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int t = lane + 64 * k;
        tab[t] = t < table_size ? __fmul_rn(table[t], alpha) : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < kSwRows / 64; ++k) {   // beta * y (kernel.cc:10-29: only when beta != 1)
        const int i = lane + 64 * k;
        float v = 0.0f;
        if (i < nr) {
            v = y[r0 + i];
            if (beta != 1.0f) v = __fmul_rn(v, beta);
        }
        yacc[i] = v;
    }
    __syncthreads();
    const int64_t c0 = block_chunk[b], c1 = block_chunk[b + 1];
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x, (uint64_t)n_cols * 4);
    auto shr1 = [](float v) {   // lane i <- lane i-1
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto sel = [](uint64_t m, float a, float bb) -> float {   // lane i: bit i of m ? bb : a
        float r;
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(bb), "s"(m));
        return r;
    };
    auto load_group = [&](int64_t c, uint2 *e) {
#pragma unroll
        for (int u = 0; u < kSwGroup; ++u) {
            const int64_t cc = min(c + u, c1 - 1);   // past the block: a real slot, not applied
            e[u] = ent[cc * 64 + lane];
        }
    };
    uint2 en[kSwGroup];
    if (c0 < c1) load_group(c0, en);
    for (int64_t c = c0; c < c1; c += kSwGroup) {
        uint2 e[kSwGroup];
        float xv[kSwGroup];
#pragma unroll
        for (int u = 0; u < kSwGroup; ++u) {
            e[u] = en[u];
            xv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(x_src, 4u * e[u].x, 0, 0));
        }
        if (c + kSwGroup < c1) load_group(c + kSwGroup, en);   // the next group's slots fly meanwhile
#pragma unroll
        for (int u = 0; u < kSwGroup; ++u) {
            if (c + u >= c1) break;   // wave-uniform
            const uint32_t meta = e[u].y;
            const uint32_t id = (meta >> 16) & 0xFFu;
            const uint32_t row = meta & 0xFFFu;
            const bool live = id != kSwDummyId;
            const uint64_t cont = __ballot((meta & kSwContBit) != 0);
            const float tm = __fmul_rn(xv[u], tab[id]);
            float acc = __fadd_rn(yacc[row], tm);
            for (uint64_t R = cont & ~(cont << 1); R; R = cont & (R << 1))
                acc = sel(R, acc, __fadd_rn(shr1(acc), tm));
            const uint64_t last = __ballot(live) & ~(cont >> 1);
            if ((last >> lane) & 1) yacc[row] = acc;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSwRows / 64; ++k) {
        const int i = lane + 64 * k;
        if (i < nr) y[r0 + i] = yacc[i];
    }
}

}  // namespace

hipError_t launch_spmv_sweep(const SweepDev &sd, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (sd.n_blocks <= 0) return hipSuccess;
    if (!sd.d_block_chunk || !sd.d_table || (sd.n_chunks > 0 && !sd.d_ent) || sd.table_size < 0 ||
        sd.table_size > 255 || sd.n_blocks > 0x7FFFFFFF)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(spmv_sweep_kernel, dim3((unsigned)sd.n_blocks), dim3(64), 0, s, n_rows, n_cols,
                       sd.d_block_chunk, reinterpret_cast<const uint2 *>(sd.d_ent), sd.d_table,
                       sd.table_size, x, y, alpha, beta);
    return hipGetLastError();
}

}  // namespace smamd
