// rowgather.hip -- the floor under config 3's SpMM (VERDICT r2 "show the floor"):
// 2^20 output rows x 16 random distinct columns, each term gathering one 128-byte row
// of X (2^20 x 32 fp32 = 128 MiB), 8 lanes per output row holding a float4 of it,
// exactly the access pattern of spmm_rowpanel2_kernel<8> (kernels.hip) without its
// arithmetic order, codebook and beta -- so its time is what the gathers alone cost.
// Variants (each over 4 rotating replicas of the index stream / X / Y so the working
// set exceeds the 256 MiB Infinity Cache, like bench.py):
//   idx     the index stream alone (64 MiB of int32 column ids, 16 per row)
//   gather  + the 16.7M X-row gathers, summed per lane, one float4 per lane stored
//   full    + Y read and written (beta * Y + sum), the SpMM's whole traffic
//   sorted  full, with the output rows visited in an order that groups rows sharing
//           X rows onto one XCD? -- not possible for uniform columns; instead the
//           columns are made XCD-local (bucketed by column % 8 == xcd) to show what
//           L2 reuse would buy (an upper bound, not a layout the matrix has)
// Build: hipcc --offload-arch=gfx950 -O3 tools/rowgather.hip -o build/rowgather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr int kRows = 1 << 20, kCols = 1 << 20, kPer = 16, kN = 32, kG = kN / 4;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// Column ids: 16 per row; mode 1 puts row r's columns on XCD-local X rows (c % 8 == r % 8
// after the workgroup -> XCD round robin: rows of workgroup b map to XCD b % 8).
__global__ void make_idx(int32_t *idx, uint32_t seed, int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)kRows * kPer) return;
    uint32_t c = hash32((uint32_t)i * 2654435761u + seed) & (kCols - 1);
    if (mode == 1) {
        const int64_t r = i / kPer;
        const int32_t wg = (int32_t)(r * kG / 256);   // 256-thread workgroups, kG lanes per row
        c = (c & ~7u) | (uint32_t)(wg & 7);
    }
    idx[i] = (int32_t)c;
}

template <int MODE>   // 0 idx only, 1 gather, 2 full
__global__ __launch_bounds__(256) void rowgather(const int32_t *__restrict__ idx,
                                                 const float4 *__restrict__ X,
                                                 float4 *__restrict__ Y, float beta) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = t / kG;
    const int g = (int)(t % kG);
    if (r >= kRows) return;
    const int4 *ip = reinterpret_cast<const int4 *>(idx + r * kPer);
    int4 c4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c4[k] = ip[k];
    const int32_t c[16] = {c4[0].x, c4[0].y, c4[0].z, c4[0].w, c4[1].x, c4[1].y, c4[1].z, c4[1].w,
                           c4[2].x, c4[2].y, c4[2].z, c4[2].w, c4[3].x, c4[3].y, c4[3].z, c4[3].w};
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 0) {
        int s = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) s += c[k];
        acc.x = (float)s;
    } else {
        float4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = X[(int64_t)c[k] * kG + g];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
        }
    }
    float4 *yp = Y + r * kG + g;
    if (MODE == 2) {
        const float4 y = *yp;
        acc.x += beta * y.x; acc.y += beta * y.y; acc.z += beta * y.z; acc.w += beta * y.w;
    }
    *yp = acc;
}

int main() {
    const int R = 4;
    std::vector<int32_t *> idx(R), idx_local(R);
    std::vector<float4 *> X(R), Y(R);
    const size_t ni = (size_t)kRows * kPer;
    for (int k = 0; k < R; ++k) {
        CK(hipMalloc(&idx[k], ni * 4));
        CK(hipMalloc(&idx_local[k], ni * 4));
        CK(hipMalloc(&X[k], (size_t)kCols * kN * 4));
        CK(hipMalloc(&Y[k], (size_t)kRows * kN * 4));
        CK(hipMemset(X[k], 0, (size_t)kCols * kN * 4));
        CK(hipMemset(Y[k], 0, (size_t)kRows * kN * 4));
        hipLaunchKernelGGL(make_idx, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, 0, idx[k], 17u + k, 0);
        hipLaunchKernelGGL(make_idx, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, 0, idx_local[k], 17u + k, 1);
    }
    CK(hipDeviceSynchronize());
    const unsigned grid = (unsigned)(((int64_t)kRows * kG + 255) / 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *name, int mode, bool local) {
        for (int w = 0; w < 3; ++w) {   // warm
            const int k = w % R;
            int32_t *ix = local ? idx_local[k] : idx[k];
            if (mode == 0) hipLaunchKernelGGL(rowgather<0>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
            if (mode == 1) hipLaunchKernelGGL(rowgather<1>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
            if (mode == 2) hipLaunchKernelGGL(rowgather<2>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
        }
        const int reps = 40;
        CK(hipEventRecord(a, 0));
        for (int it = 0; it < reps; ++it) {
            const int k = it % R;
            int32_t *ix = local ? idx_local[k] : idx[k];
            if (mode == 0) hipLaunchKernelGGL(rowgather<0>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
            if (mode == 1) hipLaunchKernelGGL(rowgather<1>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
            if (mode == 2) hipLaunchKernelGGL(rowgather<2>, dim3(grid), dim3(256), 0, 0, ix, X[k], Y[k], 0.5f);
        }
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        const double bytes = 4.0 * ni + (mode >= 1 ? 128.0 * ni : 0) + (mode == 2 ? 2.0 : 1.0) * kRows * kN * 4;
        printf("%-34s %8.1f us  %7.1f GB/s moved (idx + X rows + Y)\n", name, ms * 1e3, bytes / ms / 1e6);
    };
    run("idx stream + Y store", 0, false);
    run("gather 16.7M x 128 B rows", 1, false);
    run("full: gather + Y read/write", 2, false);
    run("full, XCD-local columns (bound)", 2, true);
    return 0;
}
