// tools/ta_bench.hip -- per-CU vector-memory issue cost on MI355X (development).
// One 1024-thread workgroup per CU (256), every wave issues ITERS x 8 buffer loads
// of one kind, 8 in flight; prints ns per wave-instruction per CU and GB/s.
// Question it answers: is the cost of a load per instruction (address processing)
// or per byte (cache/fabric)?  Kinds: L2-resident dword/dwordx2/dwordx4, the same
// with the descriptor range 0 (no memory request), HBM streaming dword/dwordx4,
// LDS-DMA dwordx4 from L2, and mixes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ta_bench.hip -o build/ta_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes,
                                             0x00020000);
}

// KIND: 1 dword, 2 dwordx2, 4 dwordx4 (register loads); 8 LDS-DMA dwordx4;
// 9: one LDS-DMA dwordx4 + 2 dword loads per step (the SpMV band mix).
// WS: bytes of the window each workgroup walks (L2-resident when small).
template <int KIND>
__global__ __launch_bounds__(1024) void ta_kernel(const float *buf, uint32_t range, uint64_t ws,
                                                  int iters, float *out, int hbm) {
    __shared__ __attribute__((aligned(16))) float lds[16 * 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float *base = buf + (hbm ? (uint64_t)blockIdx.x * (ws / 4) : 0);
    const __amdgpu_buffer_rsrc_t r = rsrc(base, range);
    constexpr int W = KIND == 8 || KIND == 9 ? 16 : KIND * 4;   // bytes per lane
    uint32_t off = (uint32_t)((wave * 64 + lane) * W);
    const uint32_t step = 16u * 64u * W;                       // all 16 waves, one instr each
    const uint32_t wrap = (uint32_t)ws;
    float s = 0.f;
    const uint32_t lds_base = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&lds[0];
    for (int it = 0; it < iters; ++it) {
        if constexpr (KIND == 1) {
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                v[k] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
                off += step; off = off >= wrap ? off - wrap : off;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) s += __uint_as_float(v[k]);
        } else if constexpr (KIND == 2) {
            u32x2 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                v[k] = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
                off += step; off = off >= wrap ? off - wrap : off;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) s += __uint_as_float(v[k].x) + __uint_as_float(v[k].y);
        } else if constexpr (KIND == 4) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
                off += step; off = off >= wrap ? off - wrap : off;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) s += __uint_as_float(v[k].x) + __uint_as_float(v[k].w);
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t lds = __builtin_amdgcn_readfirstlane(
                    lds_base + 4u * (uint32_t)(((wave * 8 + k) & 15) * 1024));
                uint32_t keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                    "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(off), "s"(r), "s"(lds)
                    : "memory");
                off += step; off = off >= wrap ? off - wrap : off;
            }
            if constexpr (KIND == 9) {
                uint32_t v[16];
                uint32_t o2 = off >> 2;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    v[k] = __builtin_amdgcn_raw_buffer_load_b32(r, o2, 0, 0);
                    o2 += 4096;
                    o2 = o2 >= wrap ? o2 - wrap : o2;
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) s += __uint_as_float(v[k]);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    if (s == 1234.5f) out[threadIdx.x] = s + lds[threadIdx.x];
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float *out;
    CK(hipMalloc(&out, 4096 * 4));
    const size_t big = (size_t)1 << 30;
    float *buf;
    CK(hipMalloc(&buf, big));
    CK(hipMemset(buf, 0, big));
    auto timeit = [&](auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 7; r++) {
            CK(hipEventRecord(e0, 0));
            fn();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    };
    const int grid = 256;
    auto run = [&](const char *name, auto kern, int width, uint32_t range, uint64_t ws, int iters,
                   int hbm, int instr_per_iter) {
        float ms = timeit([&] {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), 0, 0, buf, range, ws, iters, out, hbm);
        });
        const double instr_per_cu = 16.0 * iters * instr_per_iter;
        const double bytes = 256.0 * instr_per_cu * 64 * width;
        printf("%-34s %8.3f ms  %6.2f ns/instr/CU  %8.1f GB/s (%s)\n", name, ms,
               ms * 1e6 / instr_per_cu, bytes / ms / 1e6, range ? "requests" : "no request");
    };
    const uint32_t l2 = 1u << 20;   // 1 MiB window: L2-resident (shared by all CUs)
    run("L2 dword", ta_kernel<1>, 4, l2, l2, 256, 0, 8);
    run("L2 dwordx2", ta_kernel<2>, 8, l2, l2, 128, 0, 8);
    run("L2 dwordx4", ta_kernel<4>, 16, l2, l2, 64, 0, 8);
    run("OOR dword", ta_kernel<1>, 4, 0, l2, 256, 0, 8);
    run("OOR dwordx4", ta_kernel<4>, 16, 0, l2, 64, 0, 8);
    run("L2 LDS-DMA dwordx4", ta_kernel<8>, 16, l2, l2, 64, 0, 8);
    const uint64_t per_cu = big / 256;   // 4 MiB per CU, streamed once
    run("HBM dword (4 MiB/CU)", ta_kernel<1>, 4, (uint32_t)per_cu, per_cu, 128, 1, 8);
    run("HBM dwordx4 (4 MiB/CU)", ta_kernel<4>, 16, (uint32_t)per_cu, per_cu, 32, 1, 8);
    run("HBM LDS-DMA dwordx4 (4 MiB/CU)", ta_kernel<8>, 16, (uint32_t)per_cu, per_cu, 32, 1, 8);
    run("L2 LDS-DMA x4 + 2 dword/step", ta_kernel<9>, 16, l2, l2, 64, 0, 8);
    return 0;
}
