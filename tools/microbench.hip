// tools/microbench.hip -- calibration kernels for the SpMV roofline on MI355X.
//   copy      : float4 stream read + write (achievable HBM rate)
//   read      : float4 stream read only
//   gather T  : stream an int32 index array (16.7M) + gather 4-byte values
//               from a table of T bytes (the x-vector access of SpMV)
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o build/microbench
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

__global__ void copy_kernel(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ void read_kernel(const float4 *__restrict__ a, size_t n, float *out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// each thread: 4 consecutive indices (int4), 4 gathers, accumulate
__global__ void gather_kernel(const int4 *__restrict__ idx, size_t n4, const float *__restrict__ t,
                              float *out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x) {
        int4 c = idx[i];
        s += t[c.x] + t[c.y] + t[c.z] + t[c.w];
    }
    if (s == 1234.5f) out[0] = s;
}

// 16 gathers in flight per thread
__global__ void gather16_kernel(const int4 *__restrict__ idx, size_t n4, const float *__restrict__ t,
                                float *out) {
    float s = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += 4 * stride) {
        int4 c[4];
#pragma unroll
        for (int k = 0; k < 4; k++) c[k] = (i + k * stride < n4) ? idx[i + k * stride] : make_int4(0, 0, 0, 0);
        float v[16];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[4 * k] = t[c[k].x]; v[4 * k + 1] = t[c[k].y]; v[4 * k + 2] = t[c[k].z]; v[4 * k + 3] = t[c[k].w];
        }
#pragma unroll
        for (int k = 0; k < 16; k++) s += v[k];
    }
    if (s == 1234.5f) out[0] = s;
}

// LDS gather: table slice of `te` floats staged in LDS, random indices streamed
template <int TE>
__global__ __launch_bounds__(1024) void lds_gather_kernel(const int4 *__restrict__ idx, size_t n4,
                                                          const float *__restrict__ t, float *out) {
    __shared__ float tab[TE];
    for (int i = threadIdx.x; i < TE; i += blockDim.x) tab[i] = t[i];
    __syncthreads();
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x) {
        int4 c = idx[i];
        s += tab[c.x & (TE - 1)] + tab[c.y & (TE - 1)] + tab[c.z & (TE - 1)] + tab[c.w & (TE - 1)];
    }
    if (s == 1234.5f) out[0] = s;
}

// LDS read-modify-write at random rows (the y-accumulator update)
template <int TE>
__global__ __launch_bounds__(1024) void lds_rmw_kernel(const int4 *__restrict__ idx, size_t n4,
                                                       float *out) {
    __shared__ float acc[TE];
    for (int i = threadIdx.x; i < TE; i += blockDim.x) acc[i] = 0;
    __syncthreads();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x) {
        int4 c = idx[i];
        atomicAdd(&acc[c.x & (TE - 1)], 1.0f);
        atomicAdd(&acc[c.y & (TE - 1)], 1.0f);
        atomicAdd(&acc[c.z & (TE - 1)], 1.0f);
        atomicAdd(&acc[c.w & (TE - 1)], 1.0f);
    }
    __syncthreads();
    if (acc[threadIdx.x] == 1234.5f) out[0] = 1;
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float *out;
    CK(hipMalloc(&out, 4));
    auto timeit = [&](auto fn, int reps) {
        fn();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < reps; r++) {
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
    // --- stream copy / read, 1 GiB
    const size_t n = (size_t)1 << 26;   // float4 -> 1 GiB
    float4 *a, *b;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMemset(a, 0, n * 16));
    const int grid = 256 * 16;
    float ms = timeit([&] { hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, a, b, n); }, 10);
    printf("copy      1 GiB: %.3f ms  %.1f GB/s (read+write)\n", ms, 2.0 * n * 16 / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, a, n, out); }, 10);
    printf("read      1 GiB: %.3f ms  %.1f GB/s\n", ms, 1.0 * n * 16 / ms / 1e6);
    // --- gathers
    const size_t ng = (size_t)1 << 24;   // 16.7M gathers
    std::vector<int> hidx(ng);
    float *tab;
    CK(hipMalloc(&tab, (size_t)256 << 20));
    CK(hipMemset(tab, 0, (size_t)256 << 20));
    int4 *didx;
    CK(hipMalloc(&didx, ng * 4));
    for (size_t T : {(size_t)64 << 10, (size_t)1 << 20, (size_t)4 << 20, (size_t)16 << 20,
                     (size_t)64 << 20, (size_t)256 << 20}) {
        const size_t te = T / 4;
        srand(1);
        for (size_t i = 0; i < ng; i++) hidx[i] = (int)(((size_t)rand() * 2654435761u + rand()) % te);
        CK(hipMemcpy(didx, hidx.data(), ng * 4, hipMemcpyHostToDevice));
        ms = timeit([&] { hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, 0, didx, ng / 4, tab, out); }, 10);
        float ms16 = timeit([&] { hipLaunchKernelGGL(gather16_kernel, dim3(grid), dim3(256), 0, 0, didx, ng / 4, tab, out); }, 10);
        printf("gather table %7zu KiB: 16.7M gathers %.3f ms (%.2f Ggather/s)  16-in-flight %.3f ms (%.2f Ggather/s)\n",
               T >> 10, ms, ng / ms / 1e6, ms16, ng / ms16 / 1e6);
    }
    // LDS gathers (the table slice lives in LDS; one 1024-thread block per CU)
    {
        srand(1);
        for (size_t i = 0; i < ng; i++) hidx[i] = (int)(((size_t)rand() * 2654435761u + rand()) & 0xffffff);
        CK(hipMemcpy(didx, hidx.data(), ng * 4, hipMemcpyHostToDevice));
        ms = timeit([&] { hipLaunchKernelGGL(lds_gather_kernel<32768>, dim3(256), dim3(1024), 0, 0, didx, ng / 4, tab, out); }, 10);
        printf("LDS gather (128 KiB slice, 256 x 1024 thr): %.3f ms (%.2f Ggather/s)\n", ms, ng / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(lds_gather_kernel<16384>, dim3(512), dim3(1024), 0, 0, didx, ng / 4, tab, out); }, 10);
        printf("LDS gather (64 KiB slice, 512 x 1024 thr): %.3f ms (%.2f Ggather/s)\n", ms, ng / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(lds_rmw_kernel<4096>, dim3(256), dim3(1024), 0, 0, didx, ng / 4, out); }, 10);
        printf("LDS atomicAdd f32 (16 KiB acc): %.3f ms (%.2f Gop/s)\n", ms, ng / ms / 1e6);
    }
    // windowed gathers: each wave-instruction's 64 addresses fall in one random W-byte window
    // of a T-byte table (column-sorted entries of a band: ~8 entries per 128-byte line at W = 1 KiB)
    for (size_t T : {(size_t)1 << 20, (size_t)4 << 20}) {
        for (size_t W : {(size_t)512, (size_t)1024, (size_t)2048, (size_t)4096}) {
            const size_t te = T / 4, we = W / 4;
            srand(2);
            // gather_kernel: wave-instruction j of wave block b reads idx[4*(64*b + l) + j], l < 64
            for (size_t b = 0; b < ng / 256; b++)
                for (int j = 0; j < 4; j++) {
                    const size_t base = ((size_t)rand() * 2654435761u) % (te - we);
                    for (int l = 0; l < 64; l++) hidx[4 * (64 * b + l) + j] = (int)(base + (size_t)rand() % we);
                }
            CK(hipMemcpy(didx, hidx.data(), ng * 4, hipMemcpyHostToDevice));
            ms = timeit([&] { hipLaunchKernelGGL(gather16_kernel, dim3(grid), dim3(256), 0, 0, didx, ng / 4, tab, out); }, 10);
            printf("windowed gather table %5zu KiB window %5zu B: %.3f ms (%.2f Ggather/s)\n", T >> 10, W, ms, ng / ms / 1e6);
        }
    }
    // sequential "gather" (idx[i] = i) for reference
    for (size_t i = 0; i < ng; i++) hidx[i] = (int)i;
    CK(hipMemcpy(didx, hidx.data(), ng * 4, hipMemcpyHostToDevice));
    ms = timeit([&] { hipLaunchKernelGGL(gather16_kernel, dim3(grid), dim3(256), 0, 0, didx, ng / 4, tab, out); }, 10);
    printf("sequential idx (64 MiB table): %.3f ms (%.2f Ggather/s)\n", ms, ng / ms / 1e6);
    return 0;
}
