// tools/xstream.hip -- the cband kernel's memory path alone (no apply): how fast can one
// CU stream its 1 MiB slab of x from L2 into LDS windows, beside the entry stream from HBM,
// with one barrier per window?  DESIGN.md §3.4b / §7 item 1.
//
// One 1024-thread workgroup per CU (256), tile t reads slab t % 4 of a 4 MiB x (the
// config-2 geometry: 64 row blocks x 4 slabs) in windows of W KiB, NBUF = A + 1 LDS
// buffers, window q + A issued at band q.  Variants (template):
//   NLD > 0: NLD loader waves (the last ones) issue the LDS-DMA pieces, the other waves
//            load 8 B of entries per lane per band, AE bands ahead (dma3 = NLD 1, W 30, A 2)
//   NLD = 0: every wave issues W / 16 pieces of the window and its entry load (DMA first)
//   E = 0  : no entry stream
// Build: hipcc --offload-arch=gfx950 -O3 tools/xstream.hip -o build/xstream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint64_t bytes) {
    const uint32_t n = bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)n, 0x00020000);
}

constexpr int kSlabBytes = 1 << 20;

// One LDS read that hipcc cannot turn into a flat load (a volatile LDS pointer becomes a
// flat_load, counted in vmcnt, and hipcc then drains vmcnt(0) before it).
__device__ __forceinline__ uint32_t lds_touch(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
constexpr int kLdsBytes = 160 * 1024;

// One 1 KiB piece of x (byte offset voff per lane) into LDS at lds (wave-uniform).
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t src, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(src), "s"(lds)
        : "memory");
}

template <int NLD, int WK, int A, int AE, bool E, int CS = 0, int EP = 2>
__global__ __launch_bounds__(1024) void xstream_kernel(const float *__restrict__ x,
                                                       const uint32_t *__restrict__ ent,
                                                       uint32_t *__restrict__ out) {
    constexpr int NBUF = A + 1;
    constexpr int W = WK * 1024;   // window bytes
    static_assert(NBUF * W <= kLdsBytes, "LDS");
    constexpr int NB = (kSlabBytes + W - 1) / W;   // bands per tile
    constexpr int PIECES = WK;                     // 1 KiB pieces per window
    constexpr int NAPPLY = NLD > 0 ? 16 - NLD : 16;
    constexpr int PPL = NLD > 0 ? (PIECES + NLD - 1) / NLD : (PIECES + 15) / 16;   // pieces per issuing wave
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slab = blockIdx.x & 3;
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x + (size_t)slab * (kSlabBytes / 4), kSlabBytes);
    const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)&lds[0];
    // entries: tile-private, 8 B per lane of each applying wave per band
    constexpr uint32_t kBandEnt = 8u * 64u * NAPPLY;
    const __amdgpu_buffer_rsrc_t e_src = rsrc(ent + (size_t)blockIdx.x * (kBandEnt / 4) * NB, (uint64_t)kBandEnt * NB);
    auto load_e = [&](int q) -> u32x2 {
        const uint32_t off = (E && wid < NAPPLY && q < NB) ? kBandEnt * (uint32_t)q + 8u * (uint32_t)tid : 0xFFFFFFF0u;
        u32x2 v;   // asm: hipcc tracks no load here, so it inserts no vmcnt drains of its own
        if constexpr (EP == 2)
            asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(e_src) : "memory");
        else if constexpr (EP == 1)
            asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen sc0" : "=v"(v) : "v"(off), "s"(e_src) : "memory");
        else if constexpr (EP == 3)
            asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen sc0 sc1" : "=v"(v) : "v"(off), "s"(e_src) : "memory");
        else
            asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(e_src) : "memory");
        return v;
    };
    // wait until only N younger vector-memory ops are pending, then use v
    auto wait_use = [](u32x2 &v, auto n) {
        asm volatile("s_waitcnt vmcnt(%2)" : "+v"(v.x), "+v"(v.y) : "n"(decltype(n)::value) : "memory");
    };
    // issue the pieces of window q owned by this wave
    auto issue = [&](int q) {
        const int first = NLD > 0 ? wid - (16 - NLD) : wid;
        const int step = NLD > 0 ? NLD : 16;
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
            const int m = first + k * step;
            const bool ok = q < NB && m < PIECES;
            const uint32_t voff = ok ? (uint32_t)(q * W + m * 1024 + lane * 16) : 0xFFFFFFF0u;
            dma_piece(x_src, voff, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((q % NBUF) * W + (m % PIECES) * 1024)));
        }
    };
    uint32_t acc = 0;
    u32x2 ev[AE];
    const bool loader = NLD > 0 && wid >= NAPPLY;
    // prologue: windows 0..A-1, entries 0..AE-1
    if (NLD == 0 || loader)
        for (int q = 0; q < A; ++q) issue(q);
    if (!loader) {
#pragma unroll
        for (int v = 0; v < AE; ++v) ev[v] = load_e(v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    constexpr int U = AE;   // unroll so the entry ring indices are static
    if constexpr (NLD > 0) {
        if (loader) {   // its own loop: no entry registers flow through it (hipcc would drain vmcnt)
            for (int q = 0; q < NB; ++q) {
                issue(q + A);   // into the buffer window q-1 left
                // window q+1 landed: the younger (A-1) windows' pieces may fly
                if constexpr (A == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if constexpr (A == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL) : "memory");
                else if constexpr (A == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPL) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPL) : "memory");
                __syncthreads();
            }
        } else {
            for (int p = 0; p < NB; p += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int q = p + u;
                    wait_use(ev[u], std::integral_constant<int, AE - 1>());
                    acc ^= ev[u].x ^ ev[u].y;
                    ev[u] = load_e(q + AE);
                    acc += lds_touch(lds0 + (uint32_t)((q % NBUF) * W + lane * 4));
                    if constexpr (CS > 0) {   // the apply's LDS traffic: per chunk x, table, sum reads, sum write
                        constexpr uint32_t kAcc = NBUF * W, kTab = kAcc + 65536;
                        static_assert(kTab + 4096 <= kLdsBytes, "LDS");
#pragma unroll
                        for (int k = 0; k < CS; ++k) {
                            const uint32_t h = (uint32_t)lane * 2654435761u ^ (uint32_t)q * 40503u ^ (uint32_t)(wid * CS + k) * 2246822519u;
                            const uint32_t ax = lds0 + (uint32_t)((q % NBUF) * W) + ((h >> 7) % (uint32_t)(W / 4)) * 4u;
                            const uint32_t aa = lds0 + kAcc + ((h >> 3) & 16383u) * 4u;
                            const uint32_t at = lds0 + kTab + ((h >> 20) & 255u) * 16u + (lane & 3) * 4u;
                            uint32_t vx, va, vt;
                            asm volatile("ds_read_b32 %0, %3\n\tds_read_b32 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)\n\t"
                                         "v_add_u32 %1, %1, %0\n\tv_add_u32 %1, %1, %2\n\tds_write_b32 %4, %1"
                                         : "=&v"(vx), "=&v"(va), "=&v"(vt) : "v"(ax), "v"(aa), "v"(at) : "memory");
                            acc += va;
                        }
                    }
                    if (q < NB) __syncthreads();
                }
            }
        }
    } else {
        for (int p = 0; p < NB; p += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = p + u;
                // window q and entries q landed: the ops younger than the younger of the two
                // may fly (issue order per band r: window r+A's pieces, then entries r+AE)
                constexpr int X = AE <= A ? (AE - 1) * (PPL + 1) : 1 + (A - 1) * (PPL + 1);
                wait_use(ev[u], std::integral_constant<int, X>());
                if (q < NB) __syncthreads();   // every wave's pieces of window q
                acc ^= ev[u].x ^ ev[u].y;
                acc += lds_touch(lds0 + (uint32_t)((q % NBUF) * W + lane * 4));
                issue(q + A);      // into the buffer window q-1 left (every wave is past it)
                ev[u] = load_e(q + AE);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// Pure streaming, no barrier: NLD waves each keep K 1 KiB LDS-DMA pieces in flight
// (s_waitcnt vmcnt(K) after every issue) until the tile's 1 MiB slab is in LDS (written
// round-robin over a 64 KiB region; the data is not used).  Per-CU L2 -> LDS rate against
// the number of pieces in flight.
template <int NLD, int K>
__global__ __launch_bounds__(1024) void xflow_kernel(const float *__restrict__ x, uint32_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slab = blockIdx.x & 3;
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x + (size_t)slab * (kSlabBytes / 4), kSlabBytes);
    const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)&lds[0];
    if (wid < NLD) {
        constexpr int P = kSlabBytes / 1024 / NLD;   // pieces per loader
        for (int k = 0; k < P; ++k) {
            const int m = wid + k * NLD;
            dma_piece(x_src, (uint32_t)(m * 1024 + lane * 16),
                      __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((m & 63) * 1024)));
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0 && lds_touch(lds0) == 0x12345678u) out[blockIdx.x] = 1;
}

template <int NLD, int K>
void run_flow(const float *x, uint32_t *out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((xflow_kernel<NLD, K>), dim3(256), dim3(1024), 0, 0, x, out);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((xflow_kernel<NLD, K>), dim3(256), dim3(1024), 0, 0, x, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const float us = 1000.f * ms / reps;
    printf("flow: %2d loader waves x %2d pieces in flight (%4d KiB per CU): %7.2f us/launch  %6.1f GB/s per CU\n",
           NLD, K, NLD * K, us, (double)kSlabBytes / (us * 1e3));
}

template <int NLD, int WK, int A, int AE, bool E, int CS = 0, int EP = 2>
float run(const float *x, const uint32_t *ent, uint32_t *out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // four copies of the entry stream rotate (4 x <= 128 MiB > the 256 MiB Infinity Cache
    // with x), so entries come from HBM as in the bench
    constexpr size_t kCopy = (size_t)32 << 20;   // uint32 words = 128 MiB
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((xstream_kernel<NLD, WK, A, AE, E, CS, EP>), dim3(256), dim3(1024), 0, 0, x, ent + (i & 3) * kCopy, out);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((xstream_kernel<NLD, WK, A, AE, E, CS, EP>), dim3(256), dim3(1024), 0, 0, x, ent + (i & 3) * kCopy, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const float us = 1000.f * ms / reps;
    constexpr int NB = (kSlabBytes + WK * 1024 - 1) / (WK * 1024);
    printf("NLD %d  W %3d KiB  A %d  AE %d  entries %d (policy %d)  apply-sim %d chunks  bands %3d : %7.2f us/launch  x %6.1f GB/s per CU  %5.3f us/band\n",
           NLD, WK, A, AE, (int)E, EP, CS, NB, us, (double)NB * WK * 1024 / (us * 1e3), us / NB);
    return us;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    float *x;
    uint32_t *ent, *out;
    CK(hipMalloc(&x, 4 << 20));
    CK(hipMemset(x, 0, 4 << 20));
    const size_t ent_bytes = (size_t)512 << 20;   // four 128 MiB copies
    CK(hipMalloc(&ent, ent_bytes));
    CK(hipMemset(ent, 0, ent_bytes));
    CK(hipMalloc(&out, 4096));
    if (argc > 2 && argv[2][0] == 'c') {   // entry cache policy: 0 default, 1 sc0, 2 nt, 3 sc0 sc1
        run<4, 45, 1, 4, true, 0, 0>(x, ent, out, reps);
        run<4, 45, 1, 4, true, 0, 1>(x, ent, out, reps);
        run<4, 45, 1, 4, true, 0, 2>(x, ent, out, reps);
        run<4, 45, 1, 4, true, 0, 3>(x, ent, out, reps);
        run<1, 30, 2, 2, true, 0, 0>(x, ent, out, reps);
        run<1, 30, 2, 2, true, 0, 2>(x, ent, out, reps);
        run<8, 45, 1, 4, true, 0, 0>(x, ent, out, reps);
        run<8, 45, 1, 4, true, 6, 0>(x, ent, out, reps);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'b') {   // two buffers, entries further ahead, simulated apply
        run<1, 30, 2, 2, true, 2>(x, ent, out, reps);    // dma3 with its apply's LDS traffic
        run<2, 40, 1, 4, true>(x, ent, out, reps);
        run<2, 40, 1, 4, false>(x, ent, out, reps);
        run<4, 45, 1, 4, true>(x, ent, out, reps);
        run<4, 45, 1, 6, true>(x, ent, out, reps);
        run<8, 45, 1, 4, true>(x, ent, out, reps);
        run<2, 40, 1, 4, true, 3>(x, ent, out, reps);    // 14 appliers x 3 chunks
        run<4, 45, 1, 4, true, 4>(x, ent, out, reps);    // 12 appliers x 4 chunks
        run<4, 40, 1, 4, true, 4>(x, ent, out, reps);
        run<8, 45, 1, 4, true, 6>(x, ent, out, reps);    // 8 appliers x 6 chunks
        run<2, 30, 2, 4, true, 2>(x, ent, out, reps);
        run<4, 30, 2, 4, true, 3>(x, ent, out, reps);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'a') {   // two buffers (window q+1 issued at band q)
        run<1, 46, 1, 2, true>(x, ent, out, reps);
        run<2, 46, 1, 2, true>(x, ent, out, reps);
        run<4, 46, 1, 2, true>(x, ent, out, reps);
        run<8, 46, 1, 2, true>(x, ent, out, reps);
        run<4, 46, 1, 2, false>(x, ent, out, reps);
        run<4, 40, 1, 2, true>(x, ent, out, reps);
        run<4, 32, 1, 2, true>(x, ent, out, reps);
        run<8, 32, 1, 2, true>(x, ent, out, reps);
        run<4, 30, 2, 2, true>(x, ent, out, reps);
        run<8, 30, 2, 2, true>(x, ent, out, reps);
        run<1, 30, 2, 2, true>(x, ent, out, reps);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'f') {   // streaming ceiling only
        run_flow<1, 8>(x, out, reps);
        run_flow<1, 16>(x, out, reps);
        run_flow<1, 32>(x, out, reps);
        run_flow<1, 56>(x, out, reps);
        run_flow<2, 16>(x, out, reps);
        run_flow<2, 32>(x, out, reps);
        run_flow<2, 56>(x, out, reps);
        run_flow<4, 8>(x, out, reps);
        run_flow<4, 16>(x, out, reps);
        run_flow<4, 32>(x, out, reps);
        run_flow<4, 56>(x, out, reps);
        run_flow<8, 8>(x, out, reps);
        run_flow<8, 16>(x, out, reps);
        run_flow<8, 32>(x, out, reps);
        run_flow<16, 4>(x, out, reps);
        run_flow<16, 8>(x, out, reps);
        run_flow<16, 16>(x, out, reps);
        run_flow<16, 32>(x, out, reps);
        return 0;
    }
    // dma3 as built: 1 loader, 30 KiB windows, 3 buffers
    run<1, 30, 2, 2, true>(x, ent, out, reps);
    run<1, 30, 2, 2, false>(x, ent, out, reps);
    run<2, 30, 2, 2, true>(x, ent, out, reps);
    run<4, 30, 2, 2, true>(x, ent, out, reps);
    run<0, 32, 2, 2, true>(x, ent, out, reps);
    run<0, 32, 2, 3, true>(x, ent, out, reps);
    // windows and depth
    run<1, 20, 3, 2, true>(x, ent, out, reps);
    run<2, 20, 3, 2, true>(x, ent, out, reps);
    run<1, 45, 2, 2, true>(x, ent, out, reps);
    run<2, 45, 2, 2, true>(x, ent, out, reps);
    run<4, 45, 2, 2, true>(x, ent, out, reps);
    run<2, 48, 2, 2, true>(x, ent, out, reps);
    run<1, 16, 4, 2, true>(x, ent, out, reps);
    run<2, 16, 4, 2, true>(x, ent, out, reps);
    run<4, 16, 4, 2, true>(x, ent, out, reps);
    run<2, 36, 3, 2, true>(x, ent, out, reps);
    run<4, 36, 3, 2, true>(x, ent, out, reps);
    run<4, 30, 3, 2, true>(x, ent, out, reps);   // 4 buffers of 30 KiB: more in flight (120 KiB, not available)
    run<2, 23, 3, 2, true>(x, ent, out, reps);   // 4 buffers of 23 KiB = 92 KiB (what fits beside the sums)
    run<4, 23, 3, 2, true>(x, ent, out, reps);
    run<3, 30, 2, 2, true>(x, ent, out, reps);
    run<0, 48, 2, 2, true>(x, ent, out, reps);
    run<0, 36, 3, 2, true>(x, ent, out, reps);
    return 0;
}
