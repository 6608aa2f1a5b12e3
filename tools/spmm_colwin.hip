// spmm_colwin.hip -- VERDICT r5 item 6: one measured column-ordered pull for config 3 instead of
// the paper estimate ("X fabric traffic ~ 8 XCDs x 4 generations x
// 128 MiB = 4.3 GB > 2.50 GB").  A development experiment, not a product kernel.
//
// Config 3: Y (2^20 x 32) = alpha * B X + beta * Y, B 2^20 x 2^20 with 16 distinct uniform
// columns per row, values from a 255-entry table, X 2^20 x 32 fp32 (128 MiB).
// Pull order: 1024 tiles of 1024 rows; a tile's Y rows live in LDS (128 KiB: one workgroup per
// CU, four generations on 256 CUs); the tile's terms are sorted by column, so every tile sweeps
// X from its first row to its last and the 32 tiles an XCD runs at once gather from the same
// region of X at about the same time -- an X line fetched into an XCD's L2 serves the other
// tiles there that need it (only the lines terms touch move, not whole windows).  Each half-wave
// takes one term: 32 lanes gather the term's X row (128 B) and add fl(v alpha) x into the LDS
// row with ds_add_f32 -- the order of a row's additions is not fixed, so results are checked
// against a double-precision reference within 1e-6 * sum|terms| (sampled rows), not bit for bit.
//
//   build/spmm_colwin [reps]     prints the kernel's median time and the check
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <random>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                             \
        }                                                                                        \
    } while (0)

constexpr int kN = 32;                 // right-hand sides
constexpr int kTileRows = 1024;        // Y rows per tile: 128 KiB of LDS
constexpr int kThreads = 1024;

// Term word: column << 10 | row in tile (columns < 2^22).
__global__ __launch_bounds__(kThreads) void colwin_kernel(const int64_t *__restrict__ toff,
                                                          const uint32_t *__restrict__ tw,
                                                          const float *__restrict__ tv,
                                                          const float *__restrict__ X, float *__restrict__ Y,
                                                          int32_t n_rows, float alpha, float beta) {
    __shared__ float ys[kTileRows * kN];
    const int t = blockIdx.x;
    const int32_t r0 = t * kTileRows;
    const int32_t nr = min(kTileRows, n_rows - r0);
    for (int i = threadIdx.x; i < nr * kN; i += kThreads) {
        const float v = Y[(int64_t)r0 * kN + i];
        ys[i] = beta != 1.0f ? v * beta : v;
    }
    __syncthreads();
    const int64_t e0 = toff[t], e1 = toff[t + 1];
    const int half = threadIdx.x >> 5, j = threadIdx.x & 31;   // 32 half-waves, lane = X column
    for (int64_t e = e0 + half; e < e1; e += kThreads / 32) {
        const uint32_t w = tw[e];
        const float a = __fmul_rn(tv[e], alpha);
        const float x = X[(int64_t)(w >> 10) * kN + j];
        atomicAdd(&ys[(w & 1023u) * kN + j], __fmul_rn(x, a));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nr * kN; i += kThreads) Y[(int64_t)r0 * kN + i] = ys[i];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const int32_t n = 1 << 20, per = 16;
    const int64_t nnz = (int64_t)n * per;
    std::mt19937_64 rng(3);
    std::vector<float> table(255);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (auto &v : table) v = U(rng);
    // Rows: 16 distinct uniform columns; then per tile its terms sorted by column.
    const int n_tiles = (n + kTileRows - 1) / kTileRows;
    std::vector<int64_t> toff(n_tiles + 1, 0);
    std::vector<uint32_t> tw((size_t)nnz);
    std::vector<float> tv((size_t)nnz);
    std::vector<int32_t> rcol((size_t)nnz);   // row-major copy for the check
    std::vector<float> rval((size_t)nnz);
    std::vector<std::pair<uint64_t, float>> buf;
    for (int t = 0; t < n_tiles; t++) {
        buf.clear();
        for (int32_t r = t * kTileRows; r < std::min(n, (t + 1) * kTileRows); r++) {
            int32_t c[per];
            for (int k = 0; k < per; k++) {
                bool dup;
                do {
                    c[k] = (int32_t)(rng() % (uint64_t)n);
                    dup = false;
                    for (int q = 0; q < k; q++) dup |= c[q] == c[k];
                } while (dup);
            }
            std::sort(c, c + per);
            for (int k = 0; k < per; k++) {
                const float v = table[rng() % 255];
                rcol[(size_t)r * per + k] = c[k];
                rval[(size_t)r * per + k] = v;
                buf.push_back({((uint64_t)c[k] << 10) | (uint64_t)(r - t * kTileRows), v});
            }
        }
        std::stable_sort(buf.begin(), buf.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        toff[t + 1] = toff[t] + (int64_t)buf.size();
        for (size_t i = 0; i < buf.size(); i++) {
            tw[(size_t)toff[t] + i] = (uint32_t)buf[i].first;
            tv[(size_t)toff[t] + i] = buf[i].second;
        }
    }
    std::vector<float> X((size_t)n * kN), Y0((size_t)n * kN);
    for (auto &v : X) v = U(rng);
    for (auto &v : Y0) v = U(rng);
    int64_t *d_off;
    uint32_t *d_w;
    float *d_v, *d_x, *d_y;
    CK(hipMalloc(&d_off, toff.size() * 8));
    CK(hipMalloc(&d_w, tw.size() * 4));
    CK(hipMalloc(&d_v, tv.size() * 4));
    CK(hipMalloc(&d_x, X.size() * 4));
    CK(hipMalloc(&d_y, Y0.size() * 4));
    CK(hipMemcpy(d_off, toff.data(), toff.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w, tw.data(), tw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_v, tv.data(), tv.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, X.data(), X.size() * 4, hipMemcpyHostToDevice));
    const float alpha = 1.0f, beta = 0.5f;
    // correctness: one product from Y0
    CK(hipMemcpy(d_y, Y0.data(), Y0.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(colwin_kernel, dim3(n_tiles), dim3(kThreads), 0, 0, d_off, d_w, d_v, d_x, d_y, n, alpha, beta);
    CK(hipGetLastError());
    std::vector<float> Y((size_t)n * kN);
    CK(hipMemcpy(Y.data(), d_y, Y.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    double worst = 0;
    for (int s = 0; s < 4096; s++) {
        const int32_t r = (int32_t)(rng() % (uint64_t)n);
        for (int j = 0; j < kN; j++) {
            double ref = (double)Y0[(size_t)r * kN + j] * beta, mag = std::fabs(ref);
            for (int k = 0; k < per; k++) {
                const double term = (double)X[(size_t)rcol[(size_t)r * per + k] * kN + j] * (double)(rval[(size_t)r * per + k] * alpha);
                ref += term;
                mag += std::fabs(term);
            }
            const double err = std::fabs((double)Y[(size_t)r * kN + j] - ref), bound = 1e-6 * mag + 1e-37;
            worst = std::max(worst, err / bound);
            bad += err > bound;
        }
    }
    // timing: reps products (Y keeps being updated in place)
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int i = 0; i < reps; i++) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(colwin_kernel, dim3(n_tiles), dim3(kThreads), 0, 0, d_off, d_w, d_v, d_x, d_y, n, alpha, beta);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("spmm_colwin: config 3 (2^20 x 2^20, 16/row, N = 32), %d tiles of %d rows, median %.1f us over %d "
           "(min %.1f); check: %d of %d sampled outputs out of 1e-6*sum|terms| (worst ratio %.3g)\n",
           n_tiles, kTileRows, 1e3 * ms[ms.size() / 2], reps, 1e3 * ms[0], bad, 4096 * kN, worst);
    return bad ? 1 : 0;
}
