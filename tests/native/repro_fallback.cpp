// Standalone C-ABI reproduction of test_xband_not_applicable_falls_back (no torch):
// xband matrix, SpMV with a 4-byte-misaligned x (stream fallback), D2H copy, and the
// same sequence with xband forced on a matrix that has the layout.  Each step is
// synchronised and checked.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <algorithm>
#include "sparsematrix.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define SM(x) do { sm_status s = (x); if (s != SM_OK) { printf("SM %d %s at %d\n", (int)s, sm_last_error(), __LINE__); return 1; } } while (0)

int main() {
    const int n = 5000, k = 40000, per = 8;
    std::mt19937 rng(5);
    std::vector<int32_t> rp(n + 1), col;
    std::vector<float> val;
    for (int r = 0; r < n; r++) {
        std::vector<int32_t> c(per);
        for (auto &v : c) v = rng() % k;
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (auto v : c) { col.push_back(v); val.push_back(1.0f); }
        rp[r + 1] = (int32_t)col.size();
    }
    setenv("SM_XBAND", "1", 1);
    sm_matrix *m = nullptr;
    SM(sm_create_from_csr(n, k, (int64_t)col.size(), rp.data(), col.data(), val.data(), 0, &m));
    sm_info inf;
    SM(sm_get_info(m, &inf));
    printf("has_xband=%d blocks=%d bands=%d\n", inf.has_xband, inf.xband_blocks, inf.xband_bands);
    float *xbuf, *y;
    CK(hipMalloc(&xbuf, (k + 4) * sizeof(float)));
    CK(hipMalloc(&y, n * sizeof(float)));
    std::vector<float> xh(k + 4, 1.0f), yh(n, 0.0f);
    CK(hipMemcpy(xbuf, xh.data(), xh.size() * 4, hipMemcpyHostToDevice));
    for (int shift : {0, 1}) {
        for (int algo : {SM_ALGO_STREAM, SM_ALGO_XBAND, SM_ALGO_PARITY}) {
            CK(hipMemcpy(y, yh.data(), n * 4, hipMemcpyHostToDevice));
            SM(sm_spmv(m, 1.0f, xbuf + shift, 1.0f, y, (sm_algo)algo, nullptr));
            CK(hipDeviceSynchronize());
            std::vector<float> out(n);
            CK(hipMemcpy(out.data(), y, n * 4, hipMemcpyDeviceToHost));
            double s = 0;
            for (float v : out) s += v;
            printf("shift=%d algo=%d sum=%.1f (expect %zu)\n", shift, algo, s, col.size());
        }
    }
    sm_destroy(m);
    CK(hipFree(xbuf));
    CK(hipFree(y));
    printf("repro done\n");
    return 0;
}
