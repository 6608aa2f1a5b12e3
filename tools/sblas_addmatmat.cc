// sblas_addmatmat -- one AddMatMat through the reference's C++ surface
// (include/sblas/sparse-matrix.h over libsblas.so), as a reference user would call it:
// CopyForm from a dense uint8 index, then AddMatMat on device or host buffers.  Used by
// tests/test_gpu_shim.py (bit-exact against the oracle's restatement of
// /root/reference/src/sparse/sparse-matrix.cc:139-194) and for the shim-vs-AUTO timing.
//
//   sblas_addmatmat DIR rows cols stride table_size trans m alpha beta device|host reps
//
// Reads DIR/index.bin (rows x stride bytes), DIR/table.bin (table_size floats),
// DIR/a.bin (m x k floats, lda = k), DIR/c.bin (m x n floats, ldc = n); writes the result
// of the first call to DIR/out.bin and prints one JSON line: the matrix's layout, the
// algorithm SM_ALGO_EXACT runs, and the median time of `reps` further calls of
// AddMatMat (C reset before each, device drained after) next to sm_addmatmat with
// SM_ALGO_AUTO on the same buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sparse-matrix.h"
#include "sparsematrix.h"

namespace {

template <class T>
std::vector<T> read_file(const std::string &path, size_t count) {
    std::vector<T> v(count);
    FILE *f = fopen(path.c_str(), "rb");
    if (!f || fread(v.data(), sizeof(T), count, f) != count) {
        fprintf(stderr, "sblas_addmatmat: cannot read %zu items from %s\n", count, path.c_str());
        exit(2);
    }
    fclose(f);
    return v;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

#define HIP_OK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "sblas_addmatmat: %s: %s\n", #x, hipGetErrorString(e_));       \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

template <class F>
double median_ms(int reps, F &&one) {
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) t.push_back(one());
    if (t.empty()) return 0.0;
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 12) {
        fprintf(stderr, "usage: %s DIR rows cols stride table_size trans m alpha beta device|host reps\n",
                argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    const int rows = atoi(argv[2]), cols = atoi(argv[3]), stride = atoi(argv[4]);
    const int table_size = atoi(argv[5]), trans = atoi(argv[6]), m = atoi(argv[7]);
    const float alpha = (float)atof(argv[8]), beta = (float)atof(argv[9]);
    const bool device = strcmp(argv[10], "device") == 0;
    const int reps = atoi(argv[11]);

    const auto index = read_file<uint8>(dir + "/index.bin", (size_t)rows * stride);
    const auto table = read_file<float>(dir + "/table.bin", (size_t)table_size);
    sblas::SparseMatrix<uint8, uint8, float> B;
    const double tb = now_ms();
    B.CopyForm(index.data(), rows, cols, stride, table.data(), table_size,
               trans ? sblas::SblasTrans : sblas::SblasNoTrans);
    const double build_ms = now_ms() - tb;
    const int k = B.NumRows(), n = B.NumCols();
    const auto A = read_file<float>(dir + "/a.bin", (size_t)m * k);
    const auto C0 = read_file<float>(dir + "/c.bin", (size_t)m * n);
    std::vector<float> C = C0;
    double ms_shim = 0.0, ms_auto = 0.0;
    if (device) {
        float *dA = nullptr, *dC = nullptr, *dC0 = nullptr;
        HIP_OK(hipMalloc((void **)&dA, A.size() * 4 + 16));
        HIP_OK(hipMalloc((void **)&dC, C0.size() * 4 + 16));
        HIP_OK(hipMalloc((void **)&dC0, C0.size() * 4 + 16));
        HIP_OK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(dC0, C0.data(), C0.size() * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(dC, dC0, C0.size() * 4, hipMemcpyDeviceToDevice));
        B.AddMatMat(dA, m, k, dC, n, alpha, beta);   // the checked result
        {   // read C on a non-blocking stream, not ordered behind the null stream: the
            // reference's AddMatMat is synchronous, so C must be final on return
            hipStream_t rs;
            HIP_OK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
            HIP_OK(hipMemcpyAsync(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost, rs));
            HIP_OK(hipStreamSynchronize(rs));
            HIP_OK(hipStreamDestroy(rs));
        }
        auto timed = [&](auto &&call) {
            return median_ms(reps, [&] {
                HIP_OK(hipMemcpy(dC, dC0, C0.size() * 4, hipMemcpyDeviceToDevice));
                HIP_OK(hipDeviceSynchronize());
                const double t0 = now_ms();
                call();
                HIP_OK(hipDeviceSynchronize());
                return now_ms() - t0;
            });
        };
        ms_shim = timed([&] { B.AddMatMat(dA, m, k, dC, n, alpha, beta); });
        ms_auto = timed([&] {
            if (sm_addmatmat(B.handle(), dA, m, k, dC, n, alpha, beta, SM_ALGO_AUTO, nullptr) != SM_OK) {
                fprintf(stderr, "sm_addmatmat: %s\n", sm_last_error());
                exit(2);
            }
        });
        HIP_OK(hipFree(dA));
        HIP_OK(hipFree(dC));
        HIP_OK(hipFree(dC0));
    } else {
        std::vector<float> Ah = A;
        B.AddMatMat(Ah.data(), m, k, C.data(), n, alpha, beta);
        std::vector<float> Ct;
        ms_shim = median_ms(reps, [&] {
            Ct = C0;
            const double t0 = now_ms();
            B.AddMatMat(Ah.data(), m, k, Ct.data(), n, alpha, beta);
            return now_ms() - t0;
        });
    }
    FILE *f = fopen((dir + "/out.bin").c_str(), "wb");
    if (!f || fwrite(C.data(), 4, C.size(), f) != C.size()) {
        fprintf(stderr, "sblas_addmatmat: cannot write out.bin\n");
        return 2;
    }
    fclose(f);
    sm_info info;
    if (sm_get_info(B.handle(), &info) != SM_OK) return 2;
    printf("{\"k\": %d, \"n\": %d, \"nnz\": %lld, \"m\": %d, \"where\": \"%s\", \"has_xband\": %d, "
           "\"xband_slabs\": %d, \"sell_slices\": %lld, \"exact_sell_slices\": %lld, \"exact_algo\": %d, "
           "\"max_row_nnz\": %d, \"build_ms\": %.3f, \"ms_shim\": %.5f, \"ms_auto\": %.5f, \"reps\": %d}\n",
           k, n, (long long)info.nnz, m, device ? "device" : "host", info.has_xband, info.xband_slabs,
           (long long)info.sell_slices, (long long)info.exact_sell_slices, info.exact_algo,
           info.max_row_nnz, build_ms, ms_shim, ms_auto, reps);
    return 0;
}
