// blas_test -- the reference harness's command line over the GPU backend
// (the reference's src/test/blas_test.{h,cc}).
//
//   blas_test [m[:m2]] [n[:n2]] [k[:k2]] [check 0|1] [filter]
//
// m, n, k sweep by doubling from the first to the second value (defaults 117, 1023,
// 2047 -- blas_test.cc:33); `check` (default 1) compares every result with a CPU
// dense sgemm; `filter` is a ';'-separated list of patterns matched anywhere in the
// function name, a leading '-' excluding (blas_test.h:17-46).  Output: the timing
// table in markdown (blas_test.h:65-98), and a "check <func> result failed" line
// for a result outside the reference's tolerance (10 % relative, more than
// size/1e4 outliers: blas_test.h:160-182).
//
// Functions (C = alpha*A*B^T + beta*C, A m x k, B n x k, C m x n, B sparse at 25 %
// density from a 255-entry table, encoded Trans as the reference's harness does):
//   sgemm_sparse          sblas::SparseMatrix::AddMatMat on host buffers (the
//                         reference-exact parity path, transfers included)
//   sgemm_sparse_device   the same product with A and C resident on the GPU (fast
//                         kernels; the time covers the kernels only)
//   sm_addmatmat_auto     the C ABI's sm_addmatmat with SM_ALGO_AUTO on the same
//                         device buffers (the library's own speed, for comparison:
//                         the C++ surface runs SM_ALGO_EXACT, the reference's order)
//   cpu_sgemm_baseline    the dense CPU product used as the checker (the reference
//                         uses OpenBLAS cblas_sgemm, absent from this image)
//
// Timing: one call, as the reference's harness does (its repeat loop is commented out,
// blas_test.h:199).  SBLAS_REPS=r > 1: one untimed call first, then the median of r
// timed calls (each on fresh copies of C).
//
// Unlike the reference (srand(time)), the generator is seeded (SBLAS_SEED, default
// 1) so a run can be repeated.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <regex>
#include <string>
#include <vector>

#include "sparse-matrix.h"
#include "sparsematrix.h"   // the C ABI (sm_addmatmat AUTO row)

namespace {

struct Range {
    int lo, hi;
    explicit Range(const char *s) {
        lo = atoi(s);
        const char *c = strchr(s, ':');
        hi = c ? atoi(c + 1) : lo;
    }
};

class Filter {   // patterns matched anywhere; the first match decides; none given = all
  public:
    explicit Filter(const char *spec) {
        std::string cur;
        auto flush = [&] {
            if (cur.empty()) return;
            const bool neg = cur[0] == '-';
            rules_.push_back({std::regex(".*" + cur.substr(neg ? 1 : 0) + ".*"), !neg});
            cur.clear();
        };
        for (const char *p = spec ? spec : ""; *p; ++p) {
            if (*p == ';') flush();
            else if ((unsigned char)*p > ' ') cur += *p;
        }
        flush();
    }
    bool Match(const std::string &name) const {
        if (rules_.empty()) return true;
        for (const auto &r : rules_)
            if (std::regex_match(name, r.re)) return r.keep;
        return false;
    }

  private:
    struct Rule { std::regex re; bool keep; };
    std::vector<Rule> rules_;
};

class Table {   // name -> (shape, ms) in first-seen order, printed as markdown
  public:
    void Add(const std::string &name, int m, int n, int k, double ms) {
        if (rows_.find(name) == rows_.end()) order_.push_back(name);
        rows_[name].push_back({m, n, k, ms});
    }
    void Print() const {
        for (size_t i = 0; i < order_.size(); ++i) {
            const auto &r = rows_.at(order_[i]);
            if (i == 0) {
                printf("| |");
                for (const auto &e : r) printf(" %dx%dx%d |", e.m, e.n, e.k);
                printf("\n");
            }
            printf("| %s |", order_[i].c_str());
            for (const auto &e : r) printf(" %gms |", e.ms);
            printf("\n");
        }
    }

  private:
    struct E { int m, n, k; double ms; };
    std::map<std::string, std::vector<E>> rows_;
    std::vector<std::string> order_;
};

std::mt19937 g_rng;

float rand_value() {   // the reference's magnitude profile: integers folded into [-1000, 1000]
    float v = (float)((int64_t)g_rng() % 2000001 - 1000000);
    while (v > 1000.0f || v < -1000.0f) v /= 100.0f;
    return v;
}

std::vector<float> random_matrix(size_t count) {
    std::vector<float> a(count);
    for (auto &v : a) v = rand_value();
    return a;
}

// B (n x k, row-major): 25 % of the positions carry a random id < 255, the rest the
// out-of-range id 255 (dropped by CopyForm); encoded Trans like the reference harness.
void random_sparse(int n, int k, sblas::SparseMatrix<uint8, uint8, float> &B) {
    std::vector<uint8> index((size_t)n * k, 255);
    std::vector<float> table = random_matrix(256);
    for (auto &v : index)
        if (g_rng() % 4 == 0) v = (uint8)(g_rng() % 255);
    B.CopyForm(index.data(), n, k, k, table.data(), 255, sblas::SblasTrans);
}

// C = alpha * A * Bd^T + beta * C (the checker; Bd dense n x k).
void cpu_sgemm(int m, int n, int k, const float *A, const float *Bd, float *C, float alpha,
               float beta) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            const float *a = A + (size_t)i * k, *b = Bd + (size_t)j * k;
            for (int l = 0; l < k; ++l) acc += (double)a[l] * b[l];
            C[(size_t)i * n + j] = (float)(alpha * acc + beta * C[(size_t)i * n + j]);
        }
}

bool check(const char *name, const std::vector<float> &c, const std::vector<float> &want) {
    size_t bad = 0;
    for (size_t i = 0; i < c.size(); ++i) {
        const float z = c[i] == 0.0f ? 1e-6f : c[i];
        const float rel = (want[i] - c[i]) / z;
        if (rel < -0.1f || rel > 0.1f) {
            if (bad++ > c.size() / 10000) {
                printf("check %s result failed, [%zu] c:%g, check:%g, diff:%g, diff_count:%zu\n",
                       name, i, c[i], want[i], rel, bad);
                return false;
            }
        }
    }
    return true;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

#define HIP_OK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "blas_test: %s: %s\n", #x, hipGetErrorString(e_));             \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

}  // namespace

// Median over `reps` runs of fn() (one untimed run first when reps > 1).
template <class F>
double timed_ms(int reps, F &&fn) {
    if (reps <= 1) {
        const double t0 = now_ms();
        fn();
        return now_ms() - t0;
    }
    fn();
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_ms();
        fn();
        t.push_back(now_ms() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    Range rm(argc > 1 ? argv[1] : "117"), rn(argc > 2 ? argv[2] : "1023"),
        rk(argc > 3 ? argv[3] : "2047");
    const bool do_check = argc > 4 ? argv[4][0] == '1' : true;
    const Filter filter(argc > 5 ? argv[5] : nullptr);
    const char *seed = getenv("SBLAS_SEED");
    g_rng.seed(seed ? (unsigned)atoi(seed) : 1u);
    const char *reps_env = getenv("SBLAS_REPS");
    const int reps = reps_env ? std::max(1, atoi(reps_env)) : 1;
    const float alpha = 1.0f, beta = 1.0f;   // the reference's sparse invoker (blas_test.h:307)
    Table table;
    int failures = 0;

    for (int m = rm.lo; m <= rm.hi; m <<= 1)
        for (int n = rn.lo; n <= rn.hi; n <<= 1)
            for (int k = rk.lo; k <= rk.hi; k <<= 1) {
                const std::vector<float> A = random_matrix((size_t)m * k);
                const std::vector<float> C0 = random_matrix((size_t)m * n);
                sblas::SparseMatrix<uint8, uint8, float> B;
                random_sparse(n, k, B);
                std::vector<float> want;
                if (do_check) {   // dense B (n x k) from the sparse encoding, then the CPU product
                    std::vector<float> Bd((size_t)n * k);
                    B.CopyTo(Bd.data(), k, sblas::SblasTrans);
                    want = C0;
                    const double t0 = now_ms();
                    cpu_sgemm(m, n, k, A.data(), Bd.data(), want.data(), alpha, beta);
                    if (filter.Match("cpu_sgemm_baseline"))
                        table.Add("cpu_sgemm_baseline", m, n, k, now_ms() - t0);
                }
                if (filter.Match("sgemm_sparse")) {
                    std::vector<float> Ah = A, C = C0;
                    const double ms = timed_ms(reps, [&] {
                        C = C0;
                        B.AddMatMat(Ah.data(), m, k, C.data(), n, alpha, beta);
                    });
                    table.Add("sgemm_sparse", m, n, k, ms);
                    if (do_check && !check("sgemm_sparse", C, want)) ++failures;
                }
                const bool dev_fn = filter.Match("sgemm_sparse_device");
                const bool auto_fn = filter.Match("sm_addmatmat_auto");
                if (dev_fn || auto_fn) {
                    float *dA = nullptr, *dC = nullptr, *dC0 = nullptr;
                    HIP_OK(hipMalloc((void **)&dA, A.size() * sizeof(float)));
                    HIP_OK(hipMalloc((void **)&dC, C0.size() * sizeof(float)));
                    HIP_OK(hipMalloc((void **)&dC0, C0.size() * sizeof(float)));
                    HIP_OK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
                    HIP_OK(hipMemcpy(dC0, C0.data(), C0.size() * 4, hipMemcpyHostToDevice));
                    // Kernel time: C reset outside the timed call, device drained after it.
                    auto run = [&](const char *name, auto &&call) {
                        std::vector<double> t;
                        for (int r = 0; r < (reps > 1 ? reps + 1 : 1); ++r) {
                            HIP_OK(hipMemcpy(dC, dC0, C0.size() * 4, hipMemcpyDeviceToDevice));
                            HIP_OK(hipDeviceSynchronize());
                            const double t0 = now_ms();
                            call();
                            HIP_OK(hipDeviceSynchronize());
                            if (reps <= 1 || r > 0) t.push_back(now_ms() - t0);
                        }
                        std::sort(t.begin(), t.end());
                        table.Add(name, m, n, k, t[t.size() / 2]);
                        std::vector<float> C(C0.size());
                        HIP_OK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
                        if (do_check && !check(name, C, want)) ++failures;
                    };
                    if (dev_fn)
                        run("sgemm_sparse_device", [&] { B.AddMatMat(dA, m, k, dC, n, alpha, beta); });
                    if (auto_fn)
                        run("sm_addmatmat_auto", [&] {
                            const sm_status st = sm_addmatmat(B.handle(), dA, m, k, dC, n, alpha, beta,
                                                              SM_ALGO_AUTO, nullptr);
                            if (st != SM_OK) {
                                fprintf(stderr, "sm_addmatmat: %s\n", sm_last_error());
                                exit(2);
                            }
                        });
                    HIP_OK(hipFree(dA));
                    HIP_OK(hipFree(dC));
                    HIP_OK(hipFree(dC0));
                }
            }
    table.Print();
    return failures ? 1 : 0;
}
