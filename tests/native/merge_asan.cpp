// Host-only check of the merge path's plan (sparsematrix_amd/csrc/merge.cpp), built with
// AddressSanitizer by tests/test_xband_builder.py.  For random, skewed and edge shapes:
//  - merge_corners equals a sequential walk of the merge (row i's end is taken once all its
//    terms are, i.e. before the term with the same index) sampled every kMgTile items;
//  - merge_stage_build: per slice, z is a permutation of the slice's terms, the words are
//    column << 8 | id of those terms in ascending column order (ties in CSR order), and the
//    table maps every id back to the term's value bits; it declines more than 255 distinct
//    values and more than 2^24 columns.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "merge.h"

using namespace smamd;

static int check(const std::vector<int32_t> &rp, const std::vector<int32_t> &col, const std::vector<float> &val,
                 int64_t n_cols, const char *name) {
    const int64_t n = (int64_t)rp.size() - 1, nnz = (int64_t)col.size();
    std::vector<int32_t> corners;
    merge_corners(rp.data(), n, nnz, corners);
    const int64_t nb = merge_blocks(n, nnz);
    if ((int64_t)corners.size() != 2 * (nb + 1)) { printf("FAIL %s corner count\n", name); return 1; }
    int64_t i = 0, j = 0;
    for (int64_t d = 0;; ++d) {
        if (d % kMgTile == 0 || d == n + nnz) {
            const int64_t b = d % kMgTile == 0 ? d / kMgTile : nb;
            if (corners[(size_t)(2 * b)] != i || corners[(size_t)(2 * b + 1)] != j) {
                printf("FAIL %s corner %lld: (%d, %d) want (%lld, %lld)\n", name, (long long)b,
                       corners[(size_t)(2 * b)], corners[(size_t)(2 * b + 1)], (long long)i, (long long)j);
                return 1;
            }
        }
        if (d == n + nnz) break;
        if (i < n && j >= rp[(size_t)(i + 1)]) ++i;   // row i's end
        else ++j;                                     // term j
    }
    std::vector<uint32_t> w;
    std::vector<uint16_t> z;
    std::vector<float> table;
    if (!merge_stage_build(rp.data(), col.data(), val.data(), n, n_cols, nnz, w, z, table)) {
        printf("FAIL %s stage declined\n", name);
        return 1;
    }
    if ((int64_t)w.size() != nnz || (int64_t)z.size() != nnz || table.size() != 256) {
        printf("FAIL %s stage sizes\n", name);
        return 1;
    }
    for (int64_t b = 0; b < nb; ++b) {
        const int32_t z0 = corners[(size_t)(2 * b + 1)], z1 = corners[(size_t)(2 * b + 3)];
        std::vector<char> seen((size_t)(z1 - z0), 0);
        for (int32_t k = 0; k < z1 - z0; ++k) {
            const int32_t p = z[(size_t)(z0 + k)];
            if (p < 0 || p >= z1 - z0 || seen[(size_t)p]) { printf("FAIL %s slice %lld not a permutation\n", name, (long long)b); return 1; }
            seen[(size_t)p] = 1;
            const int32_t e = z0 + p;
            const uint32_t wd = w[(size_t)(z0 + k)];
            const float tv = table[wd & 0xffu];
            if ((int32_t)(wd >> 8) != col[(size_t)e] || memcmp(&tv, &val[(size_t)e], 4) != 0 || (wd & 0xffu) == 0xffu) {
                printf("FAIL %s slice %lld word %d\n", name, (long long)b, k);
                return 1;
            }
            if (k > 0) {
                const int32_t pc = col[(size_t)(z0 + z[(size_t)(z0 + k - 1)])];
                if (pc > col[(size_t)e] || (pc == col[(size_t)e] && z[(size_t)(z0 + k - 1)] > p)) {
                    printf("FAIL %s slice %lld order at %d\n", name, (long long)b, k);
                    return 1;
                }
            }
        }
    }
    return 0;
}

static void csr(std::mt19937_64 &g, int64_t n, int64_t n_cols, const std::vector<int32_t> &lens,
                std::vector<int32_t> &rp, std::vector<int32_t> &col, std::vector<float> &val, int n_values,
                bool skew) {
    std::vector<float> vals((size_t)n_values);
    for (int k = 0; k < n_values; ++k) vals[(size_t)k] = (float)(k - n_values / 2) * 0.37f + (k == 0 ? -0.0f : 0.0f);
    rp.assign((size_t)n + 1, 0);
    col.clear();
    val.clear();
    for (int64_t r = 0; r < n; ++r) {
        std::vector<int32_t> c;
        for (int32_t k = 0; k < lens[(size_t)r]; ++k) {
            const uint64_t u = g();
            c.push_back(skew ? (int32_t)((u % 64 < 48 ? u % 97 : u) % (uint64_t)n_cols) : (int32_t)(u % (uint64_t)n_cols));
        }
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (int32_t x : c) {
            col.push_back(x);
            val.push_back(vals[(size_t)(g() % (uint64_t)n_values)]);
        }
        rp[(size_t)r + 1] = (int32_t)col.size();
    }
}

int main() {
    std::mt19937_64 g(7);
    int fails = 0;
    std::vector<int32_t> rp, col;
    std::vector<float> val;
    {   // uniform rows
        std::vector<int32_t> lens(30001, 16);
        csr(g, 30001, 40000, lens, rp, col, val, 255, false);
        fails += check(rp, col, val, 40000, "uniform");
    }
    {   // power-law rows, runs of empty rows, a few rows spanning many slices, hot columns
        std::vector<int32_t> lens(50000);
        for (auto &l : lens) l = (g() % 10 < 3) ? 0 : (int32_t)(1 + (g() % 1000 == 0 ? g() % 20000 : g() % 12));
        csr(g, 50000, 1 << 20, lens, rp, col, val, 200, true);
        fails += check(rp, col, val, 1 << 20, "skewed");
    }
    {   // one row; no terms in a slice's middle; a single term
        std::vector<int32_t> lens(1, 5000);
        csr(g, 1, 1 << 16, lens, rp, col, val, 3, false);
        fails += check(rp, col, val, 1 << 16, "one_row");
        std::vector<int32_t> l2(9000, 0);
        l2[4500] = 1;
        csr(g, 9000, 10, l2, rp, col, val, 1, false);
        fails += check(rp, col, val, 10, "single_term");
    }
    {   // declines: 256 distinct values, columns past 2^24, no terms
        std::vector<int32_t> lens(100, 30);
        csr(g, 100, 1000, lens, rp, col, val, 255, false);
        for (size_t k = 0; k < val.size(); ++k) val[k] = (float)k;   // 3000 distinct
        std::vector<uint32_t> w;
        std::vector<uint16_t> z;
        std::vector<float> t;
        if (merge_stage_build(rp.data(), col.data(), val.data(), 100, 1000, (int64_t)col.size(), w, z, t)) {
            printf("FAIL accepted > 255 values\n");
            ++fails;
        }
        csr(g, 100, 1000, lens, rp, col, val, 10, false);
        if (merge_stage_build(rp.data(), col.data(), val.data(), 100, (1 << 24) + 1, (int64_t)col.size(), w, z, t)) {
            printf("FAIL accepted > 2^24 columns\n");
            ++fails;
        }
        std::vector<int32_t> rp0(11, 0);
        if (merge_stage_build(rp0.data(), nullptr, nullptr, 10, 10, 0, w, z, t)) {
            printf("FAIL accepted nnz = 0\n");
            ++fails;
        }
    }
    if (fails) return 1;
    printf("merge_asan: ok\n");
    return 0;
}
