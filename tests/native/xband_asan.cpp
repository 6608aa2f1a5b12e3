// Host-only check of the column-band builder (sparsematrix_amd/csrc/xband.cpp)
// under AddressSanitizer: builds the layout for several shapes and verifies
// that every term appears exactly once, in (row, column) order per band, with
// correct ranks and no segment straddling a chunk.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <algorithm>
#include "xband.h"

using namespace smamd;

static int check(int64_t n_rows, int64_t n_cols, int per_row, unsigned seed, bool expect_ok) {
    std::mt19937 rng(seed);
    std::vector<int32_t> rp(n_rows + 1), col;
    std::vector<float> val;
    for (int64_t r = 0; r < n_rows; r++) {
        std::vector<int32_t> c(per_row);
        for (auto &v : c) v = (int32_t)(rng() % n_cols);
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (auto v : c) { col.push_back(v); val.push_back((float)(rng() % 1000)); }
        rp[r + 1] = (int32_t)col.size();
    }
    XbandHost xh;
    const bool ok = xband_build(rp.data(), col.data(), val.data(), n_rows, n_cols, kXbBlockRows,
                                kXbBandCols, xh);
    if (ok != expect_ok) { printf("FAIL build=%d expected %d\n", ok, expect_ok); return 1; }
    if (!ok) return 0;
    // reconstruct per row the (col, val) list in processing order
    std::vector<std::vector<std::pair<int32_t, float>>> got(n_rows);
    for (int64_t b = 0; b < xh.n_blocks; b++)
        for (int64_t p = 0; p < xh.n_bands; p++) {
            const int64_t c0 = xh.chunk_start[b * xh.n_bands + p], c1 = xh.chunk_start[b * xh.n_bands + p + 1];
            for (int64_t c = c0; c < c1; c++) {
                std::vector<int> seen_rows;
                for (int l = 0; l < 64; l++) {
                    const uint32_t w = xh.word[c * 64 + l];
                    const uint32_t rank = (w >> kXbColBits) & 63u;
                    if (rank == kXbDummyRank) continue;
                    const uint32_t cl = w & ((1u << kXbColBits) - 1u);
                    const uint32_t rl = w >> (kXbColBits + kXbRankBits);
                    const int64_t r = b * xh.block_rows + rl;
                    if (r >= n_rows) { printf("FAIL row out of range\n"); return 1; }
                    if ((int64_t)rank != (int64_t)std::count(seen_rows.begin(), seen_rows.end(), (int)rl)) {
                        printf("FAIL rank\n"); return 1; }
                    seen_rows.push_back((int)rl);
                    got[r].push_back({(int32_t)(p * xh.band_cols + cl), xh.val[c * 64 + l]});
                }
            }
        }
    for (int64_t r = 0; r < n_rows; r++) {
        if ((int64_t)got[r].size() != rp[r + 1] - rp[r]) { printf("FAIL count row %lld\n", (long long)r); return 1; }
        for (int32_t e = rp[r]; e < rp[r + 1]; e++)
            if (got[r][e - rp[r]].first != col[e] || got[r][e - rp[r]].second != val[e]) {
                printf("FAIL order row %lld\n", (long long)r); return 1; }
    }
    return 0;
}

int main() {
    int bad = 0;
    bad += check(200003, 300001, 16, 1, true);
    bad += check(9000, 70001, 40, 2, true);
    bad += check(4096, 32768, 7, 3, true);
    bad += check(5000, 1000, 5, 4, true);
    bad += check(5000, 40000, 8, 5, true);
    bad += check(300, 20000, 400, 6, false);   // > 63 terms in one band
    printf(bad ? "xband_asan: FAILED\n" : "xband_asan: ok\n");
    return bad ? 1 : 0;
}
