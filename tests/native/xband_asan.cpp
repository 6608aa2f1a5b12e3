// Host-only check of the column-band builder (sparsematrix_amd/csrc/xband.cpp),
// built with AddressSanitizer by tests/test_xband_builder.py: for the three layouts
// (exact, blocked, gather = blocked bits with column-ordered segments) and several
// shapes, every term appears exactly once, per row
// in ascending column order (bands ascend, ranks ascend inside a band), with
// correct ranks, no row's segment split across chunks, the register capacity
// respected, padding decoding as dummies, and (gather) a band's chunks in ascending
// order of their segments' first columns.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "xband.h"

using namespace smamd;

static int check(XbBits bits, int waves, int64_t n_rows, int64_t n_cols, int per_row,
                 unsigned seed, bool expect_ok, bool col_order = false) {
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
    const bool ok = xband_build(rp.data(), col.data(), val.data(), n_rows, n_cols, bits, waves, xh,
                                col_order);
    if (ok != expect_ok) { printf("FAIL build=%d expected %d\n", ok, expect_ok); return 1; }
    if (!ok) return 0;
    if (xh.block_rows > (1 << bits.row) || xh.band_cols != (1 << bits.col)) {
        printf("FAIL geometry\n"); return 1; }
    if (xh.max_chunks_per_band > kXbMaxCap * waves) {
        printf("FAIL register capacity\n"); return 1; }
    const uint32_t colmask = (1u << bits.col) - 1u, rankmask = (1u << bits.rank) - 1u;
    std::vector<std::vector<std::pair<int32_t, float>>> got(n_rows);
    for (int64_t b = 0; b < xh.n_blocks; b++)
        for (int64_t p = 0; p < xh.n_bands; p++) {
            const int64_t c0 = xh.chunk_start[b * xh.n_bands + p];
            const int64_t c1 = xh.chunk_start[b * xh.n_bands + p + 1];
            std::vector<int64_t> owner(xh.block_rows, -1);   // chunk holding the row's segment
            uint32_t prev_max = 0;                             // col_order: previous chunk's last first-column
            for (int64_t c = c0; c < c1; c++) {
                std::vector<int> seen_rows;
                uint32_t cmin = 0xFFFFFFFFu, cmax = 0;
                for (int l = 0; l < 64; l++) {
                    const size_t idx = (size_t)(c * 64 + l);
                    const uint32_t w = xh.word[idx] ^ bits.dummy_word();
                    const uint32_t rank = (w >> bits.col) & rankmask;
                    if (rank == bits.dummy_rank()) {
                        if (xh.val[idx] != 0.0f) { printf("FAIL dummy value\n"); return 1; }
                        continue;
                    }
                    const uint32_t cl = w & colmask;
                    const uint32_t rl = w >> (bits.col + bits.rank);
                    const int64_t r = b * xh.block_rows + rl;
                    if (rl >= (uint32_t)xh.block_rows || r >= n_rows) {
                        printf("FAIL row out of range\n"); return 1; }
                    if (owner[rl] != -1 && owner[rl] != c) {
                        printf("FAIL segment split across chunks\n"); return 1; }
                    owner[rl] = c;
                    if ((int64_t)rank != (int64_t)std::count(seen_rows.begin(), seen_rows.end(), (int)rl)) {
                        printf("FAIL rank\n"); return 1; }
                    seen_rows.push_back((int)rl);
                    got[r].push_back({(int32_t)(p * xh.band_cols + cl), xh.val[idx]});
                    if (rank == 0) { cmin = std::min(cmin, cl); cmax = std::max(cmax, cl); }
                }
                if (col_order && cmin != 0xFFFFFFFFu) {
                    if (cmin < prev_max) { printf("FAIL column order across chunks\n"); return 1; }
                    prev_max = cmax;
                }
            }
        }
    for (int64_t r = 0; r < n_rows; r++) {
        if ((int64_t)got[r].size() != rp[r + 1] - rp[r]) {
            printf("FAIL count row %lld\n", (long long)r); return 1; }
        for (int32_t e = rp[r]; e < rp[r + 1]; e++)
            if (got[r][e - rp[r]].first != col[e] || got[r][e - rp[r]].second != val[e]) {
                printf("FAIL order row %lld\n", (long long)r); return 1; }
    }
    return 0;
}

int main() {
    const XbBits exact = xb_bits(kXbExactBandLog2, kXbExactRowsLog2);
    const XbBits blocked = xb_bits(kXbBlockedBandLog2, kXbBlockedRowsLog2);
    int bad = 0;
    const XbBits gather = xb_bits(kXbGatherBandLog2, kXbGatherRowsLog2);
    const struct { XbBits bits; int waves; bool col_order; } kinds[] = {
        {exact, kXbThreads / 64, false}, {blocked, kXbComputeWaves, false},
        {gather, kXbThreads / 64, true}};
    for (const auto &k : kinds) {
        const bool co = k.col_order;
        bad += check(k.bits, k.waves, 200003, 300001, 16, 1, true, co);
        bad += check(k.bits, k.waves, 9000, 70001, 40, 2, true, co);    // dense bands: smaller blocks
        bad += check(k.bits, k.waves, 4096, 32768, 7, 3, true, co);
        bad += check(k.bits, k.waves, 5000, 1000, 5, 4, true, co);
        bad += check(k.bits, k.waves, 5000, 40000, 8, 5, true, co);
        bad += check(k.bits, k.waves, 70000, 1000003, 16, 7, true, co);
        bad += check(k.bits, k.waves, 300, 20000, 400, 6, false, co);   // a row's segment too long for the rank field
    }
    printf(bad ? "xband_asan: FAILED\n" : "xband_asan: ok\n");
    return bad ? 1 : 0;
}
