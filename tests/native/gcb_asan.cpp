// Host-only check of the gathered-chunk-band builder (sparsematrix_amd/csrc/gcb.cpp), built
// with AddressSanitizer by tests/test_xband_builder.py.  Decodes every band exactly as
// kernels_gcb.hip does (lane 0 of a chunk = its base row; row = base + offset; live and
// continuation bits) and checks: every term appears exactly once with its value; each row's
// terms come out in ascending column order over the tile's bands and, inside a band, as one
// run of consecutive lanes of one chunk whose lanes after the first are continuations;
// columns stay within the band's window and the tile's slab; a row appears in at most one
// chunk per band; padding decodes as dummies with value 0.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "gcb.h"

using namespace smamd;

static int check(const std::vector<int32_t> &rp, const std::vector<int32_t> &col, const std::vector<float> &val,
                 int64_t n_rows, int64_t n_cols, int rows_log2, int slabs, int32_t window) {
    GcbHost h;
    if (!gcb_build(rp.data(), col.data(), val.data(), n_rows, n_cols, rows_log2, slabs, window, h)) {
        printf("FAIL build\n");
        return 1;
    }
    if ((int64_t)h.band_clo.size() != h.n_bands || (int64_t)h.ent.size() != h.n_bands * kGcbBandWords) {
        printf("FAIL sizes\n");
        return 1;
    }
    std::vector<std::vector<std::pair<int32_t, float>>> got((size_t)n_rows);
    int64_t terms = 0;
    for (int64_t t = 0; t < (int64_t)h.n_blocks * h.n_slabs; t++) {
        const int64_t b = t / h.n_slabs, s = t % h.n_slabs;
        const int64_t c0 = s * h.slab_cols, c1 = std::min<int64_t>(n_cols, c0 + h.slab_cols);
        std::vector<int64_t> seen_in((size_t)h.block_rows, -1);   // last band a row started a segment in
        for (int64_t g = h.tile_band_start[(size_t)t]; g < h.tile_band_start[(size_t)t + 1]; g++) {
            const int64_t clo = h.band_clo[(size_t)g];
            for (int c = 0; c < kGcbChunks; c++) {
                const int wave = c >> 1, k = c & 1;
                auto word = [&](int l) { return h.ent[(size_t)g * kGcbBandWords + (size_t)(wave * 64 + l) * 4 + k]; };
                auto value = [&](int l) {
                    float v;
                    memcpy(&v, &h.ent[(size_t)g * kGcbBandWords + (size_t)(wave * 64 + l) * 4 + 2 + k], 4);
                    return v;
                };
                const uint32_t hdr = word(0);
                if (hdr & (kGcbLive | kGcbCont)) { printf("FAIL header flags\n"); return 1; }
                const int64_t base = hdr & kGcbColMask;
                int32_t prev_row = -1;
                for (int l = 1; l < 64; l++) {
                    const uint32_t w = word(l);
                    if (!(w & kGcbLive)) {
                        if (w != 0 || value(l) != 0.0f) { printf("FAIL dummy\n"); return 1; }
                        prev_row = -1;
                        continue;
                    }
                    const int64_t rl = base + ((w >> kGcbColBits) & kGcbOffMask);
                    const int64_t r = b * h.block_rows + rl;
                    const int64_t cc = clo + (w & kGcbColMask);
                    if (r >= n_rows || rl >= h.block_rows) { printf("FAIL row\n"); return 1; }
                    if (cc - clo >= window || cc < c0 || cc >= c1) { printf("FAIL window\n"); return 1; }
                    const bool cont = (w & kGcbCont) != 0;
                    if (cont != (prev_row == (int32_t)rl)) { printf("FAIL continuation\n"); return 1; }
                    if (!cont) {
                        if (seen_in[(size_t)rl] == g) {
                            printf("FAIL row twice in a band\n");
                            return 1;
                        }
                        seen_in[(size_t)rl] = g;
                    }
                    prev_row = (int32_t)rl;
                    got[(size_t)r].push_back({(int32_t)cc, value(l)});
                    terms++;
                }
            }
        }
    }
    if (terms != rp[(size_t)n_rows]) { printf("FAIL term count %lld vs %d\n", (long long)terms, rp[(size_t)n_rows]); return 1; }
    for (int64_t r = 0; r < n_rows; r++) {
        // per slab in ascending column order; concatenated over slabs the row's own order
        std::vector<std::pair<int32_t, float>> want;
        for (int32_t e = rp[(size_t)r]; e < rp[(size_t)r + 1]; e++) want.push_back({col[(size_t)e], val[(size_t)e]});
        if (got[(size_t)r].size() != want.size()) { printf("FAIL row %lld size\n", (long long)r); return 1; }
        std::vector<std::pair<int32_t, float>> g = got[(size_t)r];
        // decoded in tile order (slabs ascend within a block), bands ascend within a tile
        for (size_t i = 0; i < g.size(); i++)
            if (g[i].first != want[i].first || memcmp(&g[i].second, &want[i].second, 4) != 0) {
                printf("FAIL row %lld order\n", (long long)r);
                return 1;
            }
    }
    return 0;
}

int main() {
    std::mt19937_64 rng(42);
    int fails = 0;
    struct Case { int64_t rows, cols; int per, rows_log2, slabs; int32_t window; };
    for (const Case &c : {Case{20000, 3000001, 16, 15, 1, 1 << 18}, Case{20000, 3000001, 16, 14, 3, 1 << 18},
                          Case{9000, 70001, 40, 14, 1, 4096}, Case{5000, 1000, 5, 14, 2, 1 << 18},
                          Case{1, 50000, 300, 14, 1, 1 << 18}, Case{20000, 20000, 3, 15, 4, 1 << 12}}) {
        std::vector<int32_t> rp(1, 0), col;
        std::vector<float> val;
        for (int64_t r = 0; r < c.rows; r++) {
            std::vector<int32_t> cs;
            for (int i = 0; i < c.per; i++) cs.push_back((int32_t)(rng() % (uint64_t)c.cols));
            std::sort(cs.begin(), cs.end());
            cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
            for (int32_t x : cs) {
                col.push_back(x);
                val.push_back((float)((int64_t)(rng() % 2001) - 1000) / 7.0f);
            }
            rp.push_back((int32_t)col.size());
        }
        fails += check(rp, col, val, c.rows, c.cols, c.rows_log2, c.slabs, c.window);
    }
    {   // long consecutive runs (segments cut at 63 terms) and hub columns in every row
        const int64_t rows = 2000, cols = 700000;
        std::vector<int32_t> rp(1, 0), col;
        std::vector<float> val;
        for (int64_t r = 0; r < rows; r++) {
            const int32_t s = (int32_t)(10 + rng() % (uint64_t)(cols - 200));
            std::vector<int32_t> cs = {5, 600000};
            for (int i = 0; i < 90; i++) cs.push_back(s + i);
            std::sort(cs.begin(), cs.end());
            cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
            for (int32_t x : cs) {
                col.push_back(x);
                val.push_back((float)(rng() % 1000));
            }
            rp.push_back((int32_t)col.size());
        }
        fails += check(rp, col, val, rows, cols, 14, 1, 1 << 18);
        fails += check(rp, col, val, rows, cols, 14, 2, 1 << 18);
    }
    {   // x of 4 GiB or more: the kernel's 32-bit byte offsets into x would wrap, so the
        // builder must decline -- here and in band2_build.
        const std::vector<int32_t> rp = {0, 2}, col = {3, (1 << 30) + 5};
        const std::vector<float> val = {1.0f, 2.0f};
        GcbHost h;
        for (int64_t cols : {(int64_t)1 << 30, ((int64_t)1 << 31) - 1})
            if (gcb_build(rp.data(), col.data(), val.data(), 1, cols, 14, 1, 1 << 18, h)) {
                printf("gcb_build accepted %lld columns (x >= 4 GiB)\n", (long long)cols);
                fails++;
            }
        const std::vector<int32_t> col2 = {3, (1 << 30) - 5};
        if (!gcb_build(rp.data(), col2.data(), val.data(), 1, ((int64_t)1 << 30) - 1, 14, 1, 1 << 18, h)) {
            printf("gcb_build declined 2^30 - 1 columns\n");
            fails++;
        }
    }
    if (fails) return 1;
    printf("gcb_asan: ok\n");
    return 0;
}
