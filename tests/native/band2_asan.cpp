// Host-only check of the balanced-band builder (sparsematrix_amd/csrc/band2.cpp),
// built with AddressSanitizer by tests/test_xband_builder.py.  For several shapes
// and slab counts: every term appears exactly once, each row's terms come out in
// ascending column order across the tile's bands (bands ascend, ranks ascend in a
// band), ranks are the term's index in its segment, a segment never spans two
// chunks, columns stay inside the band's 8192-column window, bands ascend and never
// overlap, and padding decodes as dummies with value 0.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "xband.h"

using namespace smamd;

// Builder-only geometries (the kernel runs wide and dma3): tall tiles, three and six chunks
// per wave -- the builder's parameterisation (row and column field widths, chunk counts).
constexpr B2Geom kB2TallB2{1 << 15, 4096, 13};
constexpr B2Geom kB2TallCb{1 << 15, 3840, 13, 2, kCbColBits, 1};
constexpr B2Geom kB2Wide3Cb{1 << 14, 12160, 14, 3, 14, 1};
constexpr B2Geom kB2DmawCb{1 << 14, 11520, 14, 6, 14, 4, 48};


static int check_layout(const std::vector<int32_t> &rp, const std::vector<int32_t> &col,
                        const std::vector<float> &val, int64_t n_rows, int64_t n_cols, int slabs,
                        bool expect_ok, B2Geom geom = kB2Wide, int permille = 1000) {
    Band2Host h;
    const bool ok = band2_build(rp.data(), col.data(), val.data(), n_rows, n_cols, slabs, h, nullptr, geom, permille);
    const uint32_t kDummy = geom.dummy_word();
    const int kCol = geom.col_bits;
    if (ok != expect_ok) { printf("FAIL build=%d expected %d\n", ok, expect_ok); return 1; }
    if (!ok) return 0;
    if ((int64_t)h.band_clo.size() != h.n_bands || (int64_t)h.ent.size() != h.n_bands * 4096) {
        printf("FAIL sizes\n"); return 1; }
    std::vector<std::vector<std::pair<int32_t, float>>> got(n_rows);
    int64_t terms = 0;
    for (int64_t t = 0; t < (int64_t)h.n_blocks * h.n_slabs; t++) {
        const int64_t b = t / h.n_slabs, s = t % h.n_slabs;
        // slab 0 = [0, slab0_cols), slab s >= 1 = [slab0 + (s-1) slab_cols, + slab_cols)
        const int64_t c0 = s == 0 ? 0 : h.slab0_cols + (s - 1) * (int64_t)h.slab_cols;
        const int64_t c1 = std::min<int64_t>(n_cols, s == 0 ? h.slab0_cols : c0 + h.slab_cols);
        int64_t prev_hi = c0;
        for (int64_t g = h.tile_band_start[t]; g < h.tile_band_start[t + 1]; g++) {
            const int64_t clo = h.band_clo[g];
            if (clo % 4) { printf("FAIL clo alignment\n"); return 1; }
            int64_t lo_col = INT64_MAX, hi_col = -1;
            for (int c = 0; c < kB2Chunks; c++) {
                const int wave = c >> 1, k = c & 1;
                std::vector<int> rows_seen;
                for (int l = 0; l < 64; l++) {
                    const uint32_t *e = &h.ent[(size_t)g * 4096 + (size_t)(wave * 64 + l) * 4];
                    const uint32_t w = e[k] ^ kDummy;
                    const uint32_t rank = (w >> kCol) & kB2DummyRank;
                    float v;
                    memcpy(&v, &e[2 + k], 4);
                    if (rank == kB2DummyRank) {
                        if (v != 0.0f || (w & ((1u << kCol) - 1u)) != 0) {
                            printf("FAIL dummy\n"); return 1; }
                        continue;
                    }
                    const uint32_t rl = w >> (kCol + kB2RankBits);
                    const int64_t r = b * h.block_rows + rl;
                    const int64_t cc = clo + (w & ((1u << kCol) - 1u));
                    if (r >= n_rows || (int64_t)rl >= h.block_rows) { printf("FAIL row\n"); return 1; }
                    if (cc - clo >= geom.window || cc < c0 || cc >= c1) { printf("FAIL window\n"); return 1; }
                    if ((int)rank != (int)std::count(rows_seen.begin(), rows_seen.end(), (int)rl)) {
                        printf("FAIL rank\n"); return 1; }
                    if (rank > 0 && (l == 0 || ((h.ent[(size_t)g * 4096 + (size_t)(wave * 64 + l - 1) * 4 + k] ^
                                                 kDummy) >> (kCol + kB2RankBits)) != rl)) {
                        printf("FAIL segment not on consecutive lanes\n"); return 1; }
                    rows_seen.push_back((int)rl);
                    got[r].push_back({(int32_t)cc, v});
                    lo_col = std::min(lo_col, cc);
                    hi_col = std::max(hi_col, cc);
                    terms++;
                }
            }
            if (hi_col < 0) { printf("FAIL empty band\n"); return 1; }
            // Bands never overlap, except the one-column bands a dense column is split
            // into (by rows): those repeat the previous band's single column.
            const bool split_piece = lo_col == hi_col && lo_col == prev_hi - 1;
            if (lo_col < prev_hi && !split_piece) { printf("FAIL bands overlap\n"); return 1; }
            prev_hi = hi_col + 1;
        }
    }
    // A row's segment inside one band sits in one chunk: implied by consecutive lanes +
    // per-chunk ranks starting at 0 (checked above); the order check covers the rest.
    for (int64_t r = 0; r < n_rows; r++) {
        if ((int64_t)got[r].size() != rp[r + 1] - rp[r]) { printf("FAIL count row %lld\n", (long long)r); return 1; }
        // terms of a row arrive band by band; within the tile's walk the bands ascend,
        // but tiles (slabs) were walked in order too, so plain ascending order is required
        for (int32_t e = rp[r]; e < rp[r + 1]; e++)
            if (got[r][e - rp[r]].first != col[e] || got[r][e - rp[r]].second != val[e]) {
                printf("FAIL order row %lld\n", (long long)r); return 1; }
    }
    if (terms != h.real_terms) { printf("FAIL real_terms\n"); return 1; }
    return 0;
}

// cband encoding: rebuild every row from the 32-bit words (header base + offset,
// codebook id, column), check segments sit on consecutive lanes, rows stay within
// the chunk's 2048-row span, ids decode to the term's exact value bits.
static int check_layout_cb(const std::vector<int32_t> &rp, const std::vector<int32_t> &col,
                           const std::vector<float> &val, int64_t n_rows, int64_t n_cols, int slabs,
                           B2Geom geom = kB2Wide, int permille = 1000) {
    std::vector<float> table;
    std::vector<uint8_t> ids;
    if (!codebook_ids(val.data(), (int64_t)val.size(), table, ids)) { printf("FAIL codebook\n"); return 1; }
    for (size_t e = 0; e < val.size(); e++)
        if (memcmp(&table[ids[e]], &val[e], 4) != 0) { printf("FAIL codebook id\n"); return 1; }
    Band2Host h;
    if (!band2_build(rp.data(), col.data(), val.data(), n_rows, n_cols, slabs, h, ids.data(), geom, permille)) {
        printf("FAIL cband build\n"); return 1; }
    const int cpw = geom.cpw, nch = geom.chunks();
    const size_t bw = (size_t)64 * nch;
    const uint32_t dmy = geom.cb_dummy_word(), cmask = (1u << geom.cb_col) - 1u;
    const int osh = geom.cb_off_shift();
    const uint32_t omask = geom.cb_off_mask();
    if (!h.codebook || h.ent.size() != (size_t)h.n_bands * bw) { printf("FAIL cband sizes\n"); return 1; }
    std::vector<std::vector<std::pair<int32_t, float>>> got(n_rows);
    int64_t terms = 0;
    for (int64_t t = 0; t < (int64_t)h.n_blocks * h.n_slabs; t++) {
        const int64_t b = t / h.n_slabs, s = t % h.n_slabs;
        // slab 0 = [0, slab0_cols), slab s >= 1 = [slab0 + (s-1) slab_cols, + slab_cols)
        const int64_t c0 = s == 0 ? 0 : h.slab0_cols + (s - 1) * (int64_t)h.slab_cols;
        const int64_t c1 = std::min<int64_t>(n_cols, s == 0 ? h.slab0_cols : c0 + h.slab_cols);
        for (int64_t g = h.tile_band_start[t]; g < h.tile_band_start[t + 1]; g++) {
            const int64_t clo = h.band_clo[g];
            for (int c = 0; c < nch; c++) {
                const int wave = c / cpw, k = c % cpw;
                auto word = [&](int l) { return h.ent[(size_t)g * bw + (size_t)(wave * 64 + l) * cpw + k] ^ dmy; };
                const uint32_t hd = word(0);
                if (((hd >> geom.cb_col) & kCbDummyId) != kCbDummyId) { printf("FAIL header id\n"); return 1; }
                const uint32_t base = (hd & cmask) | (((hd >> osh) & omask) << geom.cb_col);
                if (hd >> kCbContBit) { printf("FAIL header cont\n"); return 1; }
                std::vector<int> rows_seen;
                int prev_row = -1;
                for (int l = 1; l < 64; l++) {
                    const uint32_t w = word(l);
                    const uint32_t id = (w >> geom.cb_col) & kCbDummyId;
                    if (id == kCbDummyId) {
                        if (w != dmy) { printf("FAIL cband dummy\n"); return 1; }
                        prev_row = -1;
                        continue;
                    }
                    if (id >= table.size()) { printf("FAIL id range\n"); return 1; }
                    const uint32_t rl = base + ((w >> osh) & omask);
                    const bool cont = (w >> kCbContBit) != 0;
                    const int64_t r = b * h.block_rows + rl;
                    const int64_t cc = clo + (w & cmask);
                    if (r >= n_rows || (int64_t)rl >= h.block_rows) { printf("FAIL cband row\n"); return 1; }
                    if (cc - clo >= geom.window || cc < c0 || cc >= c1) { printf("FAIL cband window\n"); return 1; }
                    const int seen = (int)std::count(rows_seen.begin(), rows_seen.end(), (int)rl);
                    if (seen > 0 && prev_row != (int)rl) { printf("FAIL cband segment lanes\n"); return 1; }
                    if (cont != (seen > 0)) { printf("FAIL cband cont flag\n"); return 1; }
                    rows_seen.push_back((int)rl);
                    prev_row = (int)rl;
                    got[r].push_back({(int32_t)cc, table[id]});
                    terms++;
                }
            }
        }
    }
    for (int64_t r = 0; r < n_rows; r++) {
        if ((int64_t)got[r].size() != rp[r + 1] - rp[r]) { printf("FAIL cband count row %lld\n", (long long)r); return 1; }
        for (int32_t e = rp[r]; e < rp[r + 1]; e++)
            if (got[r][e - rp[r]].first != col[e] || memcmp(&got[r][e - rp[r]].second, &val[e], 4) != 0) {
                printf("FAIL cband order row %lld\n", (long long)r); return 1; }
    }
    if (terms != h.real_terms) { printf("FAIL cband real_terms\n"); return 1; }
    return 0;
}

static int check_random(int64_t n_rows, int64_t n_cols, int per_row, unsigned seed, int slabs,
                        bool expect_ok) {
    std::mt19937 rng(seed);
    std::vector<int32_t> rp(n_rows + 1), col;
    std::vector<float> val;
    for (int64_t r = 0; r < n_rows; r++) {
        std::vector<int32_t> c(per_row);
        for (auto &v : c) v = (int32_t)(rng() % n_cols);
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (auto v : c) { col.push_back(v); val.push_back((float)(rng() % 1000) + 1.0f); }
        rp[r + 1] = (int32_t)col.size();
    }
    int bad = check_layout(rp, col, val, n_rows, n_cols, slabs, expect_ok);
    bad += check_layout(rp, col, val, n_rows, n_cols, slabs, expect_ok, kB2TallB2);
    if (expect_ok) {   // the same pattern with a 255-value codebook (incl. -0.0 and +0.0)
        for (size_t e = 0; e < val.size(); e++) {
            const uint32_t i = rng() % 255;
            val[e] = i == 0 ? -0.0f : (float)i * 0.37f - 40.0f;
        }
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2TallCb);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2Wide3Cb);
        // the AUTO geometry (dma3) with slab 0 narrower, as sm_create_* builds it
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2Dma3Cb, 930);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2DmawCb);   // six chunks per wave
    }
    return bad;
}

int main() {
    int bad = 0;
    for (int slabs : {1, 4, 16}) {
        bad += check_random(20011, 300001, 16, 1, slabs, true);
        bad += check_random(3001, 70001, 40, 2, slabs, true);
        bad += check_random(5000, 1000, 5, 4, slabs, true);
        bad += check_random(8009, 1000003, 16, 7, slabs, true);
        bad += check_random(1, 50000, 30, 8, slabs, true);
    }
    // Contiguous runs of 40 columns: bands are cut inside them (<= 14 terms per row).
    {
        const int64_t n_rows = 3000, n_cols = 7000, w = 40;
        std::mt19937 rng(9);
        std::vector<int32_t> rp(n_rows + 1), col;
        std::vector<float> val;
        for (int64_t r = 0; r < n_rows; r++) {
            const int32_t s = (int32_t)(rng() % (n_cols - w));
            for (int j = 0; j < w; j++) { col.push_back(s + j); val.push_back(1.0f + j); }
            rp[r + 1] = (int32_t)col.size();
        }
        bad += check_layout(rp, col, val, n_rows, n_cols, 1, true);
        bad += check_layout(rp, col, val, n_rows, n_cols, 5, true);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, 1);   // 40-term segments fit a chunk
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, 1, kB2Wide3Cb);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, 5);
    }
    // Rows of 70 consecutive columns: cband cuts bands inside them (<= 63 terms).
    {
        const int64_t n_rows = 500, n_cols = 5000, w = 70;
        std::mt19937 rng(10);
        std::vector<int32_t> rp(n_rows + 1), col;
        std::vector<float> val;
        for (int64_t r = 0; r < n_rows; r++) {
            const int32_t s = (int32_t)(rng() % (n_cols - w));
            for (int j = 0; j < w; j++) { col.push_back(s + j); val.push_back((float)(j % 7)); }
            rp[r + 1] = (int32_t)col.size();
        }
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, 1);
    }
    // Sparse rows far apart: chunks close at the 2048-row span.
    {
        const int64_t n_rows = 16384, n_cols = 9000;
        std::vector<int32_t> rp(n_rows + 1, 0), col;
        std::vector<float> val;
        for (int64_t r = 0; r < n_rows; r++) {
            if (r % 3000 == 0) { col.push_back((int32_t)(r % n_cols)); val.push_back(2.0f); }
            rp[r + 1] = (int32_t)col.size();
        }
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, 1);
    }
    // Dense (hub) columns: every row of a 16K-row block holds column 4097, every third
    // row column 9000 (more than 32 chunks of one column in one band: the builder used
    // to loop forever here; now it splits such a column by rows over one-column bands).
    for (int slabs : {1, 3}) {
        const int64_t n_rows = 40000, n_cols = 20000;
        std::mt19937 rng(11);
        std::vector<int32_t> rp(n_rows + 1), col;
        std::vector<float> val;
        for (int64_t r = 0; r < n_rows; r++) {
            std::vector<int32_t> c = {4097};
            if (r % 3 == 0) c.push_back(9000);
            for (int j = 0; j < 6; j++) c.push_back((int32_t)(rng() % n_cols));
            std::sort(c.begin(), c.end());
            c.erase(std::unique(c.begin(), c.end()), c.end());
            for (auto v : c) { col.push_back(v); val.push_back((float)(rng() % 200) * 0.5f - 7.0f); }
            rp[r + 1] = (int32_t)col.size();
        }
        bad += check_layout(rp, col, val, n_rows, n_cols, slabs, true);
        bad += check_layout(rp, col, val, n_rows, n_cols, slabs, true, kB2TallB2);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2TallCb);
        bad += check_layout_cb(rp, col, val, n_rows, n_cols, slabs, kB2Wide3Cb);
    }
    // More than 255 distinct values: no codebook.
    {
        std::vector<float> v(1000), table;
        std::vector<uint8_t> ids;
        for (int i = 0; i < 1000; i++) v[i] = (float)(i % 256);
        if (codebook_ids(v.data(), 1000, table, ids)) { printf("FAIL codebook accepted 256 values\n"); bad++; }
        for (int i = 0; i < 1000; i++) v[i] = (float)(i % 255);
        if (!codebook_ids(v.data(), 1000, table, ids) || table.size() != 255) { printf("FAIL codebook 255\n"); bad++; }
    }
    // Unsorted columns are rejected.
    {
        std::vector<int32_t> rp = {0, 3}, col = {5, 2, 9};
        std::vector<float> val = {1, 2, 3};
        bad += check_layout(rp, col, val, 1, 10, 1, false);
    }
    {   // x of 4 GiB or more: 32-bit byte offsets into x would wrap, so the builder declines
        const std::vector<int32_t> rp = {0, 2}, col = {3, (1 << 30) + 5};
        const std::vector<float> val = {1.0f, 2.0f};
        Band2Host h;
        if (band2_build(rp.data(), col.data(), val.data(), 1, (int64_t)1 << 30, 1, h)) {
            printf("band2_build accepted 2^30 columns\n");
            bad++;
        }
    }
    printf(bad ? "band2_asan: FAILED\n" : "band2_asan: ok\n");
    return bad ? 1 : 0;
}
