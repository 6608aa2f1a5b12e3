// Host-only check of the row-owner band builder (sparsematrix_amd/csrc/ro.cpp), built with
// AddressSanitizer by tests/test_xband_builder.py.  Decodes every chunk as kernels_ro.hip
// does (header: window, base row relative to the wave; terms: column in window, id, row
// offset, continuation) and checks: every term exactly once, each row's terms in ascending
// column order in stream order, rows inside the owning wave's range, chunk windows
// non-decreasing along a wave's stream, segments on consecutive lanes, ids exact.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ro.h"
#include "xband.h"

using namespace smamd;

static int check(const std::vector<int32_t> &rp, const std::vector<int32_t> &col, const std::vector<float> &val,
                 int64_t n_rows, int64_t n_cols, int slabs) {
    std::vector<float> table;
    std::vector<uint8_t> ids;
    if (!codebook_ids(val.data(), (int64_t)val.size(), table, ids)) { printf("FAIL codebook\n"); return 1; }
    RoHost h;
    if (!ro_build(rp.data(), col.data(), ids.data(), n_rows, n_cols, slabs, h)) { printf("FAIL build\n"); return 1; }
    const uint32_t dmy = kCbDummyWord;
    std::vector<std::vector<std::pair<int32_t, float>>> got((size_t)n_rows);
    for (int64_t t = 0; t < (int64_t)h.n_blocks * h.n_slabs; t++) {
        const int64_t b = t / h.n_slabs, s = t % h.n_slabs;
        const int64_t c0 = s * (int64_t)h.slab_cols, c1 = std::min<int64_t>(n_cols, c0 + h.slab_cols);
        for (int w = 0; w < kRoApplyWaves; w++) {
            const int32_t cs = h.wave_start[(size_t)(t * kRoApplyWaves + w)], ce = h.wave_start[(size_t)(t * kRoApplyWaves + w + 1)];
            const int64_t wr0 = b * h.block_rows + (int64_t)w * kRoWaveRows;
            int32_t prev_q = -1;
            for (int32_t c = cs; c < ce; c++) {
                const uint32_t *e = &h.ent[(size_t)c * 64];
                const uint32_t hd = e[0] ^ dmy;
                if (((hd >> 13) & kCbDummyId) != kCbDummyId) { printf("FAIL header id\n"); return 1; }
                const int32_t q = (int32_t)(hd & (uint32_t)(kRoMaxWindows - 1));
                const int32_t stage = (int32_t)((hd >> kRoStageShift) & 3u);
                const int32_t brel = (int32_t)(((hd >> 21) & kCbOffMask) | ((hd >> 31) << 10));
                if (q < prev_q) { printf("FAIL window order\n"); return 1; }
                prev_q = q;
                const int64_t clo = c0 + (int64_t)q * kRoWindow;
                // the stage: 1 + the highest stage of the earlier chunks of its group (kRoGroup
                // aligned in the wave's stream) it shares a row with, else 0
                {
                    const int32_t gi = (c - cs) % kRoGroup;
                    std::vector<int32_t> mine;
                    for (int l = 1; l < 64; l++) {
                        const uint32_t wc = e[l] ^ dmy;
                        if (((wc >> 13) & kCbDummyId) != kCbDummyId) mine.push_back(brel + (int32_t)((wc >> 21) & kCbOffMask));
                    }
                    int32_t want = 0;
                    for (int32_t j = c - gi; j < c; j++) {
                        const uint32_t ph = h.ent[(size_t)j * 64] ^ dmy;
                        const int32_t pb = (int32_t)(((ph >> 21) & kCbOffMask) | ((ph >> 31) << 10));
                        bool share = false;
                        for (int l = 1; l < 64 && !share; l++) {
                            const uint32_t wp = h.ent[(size_t)j * 64 + l] ^ dmy;
                            if (((wp >> 13) & kCbDummyId) == kCbDummyId) continue;
                            share = std::count(mine.begin(), mine.end(), pb + (int32_t)((wp >> 21) & kCbOffMask)) > 0;
                        }
                        if (share) want = std::max(want, (int32_t)((ph >> kRoStageShift) & 3u) + 1);
                    }
                    if (want != stage) { printf("FAIL stage\n"); return 1; }
                }
                int32_t prev_row = -1;
                std::vector<int32_t> seen;
                for (int l = 1; l < 64; l++) {
                    const uint32_t wd = e[l] ^ dmy;
                    const uint32_t id = (wd >> 13) & kCbDummyId;
                    if (id == kCbDummyId) {
                        if (wd != dmy) { printf("FAIL dummy\n"); return 1; }
                        prev_row = -1;
                        continue;
                    }
                    if (id >= table.size()) { printf("FAIL id range\n"); return 1; }
                    const int64_t r = wr0 + brel + ((wd >> 21) & kCbOffMask);
                    const bool cont = (wd >> 31) != 0;
                    const int64_t cc = clo + (wd & 8191u);
                    if (r < wr0 || r >= wr0 + kRoWaveRows || r >= n_rows) { printf("FAIL row range\n"); return 1; }
                    if (cc < c0 || cc >= c1 || (wd & 8191u) >= (uint32_t)kRoWindow) { printf("FAIL window\n"); return 1; }
                    const bool again = std::count(seen.begin(), seen.end(), (int32_t)r) > 0;
                    if (again && prev_row != (int32_t)r) { printf("FAIL segment lanes\n"); return 1; }
                    if (cont != again) { printf("FAIL cont flag\n"); return 1; }
                    seen.push_back((int32_t)r);
                    prev_row = (int32_t)r;
                    got[(size_t)r].push_back({(int32_t)cc, table[id]});
                }
            }
        }
    }
    for (int64_t r = 0; r < n_rows; r++) {
        // per slab in stream order; slabs in tile order: concatenated they are the row
        if ((int64_t)got[(size_t)r].size() != rp[r + 1] - rp[r]) { printf("FAIL count row %lld\n", (long long)r); return 1; }
        for (int32_t e = rp[r]; e < rp[r + 1]; e++) {
            const auto &g = got[(size_t)r][(size_t)(e - rp[r])];
            if (g.first != col[e] || memcmp(&g.second, &val[e], 4) != 0) { printf("FAIL term order row %lld\n", (long long)r); return 1; }
        }
    }
    return 0;
}

int main() {
    std::mt19937_64 rng(7);
    int bad = 0;
    struct Case { int64_t rows, cols; int per; int slabs; int run; };
    for (const Case &c : {Case{40000, 300001, 16, 4, 0}, Case{20011, 100003, 16, 1, 0}, Case{5000, 1000, 5, 2, 0},
                          Case{3000, 70001, 40, 3, 0}, Case{2000, 20000, 0, 2, 150}, Case{1, 50000, 300, 1, 0}}) {
        std::vector<int32_t> rp(1, 0), col;
        std::vector<float> val;
        for (int64_t r = 0; r < c.rows; r++) {
            std::vector<int32_t> cs;
            if (c.run) {   // long consecutive runs: rows cut over several chunks
                const int32_t s = (int32_t)(rng() % (uint64_t)(c.cols - c.run));
                for (int i = 0; i < c.run; i++) cs.push_back(s + i);
            } else {
                for (int i = 0; i < c.per; i++) cs.push_back((int32_t)(rng() % (uint64_t)c.cols));
            }
            std::sort(cs.begin(), cs.end());
            cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
            for (int32_t x : cs) {
                col.push_back(x);
                const uint32_t i = (uint32_t)(rng() % 255);
                val.push_back(i == 0 ? -0.0f : (float)i * 0.37f - 40.0f);
            }
            rp.push_back((int32_t)col.size());
        }
        bad += check(rp, col, val, c.rows, c.cols, c.slabs);
    }
    printf(bad ? "ro_asan: FAILED\n" : "ro_asan: ok\n");
    return bad ? 1 : 0;
}
