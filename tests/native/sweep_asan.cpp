// Host-only check of the column-swept row-block builder (sparsematrix_amd/csrc/sweep.cpp),
// built with AddressSanitizer by tests/test_xband_builder.py.  Walking each block's
// chunks in order: every row's terms come out exactly once, in ascending column order,
// with their ids; inside a chunk a row's terms sit in consecutive lanes with the
// continuation bit on all but the first; padding slots carry the dummy id; the chunk
// counts match; unsorted rows decline.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "sweep.h"

using namespace smamd;

static int fails = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);                \
            fails++;                                                          \
        }                                                                     \
    } while (0)

static void check(int64_t n_rows, int64_t n_cols, int per_lo, int per_hi, uint32_t seed) {
    std::mt19937 rng(seed);
    std::vector<int32_t> rp(1, 0), col;
    std::vector<uint8_t> ids;
    for (int64_t r = 0; r < n_rows; r++) {
        const int n = per_lo + (int)(rng() % (uint32_t)(per_hi - per_lo + 1));
        std::vector<int32_t> c;
        for (int k = 0; k < n; k++) c.push_back((int32_t)(rng() % (uint32_t)n_cols));
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (int32_t v : c) { col.push_back(v); ids.push_back((uint8_t)(rng() % 255)); }
        rp.push_back((int32_t)col.size());
    }
    SweepHost h;
    CHECK(sweep_build(rp.data(), col.data(), ids.data(), n_rows, h));
    CHECK(h.n_blocks == (n_rows + kSwRows - 1) / kSwRows);
    std::vector<int32_t> seen(n_rows, 0);
    for (int64_t b = 0; b < h.n_blocks; b++) {
        const int64_t r0 = b * kSwRows;
        const int64_t r1 = std::min(n_rows, r0 + kSwRows);
        CHECK(h.block_chunk[b + 1] - h.block_chunk[b] == (rp[r1] - rp[r0] + 63) / 64);
        std::vector<int64_t> pos(kSwRows, 0);   // next term of each row
        for (int64_t c = h.block_chunk[b]; c < h.block_chunk[b + 1]; c++) {
            const uint32_t *ch = h.ent.data() + c * 128;
            std::vector<char> in_chunk(kSwRows, 0);
            int32_t prev_row = -1;
            for (int l = 0; l < 64; l++) {
                const uint32_t cl = ch[2 * l], meta = ch[2 * l + 1];
                const uint32_t id = (meta >> 16) & 0xFF, row = meta & 0xFFF;
                const bool cont = (meta & kSwContBit) != 0;
                if (id == kSwDummyId) { CHECK(!cont); prev_row = -1; continue; }
                CHECK(row < (uint32_t)(r1 - r0));
                CHECK(cont == (prev_row == (int32_t)row));
                if (!cont) { CHECK(!in_chunk[row]); in_chunk[row] = 1; }
                const int64_t r = r0 + row;
                const int64_t e = rp[r] + pos[row];
                CHECK(e < rp[r + 1]);
                if (e < rp[r + 1]) {
                    CHECK((int32_t)cl == col[e]);
                    CHECK(id == ids[e]);
                }
                pos[row]++;
                seen[r]++;
                prev_row = (int32_t)row;
            }
        }
    }
    for (int64_t r = 0; r < n_rows; r++) CHECK(seen[r] == rp[r + 1] - rp[r]);
}

int main() {
    check(1, 10, 0, 0, 1);
    check(1000, 1 << 20, 0, 40, 2);              // empty and ragged rows, not a multiple of 256
    check(3000, 1 << 23, 16, 16, 3);             // wide, uniform
    check(700, 5000, 100, 300, 4);               // rows longer than a chunk: segments across chunks
    check(513, 300, 0, 300, 5);                  // dense-ish: long segments inside one chunk
    {   // unsorted row declines
        std::vector<int32_t> rp = {0, 2}, col = {5, 3};
        std::vector<uint8_t> ids = {0, 1};
        SweepHost h;
        CHECK(!sweep_build(rp.data(), col.data(), ids.data(), 1, h));
    }
    if (fails) {
        printf("sweep_asan: %d failures\n", fails);
        return 1;
    }
    printf("sweep_asan: ok\n");
    return 0;
}
