// Host-only check of the column-chunked sliced-ELL builder (sparsematrix_amd/csrc/
// ccsell.cpp), built with AddressSanitizer by tests/test_xband_builder.py.  Walking the
// chunks in order and every slice's lanes, each row's terms come out exactly once, in
// ascending column order, with their values (codebook ids or plain); each row's first
// unit (and only it) carries the first flag, rows without terms get one empty unit in
// chunk 0, units of a slice are sorted by length (or kept in row order), a unit's
// columns stay inside its chunk, a slice is as long as its longest unit with zero
// words past each unit, and oversized units decline.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ccsell.h"
#include "sell.h"

using namespace smamd;

static int check(const std::vector<int32_t> &rp, const std::vector<int32_t> &col,
                 const std::vector<float> &val, int64_t n_rows, int64_t n_cols, int chunk_log2,
                 bool codebook, bool by_length = true) {
    std::vector<uint8_t> ids;
    std::vector<float> table;
    if (codebook) {
        for (float v : val) {
            auto it = std::find(table.begin(), table.end(), v);
            if (it == table.end()) { table.push_back(v); it = table.end() - 1; }
            ids.push_back((uint8_t)(it - table.begin()));
        }
        if (table.size() > 255) { printf("FAIL test codebook\n"); return 1; }
    }
    CcsellHost h;
    if (!ccsell_build(rp.data(), col.data(), val.data(), codebook ? ids.data() : nullptr, n_rows,
                      n_cols, chunk_log2, h, by_length)) { printf("FAIL build\n"); return 1; }
    const int64_t nch = (n_cols + ((int64_t)1 << chunk_log2) - 1) >> chunk_log2;
    if (h.n_chunks != nch || (int64_t)h.chunk_slice.size() != nch + 1) { printf("FAIL chunks\n"); return 1; }
    std::vector<std::vector<std::pair<int32_t, float>>> got(n_rows);
    std::vector<int> firsts(n_rows, 0);
    std::vector<int64_t> last_chunk(n_rows, -1);
    const uint32_t cmask = (uint32_t)((1ull << chunk_log2) - 1);
    for (int64_t c = 0; c < nch; c++) {
        for (int64_t s = h.chunk_slice[c]; s < h.chunk_slice[c + 1]; s++) {
            int prev_n = 1 << 30, longest = 0, prev_row = -1;
            for (int l = 0; l < kSellLanes; l++) {
                const int32_t rw = h.row[s * kSellLanes + l];
                const int n = h.row_len[s * kSellLanes + l];
                if (rw == -1) { if (n) { printf("FAIL empty lane len\n"); return 1; } continue; }
                if (by_length && n > prev_n) { printf("FAIL slice not sorted\n"); return 1; }
                if (!by_length && (rw & 0x7FFFFFFF) <= prev_row) { printf("FAIL not in row order\n"); return 1; }
                prev_n = n;
                prev_row = rw & 0x7FFFFFFF;
                longest = std::max(longest, n);
                if (n > h.len[s]) { printf("FAIL unit longer than slice\n"); return 1; }
                const int32_t r = rw & 0x7FFFFFFF;
                if (r >= n_rows) { printf("FAIL row range\n"); return 1; }
                if (last_chunk[r] >= c) { printf("FAIL two units of a row in one chunk\n"); return 1; }
                last_chunk[r] = c;
                if (rw & (int32_t)kCcFirst) {
                    if (!got[r].empty() || firsts[r]) { printf("FAIL first flag not first\n"); return 1; }
                    firsts[r]++;
                } else if (!firsts[r]) { printf("FAIL unit before the first\n"); return 1; }
                for (int j = 0; j < h.len[s]; j++) {
                    const uint32_t w = h.word[h.off[s] + (int64_t)j * kSellLanes + l];
                    if (j >= n) {
                        if (w != 0 || (!codebook && h.val[h.off[s] + (int64_t)j * kSellLanes + l] != 0.0f)) {
                            printf("FAIL padding\n"); return 1; }
                        continue;
                    }
                    const int32_t cc = (int32_t)((c << chunk_log2) + (w & cmask));
                    const float v = codebook ? table[w >> chunk_log2]
                                             : h.val[h.off[s] + (int64_t)j * kSellLanes + l];
                    got[r].push_back({cc, v});
                }
            }
            if (longest != h.len[s]) { printf("FAIL slice length is not its longest unit\n"); return 1; }
        }
    }
    for (int64_t r = 0; r < n_rows; r++) {
        if (firsts[r] != 1) { printf("FAIL row %lld has %d first units\n", (long long)r, firsts[r]); return 1; }
        if ((int64_t)got[r].size() != rp[r + 1] - rp[r]) { printf("FAIL count row %lld\n", (long long)r); return 1; }
        for (int32_t e = rp[r]; e < rp[r + 1]; e++)
            if (got[r][e - rp[r]].first != col[e] || memcmp(&got[r][e - rp[r]].second, &val[e], 4) != 0) {
                printf("FAIL order row %lld\n", (long long)r); return 1; }
    }
    return 0;
}

static int random_case(int64_t n_rows, int64_t n_cols, int per_row, unsigned seed, int chunk_log2,
                       bool codebook, bool by_length = true) {
    std::mt19937 rng(seed);
    std::vector<int32_t> rp(n_rows + 1), col;
    std::vector<float> val;
    for (int64_t r = 0; r < n_rows; r++) {
        std::vector<int32_t> c;
        const int k = (r % 11 == 0) ? 0 : (int)(rng() % (2 * per_row + 1));
        for (int j = 0; j < k; j++) c.push_back((int32_t)(rng() % n_cols));
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        for (auto v : c) {
            col.push_back(v);
            val.push_back(codebook ? (float)(rng() % 200) * 0.25f - 9.0f : (float)(rng() % 100000) * 1e-3f);
        }
        rp[r + 1] = (int32_t)col.size();
    }
    return check(rp, col, val, n_rows, n_cols, chunk_log2, codebook, by_length);
}

int main() {
    int bad = 0;
    for (bool cb : {true, false}) {
        bad += random_case(20000, 1 << 20, 16, 1, 16, cb);
        bad += random_case(5000, 300001, 40, 2, 12, cb);
        bad += random_case(3, 1000, 300, 3, 8, cb);
        bad += random_case(100000, 5000000, 4, 4, 20, cb);
        bad += random_case(20000, 1 << 20, 16, 5, 16, cb, false);
    }
    // A run of more than 2048 terms inside one chunk declines.
    {
        std::vector<int32_t> rp = {0, 3000}, col(3000);
        std::vector<float> val(3000, 1.0f);
        for (int i = 0; i < 3000; i++) col[i] = i;
        CcsellHost h;
        if (ccsell_build(rp.data(), col.data(), val.data(), nullptr, 1, 1 << 20, 20, h)) {
            printf("FAIL oversized unit accepted\n"); bad++; }
        if (!ccsell_build(rp.data(), col.data(), val.data(), nullptr, 1, 1 << 20, 10, h)) {
            printf("FAIL 1024-column chunks should fit\n"); bad++; }
    }
    // Unsorted columns decline.
    {
        std::vector<int32_t> rp = {0, 3}, col = {5, 2, 9};
        std::vector<float> val = {1, 2, 3};
        CcsellHost h;
        if (ccsell_build(rp.data(), col.data(), val.data(), nullptr, 1, 10, 8, h)) {
            printf("FAIL unsorted accepted\n"); bad++; }
    }
    printf(bad ? "ccsell_asan: FAILED\n" : "ccsell_asan: ok\n");
    return bad ? 1 : 0;
}
