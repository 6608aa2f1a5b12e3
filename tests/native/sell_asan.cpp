// Host-only check of the sorted sliced-ELL builder (sparsematrix_amd/csrc/sell.cpp),
// built with AddressSanitizer by tests/test_xband_builder.py.  For random and skewed
// shapes: every row of at most max_len terms sits in exactly one lane with its terms
// in stored order, every longer row in consecutive max_len-term segments (one lane
// each, partials in segment order), slices are sorted by length (longest first; with
// sigma windows: within a slice, whose units share one window, dealt to the stream of
// the slice's group) and padded to multiples of kSellUnroll with column 0 / value 0, lanes past the units
// hold -1.  Codebook form (ids): every slot is column | id << 24, padding 0, no values.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "sell.h"

using namespace smamd;

static int check(const std::vector<int32_t> &rp, const std::vector<int32_t> &col,
                 const std::vector<float> &val, int64_t n_rows, int32_t max_len,
                 int64_t sigma = 0, int streams = 1, bool cb = false) {
    SellHost h;
    std::vector<uint8_t> ids(val.size());
    for (size_t i = 0; i < val.size(); i++) ids[i] = (uint8_t)(val[i] + 48.0f);   // values in [-48, 48]
    sell_build(rp.data(), col.data(), val.data(), n_rows, max_len, h, sigma, streams,
               cb ? ids.data() : nullptr);
    if (cb ? !h.val.empty() : h.val.size() != h.col.size()) { printf("FAIL value slots\n"); return 1; }
    // term i as stored: (column, value) or the codebook word with value 0
    auto same = [&](size_t k, int64_t i) {
        if (cb) return (uint32_t)h.col[k] == (i < 0 ? 0u : ((uint32_t)col[(size_t)i] | (uint32_t)ids[(size_t)i] << kSellCbColBits));
        return h.col[k] == (i < 0 ? 0 : col[(size_t)i]) && h.val[k] == (i < 0 ? 0.0f : val[(size_t)i]);
    };
    std::vector<int> seen((size_t)n_rows, 0);
    // Segments: partial p -> (long row, first term); long_ptr gives each row's partials.
    const int32_t n_parts = h.long_ptr.back();
    std::vector<int> part_seen((size_t)n_parts, 0);
    std::vector<int32_t> part_row((size_t)n_parts), part_start((size_t)n_parts);
    for (size_t i = 0; i < h.long_rows.size(); i++) {
        const int32_t r = h.long_rows[i];
        if (rp[r + 1] - rp[r] <= max_len) { printf("FAIL long row\n"); return 1; }
        if (h.long_ptr[i + 1] - h.long_ptr[i] != (rp[r + 1] - rp[r] + max_len - 1) / max_len) {
            printf("FAIL segment count\n"); return 1; }
        for (int32_t p = h.long_ptr[i]; p < h.long_ptr[i + 1]; p++) {
            part_row[(size_t)p] = r;
            part_start[(size_t)p] = rp[r] + (p - h.long_ptr[i]) * max_len;
        }
        seen[(size_t)r] = 1;
    }
    int64_t slots = 0;
    int32_t prev_len = INT32_MAX;
    for (int64_t s = 0; s < h.n_slices; s++) {
        const int32_t L = h.len[(size_t)s];
        if (sigma > 0) prev_len = INT32_MAX;   // sorted within windows: order per slice
        int64_t slice_win = -1;               // every unit of a slice in one window
        auto same_window = [&](int32_t row) {   // ... and in the stream its group belongs to
            if (sigma <= 0) return true;
            if (slice_win < 0) slice_win = row / sigma;
            return row / sigma == slice_win && slice_win % streams == (s / kSellGroup) % streams;
        };
        if (h.off[(size_t)s] != slots || L % kSellUnroll) { printf("FAIL slice offsets\n"); return 1; }
        slots += (int64_t)L * kSellLanes;
        for (int l = 0; l < kSellLanes; l++) {
            const int32_t r = h.row[(size_t)(s * kSellLanes + l)];
            const int32_t n = h.row_len[(size_t)(s * kSellLanes + l)];
            if (r < -1) {   // a segment of a long row
                const int32_t p = -2 - r;
                if (p >= n_parts) { printf("FAIL partial index\n"); return 1; }
                part_seen[(size_t)p]++;
                const int32_t lr = part_row[(size_t)p], a = part_start[(size_t)p];
                if (n != std::min(max_len, rp[lr + 1] - a) || n > L) { printf("FAIL segment length\n"); return 1; }
                if (n > prev_len || !same_window(lr)) { printf("FAIL order\n"); return 1; }
                prev_len = n;
                for (int32_t j = 0; j < n; j++) {
                    const size_t k = (size_t)(h.off[(size_t)s] + (int64_t)j * kSellLanes + l);
                    if (!same(k, a + j)) { printf("FAIL segment term\n"); return 1; }
                }
                continue;
            }
            if (r < 0) {
                if (n != 0) { printf("FAIL empty lane\n"); return 1; }
                for (int32_t j = 0; j < L; j++)
                    if (h.col[(size_t)(h.off[(size_t)s] + (int64_t)j * kSellLanes + l)] != 0) { printf("FAIL pad\n"); return 1; }
                continue;
            }
            if (r >= n_rows || n != rp[r + 1] - rp[r] || n > max_len || n > L) { printf("FAIL row\n"); return 1; }
            if (n > prev_len || !same_window(r)) { printf("FAIL order\n"); return 1; }
            prev_len = n;
            seen[(size_t)r]++;
            for (int32_t j = 0; j < L; j++) {
                const size_t k = (size_t)(h.off[(size_t)s] + (int64_t)j * kSellLanes + l);
                if (!same(k, j < n ? (int64_t)rp[r] + j : -1)) { printf("FAIL term\n"); return 1; }
            }
        }
    }
    if (slots != h.padded || (int64_t)h.col.size() != slots) { printf("FAIL sizes\n"); return 1; }
    for (int64_t r = 0; r < n_rows; r++)
        if (seen[(size_t)r] != 1) { printf("FAIL coverage row %lld\n", (long long)r); return 1; }
    for (int32_t p = 0; p < n_parts; p++)
        if (part_seen[(size_t)p] != 1) { printf("FAIL segment coverage %d\n", p); return 1; }
    return 0;
}

int main() {
    int bad = 0;
    std::mt19937 rng(5);
    for (int64_t n_rows : {1, 63, 64, 65, 1000, 70001}) {
        for (int skew = 0; skew < 2; skew++) {
            std::vector<int32_t> rp((size_t)n_rows + 1, 0), col;
            std::vector<float> val;
            for (int64_t r = 0; r < n_rows; r++) {
                int32_t n = skew ? (int32_t)(std::pow(1.0 - (rng() % 10000) / 10000.0, -1.5) - 1) : (int32_t)(rng() % 20);
                n = std::min<int32_t>(n, 5000);
                for (int32_t j = 0; j < n; j++) { col.push_back((int32_t)(rng() % 100000)); val.push_back((float)(rng() % 97) - 48.0f); }
                rp[(size_t)r + 1] = (int32_t)col.size();
            }
            for (int32_t mx : {1, 16, 2048}) {
                bad += check(rp, col, val, n_rows, mx);
                bad += check(rp, col, val, n_rows, mx, 1000, 1);
                bad += check(rp, col, val, n_rows, mx, 4096, 8);
                bad += check(rp, col, val, n_rows, mx, 64, 3);
                bad += check(rp, col, val, n_rows, mx, 0, 1, true);
                bad += check(rp, col, val, n_rows, mx, 1000, 8, true);
            }
        }
    }
    printf(bad ? "sell_asan: FAILED\n" : "sell_asan: ok\n");
    return bad ? 1 : 0;
}
