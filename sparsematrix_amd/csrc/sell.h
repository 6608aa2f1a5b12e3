// sell.h -- sorted sliced-ELL layout ("sell") for skewed matrices (power-law rows and
// columns, e.g. R-MAT) that no band layout serves (see sell.cpp, kernels_sell.hip).
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kSellLanes = 64;    // rows per slice: one wavefront
constexpr int kSellUnroll = 8;    // slice lengths are padded to a multiple of this
constexpr int kSellMaxLen = 2048;  // longer rows run as long-row chunks (tree sums)

// Rows of at most `max_len` terms, sorted by length (longest first, ties in row
// order), cut into slices of 64; slice s holds its rows' terms column-interleaved:
// term j of lane l at off[s] + 64 * j + l, j < len[s] (padded with column 0, value 0,
// never added: a lane stops at its own row length).  Rows longer than max_len are
// left to the stream plan's long-row chunks.
struct SellHost {
    int64_t n_slices = 0;
    int64_t padded = 0;                 // stored slots (terms + padding)
    std::vector<int64_t> off;           // n_slices: first slot of each slice
    std::vector<int32_t> len;           // n_slices: padded slice length (multiple of kSellUnroll)
    std::vector<int32_t> row;           // n_slices * 64: original row of each lane, -1 = none
    std::vector<int32_t> row_len;       // n_slices * 64: that row's length
    std::vector<int32_t> col;           // padded slots
    std::vector<float> val;
};

// col: the matrix's (possibly relabeled) columns.
void sell_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
                int32_t max_len, SellHost &out);

}  // namespace smamd
