// sell.h -- sorted sliced-ELL layout ("sell") for skewed matrices (power-law rows and
// columns, e.g. R-MAT) that no band layout serves (see sell.cpp, kernels_sell.hip).
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kSellLanes = 64;    // rows per slice: one wavefront
constexpr int kSellUnroll = 8;    // slice lengths are padded to a multiple of this
constexpr int kSellMaxLen = 2048;  // longer rows are cut in segments of this many terms
constexpr int kSellGroup = 4;     // slices per 256-thread workgroup (kernels_sell.hip)

// Rows of at most `max_len` terms, and segments of max_len terms of the longer rows,
// sorted by length (longest first, ties in row / segment order), cut into slices of
// 64; slice s holds its lanes' terms column-interleaved: term j of lane l at
// off[s] + 64 * j + l, j < len[s] (padded with column 0, value 0, never added: a lane
// stops at its own length).  A lane's `row` is the row (>= 0), -1 (no row) or
// -2 - p for segment partial p: segments of one long row have consecutive partials
// in order (long_ptr), added to beta * y in that order by the finalize kernel.
struct SellHost {
    int64_t n_slices = 0;
    int64_t padded = 0;                 // stored slots (terms + padding)
    std::vector<int64_t> off;           // n_slices: first slot of each slice
    std::vector<int32_t> len;           // n_slices: padded slice length (multiple of kSellUnroll)
    std::vector<int32_t> row;           // n_slices * 64: original row of each lane, -1 = none
    std::vector<int32_t> row_len;       // n_slices * 64: that row's length
    std::vector<int32_t> col;           // padded slots (codebook: words, see below)
    std::vector<float> val;             // padded slots (empty with codebook ids)
    std::vector<int32_t> long_rows;     // rows split in segments
    std::vector<int32_t> long_ptr;      // long_rows.size() + 1: their partials
};

// col: the matrix's (possibly relabeled) columns.  sigma > 0: rows are sorted only
// within windows of sigma rows (SELL-C-sigma; slices never cross a window), so the
// y entries a window's slices read and write stay few; streams > 1: the windows are
// dealt round-robin to `streams` streams and the slices ordered so that workgroup b
// (kSellGroup slices) takes group b / streams of stream b % streams -- with
// workgroups dealt round-robin over the XCDs, a window's y lines stay in one XCD's
// L2 (speed only).  Streams are padded to whole, equal numbers of groups with empty
// slices (length 0, every lane -1).  ids != nullptr (codebook sell, every column <
// 2^24): each slot is one word, column | id << 24 (the value's codebook id, as the
// reference stores it: sparse-matrix.h:46-52), and `val` stays empty -- 4 bytes per
// slot instead of 8; padding words are 0 (never added).
constexpr int kSellCbColBits = 24;
void sell_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
                int32_t max_len, SellHost &out, int64_t sigma = 0, int streams = 1,
                const uint8_t *ids = nullptr);

}  // namespace smamd
