// ccsell.h -- column-chunked sorted sliced-ELL ("ccsell") for matrices whose x is far
// larger than an XCD's L2 (BASELINE config 5: a rank's 8M x 64M slice,
// x = 256 MiB).  See ccsell.cpp, kernels_ccsell.hip.
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

// Columns are cut into chunks of 2^chunk_log2 (default 2^20 columns = 4 MiB of x, an
// XCD's L2).  A unit is one row's run of terms inside one chunk; the units of chunk c
// are sorted by length (longest first, ties in row order) and cut into slices of 64 --
// chunk c's slices hold only columns of chunk c, so while chunk c's launch runs, every
// x gather hits the 4 MiB the XCDs just pulled into their L2s.  The launches run in
// chunk order and each lane adds its unit's terms to y[row] in stored order, so every
// row's terms are added in ascending column order across the launches: the
// reference's order (kernel.cc:780-796), bit for bit.  beta is applied by the row's
// first unit (lowest chunk; rows without terms get an empty unit in chunk 0).
// Slot word (codebook form): column - chunk base (chunk_log2 bits) | id << chunk_log2;
// plain form: column - chunk base (int32) and the fp32 value.  Slot j of lane l of
// slice s at off[s] + 64 j + l.  Lane row word: row | kCcFirst when the unit is the
// row's first; -1: no row.
constexpr uint32_t kCcFirst = 0x80000000u;
constexpr int kCcDefaultChunkLog2 = 20;
constexpr int kCcMaxUnit = 2048;       // a longer run inside one chunk: layout declines

struct CcsellHost {
    int32_t chunk_log2 = kCcDefaultChunkLog2;
    int32_t n_chunks = 0;
    int64_t n_slices = 0, padded = 0, n_units = 0;
    std::vector<int64_t> chunk_slice;   // n_chunks + 1: first slice of each chunk
    std::vector<int64_t> off;           // n_slices
    std::vector<int32_t> len;           // n_slices: the slice's longest unit
    std::vector<int32_t> row;           // n_slices * 64
    std::vector<uint16_t> row_len;      // n_slices * 64
    std::vector<uint32_t> word;         // padded slots
    std::vector<float> val;             // padded slots (plain form only)
};

// ids != nullptr: codebook form (requires chunk_log2 <= 24).  Returns false when a
// unit would exceed kCcMaxUnit terms or the columns are not ascending per row.
// by_length = false keeps each chunk's units in row order (the y accesses of a slice
// then fall in a short window of rows) instead of sorting them by length.
bool ccsell_build(const int32_t *row_ptr, const int32_t *col, const float *val,
                  const uint8_t *ids, int64_t n_rows, int64_t n_cols, int32_t chunk_log2,
                  CcsellHost &out, bool by_length = true);

}  // namespace smamd
