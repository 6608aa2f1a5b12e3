// xband.h -- column-band layout for the LDS-staged SpMV (see xband.cpp).
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kXbColBits = 14;                 // column inside a band: band_cols <= 16384
constexpr int kXbRankBits = 6;                 // rank inside the row's segment
constexpr int kXbRowBits = 12;                 // row inside a block: block_rows <= 4096
constexpr int kXbMaxSeg = 63;                  // ranks 0..62; 63 marks a dummy
constexpr uint32_t kXbDummyRank = 63u;
constexpr uint32_t kXbDummyWord = kXbDummyRank << kXbColBits;
constexpr int kXbBandCols = 16384;             // 64 KiB of x per band, double-buffered in LDS
constexpr int kXbBlockRows = 4096;             // 16 KiB of accumulators in LDS
constexpr int kXbThreads = 1024;               // one workgroup per CU
constexpr int kXbMaxBands = 2048;              // chunk table in LDS: n_cols <= 32 M
constexpr int kXbMaxCap = 4;                   // chunks per wave per band held in registers

struct XbandHost {
    int32_t block_rows = 0, band_cols = 0, n_blocks = 0, n_bands = 0;
    int64_t n_chunks = 0;
    int64_t max_chunks_per_band = 0;
    bool too_dense = false;                    // a band exceeded the register capacity
    std::vector<int64_t> chunk_start;          // n_blocks * n_bands + 1
    std::vector<uint32_t> word;                // 64 per chunk
    std::vector<float> val;
};

// Returns false when the matrix does not fit the layout (a row segment longer
// than kXbMaxSeg inside one band, unsorted columns, bands too dense even for
// 64-row blocks, or size limits).  `block_rows` is the largest block height
// tried; the result's block_rows may be smaller.
bool xband_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
                 int64_t n_cols, int32_t block_rows, int32_t band_cols, XbandHost &out);

}  // namespace smamd
