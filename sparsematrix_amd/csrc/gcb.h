// gcb.h -- "gathered chunk bands" (gcb): the band layout for wide matrices whose x is
// far larger than any LDS window or L2 (BASELINE config 5's rank slices: 2^23 rows x
// 2^26 columns, x = 256 MiB), built by gcb.cpp and walked by kernels_gcb.hip.
//
// A tile is (block of 2^rows_log2 rows, slab of columns), one 1024-thread workgroup, the
// block's sums in LDS.  Its terms, sorted by (column, row), are cut into bands: runs of
// at most 32 chunks of 64 lanes whose columns span fewer than `window` (<= 2^18)
// columns.  Inside a band the terms are listed by row (each row's segment in column
// order), packed into chunks; lane 0 of a chunk is its header (the chunk's base row),
// terms take lanes 1..63.  Wave w applies chunks 2w and 2w+1 of every band with one
// 16-byte load per lane {word 2w, word 2w+1, value 2w, value 2w+1} and gathers x
// straight from memory (no x window in LDS: only the gathered lines move, and the tiles
// sweeping the same columns at the same time share them in L2).  Because a band is any
// contiguous run of the (column, row)-sorted terms, every row's terms are added in
// ascending column order across the tile's bands, and inside a band by its segment --
// the reference's order (kernel.cc:780-796) within a tile; slab sums are added in slab
// order (the blocked kinds' hand-off).
//
// Word: bits [0, 18) column - band_clo (terms) or the base row (header), [18, 30) row -
// chunk base (a chunk's rows span < 4096), bit 30 live (a term), bit 31 continuation
// (the term continues the previous lane's segment of the same row).  Zero = a dummy
// lane (padding, or a load past the tile).
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kGcbColBits = 18, kGcbOffBits = 12;
constexpr uint32_t kGcbColMask = (1u << kGcbColBits) - 1u;
constexpr uint32_t kGcbOffMask = (1u << kGcbOffBits) - 1u;
constexpr uint32_t kGcbLive = 1u << 30;
constexpr uint32_t kGcbCont = 1u << 31;
constexpr int kGcbChunks = 32;            // 16 waves x 2 chunks per band
constexpr int kGcbChunkTerms = 63;        // lane 0 is the header
constexpr int kGcbRowSpan = 1 << kGcbOffBits;
constexpr int kGcbBandWords = 4096;       // 32 chunks x 64 lanes x (word + value)
constexpr int kGcbMaxWindow = 1 << kGcbColBits;

struct GcbHost {
    int32_t rows_log2 = 0, window = 0, block_rows = 0, n_blocks = 0, n_slabs = 0, slab_cols = 0;
    int32_t max_bands_per_tile = 0;
    int64_t n_bands = 0;
    int64_t real_terms = 0;
    std::vector<int32_t> tile_band_start;   // n_blocks * n_slabs + 1 (tile t = b * S + s)
    std::vector<int32_t> band_clo;          // first column of each band
    std::vector<uint32_t> ent;              // kGcbBandWords per band
};

// Returns false when the layout does not apply (unsorted or repeated columns in a row,
// size limits).  rows_log2 <= 15 (the block's sums in LDS), window <= 2^18.
bool gcb_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
               int64_t n_cols, int rows_log2, int32_t n_slabs, int32_t window, GcbHost &out);

}  // namespace smamd
