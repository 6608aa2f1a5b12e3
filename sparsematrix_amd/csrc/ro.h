// ro.h -- "row-owner" codebook bands (kernels_ro.hip, ro.cpp).
//
// Same tiles as the balanced codebook bands (cband, xband.h): a tile is (block of <= 16384
// rows, slab of columns), one 1024-thread workgroup per CU, the block's row sums in LDS,
// x streamed through LDS windows of kRoWindow columns by LDS-DMA.  What changes is who
// applies a term: applying wave w (of kRoApplyWaves) owns the block's rows
// [w * kRoWaveRows, (w + 1) * kRoWaveRows) and applies every term of them, window after
// window, so no two waves ever touch one row's sum and the waves need no barrier between
// windows -- they only wait for the loader waves to have landed a window, and the loaders
// only for every applying wave to have left the window whose buffer they refill (progress
// counters in LDS).  A wave's terms of one window are packed, row by row, into chunks of
// <= 63 terms (lane 0 the header) whose rows span < 1024; a chunk belongs to one window.
//
// Entry word (stored XOR kCbDummyWord, zero = dummy): column - window start (13 bits) |
// codebook id (8) | row - chunk base (10) | continuation (1), as cband.  Header (lane 0):
// id 255; column field = the window index (bits 0-10) | the chunk's stage (bits 11-12); row
// field + continuation bit = the chunk's base row relative to the wave's first row (11 bits).
// The kernel applies a wave's chunks in groups of kRoGroup (aligned in the wave's stream).
// Stage: 0 unless the chunk shares a row with an earlier chunk of its group (a row cut in
// 63-term pieces, or a row with terms in two windows); then 1 + the highest stage of those.
// Chunks of one stage in a group have disjoint rows and a row's chunks ascend in stage, so the
// kernel applies a group stage by stage, each stage's chunks together.
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kRoWindow = 7680;                 // columns per window (30 KiB, 30 DMA pieces)
constexpr int kRoBlockRows = 1 << 14;
constexpr int kRoApplyWaves = 14;               // waves 0..13 apply, 14..15 load x
constexpr int kRoLoadWaves = 2;
constexpr int kRoWaveRows = (kRoBlockRows + kRoApplyWaves - 1) / kRoApplyWaves;   // 1171
constexpr int kRoMaxWindows = 1 << 11;          // window index field (header bits 0-10)
constexpr int kRoStageShift = 11;               // stage field (header bits 11-12)
constexpr int kRoGroup = 4;                     // chunks a wave applies together

struct RoHost {
    int32_t block_rows = 0, n_blocks = 0, n_slabs = 0, slab_cols = 0;
    int64_t n_chunks = 0;
    std::vector<int32_t> wave_start;   // n_tiles * kRoApplyWaves + 1: first chunk of (tile, wave)
    std::vector<uint32_t> ent;         // 64 words per chunk
    int64_t real_terms = 0;
    int32_t max_chunks_per_wave = 0;   // over all (tile, wave)
};

// ids[e] = codebook id (< 255) of term e (codebook_ids, xband.h).  false when the layout does
// not apply (unsorted columns, too many windows per slab, size limits).
bool ro_build(const int32_t *row_ptr, const int32_t *col, const uint8_t *ids, int64_t n_rows,
              int64_t n_cols, int32_t n_slabs, RoHost &out);

}  // namespace smamd
