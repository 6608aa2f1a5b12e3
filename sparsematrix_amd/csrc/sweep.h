// sweep.h -- column-swept row blocks ("sweep") for wide matrices whose x is far larger
// than an XCD's L2 (BASELINE config 5's 8M x 64M rank slices, the
// 1M x 8M slices of the weak-scaled config 2).  See sweep.cpp, kernels_sweep.hip.
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

// Rows are cut into blocks of kSwRows; one wavefront owns a block, its accumulators in
// LDS, and walks the block's terms in ascending column order -- every workgroup sweeps x
// from its first column to its last at about the same pace, so the x lines in use at
// any moment are few and stay in the L2s / Infinity Cache, and no workgroup ever waits
// for another (no barrier, no slab hand-off).  The block's terms, sorted by (column,
// row), are cut into chunks of 64 slots; inside a chunk they are regrouped by row (a
// row's terms in consecutive lanes, ascending column: a segment).  A row's terms in
// later chunks have larger columns, so each row is summed in ascending column order
// from beta * y: the reference's order (kernel.cc:780-796), bit for bit.
// Slot (8 bytes): column (uint32) and meta = row in block (bits 0..11) | continuation
// (bit 12: the term continues the previous lane's row) | codebook id << 16 (bits
// 16..23; kSwDummyId = a padding slot).  Slot l of chunk c at ent[2 (64 c + l) + {0, 1}].
constexpr int kSwRows = 256;
constexpr uint32_t kSwDummyId = 255;
constexpr uint32_t kSwContBit = 1u << 12;

struct SweepHost {
    int32_t block_rows = kSwRows;
    int64_t n_blocks = 0, n_chunks = 0;
    std::vector<int64_t> block_chunk;   // n_blocks + 1: first chunk of each block
    std::vector<uint32_t> ent;          // n_chunks * 128
};

// ids: codebook id of every term (< 255).  Returns false when a row's columns are not
// strictly ascending.
bool sweep_build(const int32_t *row_ptr, const int32_t *col, const uint8_t *ids, int64_t n_rows,
                 SweepHost &out);

}  // namespace smamd
