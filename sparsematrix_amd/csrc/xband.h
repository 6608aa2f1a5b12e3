// xband.h -- column-band layout for the LDS-staged SpMV (see xband.cpp).
#pragma once

#include <cstdint>
#include <vector>

// Beta-last slab hand-off of the band2 / cband kernels (xband_dev.h combine_rows_bl): with
// several slabs every slab tile sums from -0.0 and the combine forms beta*y, so no tile loads y
// before its band loop (slab 0's 64 KiB y load made its loop 1.2 us longer than its siblings',
// r05 tile timeline).  y = (((beta*y + P_0) + P_1) + ...) + P_{S-1}; 0 restores slab 0 starting
// from beta*y (development A/B only).
#ifndef SM_B2_BL
#define SM_B2_BL 1
#endif

namespace smamd {

// Entry word: bits [0, C) column in band, [C, C+K) rank inside the row's segment
// (all ones = dummy), [C+K, 32) row in block; C = log2(band_cols), R = log2(max
// block height), K = 32 - C - R.  Stored XOR dummy_word(): zero is a dummy.
struct XbBits {
    int col, rank, row;
    constexpr uint32_t dummy_rank() const { return (1u << rank) - 1u; }
    constexpr uint32_t dummy_word() const { return dummy_rank() << col; }
    constexpr int max_seg() const { return (1 << rank) - 1; }   // ranks 0 .. max_seg-1
};
constexpr XbBits xb_bits(int band_cols_log2, int block_rows_log2) {
    return XbBits{band_cols_log2, 32 - band_cols_log2 - block_rows_log2, block_rows_log2};
}

// Two layouts over the same builder and kernel:
//  exact   -- 4096-row blocks, 16384-column bands, the whole x per block: every row
//             summed in the reference's order (bit-identical);
//  blocked -- 16384-row blocks, 8192-column bands, columns split in slabs so each
//             workgroup stages 4x less x; slab partial sums are combined in slab
//             order (within the Σ|terms| tolerance, bit-identical with one slab).
//  gather  -- blocked tiles, but x is not staged: a band's terms are listed in
//             column order so the x gathers of one wave-instruction hit a few cache
//             lines; LDS holds only the accumulators (measured slower, kept for A/B).
enum XbKind : int32_t { kXbExact = 1, kXbBlocked = 2, kXbGather = 3, kXbBand2 = 4, kXbCband = 5, kXbGcb = 6 };
constexpr int kXbExactBandLog2 = 14, kXbExactRowsLog2 = 12;
constexpr int kXbBlockedBandLog2 = 13, kXbBlockedRowsLog2 = 14;
constexpr int kXbGatherBandLog2 = 13, kXbGatherRowsLog2 = 14;
constexpr int kXbGatherWideBandLog2 = 15;      // wide slices: 32K-column bands, 3-bit ranks
constexpr int kXbThreads = 1024;               // one workgroup per CU
constexpr int kXbMaxBands = 4096;              // n_cols <= 32 M (blocked) / 64 M (exact)
constexpr int kXbMaxCap = 5;                   // chunks per wave per band held in registers
constexpr int kXbComputeWaves = 12;            // blocked kind: waves that apply (4 stage x)
constexpr int kXbTargetTiles = 256;            // blocked: >= one tile per CU

struct XbandHost {
    XbBits bits{0, 0, 0};
    int32_t block_rows = 0, band_cols = 0, n_blocks = 0, n_bands = 0;
    int64_t n_chunks = 0;
    int64_t max_chunks_per_band = 0;
    bool too_dense = false;                    // a band exceeded the register capacity
    std::vector<int64_t> chunk_start;          // n_blocks * n_bands + 1
    std::vector<uint32_t> word;                // 64 per chunk, XOR bits.dummy_word()
    std::vector<float> val;
};

// Returns false when the matrix does not fit the layout (a row segment longer
// than bits.max_seg()-1 inside one band, unsorted columns, bands too dense even
// for 64-row blocks, or size limits).  The block height starts at 2^bits.row (or
// `start_rows` when smaller and > 0) and halves while a band overflows the
// kernel's register capacity.  col_order: a band's segments are listed by their
// first column instead of by row (the gather kind).
bool xband_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
                 int64_t n_cols, XbBits bits, int waves, XbandHost &out, bool col_order = false,
                 int32_t start_rows = 0);

}  // namespace smamd

namespace smamd {

// ---------------------------------------------------------------------------
// "band2" layout (kernels_band2.hip): balanced bands.
// Tiles = (block of <= 16384 rows, slab of columns), as the blocked kind, but a
// tile's bands are variable column windows [clo, chi) of at most kB2Window columns
// holding at most kB2Chunks chunks of 64 entries -- the builder closes a band when
// either fills -- so every wave applies exactly two chunks per band and a band's
// entries are one 16-byte load per lane.  Entry word: column - clo (14 bits) |
// rank in the row's segment (4 bits, all ones = dummy) | row in block (14 bits),
// stored XOR the dummy word.  Storage per band: 4096 uint32, lane-interleaved
// [wave][lane][word of chunk 2w, word of chunk 2w+1, value bits of 2w, of 2w+1].
constexpr int kB2ColBits = 14, kB2RankBits = 4, kB2RowBits = 14;
constexpr int kB2Window = 8192;          // columns of x staged per band (32 KiB)
constexpr int kB2Chunks = 32;            // 16 waves x 2 chunks
constexpr int kB2BlockRows = 1 << kB2RowBits;
constexpr uint32_t kB2DummyRank = (1u << kB2RankBits) - 1u;
constexpr uint32_t kB2DummyWord = kB2DummyRank << kB2ColBits;

// "cband" variant (codebook balanced bands): the same tiles and bands, but every term
// is one 32-bit word -- column - clo (13 bits) | codebook id (8 bits, 255 = dummy) |
// row - chunk base (10 bits) | continuation (1 bit: the term continues the previous
// lane's segment of the same row) -- for matrices whose values take at most 255 distinct
// fp32 bit patterns (the reference's own format: uint8 ids into a table of <= 255
// floats, sparse-matrix.h:46-52).  Lane 0 of every chunk is the chunk's header: a
// dummy whose column and row fields hold the base row (rows of the chunk lie in
// [base, base + 1024)); a chunk holds <= 63 terms.  A row's segment inside a band
// is a run of consecutive lanes, all but the first flagged as continuations.  Storage per band: 2048 uint32,
// lane-interleaved [wave][lane][word of chunk 2w, word of chunk 2w+1], each stored
// XOR kCbDummyWord (zero = dummy).
constexpr int kCbColBits = 13, kCbIdBits = 8, kCbOffBits = 10, kCbContBit = 31;
constexpr uint32_t kCbDummyId = (1u << kCbIdBits) - 1u;
constexpr uint32_t kCbDummyWord = kCbDummyId << kCbColBits;
constexpr int kCbOffShift = kCbColBits + kCbIdBits;
constexpr uint32_t kCbOffMask = (1u << kCbOffBits) - 1u;
constexpr int kCbChunkTerms = 63;        // lane 0 is the header
constexpr int kCbRowSpan = 1 << kCbOffBits;
static_assert(kB2Window <= (1 << kCbColBits), "window column fits the column field");

// Tile geometry (kernels_band2.hip).  wide: 16K-row blocks, 8192-column windows (the tile's
// block sums in 64 KiB of LDS, two 32 KiB x windows), 32-chunk bands; dma3: 7680-column
// windows in three buffers staged by a loader wave, 30-chunk bands.  band2 word: column
// (col_bits) | rank (4) | row (32 - col_bits - 4); cband word: column (cb_col) | id (8) | row
// - base (23 - cb_col) | continuation (1).  The builder takes any geometry of this form (the
// ASan test builds tall, three- and six-chunk ones too); the kernel only these two -- the
// others measured slower (tall, wide3, half2, dma3 tall, dmaw: DESIGN.md §3.4b).
struct B2Geom {
    int32_t block_rows, window, col_bits;
    int32_t cpw = 2;          // chunks per wave per band
    int32_t cb_col = kCbColBits;   // cband column bits (row offset: 23 - cb_col bits)
    int32_t tab_copies = 32;  // cband: LDS copies of the scaled table (kernel)
    int32_t nch = 0;          // chunks per band when not 16 * cpw (dma3: 15 applying waves)
    constexpr uint32_t dummy_word() const { return kB2DummyRank << col_bits; }
    constexpr int chunks() const { return nch ? nch : 16 * cpw; }
    constexpr uint32_t cb_dummy_word() const { return kCbDummyId << cb_col; }
    constexpr int cb_off_shift() const { return cb_col + kCbIdBits; }
    constexpr uint32_t cb_off_mask() const { return (1u << (31 - kCbIdBits - cb_col)) - 1u; }
    constexpr int32_t cb_row_span() const { return 1 << (31 - kCbIdBits - cb_col); }
};
constexpr B2Geom kB2Wide{1 << 14, 8192, 14};
// dma3: wave 15 stages the x windows by LDS-DMA two bands ahead into three 30 KiB buffers
// (7680 columns) and applies nothing; waves 0-14 apply chunks 2w, 2w+1 of 30-chunk bands and
// never touch x in registers.  LDS: 3 x 30 KiB + 64 KiB + 4 table copies.
constexpr B2Geom kB2Dma3Cb{1 << 14, 7680, 13, 2, 13, 4, 30};
// dma3 for 8-byte band2 entries (word + fp32 value): the same loader and 30-chunk bands.
constexpr B2Geom kB2Dma3B2{1 << 14, 7680, 13, 2, kCbColBits, 1, 30};

struct Band2Host {
    bool codebook = false;               // cband encoding (ent: 2048 words per band)
    B2Geom geom = kB2Wide;
    int32_t block_rows = 0, n_blocks = 0, n_slabs = 0, slab_cols = 0;
    int32_t slab0_cols = 0;              // slab 0 = [0, slab0_cols), slab s >= 1 = [slab0 + (s-1) slab_cols, ...)
    int32_t max_bands_per_tile = 0;
    int64_t n_bands = 0;                 // over all tiles
    std::vector<int32_t> tile_band_start;   // n_blocks * n_slabs + 1 (tile t = b * S + s)
    std::vector<int32_t> band_clo;          // first column of each band's window (multiple of 4)
    std::vector<uint32_t> ent;              // 4096 per band
    int64_t real_terms = 0;                 // for the padding report
};

// Returns false when the layout does not apply: unsorted columns or size limits
// (a row segment longer than 14 terms -- 63 with ids -- cuts the band instead).
// ids != nullptr builds the cband encoding: ids[e] = codebook id (< 255) of term e.
// slab0_permille: slab 0's columns as a share of an even split (1000 = even slabs).  AUTO keeps
// even slabs: narrower slab-0 tiles measured 900: 34.0-34.2, 930: 34.1, 960: 32.9-33.2,
// 1000: 33.3-33.4 us on config 2 (profiles/r05_slab0_ab.txt).
constexpr int32_t kB2Slab0Permille = 1000;
bool band2_build(const int32_t *row_ptr, const int32_t *col, const float *val, int64_t n_rows,
                 int64_t n_cols, int32_t n_slabs, Band2Host &out, const uint8_t *ids = nullptr,
                 B2Geom geom = kB2Wide, int32_t slab0_permille = 1000);

// Codebook of a value array: table[ids[e]] has the bits of val[e] for every e; false
// when there are more than 255 distinct bit patterns (table then undefined).
bool codebook_ids(const float *val, int64_t n, std::vector<float> &table, std::vector<uint8_t> &ids);

}  // namespace smamd
