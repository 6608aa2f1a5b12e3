// encode.h -- host-side encoders and row-tile planner (see encode.cpp, plan.cpp).
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace smamd {

struct EncodeResult {
    int64_t s_rows = 0, s_cols = 0;
    int32_t table_size = 0;
    std::vector<float> table;                   // table_size + 1 (last = 0)
    std::vector<int64_t> row_ptr;               // CSR of B = S^T, s_cols + 1
    std::vector<int32_t> col;
    std::vector<float> val;
    std::vector<uint8_t> pos, val_id;           // reference stream
    std::vector<int32_t> panel_row_off, panel_col_off;
    std::vector<int64_t> panel_begin, panel_end;
};

// CopyForm (sparse-matrix.cc:20-99).  Returns 0, or -1 for a bad table_size.
int encode_dense_index(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                       const float *table, int32_t table_size, bool trans, EncodeResult &out);

// The reference encoding of a CSR matrix of B = S^T (n_rows = S columns, n_cols = S
// rows): the inverse of the CSR pass above, the stream rules of sparse-matrix.cc:32-95.
// table == nullptr: the codebook is the values' distinct fp32 bit patterns in CSR order.
// Returns 0; -1 bad table_size; -2 a value not in the table; -3 more than 255 distinct
// values; -4 S rows >= 2^23 (the reference's int32 in-panel offsets).
int encode_csr_ref(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                   int64_t n_cols, const float *table, int32_t table_size, EncodeResult &out);

struct TileHost {
    int32_t r0, r1, flags;
};
struct ChunkHost {
    int32_t lr, begin, end;
};
struct PlanHost {
    std::vector<TileHost> tiles;
    std::vector<int32_t> long_rows;
    std::vector<int32_t> long_ptr;     // long_rows.size() + 1
    std::vector<ChunkHost> chunks;
    int32_t max_row_nnz = 0;
    double avg_row_nnz = 0.0;
};

// Partition rows into nnz-balanced tiles (<= tile_nnz terms, <= tile_rows rows);
// rows longer than tile_nnz become long rows split into chunk_nnz chunks.
void plan_rows(const int32_t *row_ptr, int64_t n_rows, int32_t tile_nnz, int32_t tile_rows,
               int32_t chunk_nnz, int32_t serial_max, PlanHost &out);

}  // namespace smamd
