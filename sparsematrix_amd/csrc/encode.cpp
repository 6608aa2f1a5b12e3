// encode.cpp -- host-side construction of a matrix from the reference's dense
// codebook-index input (CopyForm semantics, sparse-matrix.cc:20-99).
//
// Produces two things from one scan of the index matrix:
//   1. the reference encoding itself (panels of 256 S-columns, uint8 delta
//      positions with 255-step fillers, uint8 ids), kept on the host for
//      sm_copy_ref_stream / sm_equal; and
//   2. CSR of B = S^T (row j = S column j, columns = S rows ascending), which
//      is what the device kernels consume.
// Indexing is 64-bit (the reference's int32 `i*stride+j` overflows above ~46k^2,
// SURVEY.md §0.4); everything else follows the reference rule for rule.
#include <cstring>
#include <unordered_map>

#include "encode.h"

namespace smamd {

namespace {
constexpr int kPanelShift = 8;          // SBLAS_BLOCK_COL_SHIFT (kernel.h:26)
constexpr int kPanelW = 1 << kPanelShift;
constexpr int kMaxStep = 255;           // uint8 delta range (sparse-matrix.cc:24)
}  // namespace

int encode_dense_index(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                       const float *table, int32_t table_size, bool trans, EncodeResult &out) {
    out = EncodeResult();
    if (table_size < 0 || table_size > kMaxStep) return -1;       // :25
    if (table_size == 0) return 0;                                 // :26 (empty matrix)
    out.table.assign(table, table + table_size);                   // :29-31
    out.table.push_back(0.0f);
    out.table_size = table_size;

    // S view: NoTrans S[r][c] = dm[r*stride + c]; Trans S[r][c] = dm[c*stride + r].
    const int64_t s_rows = trans ? cols : rows;
    const int64_t s_cols = trans ? rows : cols;
    out.s_rows = s_rows;
    out.s_cols = s_cols;
    auto at = [&](int64_t r, int64_t c) -> uint8_t {
        return trans ? dm[c * (int64_t)stride + r] : dm[r * (int64_t)stride + c];
    };
    const uint8_t T = (uint8_t)table_size;

    // ---- CSR of B (n = s_cols rows, k = s_rows columns) ------------------------
    std::vector<int64_t> cnt((size_t)s_cols + 1, 0);
    if (trans) {
        // B = dm (rows x cols), read row by row.
        for (int64_t j = 0; j < s_cols; j++) {
            const uint8_t *row = dm + j * (int64_t)stride;
            int64_t c = 0;
            for (int64_t i = 0; i < s_rows; i++) c += row[i] < T;
            cnt[j + 1] = c;
        }
    } else {
        for (int64_t r = 0; r < s_rows; r++) {
            const uint8_t *row = dm + r * (int64_t)stride;
            for (int64_t j = 0; j < s_cols; j++) cnt[j + 1] += row[j] < T;
        }
    }
    for (int64_t j = 0; j < s_cols; j++) cnt[j + 1] += cnt[j];
    const int64_t nnz = cnt[s_cols];
    out.row_ptr.assign(cnt.begin(), cnt.end());
    out.col.resize((size_t)nnz);
    out.val.resize((size_t)nnz);
    if (trans) {
        for (int64_t j = 0; j < s_cols; j++) {
            const uint8_t *row = dm + j * (int64_t)stride;
            int64_t o = cnt[j];
            for (int64_t i = 0; i < s_rows; i++) {
                if (row[i] >= T) continue;
                out.col[o] = (int32_t)i;
                out.val[o] = out.table[row[i]];
                o++;
            }
        }
    } else {
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        for (int64_t r = 0; r < s_rows; r++) {
            const uint8_t *row = dm + r * (int64_t)stride;
            for (int64_t j = 0; j < s_cols; j++) {
                if (row[j] >= T) continue;
                const int64_t o = fill[j]++;
                out.col[o] = (int32_t)r;
                out.val[o] = out.table[row[j]];
            }
        }
    }

    // ---- the reference stream (sparse-matrix.cc:32-62 / 65-95) ----------------
    // One row block (block_row_shift == 0); per panel of 256 S-columns, entries
    // row-major at in-panel position r*256 + c, delta coded from the previous
    // entry, with (255, T) filler steps while the gap exceeds 255.
    for (int64_t c0 = 0; c0 < s_cols; c0 += kPanelW) {
        const int64_t w = std::min<int64_t>(kPanelW, s_cols - c0);
        const int64_t begin = (int64_t)out.pos.size();
        int64_t prev = 0;
        for (int64_t r = 0; r < s_rows; r++) {
            for (int64_t c = 0; c < w; c++) {
                const uint8_t id = at(r, c0 + c);
                if (id >= T) continue;
                const int64_t lin = (r << kPanelShift) + c;
                int64_t gap = lin - prev;
                while (gap > kMaxStep) {
                    out.pos.push_back((uint8_t)kMaxStep);
                    out.val_id.push_back(T);
                    gap -= kMaxStep;
                }
                out.pos.push_back((uint8_t)gap);
                out.val_id.push_back(id);
                prev = lin;
            }
        }
        if ((int64_t)out.pos.size() != begin) {
            out.panel_row_off.push_back(0);
            out.panel_col_off.push_back((int32_t)c0);
            out.panel_begin.push_back(begin);
            out.panel_end.push_back((int64_t)out.pos.size());
        }
    }
    return 0;
}

int encode_csr_ref(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                   int64_t n_cols, const float *table, int32_t table_size, EncodeResult &out) {
    out = EncodeResult();
    if (n_cols >= ((int64_t)1 << (31 - kPanelShift))) return -4;
    const int64_t nnz = n_rows > 0 ? rp[n_rows] : 0;
    auto bits_of = [](float v) {
        uint32_t u;
        memcpy(&u, &v, 4);
        return u;
    };
    // Codebook: value bits -> id (the first table entry with those bits, as a dense index
    // naming either of two equal entries would decode to the same value).
    std::unordered_map<uint32_t, uint8_t> id_of;
    if (table) {
        if (table_size < 0 || table_size > kMaxStep) return -1;
        for (int32_t i = 0; i < table_size; i++) id_of.emplace(bits_of(table[i]), (uint8_t)i);
        out.table.assign(table, table + table_size);
    } else {
        for (int64_t e = 0; e < nnz; e++) {
            const uint32_t u = bits_of(val[e]);
            if (id_of.count(u)) continue;
            if ((int32_t)id_of.size() == kMaxStep) return -3;
            id_of.emplace(u, (uint8_t)id_of.size());
            out.table.push_back(val[e]);
        }
        table_size = (int32_t)out.table.size();
    }
    out.table.push_back(0.0f);
    out.table_size = table_size;
    out.s_rows = n_cols;
    out.s_cols = n_rows;
    if (table_size == 0) return nnz == 0 ? 0 : -2;
    const uint8_t T = (uint8_t)table_size;
    std::vector<std::pair<uint64_t, uint8_t>> ent;
    for (int64_t c0 = 0; c0 < n_rows; c0 += kPanelW) {
        const int64_t w = std::min<int64_t>(kPanelW, n_rows - c0);
        ent.clear();
        for (int64_t c = 0; c < w; c++)
            for (int64_t e = rp[c0 + c]; e < rp[c0 + c + 1]; e++) {
                const auto it = id_of.find(bits_of(val[e]));
                if (it == id_of.end()) return -2;
                ent.push_back({((uint64_t)(uint32_t)col[e] << kPanelShift) | (uint64_t)c, it->second});
            }
        if (ent.empty()) continue;
        // row-major in the panel (S row, then S column), as the reference scans (:65-95)
        std::stable_sort(ent.begin(), ent.end(),
                         [](const std::pair<uint64_t, uint8_t> &a, const std::pair<uint64_t, uint8_t> &b) {
                             return a.first < b.first;
                         });
        const int64_t begin = (int64_t)out.pos.size();
        int64_t prev = 0;
        for (const auto &pe : ent) {
            int64_t gap = (int64_t)pe.first - prev;
            while (gap > kMaxStep) {
                out.pos.push_back((uint8_t)kMaxStep);
                out.val_id.push_back(T);
                gap -= kMaxStep;
            }
            out.pos.push_back((uint8_t)gap);
            out.val_id.push_back(pe.second);
            prev = (int64_t)pe.first;
        }
        out.panel_row_off.push_back(0);
        out.panel_col_off.push_back((int32_t)c0);
        out.panel_begin.push_back(begin);
        out.panel_end.push_back((int64_t)out.pos.size());
    }
    return 0;
}

}  // namespace smamd
