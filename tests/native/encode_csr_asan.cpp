// Host-only check of the CSR -> reference-stream converter (sparsematrix_amd/csrc/
// encode.cpp encode_csr_ref), built with AddressSanitizer by tests/test_xband_builder.py.
// The dense-index encoder (encode_dense_index, golden-pinned against the compiled
// reference) gives both a CSR of B and the reference stream; converting that CSR back
// with the same table must give the identical stream, panels and table -- NoTrans and
// Trans, ragged shapes, filler gaps, ids at T - 1, empty matrices and empty panels.
// Without a table the derived codebook must decode to the same values; out-of-table
// values, > 255 distinct values and S rows >= 2^23 decline.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "encode.h"

using namespace smamd;

static int fails = 0;
#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);           \
            fails++;                                                     \
        }                                                                \
    } while (0)

static void round_trip(int rows, int cols, int stride, double dens, int T, bool trans, uint32_t seed) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<double> u(0, 1);
    std::vector<uint8_t> dm((size_t)rows * stride, 255);
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++)
            if (u(rng) < dens) dm[(size_t)r * stride + c] = (uint8_t)(rng() % (T + 3));   // some >= T
    std::vector<float> table(T);
    for (int i = 0; i < T; i++) table[i] = (float)(u(rng) * 2 - 1);
    if (T > 2) table[1] = -0.0f;
    EncodeResult a, b, c;
    CHECK(encode_dense_index(dm.data(), rows, cols, stride, table.data(), T, trans, a) == 0);
    std::vector<int32_t> rp(a.row_ptr.begin(), a.row_ptr.end());
    CHECK(encode_csr_ref(rp.data(), a.col.data(), a.val.data(), a.s_cols, a.s_rows, table.data(), T, b) == 0);
    CHECK(b.s_rows == a.s_rows && b.s_cols == a.s_cols && b.table_size == a.table_size);
    CHECK(b.table.size() == a.table.size() &&
          memcmp(b.table.data(), a.table.data(), a.table.size() * 4) == 0);
    CHECK(b.pos == a.pos && b.val_id == a.val_id);
    CHECK(b.panel_row_off == a.panel_row_off && b.panel_col_off == a.panel_col_off);
    CHECK(b.panel_begin == a.panel_begin && b.panel_end == a.panel_end);
    // derived codebook: same positions, ids decoding to the same bits
    CHECK(encode_csr_ref(rp.data(), a.col.data(), a.val.data(), a.s_cols, a.s_rows, nullptr, 0, c) == 0);
    CHECK(c.pos == a.pos && c.val_id.size() == a.val_id.size());
    for (size_t i = 0; i < a.val_id.size() && i < c.val_id.size(); i++) {
        const bool fa = a.val_id[i] == a.table_size, fc = c.val_id[i] == c.table_size;
        CHECK(fa == fc);
        if (!fa && !fc) CHECK(memcmp(&a.table[a.val_id[i]], &c.table[c.val_id[i]], 4) == 0);
    }
}

int main() {
    const int shapes[][3] = {{1, 1, 1}, {7, 5, 9}, {255, 256, 256}, {256, 257, 300}, {300, 1000, 1000},
                             {1024, 1024, 1024}, {3, 2000, 2000}, {2000, 3, 4}};
    uint32_t seed = 1;
    for (const auto &sh : shapes)
        for (double d : {0.0, 0.001, 0.05, 0.6})
            for (int T : {1, 17, 255})
                for (bool tr : {false, true}) round_trip(sh[0], sh[1], sh[2], d, T, tr, seed++);
    // a value outside the table
    {
        std::vector<int32_t> rp = {0, 1}, col = {0};
        std::vector<float> val = {3.0f}, table = {1.0f, 2.0f};
        EncodeResult r;
        CHECK(encode_csr_ref(rp.data(), col.data(), val.data(), 1, 1, table.data(), 2, r) == -2);
    }
    // 256 distinct values without a table
    {
        std::vector<int32_t> rp = {0, 256}, col(256);
        std::vector<float> val(256);
        for (int i = 0; i < 256; i++) { col[i] = i; val[i] = (float)i; }
        EncodeResult r;
        CHECK(encode_csr_ref(rp.data(), col.data(), val.data(), 1, 256, nullptr, 0, r) == -3);
    }
    // S rows >= 2^23
    {
        std::vector<int32_t> rp = {0, 0};
        EncodeResult r;
        CHECK(encode_csr_ref(rp.data(), nullptr, nullptr, 1, (int64_t)1 << 23, nullptr, 0, r) == -4);
    }
    if (fails) {
        printf("encode_csr_asan: %d failures\n", fails);
        return 1;
    }
    printf("encode_csr_asan: ok\n");
    return 0;
}
