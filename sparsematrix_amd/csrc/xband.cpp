// xband.cpp -- host-side builder of the column-band layout used by the
// spmv_xband kernel (kernels_xband.hip).
//
// Why: for matrices whose x does not fit the L1, every term of a CSR SpMV is a
// random 4-byte gather, and on gfx950 those run at <= ~375 G gathers/s chip
// wide (TA-bound: 64 distinct cache lines per wave instruction) -- far below
// what HBM delivers for the matrix stream (profiles/r01_microbench.txt).  The
// band layout replaces the gathers by wide, coalesced loads of x into LDS.
//
// Layout.  Rows are cut into blocks of `block_rows` (<= 4096: the per-row
// accumulators live in LDS); columns into bands of `band_cols` (the x slice
// staged in LDS).  For block b and band p the block's terms with a column in
// band p are listed in (row, column) order and packed into chunks of 64
// entries (one per lane).  A row's run of terms inside one band (its
// "segment", <= 63 terms) never straddles two chunks: the builder pads the
// chunk tail with dummy entries instead.  Each entry carries its rank inside
// its segment, so the kernel can add a chunk's terms to the LDS accumulators in
// rank rounds -- no two lanes touch one row in the same round, and a row's
// terms are added in ascending column order across bands and ranks: exactly
// the reference's order (bit-identical results, no atomics).
//
// Entry word: column in band | rank (all ones = dummy) | row in block, with
// field widths from XbBits (xband.h), stored XOR bits.dummy_word() so that a
// zero word -- padding, or a load the kernel sends past its buffer's range --
// decodes as a dummy.  Values are stored beside it (fp32).
// chunk_start[b*nb + p] indexes the first chunk of (b, p); chunk_start[nblk*nb]
// = total chunks.
#include <algorithm>
#include <thread>

#include "xband.h"

namespace smamd {

static bool xband_build_fixed(const int32_t *rp, const int32_t *col, const float *val,
                              int64_t n_rows, int64_t n_cols, int32_t block_rows, XbBits bits,
                              int waves, bool col_order, XbandHost &out);

// Largest block height (<= 2^bits.row, >= 64) whose bands fit the kernel's
// register capacity (kXbMaxCap chunks per wave per band).
bool xband_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                 int64_t n_cols, XbBits bits, int waves, XbandHost &out, bool col_order,
                 int32_t start_rows) {
    if (bits.col < 8 || bits.row < 6 || bits.rank < 2 || bits.col + bits.rank + bits.row != 32)
        return false;
    int32_t br0 = 1 << bits.row;
    while (start_rows > 0 && br0 > start_rows && br0 > 64) br0 /= 2;
    for (int32_t br = br0; br >= 64; br /= 2) {
        out.too_dense = false;
        if (xband_build_fixed(rp, col, val, n_rows, n_cols, br, bits, waves, col_order, out))
            return true;
        if (!out.too_dense) return false;   // not a capacity problem: halving will not help
    }
    return false;
}

static bool xband_build_fixed(const int32_t *rp, const int32_t *col, const float *val,
                              int64_t n_rows, int64_t n_cols, int32_t block_rows, XbBits bits,
                              int waves, bool col_order, XbandHost &out) {
    out = XbandHost();
    if (n_rows <= 0 || n_cols <= 0) return false;
    const int32_t band_cols = 1 << bits.col;
    out.bits = bits;
    const int64_t nblk = (n_rows + block_rows - 1) / block_rows;
    const int64_t nb = (n_cols + band_cols - 1) / band_cols;
    if (nblk * nb >= (int64_t)1 << 31 || nb > kXbMaxBands) return false;
    out.block_rows = block_rows;
    out.band_cols = band_cols;
    out.n_blocks = (int32_t)nblk;
    out.n_bands = (int32_t)nb;

    // Per block: chunks per band (first pass) -> offsets -> fill (second pass).
    std::vector<int64_t> chunks_of((size_t)(nblk * nb), 0);
    std::vector<uint8_t> bad((size_t)nblk, 0);
    const int nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));

    auto for_blocks = [&](auto &&fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < nthr; t++)
            th.emplace_back([&, t] {
                for (int64_t b = t; b < nblk; b += nthr) fn(b);
            });
        for (auto &x : th) x.join();
    };

    // Walk the block's terms band by band.  A cursor per row remembers where
    // the row's next band starts (columns ascend within a row).
    auto walk = [&](int64_t b, auto &&emit_seg) {
        const int64_t r0 = b * block_rows, r1 = std::min<int64_t>(n_rows, r0 + block_rows);
        std::vector<int32_t> cur((size_t)(r1 - r0));
        for (int64_t r = r0; r < r1; r++) cur[r - r0] = rp[r];
        for (int64_t p = 0; p < nb; p++) {
            const int64_t cend = (p + 1) * band_cols;
            for (int64_t r = r0; r < r1; r++) {
                int32_t &c = cur[r - r0];
                const int32_t s = c;
                while (c < rp[r + 1] && col[c] < cend) c++;
                if (c > s) emit_seg(p, (int32_t)(r - r0), s, c);
            }
        }
        for (int64_t r = r0; r < r1; r++)   // unsorted columns would leave terms behind
            if (cur[r - r0] != rp[r + 1]) return false;
        return true;
    };
    // The gather kind lists a band's segments by first column (ties: by row), so
    // the consecutive entries of a chunk -- one wave-instruction of x gathers --
    // cover a narrow column window.
    struct Seg4 { int32_t p, rl, s, e; };
    auto walk_ordered = [&](int64_t b, auto &&emit_seg) {
        if (!col_order) return walk(b, emit_seg);
        std::vector<Seg4> all;
        const bool ok = walk(b, [&](int64_t p, int32_t rl, int32_t s, int32_t e) {
            all.push_back(Seg4{(int32_t)p, rl, s, e});
        });
        std::stable_sort(all.begin(), all.end(), [&](const Seg4 &a, const Seg4 &c) {
            return a.p != c.p ? a.p < c.p : col[a.s] < col[c.s];
        });
        for (const Seg4 &g : all) emit_seg((int64_t)g.p, g.rl, g.s, g.e);
        return ok;
    };

    for_blocks([&](int64_t b) {
        std::vector<int32_t> fill((size_t)nb, 0);   // entries used in the open chunk
        int64_t *cnt = &chunks_of[(size_t)(b * nb)];
        const bool ok = walk_ordered(b, [&](int64_t p, int32_t, int32_t s, int32_t e) {
            const int32_t len = e - s;
            if (len >= bits.max_seg()) { bad[b] = 1; return; }
            if (fill[p] == 0 || fill[p] + len > 64) { cnt[p]++; fill[p] = 0; }
            fill[p] += len;
        });
        if (!ok) bad[b] = 1;
    });
    for (int64_t b = 0; b < nblk; b++)
        if (bad[b]) return false;

    out.chunk_start.resize((size_t)(nblk * nb) + 1);
    int64_t total = 0;
    for (size_t i = 0; i < chunks_of.size(); i++) {
        out.chunk_start[i] = total;
        total += chunks_of[i];
    }
    out.chunk_start.back() = total;
    if (total * 64 >= (int64_t)1 << 31) return false;
    out.n_chunks = total;
    out.max_chunks_per_band = 0;
    for (int64_t i = 0; i < nblk * nb; i++)
        out.max_chunks_per_band = std::max<int64_t>(out.max_chunks_per_band, chunks_of[i]);
    // The kernel holds a band's chunks in registers: at most kXbMaxCap per wave.
    if (out.max_chunks_per_band > (int64_t)kXbMaxCap * waves) {
        out.too_dense = true;
        return false;
    }
    out.word.assign((size_t)(total * 64), 0u);   // dummies (stored XOR dummy_word)
    out.val.assign((size_t)(total * 64), 0.0f);

    // Lanes inside a chunk.  Order matters only within a row's segment (the
    // kernel passes running sums from lane to lane and the last lane writes), so
    // segments of 2+ terms take consecutive lanes first, then each single term of
    // row r goes to lane (r mod 32) or 32 + (r mod 32) when free: the 32 lanes of
    // each half then hit 32 distinct LDS banks when reading and writing their
    // accumulators (dummy lanes write a per-lane scratch slot, bank = lane mod 32).
    struct Seg { int32_t rl, s, e; };
    auto emit_chunk = [&](int64_t p, int64_t c, const std::vector<Seg> &segs) {
        bool used[64] = {false};
        int next = 0;
        auto put = [&](const Seg &g, int32_t k, int lane) {
            const int64_t slot = c * 64 + lane;
            const uint32_t cb = (uint32_t)(col[g.s + k] - p * band_cols);
            out.word[(size_t)slot] = (cb | ((uint32_t)k << bits.col) |
                                      ((uint32_t)g.rl << (bits.col + bits.rank))) ^
                                     bits.dummy_word();
            out.val[(size_t)slot] = val[g.s + k];
            used[lane] = true;
        };
        for (const Seg &g : segs)
            if (g.e - g.s > 1)
                for (int32_t k = 0; k < g.e - g.s; k++) put(g, k, next++);
        for (const Seg &g : segs) {
            if (g.e - g.s != 1) continue;
            const int bank = g.rl & 31;
            int lane = !used[bank] ? bank : !used[32 + bank] ? 32 + bank : -1;
            if (lane < 0)
                for (lane = 63; used[lane]; lane--) {}
            put(g, 0, lane);
        }
    };
    for_blocks([&](int64_t b) {
        std::vector<int64_t> chunk((size_t)nb);
        std::vector<int32_t> fill((size_t)nb, 0);
        std::vector<std::vector<Seg>> open((size_t)nb);
        for (int64_t p = 0; p < nb; p++) chunk[p] = out.chunk_start[(size_t)(b * nb + p)] - 1;
        walk_ordered(b, [&](int64_t p, int32_t rl, int32_t s, int32_t e) {
            const int32_t len = e - s;
            if (chunk[p] < out.chunk_start[(size_t)(b * nb + p)] || fill[p] + len > 64) {
                if (!open[p].empty()) emit_chunk(p, chunk[p], open[p]);
                open[p].clear();
                chunk[p]++;
                fill[p] = 0;
            }
            open[p].push_back(Seg{rl, s, e});
            fill[p] += len;
        });
        for (int64_t p = 0; p < nb; p++)
            if (!open[p].empty()) emit_chunk(p, chunk[p], open[p]);
    });
    return true;
}

}  // namespace smamd
