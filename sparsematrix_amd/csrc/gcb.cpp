// gcb.cpp -- host builder of the gathered chunk bands (gcb.h) for spmv_gcb_kernel.
//
// Per tile (block of rows, slab of columns): the tile's terms are sorted by (column,
// row); a band is the longest next run of that order whose columns span fewer than
// `window` columns and whose terms, listed by row and packed into 64-lane chunks (lane 0
// the header, a row's segment never split across chunks, a chunk's rows spanning fewer
// than 4096), fill at most 32 chunks.  Any run of the (column, row) order keeps every
// row's terms in ascending column order across the bands (the reference's order,
// kernel.cc:780-796), including runs that cut one column's rows in two (hub columns).
#include "gcb.h"

#include <algorithm>
#include <cstring>
#include <thread>

namespace smamd {

namespace {

struct Term {
    int32_t col, rl;   // column, row in block
    int32_t e;         // index into col/val
};

struct TileOut {
    std::vector<int32_t> clo;
    std::vector<uint32_t> ent;
    int64_t terms = 0;
    bool ok = true;
};

struct Seg {
    int32_t rl, first, n;   // row in block, index of its first term in the band list, count
};

// Pack a band's terms (by row) into chunks; returns the chunk count (> kGcbChunks: no fit).
// chunk_of[i] receives the chunk of segment i when `chunk_of` is not null.
int pack(const std::vector<Seg> &segs, std::vector<int> *chunk_of) {
    int chunks = 0, fill = kGcbChunkTerms;
    int32_t base = 0;
    if (chunk_of) chunk_of->resize(segs.size());
    for (size_t i = 0; i < segs.size(); i++) {
        const Seg &g = segs[i];
        if (fill + g.n > kGcbChunkTerms || g.rl - base >= kGcbRowSpan) {
            chunks++;
            fill = 0;
            base = g.rl;
        }
        fill += g.n;
        if (chunk_of) (*chunk_of)[i] = chunks - 1;
    }
    return chunks;
}

// Segments of the band terms t[a, b) (sorted by column, then row): sorted by row, each
// row's terms in column order.  `scratch` holds the band's terms by (row, column).
void segments(const Term *t, int64_t a, int64_t b, std::vector<Term> &scratch, std::vector<Seg> &segs) {
    scratch.assign(t + a, t + b);
    std::stable_sort(scratch.begin(), scratch.end(),
                     [](const Term &x, const Term &y) { return x.rl < y.rl; });   // columns stay ascending
    segs.clear();
    for (int32_t i = 0; i < (int32_t)scratch.size(); i++) {
        if (!segs.empty() && segs.back().rl == scratch[(size_t)i].rl) segs.back().n++;
        else segs.push_back(Seg{scratch[(size_t)i].rl, i, 1});
    }
}

void build_tile(const int32_t *rp, const int32_t *col, const float *val, int64_t r0, int64_t r1,
                int64_t c0, int64_t c1, int32_t window, TileOut &out) {
    std::vector<Term> t;
    for (int64_t r = r0; r < r1; r++) {
        const int32_t *a = col + rp[r], *z = col + rp[r + 1];
        const int32_t s = (int32_t)(std::lower_bound(a, z, (int32_t)c0) - col);
        const int32_t e = (int32_t)(std::lower_bound(a, z, (int32_t)c1) - col);
        for (int32_t i = s; i < e; i++) t.push_back(Term{col[i], (int32_t)(r - r0), i});
    }
    std::sort(t.begin(), t.end(), [](const Term &x, const Term &y) {
        return x.col != y.col ? x.col < y.col : x.rl < y.rl;
    });
    const int64_t n = (int64_t)t.size();
    std::vector<Term> scratch;
    std::vector<Seg> segs;
    std::vector<int> chunk_of;
    const int64_t cap = (int64_t)kGcbChunks * kGcbChunkTerms;
    int64_t a = 0;
    while (a < n) {
        // Longest run from a within the window and the chunk capacity.
        int64_t b = std::min<int64_t>(n, a + cap);
        const int32_t clo = t[(size_t)a].col;
        b = std::lower_bound(t.begin() + a, t.begin() + b, clo + window,
                             [](const Term &x, int64_t c) { return x.col < c; }) - t.begin();
        for (;;) {
            segments(t.data(), a, b, scratch, segs);
            bool seg_ok = true;   // a row's segment must fit one chunk
            for (const Seg &g : segs)
                if (g.n > kGcbChunkTerms) seg_ok = false;
            if (seg_ok && pack(segs, nullptr) <= kGcbChunks) break;
            b = a + std::max<int64_t>(1, (b - a) * 31 / 32);
        }
        pack(segs, &chunk_of);
        // Emit: per chunk, lane 0 the header, then the segments' terms in order.
        const size_t base = out.ent.size();
        out.ent.resize(base + kGcbBandWords, 0u);
        out.clo.push_back(clo);
        uint32_t *band = out.ent.data() + base;
        int lane_next[kGcbChunks];
        int32_t cbase[kGcbChunks];
        for (int c = 0; c < kGcbChunks; c++) lane_next[c] = 0, cbase[c] = -1;
        for (size_t i = 0; i < segs.size(); i++) {
            const Seg &g = segs[i];
            const int c = chunk_of[i];
            const int wave = c >> 1, k = c & 1;
            auto slot = [&](int lane) { return band + (size_t)(wave * 64 + lane) * 4; };
            if (cbase[c] < 0) {   // header: the chunk's base row
                cbase[c] = g.rl;
                slot(0)[k] = (uint32_t)g.rl;
                lane_next[c] = 1;
            }
            for (int32_t j = 0; j < g.n; j++) {
                const Term &m = scratch[(size_t)(g.first + j)];
                uint32_t *e = slot(lane_next[c]++);
                e[k] = (uint32_t)(m.col - clo) | ((uint32_t)(g.rl - cbase[c]) << kGcbColBits) | kGcbLive |
                       (j > 0 ? kGcbCont : 0u);
                uint32_t vb;
                memcpy(&vb, &val[m.e], 4);
                e[2 + k] = vb;
            }
        }
        out.terms += b - a;
        a = b;
    }
}

}  // namespace

bool gcb_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows, int64_t n_cols,
               int rows_log2, int32_t n_slabs, int32_t window, GcbHost &out) {
    out = GcbHost();
    if (rows_log2 < 6 || rows_log2 > 15 || window < 64 || window > kGcbMaxWindow) return false;
    if (n_rows <= 0 || n_cols <= 0 || n_slabs < 1 || n_cols >= ((int64_t)1 << 30)) return false;
    // x < 4 GiB: the kernel gathers x through one buffer resource with 32-bit byte offsets
    // 4 * column; wider matrices fall back to the sliced ELL.
    for (int64_t r = 0; r < n_rows; r++)   // strictly ascending columns per row
        for (int32_t e = rp[r] + 1; e < rp[r + 1]; e++)
            if (col[e] <= col[e - 1]) return false;
    const int32_t br = (int32_t)std::min<int64_t>((int64_t)1 << rows_log2, n_rows);
    const int64_t nblk = (n_rows + br - 1) / br;
    const int64_t sc = ((n_cols + n_slabs - 1) / n_slabs + 255) & ~(int64_t)255;
    const int64_t ns = (n_cols + sc - 1) / sc;
    const int64_t ntile = nblk * ns;
    if (ntile >= ((int64_t)1 << 30)) return false;
    std::vector<TileOut> tiles((size_t)ntile);
    const int nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int k = 0; k < nthr; k++)
        th.emplace_back([&, k] {
            for (int64_t i = k; i < ntile; i += nthr) {
                const int64_t b = i / ns, s = i % ns;
                build_tile(rp, col, val, b * br, std::min<int64_t>(n_rows, (b + 1) * br), s * sc,
                           std::min<int64_t>(n_cols, (s + 1) * sc), window, tiles[(size_t)i]);
            }
        });
    for (auto &x : th) x.join();
    out.rows_log2 = rows_log2;
    out.window = window;
    out.block_rows = br;
    out.n_blocks = (int32_t)nblk;
    out.n_slabs = (int32_t)ns;
    out.slab_cols = (int32_t)sc;
    out.tile_band_start.resize((size_t)ntile + 1);
    int64_t nb = 0;
    for (int64_t i = 0; i < ntile; i++) {
        if (!tiles[(size_t)i].ok) return false;
        out.tile_band_start[(size_t)i] = (int32_t)nb;
        const int64_t k = (int64_t)tiles[(size_t)i].clo.size();
        out.max_bands_per_tile = std::max<int32_t>(out.max_bands_per_tile, (int32_t)k);
        nb += k;
        out.real_terms += tiles[(size_t)i].terms;
    }
    out.tile_band_start[(size_t)ntile] = (int32_t)nb;
    // Per-tile entry offsets are 32-bit byte offsets: a tile's bands under 4 GiB.
    if ((int64_t)out.max_bands_per_tile * kGcbBandWords * 4 >= ((int64_t)1 << 32) || nb >= INT32_MAX)
        return false;
    out.n_bands = nb;
    out.band_clo.reserve((size_t)nb);
    out.ent.reserve((size_t)(nb * kGcbBandWords));
    for (auto &x : tiles) {
        out.band_clo.insert(out.band_clo.end(), x.clo.begin(), x.clo.end());
        out.ent.insert(out.ent.end(), x.ent.begin(), x.ent.end());
        std::vector<uint32_t>().swap(x.ent);
    }
    return true;
}

}  // namespace smamd
