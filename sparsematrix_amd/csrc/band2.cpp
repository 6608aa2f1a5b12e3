// band2.cpp -- host-side builder of the balanced-band layout used by
// spmv_band2_kernel (kernels_band2.hip).  Layout: xband.h (Band2Host).
//
// Per tile (block b of rows, slab s of columns) the builder walks the slab's
// columns left to right and closes a band [clo, chi) as soon as either
//   * its window from clo rounded down to 4 columns would pass geom.window columns,
//   * its terms, packed row by row into 64-entry chunks without splitting a row's
//     segment (the row's run of terms inside the band), would need more than
//     kB2Chunks chunks, or
//   * a row would have more than 14 terms in it (the 4-bit rank field),
// so every band is one fixed-size slot of 32 chunks: the kernel's wave w applies
// chunks 2w and 2w+1 and loads them with one 16-byte load per lane.  Columns
// without terms never open a band.  Inside a band the terms are listed by row,
// each row's segment in ascending column order, so across the tile's bands (which
// ascend in column) every row's terms are added in the reference's order
// (sparse-matrix.cc:164-190, kernel.cc:780-796: per output, ascending column).
#include <algorithm>
#include <cstdlib>
#include <thread>

#include "xband.h"

namespace smamd {

namespace {

struct TileOut {
    std::vector<int32_t> clo;
    std::vector<uint32_t> ent;
    int64_t terms = 0;
    bool ok = true;
};

// A row's run of terms inside one chunk: row in block, first term index, count.
struct Seg {
    int32_t rl, s, n;
};

// Lanes inside a chunk: segments of 2+ terms take consecutive lanes first (the
// kernel passes a running sum up the lanes), then the single terms go to the two
// half-waves so that each half's LDS reads spread over the 32 banks: a ds_read_b32
// is served per 32-lane half, one LDS cycle per distinct address on its busiest bank,
// and every lane reads x[column - clo] (bank = column - clo mod 32) and the
// accumulator of its row (bank = row mod 32).  Each single goes to the half where its
// two banks are least used so far (ties: the emptier half), singles with the most
// contended banks first; lane order inside a half does not matter.  Which rows share
// a chunk and the per-row term order are unchanged (only lanes move).  cband
// (ids != nullptr): lane 0 is the header (the chunk's base row), terms take lanes
// 1..63 and carry their id, row - base and a continuation flag instead of value bits
// and rank.
void emit_chunk(uint32_t *band_ent, int c, const std::vector<Seg> &segs, const int32_t *col,
                const float *val, const uint8_t *ids, int32_t clo_al, B2Geom geom) {
    bool used[64] = {false};
    const int cpw = ids != nullptr ? geom.cpw : 2;
    const int wave = c / cpw, k = c % cpw;
    const bool cb = ids != nullptr;
    const uint32_t cb_colmask = (1u << geom.cb_col) - 1u, cb_dummy = geom.cb_dummy_word();
    const int cb_off_shift = geom.cb_off_shift();
    const bool tab_banks = cb && geom.tab_copies == 1;   // one table copy: bank = id mod 32
    // Four table copies (dma3): lane l reads copy l mod 4, bank = 4 (id mod 8) + l mod 4 --
    // the lane's class (l mod 4) matters, so singles are placed by (half, class).
#ifdef SM_DEV
    static const bool tab4_off = getenv("SM_B2_TAB4") && atoi(getenv("SM_B2_TAB4")) == 0;   // A/B
#else
    constexpr bool tab4_off = false;
#endif
    const bool tab4 = cb && geom.tab_copies == 4 && !tab4_off;
    auto tbank = [&](uint32_t id, int lane) -> int {
        return tab_banks ? (int)(id & 31) : tab4 ? (int)((4 * (id & 7) + (uint32_t)(lane & 3)) & 31) : 0;
    };
    const int32_t base = segs.empty() ? 0 : segs.front().rl;   // segments come in row order
    int next = 0;
    // Bank use per half: x reads (column bank), accumulator reads (row bank) and, with
    // one table copy, the table reads (id bank).
    uint8_t xb[2][32] = {}, yb[2][32] = {}, tb[2][32] = {};
    // A segment's lanes read one accumulator (a broadcast): its row counts once per half.
    auto note = [&](int lane, uint32_t cbits, int32_t rl, bool same_row_before, uint32_t id) {
        const int h = lane >> 5;
        xb[h][cbits & 31]++;
        if (!(same_row_before && ((lane - 1) >> 5) == h)) yb[h][rl & 31]++;
        tb[h][tbank(id, lane)]++;
    };
    if (cb) {
        const uint32_t h = ((uint32_t)base & cb_colmask) | cb_dummy |
                           ((((uint32_t)base >> geom.cb_col) & geom.cb_off_mask()) << cb_off_shift);
        band_ent[(size_t)(wave * 64) * cpw + k] = h ^ cb_dummy;
        used[0] = true;
        next = 1;
        note(0, h & cb_colmask, base + (int32_t)((h >> cb_off_shift) & geom.cb_off_mask()), false, kCbDummyId);
    }
    auto put = [&](const Seg &g, int32_t j, int lane) {
        const uint32_t cbits = (uint32_t)(col[g.s + j] - clo_al);
        if (cb) {
            const uint32_t w = cbits | ((uint32_t)ids[g.s + j] << geom.cb_col) |
                               ((uint32_t)(g.rl - base) << cb_off_shift) | ((j > 0 ? 1u : 0u) << kCbContBit);
            band_ent[(size_t)(wave * 64 + lane) * cpw + k] = w ^ cb_dummy;
        } else {
            uint32_t *e = band_ent + ((size_t)(wave * 64 + lane)) * 4;
            e[k] = (cbits | ((uint32_t)j << geom.col_bits) | ((uint32_t)g.rl << (geom.col_bits + kB2RankBits))) ^
                   geom.dummy_word();
            float v = val[g.s + j];
            uint32_t vb;
            __builtin_memcpy(&vb, &v, 4);
            e[2 + k] = vb;
        }
        used[lane] = true;
        note(lane, cbits, g.rl, j > 0, cb ? ids[g.s + j] : 0u);
    };
    for (const Seg &g : segs)
        if (g.n > 1)
            for (int32_t j = 0; j < g.n; j++) put(g, j, next++);
    // Singles: greedy, most contended banks first (pairwise swaps afterwards measured
    // 2.65 / 2.44 vs 2.70 / 2.48 cycles per half-wave read, tools/band2_banks.cpp: not kept).
    // Fixed arrays (a chunk holds <= 64 segments): no allocation per chunk.
    const Seg *single[64];
    int ns = 0;
    for (const Seg &g : segs)
        if (g.n == 1) single[ns++] = &g;
    if (ns == 0) return;
    uint8_t xcnt[32] = {}, ycnt[32] = {}, tcnt[32] = {};
    uint8_t sx[64], sy[64], st[64], half[64];
    for (int i = 0; i < ns; i++) {
        sx[i] = (uint8_t)((col[single[i]->s] - clo_al) & 31);
        sy[i] = (uint8_t)(single[i]->rl & 31);
        st[i] = tab_banks ? (uint8_t)(ids[single[i]->s] & 31) : 0;
        xcnt[sx[i]]++;
        ycnt[sy[i]]++;
        tcnt[st[i]]++;
    }
    // Most contended first, ties in segment order: a stable counting sort on the weight.
    int order[64];
    {
        int w[64], cnt[3 * 64 + 2] = {};
        int wmax = 0;
        for (int i = 0; i < ns; i++) {
            w[i] = xcnt[sx[i]] + ycnt[sy[i]] + (tab_banks ? tcnt[st[i]] : 0);
            cnt[w[i]]++;
            wmax = std::max(wmax, w[i]);
        }
        int at = 0;
        for (int v = wmax; v >= 0; v--) {   // start offsets, heaviest first
            const int c = cnt[v];
            cnt[v] = at;
            at += c;
        }
        for (int i = 0; i < ns; i++) order[cnt[w[i]]++] = i;
    }
    int free_in[2] = {0, 0};
    for (int l = 0; l < 64; l++)
        if (!used[l]) free_in[l >> 5]++;
    if (tab4) {
        // (half, lane class) per single: x and accumulator banks by half as below, the
        // table bank by half and class; then a free lane of that class in that half.
        int free_hc[2][4] = {};
        for (int l = 0; l < 64; l++)
            if (!used[l]) free_hc[l >> 5][l & 3]++;
        uint8_t cls[64];
        for (int oi = 0; oi < ns; oi++) {
            const int i = order[oi];
            const uint32_t id = ids[single[(size_t)i]->s];
            int best = -1, bcls = 0, bcost = 1 << 30;
            for (int h = 0; h < 2; h++)
                for (int c = 0; c < 4; c++) {
                    if (free_hc[h][c] == 0) continue;
                    const int a = xb[h][sx[(size_t)i]] + 1, b = yb[h][sy[(size_t)i]] + 1;
                    const int t = tb[h][tbank(id, c)] + 1;
                    const int cost = 64 * (a * a + b * b + t * t) - free_hc[h][c];
                    if (cost < bcost) { bcost = cost; best = h; bcls = c; }
                }
            half[(size_t)i] = (uint8_t)best;
            cls[(size_t)i] = (uint8_t)bcls;
            free_hc[best][bcls]--;
            xb[best][sx[(size_t)i]]++;
            yb[best][sy[(size_t)i]]++;
            tb[best][tbank(id, bcls)]++;
        }
        for (int i = 0; i < ns; i++) {
            int lane = 32 * half[(size_t)i] + cls[(size_t)i];
            while (used[lane]) lane += 4;   // a free lane of the class exists (counted above)
            put(*single[(size_t)i], 0, lane);
        }
        return;
    }
    for (int oi = 0; oi < ns; oi++) {
        const int i = order[oi];
        int best = -1, bcost = 1 << 30;
        for (int h = 0; h < 2; h++) {
            if (free_in[h] == 0) continue;
            const int a = xb[h][sx[(size_t)i]] + 1, b = yb[h][sy[(size_t)i]] + 1;
            const int t = tab_banks ? tb[h][st[(size_t)i]] + 1 : 0;
            const int cost = 64 * (a * a + b * b + t * t) - free_in[h];
            if (cost < bcost) { bcost = cost; best = h; }
        }
        half[(size_t)i] = (uint8_t)best;
        free_in[best]--;
        xb[best][sx[(size_t)i]]++;
        yb[best][sy[(size_t)i]]++;
        tb[best][st[(size_t)i]]++;
    }
    int lane_next[2] = {31, 63};
    for (int i = 0; i < ns; i++) {
        const int h = half[(size_t)i];
        int &lane = lane_next[h];
        while (used[lane]) lane--;
        put(*single[(size_t)i], 0, lane);
    }
}

// Cross-chunk balance (codebook bands): a band's chunks are cut in row order, so each single
// term could also sit in a neighbouring chunk whose rows stay within the row span.  Swapping
// singles between neighbours so each chunk's x banks (column mod 32) and accumulator banks
// (row mod 32) repeat less gives emit_chunk's half / lane-class placement a better start:
// the per-half read costs it reaches fall with the chunk-level sums of squared bank counts.
// Rows move between chunks only (each row is still one segment of one chunk), so the sums
// are unchanged.  Singles whose banks repeat at least `hot` times are the candidates.
void balance_chunks(std::vector<std::vector<Seg>> &cs, int nc, const int32_t *col, int32_t clo_al,
                    int32_t span) {
    struct Ch {
        uint8_t cx[32], cy[32];
        int32_t mn, mn2, mx, mx2;   // two smallest / largest rows
    };
    std::vector<Ch> ch((size_t)nc);
    auto xb = [&](const Seg &g) { return (int)((col[g.s] - clo_al) & 31); };
    auto stats = [&](int c) {
        Ch &h = ch[(size_t)c];
        std::fill(h.cx, h.cx + 32, 0);
        std::fill(h.cy, h.cy + 32, 0);
        h.mn = h.mn2 = INT32_MAX;
        h.mx = h.mx2 = INT32_MIN;
        for (const Seg &g : cs[(size_t)c]) {
            for (int32_t j = 0; j < g.n; j++) h.cx[(col[g.s + j] - clo_al) & 31]++;
            h.cy[g.rl & 31]++;
            if (g.rl < h.mn) { h.mn2 = h.mn; h.mn = g.rl; } else if (g.rl < h.mn2) h.mn2 = g.rl;
            if (g.rl > h.mx) { h.mx2 = h.mx; h.mx = g.rl; } else if (g.rl > h.mx2) h.mx2 = g.rl;
        }
    };
    for (int c = 0; c < nc; c++) stats(c);
    constexpr int hot = 3;
    // Per iteration, b's singles are tabulated once (structure of arrays: index, row, banks,
    // b's span without it, the a/b bank-count differences of its banks); for every hot single
    // of a, one vectorisable pass scores them all (ineligible: INT32_MAX) and the first least
    // score wins.  Same swap as the plain double loop: the first (i, j) of least d < 0.
    // Row windows: a chunk whose other rows span [mn, mx] (empty: mn = INT32_MAX) takes a row r
    // iff max(mx, r) - min(mn, r) < span, i.e. r in [mx - span + 1, mn + span - 1] when mx - mn
    // < span (always: a subset of a chunk's rows), any r when empty.
    // (64-bit: band2's span is INT32_MAX, no row limit -- the window then clamps to the int32 range)
    auto win_lo = [&](int32_t mn, int32_t mx) {
        return mn == INT32_MAX ? INT32_MIN : (int32_t)std::max<int64_t>(INT32_MIN, (int64_t)mx - span + 1);
    };
    auto win_hi = [&](int32_t mn, int32_t mx) {
        return mn == INT32_MAX ? INT32_MAX : (int32_t)std::min<int64_t>(INT32_MAX, (int64_t)mn + span - 1);
    };
    int32_t cj[64], crl[64], clo[64], chi[64], cxt[64], cyt[64], cpx[64], cpy[64], dv[64];
    for (int a = 0; a + 1 < nc; a++) {
        const int b = a + 1;
        for (int it = 0; it < 16; it++) {
            Ch &A = ch[(size_t)a], &B = ch[(size_t)b];
            int nt = 0;
            for (int j = 0; j < (int)cs[(size_t)b].size(); j++) {
                const Seg &t = cs[(size_t)b][(size_t)j];
                if (t.n != 1) continue;
                const int xt = xb(t), yt = t.rl & 31;
                const int32_t bmn = t.rl == B.mn ? B.mn2 : B.mn, bmx = t.rl == B.mx ? B.mx2 : B.mx;
                cj[nt] = j;
                crl[nt] = t.rl;
                clo[nt] = win_lo(bmn, bmx);
                chi[nt] = win_hi(bmn, bmx);
                if (bmn != INT32_MAX && bmx - bmn >= span) clo[nt] = INT32_MAX;   // (never: see above)
                cxt[nt] = xt;
                cyt[nt] = yt;
                cpx[nt] = A.cx[xt] - B.cx[xt];
                cpy[nt] = A.cy[yt] - B.cy[yt];
                nt++;
            }
            int minpx = INT32_MAX, minpy = INT32_MAX;   // lower bound of any single's best d
            for (int k = 0; k < nt; k++) {
                minpx = std::min(minpx, cpx[k]);
                minpy = std::min(minpy, cpy[k]);
            }
            int best_i = -1, best_j = -1, best = 0;
            for (int i = 0; i < (int)cs[(size_t)a].size(); i++) {
                const Seg &s_ = cs[(size_t)a][(size_t)i];
                if (s_.n != 1) continue;
                const int xs = xb(s_), ys = s_.rl & 31;
                if (A.cx[xs] < hot && A.cy[ys] < hot) continue;
                const int32_t amn = s_.rl == A.mn ? A.mn2 : A.mn, amx = s_.rl == A.mx ? A.mx2 : A.mx;
                if (amn != INT32_MAX && amx - amn >= span) continue;   // (never: see above)
                const int32_t alo = win_lo(amn, amx), ahi = win_hi(amn, amx), srl = s_.rl;
                // d = 2 (A.cx[xt] - A.cx[xs] + 1) + 2 (B.cx[xs] - B.cx[xt] + 1) if xs != xt, + the same in y
                const int qx = B.cx[xs] - A.cx[xs] + 2, qy = B.cy[ys] - A.cy[ys] + 2;
                if (nt == 0 || 2 * std::min(0, minpx + qx) + 2 * std::min(0, minpy + qy) >= best) continue;
                for (int k = 0; k < nt; k++) {   // branch-free: vectorises
                    const int d = 2 * (cpx[k] + qx) * (int)(xs != cxt[k]) + 2 * (cpy[k] + qy) * (int)(ys != cyt[k]);
                    const int ok = (int)(crl[k] >= alo) & (int)(crl[k] <= ahi) & (int)(srl >= clo[k]) & (int)(srl <= chi[k]);
                    dv[k] = ok ? d : INT32_MAX;
                }
                int mn = INT32_MAX;
                for (int k = 0; k < nt; k++) mn = std::min(mn, dv[k]);
                if (mn >= best) continue;
                int k = 0;
                while (dv[k] != mn) k++;
                best = mn;
                best_i = i;
                best_j = cj[k];
            }
            if (best_i < 0) break;
            std::swap(cs[(size_t)a][(size_t)best_i], cs[(size_t)b][(size_t)best_j]);
            stats(a);
            stats(b);
        }
    }
    for (int c = 0; c < nc; c++)   // emit_chunk: segments in row order, the first is the base
        std::sort(cs[(size_t)c].begin(), cs[(size_t)c].end(), [](const Seg &x, const Seg &y) { return x.rl < y.rl; });
}

void build_tile(const int32_t *rp, const int32_t *col, const float *val, const uint8_t *ids,
                int64_t r0, int64_t r1, int64_t c0, int64_t c1, B2Geom geom, TileOut &out) {
#ifdef SM_DEV
    static const bool kBalance = !(getenv("SM_B2_BAL") && atoi(getenv("SM_B2_BAL")) == 0);   // A/B
#else
    constexpr bool kBalance = true;
#endif
    const int64_t nr = r1 - r0;
    const bool cb = ids != nullptr;
    // Chunk capacity, longest segment and row span of one chunk.
    const int cap = cb ? kCbChunkTerms : 64;
    const int32_t max_seg = cb ? kCbChunkTerms : (int32_t)kB2DummyRank - 1;
    const int32_t span = cb ? geom.cb_row_span() : INT32_MAX;
    const int nchunks = geom.chunks();   // band2's default: kB2Chunks (32)
    const size_t band_words = (size_t)(cb ? 64 : 128) * nchunks;
    // A new chunk opens when the segment does not fit the current one (terms or rows).
    auto opens = [&](int fill, int32_t base, const Seg &g) {
        return fill + g.n > cap || g.rl - base >= span;
    };
    std::vector<int32_t> cur((size_t)nr), end((size_t)nr);
    std::vector<int32_t> hist((size_t)(c1 - c0) + 1, 0);
    for (int64_t r = r0; r < r1; r++) {
        const int32_t *a = col + rp[r], *z = col + rp[r + 1];
        cur[r - r0] = (int32_t)(std::lower_bound(a, z, (int32_t)c0) - col);
        end[r - r0] = (int32_t)(std::lower_bound(a, z, (int32_t)c1) - col);
        for (int32_t e = cur[r - r0]; e < end[r - r0]; e++) hist[(size_t)(col[e] - c0)]++;
    }
    // hist -> prefix counts H[i] = terms in columns [c0, c0 + i)
    std::vector<int64_t> H((size_t)(c1 - c0) + 1, 0);
    for (int64_t i = 0; i < c1 - c0; i++) H[(size_t)i + 1] = H[(size_t)i] + hist[(size_t)i];
    auto count = [&](int64_t a, int64_t b) { return H[(size_t)(b - c0)] - H[(size_t)(a - c0)]; };
    int64_t clo = c0;
    std::vector<Seg> segs;
    std::vector<std::vector<Seg>> chunk_segs;
    while (clo < c1 && count(clo, c1) > 0) {
        while (hist[(size_t)(clo - c0)] == 0) clo++;   // no band starts on an empty column
        const int64_t clo_al = clo & ~(int64_t)3;
#ifdef SM_DEV_B2_WINDOW   // development A/B: narrower bands (fewer terms per band)
        const int64_t lim = std::min<int64_t>(c1, clo_al + std::min<int32_t>(geom.window, SM_DEV_B2_WINDOW));
#else
        const int64_t lim = std::min<int64_t>(c1, clo_al + geom.window);
#endif
        // Largest chi <= lim with at most 32 * 64 terms (binary search on H).
        int64_t lo = clo + 1, hi = lim;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (count(clo, mid) <= (int64_t)nchunks * 64) lo = mid; else hi = mid - 1;
        }
        int64_t chi = lo;
        // A single column whose terms in this block need more than kB2Chunks chunks (a
        // hub or dense column: > 2048 terms, or rows too far apart for one chunk's row
        // span) is split by rows over several one-column bands: a band takes the rows
        // that fill its 32 chunks, the next band the same column from the next row on.
        // Each row still has one term in that column, so every row's terms stay in
        // ascending column order across the bands.
        bool split = false;
        for (;;) {   // pack; shrink chi until the band fits
            segs.clear();
            bool retry = false;
            int chunks = 0, fill = cap;
            int32_t base = 0;
            const bool single = chi == clo + 1;
            split = false;
            for (int64_t r = 0; r < nr && !retry; r++) {
                const int32_t s = cur[(size_t)r];
                int32_t n = 0;
                while (s + n < end[(size_t)r] && col[s + n] < chi) n++;
                if (n == 0) continue;
                if (n > max_seg) {   // band2: ranks 0..13 + dummy 15; cband: one chunk
                    chi = col[s + max_seg];
                    retry = true;
                    break;
                }
                const Seg g{(int32_t)r, s, n};
                if (opens(fill, base, g)) {
                    if (single && chunks == nchunks) { split = true; break; }   // rest: next band
                    chunks++; fill = 0; base = g.rl;
                }
                fill += n;
                segs.push_back(g);
            }
            if (retry) continue;
            if (chunks > nchunks) {
                chi = clo + std::max<int64_t>(1, (chi - clo) * 31 / 32);
                continue;
            }
            break;
        }
        // Emit: segments into chunks in row order.
        const size_t base = out.ent.size();
        out.ent.resize(base + band_words, 0u);   // dummies: word 0 (= dummy ^ dummy), value 0
        out.clo.push_back((int32_t)clo_al);
        chunk_segs.assign((size_t)nchunks, {});
        int c = -1, fill = cap;
        int32_t cbase = 0;
        for (const Seg &g : segs) {
            if (opens(fill, cbase, g)) { c++; fill = 0; cbase = g.rl; }
            fill += g.n;
            chunk_segs[(size_t)c].push_back(g);
            cur[(size_t)g.rl] += g.n;
            out.terms += g.n;
        }
        if (kBalance) balance_chunks(chunk_segs, c + 1, col, (int32_t)clo_al, span);
        for (int k = 0; k <= c; k++)
            emit_chunk(out.ent.data() + base, k, chunk_segs[(size_t)k], col, val, ids, (int32_t)clo_al, geom);
        if (!split) clo = chi;   // split: the column's remaining rows go to the next band
    }
    for (int64_t r = 0; r < nr; r++)
        if (cur[(size_t)r] != end[(size_t)r]) out.ok = false;   // unsorted columns
}

}  // namespace

bool band2_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                 int64_t n_cols, int32_t n_slabs, Band2Host &out, const uint8_t *ids, B2Geom geom,
                 int32_t slab0_permille) {
    out = Band2Host();
    out.codebook = ids != nullptr;
    out.geom = geom;
    if ((!ids && geom.cpw != 2) || geom.cpw < 1 || geom.cpw > 8 ||
        geom.window > (1 << geom.col_bits) || (ids && geom.window > (1 << geom.cb_col)) ||
        geom.block_rows > ((int64_t)1 << (32 - geom.col_bits - kB2RankBits)) ||
        geom.block_rows > ((int64_t)1 << (31 - kCbIdBits)))
        return false;
    const int64_t band_words = (int64_t)(ids ? 64 : 128) * geom.chunks();
    if (n_rows <= 0 || n_cols <= 0 || n_slabs < 1 || n_cols >= ((int64_t)1 << 30)) return false;   // x < 4 GiB: 32-bit buffer offsets
    for (int64_t r = 0; r < n_rows; r++)   // strictly ascending columns per row
        for (int32_t e = rp[r] + 1; e < rp[r + 1]; e++)
            if (col[e] <= col[e - 1]) return false;
    const int32_t br = (int32_t)std::min<int64_t>(geom.block_rows, n_rows);
    const int64_t nblk = (n_rows + br - 1) / br;
    // Slabs of whole 256-column pieces; slab 0 may be narrower (slab0_permille of an even
    // share), the others split the rest evenly.
    int64_t sc = ((n_cols + n_slabs - 1) / n_slabs + 255) & ~(int64_t)255;
    int64_t ns = (n_cols + sc - 1) / sc;
    int64_t s0 = sc;
    if (ns > 1 && slab0_permille > 0 && slab0_permille < 1000) {
        s0 = std::max<int64_t>(256, (sc * slab0_permille / 1000 + 255) & ~(int64_t)255);
        if (s0 < sc) {
            sc = ((n_cols - s0 + ns - 2) / (ns - 1) + 255) & ~(int64_t)255;
            ns = 1 + (n_cols - s0 + sc - 1) / sc;
        } else {
            s0 = sc;
        }
    }
    auto slab_lo = [&](int64_t s) { return s == 0 ? (int64_t)0 : std::min<int64_t>(n_cols, s0 + (s - 1) * sc); };
    const int64_t ntile = nblk * ns;
    if (ntile >= ((int64_t)1 << 30)) return false;
    std::vector<TileOut> tiles((size_t)ntile);
    const int nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nthr; t++)
        th.emplace_back([&, t] {
            for (int64_t i = t; i < ntile; i += nthr) {
                const int64_t b = i / ns, s = i % ns;
                build_tile(rp, col, val, ids, b * br, std::min<int64_t>(n_rows, (b + 1) * br), slab_lo(s),
                           slab_lo(s + 1), geom, tiles[(size_t)i]);
            }
        });
    for (auto &x : th) x.join();
    out.block_rows = br;
    out.n_blocks = (int32_t)nblk;
    out.n_slabs = (int32_t)ns;
    out.slab_cols = (int32_t)sc;
    out.slab0_cols = (int32_t)s0;
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
    if (nb * 4096 >= ((int64_t)1 << 31)) return false;   // 32-bit entry offsets (x 4 bytes per dword)
    out.n_bands = nb;
    out.band_clo.reserve((size_t)nb);
    out.ent.reserve((size_t)(nb * band_words));
    for (auto &t : tiles) {
        out.band_clo.insert(out.band_clo.end(), t.clo.begin(), t.clo.end());
        out.ent.insert(out.ent.end(), t.ent.begin(), t.ent.end());
        std::vector<uint32_t>().swap(t.ent);
    }
    return true;
}

bool codebook_ids(const float *val, int64_t n, std::vector<float> &table, std::vector<uint8_t> &ids) {
    // Open-addressing set of at most 255 bit patterns (512 slots).
    constexpr uint32_t kSlots = 512;
    uint32_t key[kSlots];
    int16_t id[kSlots];
    for (uint32_t i = 0; i < kSlots; i++) id[i] = -1;
    table.clear();
    ids.assign((size_t)n, 0);
    for (int64_t e = 0; e < n; e++) {
        uint32_t b;
        __builtin_memcpy(&b, &val[e], 4);
        uint32_t h = (b * 2654435761u) >> 23;   // 9 bits
        while (id[h] >= 0 && key[h] != b) h = (h + 1) & (kSlots - 1);
        if (id[h] < 0) {
            if (table.size() >= kCbDummyId) return false;
            key[h] = b;
            id[h] = (int16_t)table.size();
            table.push_back(val[e]);
        }
        ids[(size_t)e] = (uint8_t)id[h];
    }
    return true;
}

}  // namespace smamd
