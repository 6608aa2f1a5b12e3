// ro.cpp -- host-side builder of the row-owner codebook bands (ro.h, kernels_ro.hip).
//
// Per tile (block b of rows, slab s of columns) and applying wave w (rows [w * kRoWaveRows,
// (w + 1) * kRoWaveRows) of the block), window after window (kRoWindow columns from the
// slab's first column): the wave's terms in the window, row by row and each row's in
// ascending column order, packed into chunks of <= 63 terms whose rows span < 1024 (a
// row with more terms than fit continues in the next chunk, which the same wave applies
// after it).  So every row's terms are added in ascending column order inside the slab
// (windows ascend, chunks of a window ascend in row, a row's terms ascend inside a chunk):
// the reference's per-output order (kernel.cc:780-796), slab by slab, as cband.
// Lanes: the band builder's bank-aware placement (band2.cpp emit_chunk, balance_chunks).
#include "ro.h"

#include <algorithm>
#include <thread>

#include "xband.h"

namespace smamd {

namespace {

// The geometry emit_chunk sees: one chunk per slot (cpw 1), 13-bit window columns, the
// table in four copies as the kernel holds it.
constexpr B2Geom kRoGeom{kRoBlockRows, kRoWindow, 13, 1, 13, 4, 1};

struct RoTile {
    std::vector<uint32_t> ent;
    std::vector<int32_t> wave_chunks;   // kRoApplyWaves
    int64_t terms = 0;
    bool ok = true;
};

void build_tile(const int32_t *rp, const int32_t *col, const uint8_t *ids, int64_t r0, int64_t r1,
                int64_t c0, int64_t c1, RoTile &out) {
    const int64_t nq = (c1 - c0 + kRoWindow - 1) / kRoWindow;
    if (nq > kRoMaxWindows) { out.ok = false; return; }
    out.wave_chunks.assign(kRoApplyWaves, 0);
    const uint32_t dmy = kRoGeom.cb_dummy_word(), cmask = (1u << kRoGeom.cb_col) - 1u;
    (void)cmask;
    const int osh = kRoGeom.cb_off_shift();
    const int32_t span = kRoGeom.cb_row_span();   // 1024
    std::vector<int32_t> cur, end;
    std::vector<B2Seg> segs;
    std::vector<std::vector<B2Seg>> cs;
    std::vector<int32_t> rows;
    std::vector<std::vector<int32_t>> grp_rows(kRoGroup);   // rows (sorted) of the group's chunks so far
    int grp_stage[kRoGroup] = {};
    for (int w = 0; w < kRoApplyWaves; w++) {
        const int64_t wr0 = r0 + (int64_t)w * kRoWaveRows, wr1 = std::min<int64_t>(r1, wr0 + kRoWaveRows);
        if (wr0 >= wr1) continue;
        int32_t idx = 0;   // position in the wave's stream
        const int64_t nr = wr1 - wr0;
        cur.assign((size_t)nr, 0);
        end.assign((size_t)nr, 0);
        for (int64_t r = wr0; r < wr1; r++) {
            const int32_t *a = col + rp[r], *z = col + rp[r + 1];
            cur[(size_t)(r - wr0)] = (int32_t)(std::lower_bound(a, z, (int32_t)c0) - col);
            end[(size_t)(r - wr0)] = (int32_t)(std::lower_bound(a, z, (int32_t)c1) - col);
        }
        for (int64_t q = 0; q < nq; q++) {
            const int64_t clo = c0 + q * kRoWindow, chi = std::min<int64_t>(c1, clo + kRoWindow);
            // the wave's segments in this window, in row order; rows of more than 63 terms in
            // it are cut in 63-term pieces (consecutive chunks, applied in order)
            segs.clear();
            for (int64_t r = 0; r < nr; r++) {
                int32_t s = cur[(size_t)r];
                while (s < end[(size_t)r] && col[s] < chi) {
                    int32_t n = 0;
                    while (s + n < end[(size_t)r] && col[s + n] < chi && n < kCbChunkTerms) n++;
                    segs.push_back({(int32_t)(r + wr0 - r0), s, n});
                    s += n;
                }
                cur[(size_t)r] = s;
            }
            if (segs.empty()) continue;
            // pack: a new chunk when the segment does not fit (terms or row span)
            cs.clear();
            int fill = kCbChunkTerms;
            int32_t base = 0;
            for (const B2Seg &g : segs) {
                if (fill + g.n > kCbChunkTerms || g.rl - base >= span || (!cs.empty() && cs.back().back().rl == g.rl)) {
                    cs.emplace_back();
                    fill = 0;
                    base = g.rl;
                }
                cs.back().push_back(g);
                fill += g.n;
                out.terms += g.n;
            }
            const int nc = (int)cs.size();
            // a row cut in pieces sits in consecutive chunks: keep them out of the balance
            bool cut = false;
            for (int c = 0; c + 1 < nc && !cut; c++) cut = cs[(size_t)c].back().rl == cs[(size_t)c + 1].front().rl;
            if (!cut) b2_balance_chunks(cs, nc, col, (int32_t)clo, span);
            for (int c = 0; c < nc; c++) {
                const size_t at = out.ent.size();
                out.ent.resize(at + 64, 0u);
                b2_emit_chunk(out.ent.data() + at, 0, cs[(size_t)c], col, nullptr, ids, (int32_t)clo, kRoGeom);
                // header: window index | stage | base row relative to the wave's first row (11 bits)
                const uint32_t brel = (uint32_t)(cs[(size_t)c].front().rl - (int32_t)(wr0 - r0));
                rows.clear();
                for (const B2Seg &g : cs[(size_t)c]) rows.push_back(g.rl);
                std::sort(rows.begin(), rows.end());
                const int gi = idx % kRoGroup;
                int stage = 0;
                for (int j = 0; j < gi; j++) {
                    bool share = false;
                    for (int32_t r : rows) share = share || std::binary_search(grp_rows[(size_t)j].begin(), grp_rows[(size_t)j].end(), r);
                    if (share) stage = std::max(stage, grp_stage[j] + 1);
                }
                grp_rows[(size_t)gi].swap(rows);
                grp_stage[gi] = stage;
                idx++;
                const uint32_t h = ((uint32_t)q & (uint32_t)(kRoMaxWindows - 1)) | ((uint32_t)stage << kRoStageShift) | dmy |
                                   ((brel & 1023u) << osh) | ((brel >> 10) << kCbContBit);
                out.ent[at] = h ^ dmy;
            }
            out.wave_chunks[(size_t)w] += nc;
        }
        for (int64_t r = 0; r < nr; r++)
            if (cur[(size_t)r] != end[(size_t)r]) { out.ok = false; return; }   // unsorted columns
    }
}

}  // namespace

bool ro_build(const int32_t *rp, const int32_t *col, const uint8_t *ids, int64_t n_rows, int64_t n_cols,
              int32_t n_slabs, RoHost &out) {
    out = RoHost();
    if (!ids || n_rows <= 0 || n_cols <= 0 || n_slabs < 1 || n_cols >= ((int64_t)1 << 30)) return false;
    for (int64_t r = 0; r < n_rows; r++)   // strictly ascending columns per row
        for (int32_t e = rp[r] + 1; e < rp[r + 1]; e++)
            if (col[e] <= col[e - 1]) return false;
    const int32_t br = kRoBlockRows;
    const int64_t nblk = (n_rows + br - 1) / br;
    const int64_t sc = ((n_cols + n_slabs - 1) / n_slabs + 255) & ~(int64_t)255;
    const int64_t ns = (n_cols + sc - 1) / sc;
    const int64_t ntile = nblk * ns;
    if (ntile >= ((int64_t)1 << 24)) return false;
    std::vector<RoTile> tiles((size_t)ntile);
    const int nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nthr; t++)
        th.emplace_back([&, t] {
            for (int64_t i = t; i < ntile; i += nthr) {
                const int64_t b = i / ns, s = i % ns;
                build_tile(rp, col, ids, b * br, std::min<int64_t>(n_rows, (b + 1) * br), s * sc,
                           std::min<int64_t>(n_cols, (s + 1) * sc), tiles[(size_t)i]);
            }
        });
    for (auto &x : th) x.join();
    out.block_rows = br;
    out.n_blocks = (int32_t)nblk;
    out.n_slabs = (int32_t)ns;
    out.slab_cols = (int32_t)sc;
    out.wave_start.assign((size_t)ntile * kRoApplyWaves + 1, 0);
    int64_t nc = 0;
    for (int64_t i = 0; i < ntile; i++) {
        const RoTile &t = tiles[(size_t)i];
        if (!t.ok) return false;
        for (int w = 0; w < kRoApplyWaves; w++) {
            out.wave_start[(size_t)(i * kRoApplyWaves + w)] = (int32_t)nc;
            nc += t.wave_chunks[(size_t)w];
            out.max_chunks_per_wave = std::max(out.max_chunks_per_wave, t.wave_chunks[(size_t)w]);
        }
        out.real_terms += t.terms;
    }
    out.wave_start[(size_t)ntile * kRoApplyWaves] = (int32_t)nc;
    if (nc * 256 >= ((int64_t)1 << 32)) return false;   // 32-bit byte offsets of the entries
    out.n_chunks = nc;
    out.ent.reserve((size_t)nc * 64);
    for (auto &t : tiles) {
        out.ent.insert(out.ent.end(), t.ent.begin(), t.ent.end());
        std::vector<uint32_t>().swap(t.ent);
    }
    return true;
}

}  // namespace smamd
