// sweep.cpp -- host builder of the column-swept row blocks (sweep.h).
#include "sweep.h"

#include <algorithm>
#include <atomic>
#include <thread>

namespace smamd {

bool sweep_build(const int32_t *rp, const int32_t *col, const uint8_t *ids, int64_t n_rows,
                 SweepHost &out) {
    out = SweepHost();
    const int64_t R = out.block_rows;
    out.n_blocks = (n_rows + R - 1) / R;
    out.block_chunk.assign((size_t)out.n_blocks + 1, 0);
    for (int64_t b = 0; b < out.n_blocks; b++) {
        const int64_t r1 = std::min(n_rows, (b + 1) * R);
        out.block_chunk[(size_t)b + 1] = out.block_chunk[(size_t)b] + ((int64_t)rp[r1] - rp[b * R] + 63) / 64;
    }
    out.n_chunks = out.block_chunk.back();
    out.ent.assign((size_t)out.n_chunks * 128, 0u);
    const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<bool> ok{true};
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        struct Term {
            uint32_t col, row;
            uint8_t id;
        };
        std::vector<Term> t;
        for (;;) {
            const int64_t b = next.fetch_add(1);
            if (b >= out.n_blocks || !ok.load()) return;
            const int64_t r0 = b * R, r1 = std::min(n_rows, r0 + R);
            t.clear();
            for (int64_t r = r0; r < r1; r++)
                for (int32_t e = rp[r]; e < rp[r + 1]; e++) {
                    if (e > rp[r] && col[e] <= col[e - 1]) { ok = false; return; }
                    t.push_back(Term{(uint32_t)col[e], (uint32_t)(r - r0), ids[e]});
                }
            // The block's terms in ascending column (rows distinct within a column).
            std::sort(t.begin(), t.end(), [](const Term &a, const Term &c) {
                return a.col != c.col ? a.col < c.col : a.row < c.row;
            });
            uint32_t *ent = out.ent.data() + (size_t)out.block_chunk[(size_t)b] * 128;
            for (size_t c0 = 0; c0 < t.size(); c0 += 64) {
                const size_t c1 = std::min(t.size(), c0 + 64);
                // Inside the chunk: grouped by row, each row's terms still ascending.
                std::stable_sort(t.begin() + (int64_t)c0, t.begin() + (int64_t)c1,
                                 [](const Term &a, const Term &c) { return a.row < c.row; });
                uint32_t *ch = ent + (c0 / 64) * 128;
                for (size_t i = c0; i < c1; i++) {
                    const size_t l = i - c0;
                    const bool cont = i > c0 && t[i].row == t[i - 1].row;
                    ch[2 * l] = t[i].col;
                    ch[2 * l + 1] = t[i].row | (cont ? kSwContBit : 0u) | ((uint32_t)t[i].id << 16);
                }
                for (size_t l = c1 - c0; l < 64; l++) {   // padding: dummy id, row 0
                    ch[2 * l] = 0;
                    ch[2 * l + 1] = kSwDummyId << 16;
                }
            }
        }
    };
    std::vector<std::thread> th;
    for (int k = 0; k < nthr; k++) th.emplace_back(work);
    for (auto &x : th) x.join();
    return ok.load();
}

}  // namespace smamd
