// ccsell.cpp -- host builder of the column-chunked sorted sliced-ELL layout (ccsell.h).
//
// Two passes over the CSR, rows split over threads: pass 1 counts units per
// (chunk, length) bucket and thread; a prefix over buckets in (chunk, descending
// length) order and threads in row order gives every thread its cursors; pass 2
// recomputes the units and writes them straight to their sorted place (a stable
// counting sort: ties keep row order).  Slices of 64 units are then cut per chunk and
// their slots filled, slices split over threads.
#include "ccsell.h"

#include <algorithm>
#include <thread>

#include "sell.h"

namespace smamd {

namespace {

struct Unit {
    int32_t row;     // | kCcFirst for the row's first unit
    int32_t start;   // first term in the CSR
    int32_t n;       // terms
};

}  // namespace

bool ccsell_build(const int32_t *rp, const int32_t *col, const float *val, const uint8_t *ids,
                  int64_t n_rows, int64_t n_cols, int32_t chunk_log2, CcsellHost &out,
                  bool by_length) {
    out = CcsellHost();
    if (n_rows <= 0 || n_cols <= 0 || chunk_log2 < 8 || chunk_log2 > 30) return false;
    if (ids && chunk_log2 > 24) return false;               // column bits + 8-bit id
    if (n_rows >= ((int64_t)1 << 31)) return false;
    const int64_t nch = (n_cols + ((int64_t)1 << chunk_log2) - 1) >> chunk_log2;
    if (nch > (1 << 16)) return false;
    const int64_t nb = nch * (kCcMaxUnit + 1);              // buckets: (chunk, length)
    const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t rows_per = (n_rows + nthr - 1) / nthr;
    std::vector<std::vector<int64_t>> cnt((size_t)nthr);
    std::vector<char> bad((size_t)nthr, 0);
    // Visit the units of rows [r0, r1): f(unit, bucket).
    auto walk = [&](int64_t r0, int64_t r1, auto &&f) -> bool {
        for (int64_t r = r0; r < r1; r++) {
            const int32_t a = rp[r], b = rp[r + 1];
            if (a == b) {   // no terms: an empty unit in chunk 0 applies beta
                f(Unit{(int32_t)((uint32_t)r | kCcFirst), a, 0}, by_length ? (int64_t)kCcMaxUnit : 0);
                continue;
            }
            bool first = true;
            for (int32_t e = a; e < b;) {
                const int64_t c = col[e] >> chunk_log2;
                int32_t k = e + 1;
                while (k < b && (col[k] >> chunk_log2) == c) {
                    if (col[k] <= col[k - 1]) return false;   // unsorted / repeated
                    k++;
                }
                if (k < b && col[k] <= col[k - 1]) return false;
                const int32_t n = k - e;
                if (n > kCcMaxUnit) return false;
                f(Unit{(int32_t)((uint32_t)r | (first ? kCcFirst : 0u)), e, n},
                  c * (kCcMaxUnit + 1) + (by_length ? kCcMaxUnit - n : 0));
                first = false;
                e = k;
            }
        }
        return true;
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nthr; t++)
            th.emplace_back([&, t] {
                cnt[(size_t)t].assign((size_t)nb, 0);
                int64_t *h = cnt[(size_t)t].data();
                const int64_t r0 = std::min(n_rows, t * rows_per), r1 = std::min(n_rows, (t + 1) * rows_per);
                bad[(size_t)t] = !walk(r0, r1, [&](const Unit &, int64_t bk) { h[bk]++; });
            });
        for (auto &x : th) x.join();
    }
    for (char b : bad)
        if (b) return false;
    // Cursors: bucket-major, thread-minor; chunk c's units start at the first bucket of c.
    std::vector<int64_t> chunk_units((size_t)nch + 1, 0);
    int64_t total = 0;
    for (int64_t bk = 0; bk < nb; bk++) {
        if (bk % (kCcMaxUnit + 1) == 0) chunk_units[(size_t)(bk / (kCcMaxUnit + 1))] = total;
        for (int t = 0; t < nthr; t++) {
            const int64_t v = cnt[(size_t)t][(size_t)bk];
            cnt[(size_t)t][(size_t)bk] = total;
            total += v;
        }
    }
    chunk_units[(size_t)nch] = total;
    if (total >= ((int64_t)1 << 31)) return false;
    std::vector<Unit> units((size_t)total);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nthr; t++)
            th.emplace_back([&, t] {
                int64_t *cur = cnt[(size_t)t].data();
                const int64_t r0 = std::min(n_rows, t * rows_per), r1 = std::min(n_rows, (t + 1) * rows_per);
                walk(r0, r1, [&](const Unit &u, int64_t bk) { units[(size_t)cur[bk]++] = u; });
            });
        for (auto &x : th) x.join();
    }
    std::vector<std::vector<int64_t>>().swap(cnt);
    // Slices of 64 units, per chunk.
    out.chunk_log2 = chunk_log2;
    out.n_chunks = (int32_t)nch;
    out.n_units = total;
    out.chunk_slice.assign((size_t)nch + 1, 0);
    int64_t ns = 0;
    for (int64_t c = 0; c < nch; c++) {
        out.chunk_slice[(size_t)c] = ns;
        ns += (chunk_units[(size_t)c + 1] - chunk_units[(size_t)c] + kSellLanes - 1) / kSellLanes;
    }
    out.chunk_slice[(size_t)nch] = ns;
    out.n_slices = ns;
    out.off.resize((size_t)ns);
    out.len.resize((size_t)ns);
    out.row.assign((size_t)ns * kSellLanes, -1);
    out.row_len.assign((size_t)ns * kSellLanes, 0);
    std::vector<int64_t> slice_unit((size_t)ns);   // first unit of each slice
    int64_t slots = 0;
    for (int64_t c = 0; c < nch; c++) {
        for (int64_t s = out.chunk_slice[(size_t)c]; s < out.chunk_slice[(size_t)c + 1]; s++) {
            const int64_t u0 = chunk_units[(size_t)c] + (s - out.chunk_slice[(size_t)c]) * kSellLanes;
            slice_unit[(size_t)s] = u0;
            int32_t L = 0;   // the slice's longest unit (its first when sorted by length)
            for (int64_t u = u0; u < std::min(u0 + kSellLanes, chunk_units[(size_t)c + 1]); u++)
                L = std::max(L, units[(size_t)u].n);
            out.off[(size_t)s] = slots;
            out.len[(size_t)s] = L;   // no padding: the kernel runs the remainder one slot at a time
            slots += (int64_t)out.len[(size_t)s] * kSellLanes;
        }
    }
    out.padded = slots;
    out.word.assign((size_t)slots, 0u);
    if (!ids) out.val.assign((size_t)slots, 0.0f);
    const uint32_t cmask = (uint32_t)((1ull << chunk_log2) - 1);
    auto fill = [&](int64_t s0, int64_t s1) {
        for (int64_t s = s0; s < s1; s++) {
            const int64_t c = std::upper_bound(out.chunk_slice.begin(), out.chunk_slice.end(), s) -
                              out.chunk_slice.begin() - 1;
            const int64_t u1 = chunk_units[(size_t)c + 1];
            for (int l = 0; l < kSellLanes && slice_unit[(size_t)s] + l < u1; l++) {
                const Unit &u = units[(size_t)(slice_unit[(size_t)s] + l)];
                const size_t i = (size_t)(s * kSellLanes + l);
                out.row[i] = u.row;
                out.row_len[i] = (uint16_t)u.n;
                uint32_t *w = out.word.data() + out.off[(size_t)s] + l;
                for (int32_t j = 0; j < u.n; j++) {
                    const uint32_t cc = (uint32_t)col[u.start + j] & cmask;
                    w[(size_t)j * kSellLanes] = ids ? cc | (uint32_t)ids[u.start + j] << chunk_log2 : cc;
                }
                if (!ids) {
                    float *v = out.val.data() + out.off[(size_t)s] + l;
                    for (int32_t j = 0; j < u.n; j++) v[(size_t)j * kSellLanes] = val[u.start + j];
                }
            }
        }
    };
    if (nthr == 1 || slots < (1 << 20)) {
        fill(0, ns);
    } else {
        std::vector<std::thread> th;
        const int64_t per = (ns + nthr - 1) / nthr;
        for (int t = 0; t < nthr; t++)
            th.emplace_back(fill, std::min(ns, t * per), std::min(ns, (t + 1) * per));
        for (auto &x : th) x.join();
    }
    return true;
}

}  // namespace smamd
