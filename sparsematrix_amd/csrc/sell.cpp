// sell.cpp -- host builder of the sorted sliced-ELL layout (sell.h).  Sorting the
// rows by length makes the 64 rows of a slice nearly equally long, so a wavefront
// walks them with little padding: one lane per row adds its terms in stored order
// (the reference's order, kernel.cc:780-796), every load of a term slot is one
// coalesced 256-byte access, and no LDS or barrier sits between a slot's loads,
// its x gathers and its adds.
#include "sell.h"

#include <algorithm>
#include <thread>

namespace smamd {

void sell_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                int32_t max_len, SellHost &out, int64_t sigma, int streams, const uint8_t *ids) {
    out = SellHost();
    // Units: a row of <= max_len terms, or one segment of a longer row.
    struct Unit {
        int32_t row, start, n, part;   // part >= 0: segment partial index
    };
    std::vector<Unit> units;
    units.reserve((size_t)n_rows);
    out.long_ptr.push_back(0);
    int32_t parts = 0;
    for (int64_t r = 0; r < n_rows; r++) {
        const int32_t a = rp[r], l = rp[r + 1] - a;
        if (l <= max_len) {
            units.push_back(Unit{(int32_t)r, a, l, -1});
            continue;
        }
        for (int32_t b = 0; b < l; b += max_len)
            units.push_back(Unit{(int32_t)r, a + b, std::min(max_len, l - b), parts++});
        out.long_rows.push_back((int32_t)r);
        out.long_ptr.push_back(parts);
    }
    // Per window (units are in row order, so a window is a contiguous run of them): a
    // counting sort by descending length, stable -- ties keep row / segment order.
    // sigma <= 0: one window.  Slices are ranges [b, e) of `order`, cut per window and
    // dealt to the streams window by window.
    const int64_t win = sigma > 0 ? sigma : std::max<int64_t>(n_rows, 1);
    struct Range {
        int64_t b, e;
    };
    streams = std::max(1, streams);
    std::vector<std::vector<Range>> per((size_t)streams);
    std::vector<int32_t> order(units.size());
    std::vector<int64_t> cnt((size_t)max_len + 2);
    int64_t w = 0;
    for (size_t u0 = 0; u0 < units.size(); w++) {
        size_t u1 = u0;
        while (u1 < units.size() && units[u1].row / win == units[u0].row / win) u1++;
        std::fill(cnt.begin(), cnt.end(), (int64_t)u0);
        for (size_t i = u0; i < u1; i++) cnt[(size_t)(max_len - units[i].n) + 1]++;
        for (size_t k = 1; k < cnt.size(); k++) cnt[k] += cnt[k - 1] - (int64_t)u0;
        for (size_t i = u0; i < u1; i++) order[(size_t)cnt[(size_t)(max_len - units[i].n)]++] = (int32_t)i;
        for (int64_t i = (int64_t)u0; i < (int64_t)u1; i += kSellLanes)
            per[(size_t)(w % streams)].push_back(Range{i, std::min((int64_t)u1, i + kSellLanes)});
        u0 = u1;
    }
    std::vector<Range> slices;
    if (streams == 1) {
        slices.swap(per[0]);
    } else {
        size_t groups = 0;
        for (const auto &v : per) groups = std::max(groups, (v.size() + kSellGroup - 1) / kSellGroup);
        slices.reserve(groups * kSellGroup * (size_t)streams);
        for (size_t g = 0; g < groups; g++)
            for (const auto &v : per)
                for (size_t k = g * kSellGroup; k < (g + 1) * kSellGroup; k++)
                    slices.push_back(k < v.size() ? v[k] : Range{0, 0});
    }
    out.n_slices = (int64_t)slices.size();
    out.off.resize((size_t)out.n_slices);
    out.len.resize((size_t)out.n_slices);
    out.row.assign((size_t)out.n_slices * kSellLanes, -1);
    out.row_len.assign((size_t)out.n_slices * kSellLanes, 0);
    int64_t slots = 0;
    for (int64_t s = 0; s < out.n_slices; s++) {
        const Range &q = slices[(size_t)s];
        const int32_t L = q.e > q.b ? units[(size_t)order[(size_t)q.b]].n : 0;   // the slice's longest
        out.off[(size_t)s] = slots;
        out.len[(size_t)s] = (L + kSellUnroll - 1) / kSellUnroll * kSellUnroll;
        slots += (int64_t)out.len[(size_t)s] * kSellLanes;
    }
    out.padded = slots;
    out.col.assign((size_t)slots, 0);
    if (!ids) out.val.assign((size_t)slots, 0.0f);
    // Fill the slots, slices split across threads (disjoint lanes: no sharing).
    auto fill = [&](int64_t s0, int64_t s1) {
        for (int64_t s = s0; s < s1; s++) {
            const Range &q = slices[(size_t)s];
            for (int64_t l = 0; l < q.e - q.b; l++) {
                const Unit &u = units[(size_t)order[(size_t)(q.b + l)]];
                const size_t i = (size_t)(s * kSellLanes + l);
                out.row[i] = u.part >= 0 ? -2 - u.part : u.row;
                out.row_len[i] = u.n;
                int32_t *c = out.col.data() + out.off[(size_t)s] + l;
                if (ids) {
                    for (int32_t j = 0; j < u.n; j++)
                        c[(size_t)j * kSellLanes] =
                            (int32_t)((uint32_t)col[u.start + j] | (uint32_t)ids[u.start + j] << kSellCbColBits);
                    continue;
                }
                float *v = out.val.data() + out.off[(size_t)s] + l;
                for (int32_t j = 0; j < u.n; j++) {
                    c[(size_t)j * kSellLanes] = col[u.start + j];
                    v[(size_t)j * kSellLanes] = val[u.start + j];
                }
            }
        }
    };
    const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (nthr == 1 || slots < (1 << 20)) {
        fill(0, out.n_slices);
    } else {
        std::vector<std::thread> th;
        const int64_t per_t = (out.n_slices + nthr - 1) / nthr;
        for (int t = 0; t < nthr; t++)
            th.emplace_back(fill, std::min(out.n_slices, t * per_t), std::min(out.n_slices, (t + 1) * per_t));
        for (auto &x : th) x.join();
    }
}

}  // namespace smamd
