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
                int32_t max_len, SellHost &out) {
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
    // Counting sort by descending length (stable: ties keep row / segment order).
    std::vector<int64_t> cnt((size_t)max_len + 2, 0);
    for (const Unit &u : units) cnt[(size_t)(max_len - u.n) + 1]++;
    for (size_t i = 1; i < cnt.size(); i++) cnt[i] += cnt[i - 1];
    std::vector<int32_t> order(units.size());
    for (size_t i = 0; i < units.size(); i++) order[(size_t)cnt[(size_t)(max_len - units[i].n)]++] = (int32_t)i;
    const int64_t n_units = (int64_t)units.size();
    out.n_slices = (n_units + kSellLanes - 1) / kSellLanes;
    out.off.resize((size_t)out.n_slices);
    out.len.resize((size_t)out.n_slices);
    out.row.assign((size_t)out.n_slices * kSellLanes, -1);
    out.row_len.assign((size_t)out.n_slices * kSellLanes, 0);
    int64_t slots = 0;
    for (int64_t s = 0; s < out.n_slices; s++) {
        const int32_t L = units[(size_t)order[(size_t)(s * kSellLanes)]].n;   // the slice's longest
        out.off[(size_t)s] = slots;
        out.len[(size_t)s] = (L + kSellUnroll - 1) / kSellUnroll * kSellUnroll;
        slots += (int64_t)out.len[(size_t)s] * kSellLanes;
    }
    out.padded = slots;
    out.col.assign((size_t)slots, 0);
    out.val.assign((size_t)slots, 0.0f);
    // Fill the slots, slices split across threads (disjoint lanes: no sharing).
    auto fill = [&](int64_t s0, int64_t s1) {
        for (int64_t i = s0 * kSellLanes; i < std::min(n_units, s1 * kSellLanes); i++) {
            const int64_t s = i / kSellLanes, l = i % kSellLanes;
            const Unit &u = units[(size_t)order[(size_t)i]];
            out.row[(size_t)i] = u.part >= 0 ? -2 - u.part : u.row;
            out.row_len[(size_t)i] = u.n;
            int32_t *c = out.col.data() + out.off[(size_t)s] + l;
            float *v = out.val.data() + out.off[(size_t)s] + l;
            for (int32_t j = 0; j < u.n; j++) {
                c[(size_t)j * kSellLanes] = col[u.start + j];
                v[(size_t)j * kSellLanes] = val[u.start + j];
            }
        }
    };
    const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (nthr == 1 || slots < (1 << 20)) {
        fill(0, out.n_slices);
    } else {
        std::vector<std::thread> th;
        const int64_t per = (out.n_slices + nthr - 1) / nthr;
        for (int t = 0; t < nthr; t++)
            th.emplace_back(fill, std::min(out.n_slices, t * per), std::min(out.n_slices, (t + 1) * per));
        for (auto &x : th) x.join();
    }
}

}  // namespace smamd
