// sell.cpp -- host builder of the sorted sliced-ELL layout (sell.h).  Sorting the
// rows by length makes the 64 rows of a slice nearly equally long, so a wavefront
// walks them with little padding: one lane per row adds its terms in stored order
// (the reference's order, kernel.cc:780-796), every load of a term slot is one
// coalesced 256-byte access, and no LDS or barrier sits between a slot's loads,
// its x gathers and its adds.
#include "sell.h"

#include <algorithm>

namespace smamd {

void sell_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows,
                int32_t max_len, SellHost &out) {
    out = SellHost();
    // Counting sort by descending length (stable: ties keep row order).
    std::vector<int64_t> cnt((size_t)max_len + 2, 0);
    int64_t n_short = 0;
    for (int64_t r = 0; r < n_rows; r++) {
        const int32_t l = rp[r + 1] - rp[r];
        if (l <= max_len) { cnt[(size_t)(max_len - l) + 1]++; n_short++; }
    }
    for (size_t i = 1; i < cnt.size(); i++) cnt[i] += cnt[i - 1];
    std::vector<int32_t> order((size_t)n_short);
    for (int64_t r = 0; r < n_rows; r++) {
        const int32_t l = rp[r + 1] - rp[r];
        if (l <= max_len) order[(size_t)cnt[(size_t)(max_len - l)]++] = (int32_t)r;
    }
    out.n_slices = (n_short + kSellLanes - 1) / kSellLanes;
    out.off.resize((size_t)out.n_slices);
    out.len.resize((size_t)out.n_slices);
    out.row.assign((size_t)out.n_slices * kSellLanes, -1);
    out.row_len.assign((size_t)out.n_slices * kSellLanes, 0);
    int64_t slots = 0;
    for (int64_t s = 0; s < out.n_slices; s++) {
        const int32_t r0 = order[(size_t)(s * kSellLanes)];   // the slice's longest row
        const int32_t L = rp[r0 + 1] - rp[r0];
        out.off[(size_t)s] = slots;
        out.len[(size_t)s] = (L + kSellUnroll - 1) / kSellUnroll * kSellUnroll;
        slots += (int64_t)out.len[(size_t)s] * kSellLanes;
    }
    out.padded = slots;
    out.col.assign((size_t)slots, 0);
    out.val.assign((size_t)slots, 0.0f);
    for (int64_t i = 0; i < n_short; i++) {
        const int64_t s = i / kSellLanes, l = i % kSellLanes;
        const int32_t r = order[(size_t)i];
        const int32_t a = rp[r], n = rp[r + 1] - a;
        out.row[(size_t)i] = r;
        out.row_len[(size_t)i] = n;
        int32_t *c = out.col.data() + out.off[(size_t)s] + l;
        float *v = out.val.data() + out.off[(size_t)s] + l;
        for (int32_t j = 0; j < n; j++) {
            c[(size_t)j * kSellLanes] = col[a + j];
            v[(size_t)j * kSellLanes] = val[a + j];
        }
    }
}

}  // namespace smamd
