// merge.cpp -- host-side plan of the merge path (merge.h; kernels_merge.hip runs it):
// the slices' corners and the column-sorted staging stream.
#include "merge.h"

#include <algorithm>
#include <thread>

#include "xband.h"   // codebook_ids

namespace smamd {

int64_t merge_blocks(int64_t n_rows, int64_t nnz) { return (n_rows + nnz + kMgTile - 1) / kMgTile; }

void merge_corners(const int32_t *rp, int64_t n_rows, int64_t nnz, std::vector<int32_t> &out) {
    const int64_t nb = merge_blocks(n_rows, nnz), total = n_rows + nnz;
    out.resize((size_t)(2 * (nb + 1)));
    for (int64_t b = 0; b <= nb; ++b) {
        const int64_t d = std::min<int64_t>(b * kMgTile, total);
        int64_t lo = std::max<int64_t>(d - nnz, 0), hi = std::min<int64_t>(d, n_rows);
        while (lo < hi) {   // merge_corner, on the host
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)rp[mid + 1] <= d - mid - 1) lo = mid + 1;
            else hi = mid;
        }
        out[(size_t)(2 * b)] = (int32_t)lo;
        out[(size_t)(2 * b + 1)] = (int32_t)(d - lo);
    }
}

bool merge_stage_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows, int64_t n_cols,
                       int64_t nnz, std::vector<uint32_t> &w, std::vector<uint16_t> &z, std::vector<float> &table) {
    if (nnz <= 0 || n_cols > (1 << 24)) return false;
    std::vector<uint8_t> ids;
    if (!codebook_ids(val, nnz, table, ids)) return false;
    table.resize(256, 0.0f);
    std::vector<int32_t> corners;
    merge_corners(rp, n_rows, nnz, corners);
    const int64_t nb = (int64_t)corners.size() / 2 - 1;
    w.resize((size_t)nnz);
    z.resize((size_t)nnz);
    const int nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nthr; t++)
        th.emplace_back([&, t] {
            std::vector<int32_t> ord;
            for (int64_t b = t; b < nb; b += nthr) {
                const int32_t z0 = corners[(size_t)(2 * b + 1)], z1 = corners[(size_t)(2 * b + 3)];
                ord.resize((size_t)(z1 - z0));
                for (int32_t k = 0; k < z1 - z0; k++) ord[(size_t)k] = k;
                std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t c) { return col[z0 + a] < col[z0 + c]; });
                for (int32_t k = 0; k < z1 - z0; k++) {
                    const int32_t e = z0 + ord[(size_t)k];
                    w[(size_t)(z0 + k)] = ((uint32_t)col[e] << 8) | ids[(size_t)e];
                    z[(size_t)(z0 + k)] = (uint16_t)ord[(size_t)k];
                }
            }
        });
    for (auto &x : th) x.join();
    return true;
}

}  // namespace smamd
