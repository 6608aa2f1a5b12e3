// plan.cpp -- row-tile planner for the stream SpMV kernel.
//
// Greedy, in row order: a tile takes rows while its terms stay <= tile_nnz and
// its rows <= tile_rows, so every workgroup does a similar amount of
// (rows + terms) work whatever the row-length distribution (uniform 16/row or
// R-MAT power law).  A row with more than tile_nnz terms is a "long row": it
// gets no tile; its terms are split into chunk_nnz chunks, one workgroup each,
// whose partial sums are added in chunk order by the finalize kernel.
#include "encode.h"

namespace smamd {

void plan_rows(const int32_t *rp, int64_t n, int32_t tile_nnz, int32_t tile_rows,
               int32_t chunk_nnz, int32_t serial_max, PlanHost &out) {
    out = PlanHost();
    out.long_ptr.push_back(0);
    int64_t r = 0;
    int32_t maxlen = 0;
    while (r < n) {
        const int32_t len = rp[r + 1] - rp[r];
        maxlen = std::max(maxlen, len);
        if (len > tile_nnz) {
            const int32_t lr = (int32_t)out.long_rows.size();
            for (int32_t b = rp[r]; b < rp[r + 1]; b += chunk_nnz)
                out.chunks.push_back({lr, b, std::min(rp[r + 1], b + chunk_nnz)});
            out.long_rows.push_back((int32_t)r);
            out.long_ptr.push_back((int32_t)out.chunks.size());
            r++;
            continue;
        }
        const int64_t r0 = r;
        int32_t acc = 0, flags = 0;
        while (r < n && r - r0 < tile_rows) {
            const int32_t l = rp[r + 1] - rp[r];
            if (l > tile_nnz || acc + l > tile_nnz) break;
            maxlen = std::max(maxlen, l);
            acc += l;
            if (l > serial_max) flags |= 1;
            r++;
        }
        out.tiles.push_back({(int32_t)r0, (int32_t)r, flags});
    }
    out.max_row_nnz = maxlen;
    out.avg_row_nnz = n ? (double)rp[n] / (double)n : 0.0;
}

}  // namespace smamd
