// Host-only: LDS bank cost of the cband chunk lanes the builder emits (band2.cpp).
// Builds the cband layout of a config-2-like slice (rows x 2^20 columns, 16 random
// terms per row, 255-entry codebook) and reports, per chunk instruction and half-wave,
// the LDS cycles of the x, accumulator and codebook reads (1 = conflict-free): the most
// distinct addresses on one bank.  Geometry: argv[2] = "wide" (32 table copies: its
// table reads are conflict-free) or "dma3" (the default, 4 copies).  Dev tool:
// g++ -O2 -I sparsematrix_amd/csrc tools/band2_banks.cpp sparsematrix_amd/csrc/band2.cpp -lpthread
#include <algorithm>
#include <cstdio>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "xband.h"

using namespace smamd;

int main(int argc, char **argv) {
    const int64_t n_rows = argc > 1 ? atoll(argv[1]) : 32768, n_cols = 1 << 20;
    const bool wide = argc > 2 && std::string(argv[2]) == "wide";
    const B2Geom geom = wide ? kB2Wide : kB2Dma3Cb;
    const int copies = wide ? 32 : geom.tab_copies;
    std::mt19937_64 rng(7);
    std::vector<int32_t> rp(n_rows + 1), col;
    std::vector<float> val;
    std::vector<uint8_t> ids;
    for (int64_t r = 0; r < n_rows; r++) {
        std::set<int32_t> cs;
        while (cs.size() < 16) cs.insert((int32_t)(rng() % n_cols));
        for (int32_t c : cs) { col.push_back(c); val.push_back(1.0f); ids.push_back((uint8_t)(rng() % 255)); }
        rp[r + 1] = (int32_t)col.size();
    }
    Band2Host h;
    if (!band2_build(rp.data(), col.data(), val.data(), n_rows, n_cols, 4, h, ids.data(), geom)) { puts("build failed"); return 1; }
    const int nch = geom.chunks(), cpw = geom.cpw;
    const uint32_t colmask = (1u << geom.cb_col) - 1u, dummy = geom.cb_dummy_word();
    const int offsh = geom.cb_off_shift();
    const uint32_t offm = geom.cb_off_mask();
    double xs = 0, ys = 0, ts = 0, halves = 0;
    int64_t hist_x[8] = {}, hist_y[8] = {};
    for (int64_t g = 0; g < h.n_bands; g++)
        for (int c = 0; c < nch; c++) {
            const int wave = c / cpw, k = c % cpw;
            uint32_t w[64];
            for (int l = 0; l < 64; l++)
                w[l] = h.ent[(size_t)g * 64 * nch + (size_t)(wave * 64 + l) * cpw + k] ^ dummy;
            const uint32_t hd = w[0];
            const uint32_t base = (hd & colmask) | (((hd >> offsh) & offm) << geom.cb_col);
            for (int half = 0; half < 2; half++) {
                std::set<uint32_t> xa[32], ya[32], ta[32];
                for (int l = 32 * half; l < 32 * half + 32; l++) {
                    const uint32_t cx = w[l] & colmask;
                    const uint32_t rl = base + ((w[l] >> offsh) & offm);
                    const uint32_t id = (w[l] >> geom.cb_col) & kCbDummyId;
                    const uint32_t ta_addr = id * copies + (l & (copies - 1));
                    xa[cx & 31].insert(cx);
                    ya[rl & 31].insert(rl);
                    ta[ta_addr & 31].insert(ta_addr);
                }
                size_t mx = 0, my = 0, mt = 0;
                for (int b = 0; b < 32; b++) {
                    mx = std::max(mx, xa[b].size()); my = std::max(my, ya[b].size()); mt = std::max(mt, ta[b].size());
                }
                xs += mx; ys += my; ts += mt; halves += 1;
                hist_x[std::min<size_t>(mx, 7)]++; hist_y[std::min<size_t>(my, 7)]++;
            }
        }
    printf("bands %lld  per half-wave read: x %.3f cycles, acc %.3f cycles, table %.3f cycles\n", (long long)h.n_bands,
           xs / halves, ys / halves, ts / halves);
    printf("x hist:");  for (int i = 1; i < 8; i++) printf(" %d:%.3f", i, hist_x[i] / halves);
    printf("\nacc hist:"); for (int i = 1; i < 8; i++) printf(" %d:%.3f", i, hist_y[i] / halves);
    printf("\n");
}
