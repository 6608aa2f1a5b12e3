// merge.h -- the merge path's partition (SM_ALGO_MERGE, kernels_merge.hip)
// and its host-side plan pieces (merge.cpp).  No HIP types: the builder is checked under
// AddressSanitizer on the host (tests/native/merge_asan.cpp).
#pragma once

#include <cstdint>
#include <vector>

namespace smamd {

constexpr int kMgThreads = 256;
#ifndef SM_MERGE_IPT
#define SM_MERGE_IPT 8
#endif
constexpr int kMgIpt = SM_MERGE_IPT;               // merge items per thread (A/B builds: DEV_FLAGS)
constexpr int kMgTile = kMgThreads * kMgIpt;       // 2048 per workgroup

// Workgroups (slices of kMgTile merge items: n_rows row ends + nnz terms).
int64_t merge_blocks(int64_t n_rows, int64_t nnz);
// The (row, term) corner of every workgroup's slice, blocks + 1 of them, as (row, term) pairs:
// the rows whose end comes before the slice's first item, and the terms before it.
void merge_corners(const int32_t *rp, int64_t n_rows, int64_t nnz, std::vector<int32_t> &out);
// The staging stream (sm_build_opts.merge_stage): every slice's terms stable-sorted by column,
// as (column << 8 | codebook id) words w and their place in the slice z (term z0 + z[k] of the
// CSR), and the table (256 entries, 0 past the codebook).  False when it does not apply (values
// not a <= 255-entry codebook, columns past 2^24).  col: the columns the kernel gathers with.
bool merge_stage_build(const int32_t *rp, const int32_t *col, const float *val, int64_t n_rows, int64_t n_cols,
                       int64_t nnz, std::vector<uint32_t> &w, std::vector<uint16_t> &z, std::vector<float> &table);

}  // namespace smamd
