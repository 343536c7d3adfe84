// pfx_nblist.h -- radius-neighbour lists of grid points, materialised in HBM.
//
// For a set of query points that are points of the grid (all of them, or a masked subset),
// build_lists() produces, per query j:
//   cnt[j]  = |N_r(q_j)| (FLANN semantics: d2 < (float)(r*r), self and duplicates included)
//   list[off[j] + (m << lg[j])], m < cnt[j]  = neighbours as cell-sorted positions, in FLANN
//                                order (d2, caller index) ascending when `sorted`
// Layout: queries are ordered by cell (qpos[j] = sorted position of query j).  The lists of one
// tile (<= 16 consecutive queries of one cell) are interleaved (stride 2^lg >= tile size), so a
// consumer that gives consecutive queries to consecutive lanes reads whole cache lines per load.
#pragma once
#include "pfx_internal.h"

namespace pfx {

struct NbLists {
  int64_t nq = 0;            // number of queries
  int64_t total = 0;         // sum of cnt
  int64_t slots = 0;         // list entries allocated (total + interleave padding)
  const int32_t* qpos = nullptr;   // [nq] sorted position of each query
  const int64_t* off = nullptr;    // [nq]
  const int32_t* cnt = nullptr;    // [nq]
  const uint8_t* lg = nullptr;     // [nq] log2 of the entry stride
  const uint32_t* list = nullptr;  // [total]
};

// mask (nullable): per *caller* index, queries are the masked points (in cell order).
void build_lists(pfx_ctx* ctx, const Grid& g, const uint8_t* mask, double radius, bool sorted, NbLists& out,
                 const char* tag);

}  // namespace pfx
