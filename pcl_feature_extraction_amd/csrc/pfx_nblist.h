// pfx_nblist.h -- radius-neighbour lists of grid points, materialised in HBM.
//
// For a set of query points that are points of the grid (all of them, or a masked subset),
// build_lists() produces, per query j:
//   cnt[j]  = |N_r(q_j)| (FLANN semantics: d2 < (float)(r*r), self and duplicates included)
//   list[off[j] + (m << lg[j])], m < cnt[j]  = neighbours in FLANN order (d2, caller index)
//                                ascending when `sorted`, as run entries (below)
// Run entry: (r << 28) | off -- the neighbour is the off-th point of run r (0..8) of the query
// cell's 3x3x3 block (run r = cells (ix + r/3 - 1, iy + r%3 - 1, iz-1..iz+1), clipped to the
// grid), i.e. cell-sorted position cell_start[first cell of run r] + off.  Consumers resolve r
// through a per-cell table, so a workgroup can stage its candidate runs in LDS and index them
// directly (k_normals_chain).
// Layout: queries are ordered by cell (qpos[j] = sorted position of query j).  The lists of one
// tile (<= 16 consecutive queries of one cell) are interleaved (stride 2^lg >= tile size), so a
// consumer that gives consecutive queries to consecutive lanes reads whole cache lines per load.
#pragma once
#include "pfx_internal.h"

namespace pfx {

constexpr uint32_t kEntryOffMask = 0x0fffffffu;
__host__ __device__ __forceinline__ int entry_run(uint32_t e) { return (int)(e >> 28); }
__host__ __device__ __forceinline__ uint32_t entry_off(uint32_t e) { return e & kEntryOffMask; }
// Compact lists (round 5; builds with `compact`, the tile kernels' lists of blocks whose runs all
// hold <= 4096 points): 16-bit run entries (r << 12) | off, flagged by bit 7 of lg[j]; off[j]
// and the stride 2^(lg & 0x7f) then count 16-bit entries (entry m of query j at
// ((const uint16_t*)list)[off[j] + (m << lg)]).  Read by the normal estimation's chains and by
// FPFH's all-points weighting when it reuses those lists (list_entry); the other consumers build
// without `compact`.  Per-query tiers write them too when k <= kLaneMaxCompact, so a wave of the
// lane-per-query chains rarely mixes widths.
constexpr uint8_t kLgCompact = 0x80;

__host__ __device__ __forceinline__ uint32_t widen_entry16(uint32_t e16) {
  return ((e16 >> 12) << 28) | (e16 & 0xfffu);
}
constexpr int kLaneMaxCompact = 2048;  // compact lists are at most this long (the lane-per-query chains' cap)
// entry m of a list with offset `off` and lg byte `lgr`, either width, as a 32-bit run entry
__device__ __forceinline__ uint32_t list_entry(const uint32_t* list, int64_t off, int lgr, int m) {
  const int64_t i = off + ((int64_t)m << (lgr & 0x7f));
  return (lgr & kLgCompact) ? widen_entry16(reinterpret_cast<const uint16_t*>(list)[i]) : list[i];
}

struct NbLists {
  int64_t nq = 0;            // number of queries
  int64_t total = 0;         // sum of cnt
  int64_t long_total = 0;    // sum of cnt over the lists longer than kLongList
  int64_t long_nq = 0;       // number of those lists
  int64_t slots = 0;         // list entries allocated (total + interleave padding)
  const int32_t* qpos = nullptr;   // [nq] sorted position of each query
  const int64_t* off = nullptr;    // [nq]
  const int32_t* cnt = nullptr;    // [nq]
  const uint8_t* lg = nullptr;     // [nq] log2 of the entry stride
  const uint32_t* list = nullptr;  // [slots] run entries
  bool compact = false;            // lists may be 16-bit (kLgCompact)
  int64_t list_cap = 0;            // entries the list buffer holds (every offset is below it)
  const uint32_t* skeys = nullptr; // cell key of each sorted position (the grid's)
  // deferred builds (build_lists with defer): nq is an upper bound and the query count lives on
  // the device until build_lists_check has run; kernels read it through nq_of()
  const int64_t* nq_dev = nullptr;
};

__device__ __forceinline__ int64_t nq_of(const NbLists& L) { return L.nq_dev ? *L.nq_dev : L.nq; }

// lists longer than this are handled by per-query kernels downstream (normals: k_normals_long)
constexpr int kLongList = 1024;

// neighbour lists kept between the two normal-estimation phases (pfx_normals.hip) and reused
// by the detectors that search at the normal radius (pfx_harris.hip)
struct NormalsState {
  NbLists L;
  int64_t n = 0;
  const float *x = nullptr, *y = nullptr, *z = nullptr;  // the cloud and radius the lists belong to
  double r = 0.0;
  bool ready = false;
  uint64_t grid_gen = 0;  // grid_a's build that indexes (x, y, z, n, r) (pfx_normals_prepare_dev)
  // normals_launch_dev: the lists check still owed by normals_finish_dev, and the outputs to redo
  bool pending = false;
  // normals_grid_launch_dev: grid_a build `grid_ahead_gen` queued for (x, n, r); 0: none
  uint64_t grid_ahead_gen = 0;
  const float *grid_ahead_x = nullptr, *grid_ahead_y = nullptr, *grid_ahead_z = nullptr;
  int64_t grid_ahead_n = 0;
  double grid_ahead_r = 0.0;
  float vp[3] = {0.f, 0.f, 0.f};
  float *nx = nullptr, *ny = nullptr, *nz = nullptr, *curv = nullptr;
};

// mask (nullable): per *caller* index, queries are the points with (mask != 0) == want (in cell
// order).
// defer: launch the list kernels and return without the host readback (out.nq = an upper bound,
// out.nq_dev = the device count); consumers may be launched behind them in stream order, and
// build_lists_check must follow.
// gate: the normal estimation's builds only -- wait for (and clear) the event of
// pfx_normals_gate_dev right before the list kernels; other builds leave it for the next
// normal estimation (the pfx.h contract).
void build_lists(pfx_ctx* ctx, const Grid& g, const uint8_t* mask, double radius, bool sorted, NbLists& out,
                 const char* tag, bool defer = false, int want = 1, bool compact = false, bool gate = false);
// The deferred build's readback: true and `out` completed (exact nq, statistics) when the lists are
// valid; false when they must be rebuilt synchronously (list buffer too small, first very long
// lists, or a speculative grid with points outside its bounds) -- their consumers rerun too.
bool build_lists_check(pfx_ctx* ctx, const Grid& g, NbLists& out, const char* tag);

}  // namespace pfx
