// pfx_normals.hip -- NormalEstimationOMP<PointXYZRGB,Normal> (tools.h:22-32) on gfx950.
//
// Per query point q:
//   N(q)  = radius-r neighbours in FLANN order (d2, index)
//   accu  = sequential float sums {x^2, xy, xz, y^2, yz, z^2, x, y, z} in that order
//   C     = accu/|N| - mean mean^T;  (lambda, n) = pcl::eigen33(C);  curvature = |lambda/tr C|
//   flip n towards the viewpoint;  |N| < 3 -> NaN
//
// Two phases:
//   1. build_lists (pfx_nblist.hip): every finite point's FLANN-ordered neighbour list, as
//      cell-sorted positions, written to HBM (tile kernels + per-query fallback);
//   2. k_normals_chain: one lane per query (consecutive queries of a cell in one wave), the nine
//      strictly ordered float chains in registers, eigen33 + viewpoint flip, output scattered to
//      the caller's order; lists longer than kLaneMax (2048) go to k_normals_long (nine lanes per
//      query, one per chain).
#include <cstring>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include <rocprim/rocprim.hpp>

#include "pfx_nblist.h"
#include "pfx_neighbors.h"
#include "pfx_normal_math.h"

namespace pfx {
namespace {

constexpr int kBatch = 8;      // neighbour entries per half-batch (two in flight)
#ifndef PFX_LANE_MAX
#define PFX_LANE_MAX (2 * kLongList)
#endif
// lists longer than the lane cap go to k_normals_long.  Room (few long lists): 2048 (measured:
// 1024 0.90, 1536 0.78, 2048 0.75, 4096 0.84 ms for the chain stage; round 4: 1024 / 1536 slower
// again).  Dense clouds (many long lists, the non-forked schedule): 4096 -- the dense 10M variant's
// long-list chains 140 -> 91 ms against chain_big 17 -> 28 ms (14.0 -> 14.7 Mpoints/s).
constexpr int kLaneMax = PFX_LANE_MAX;
// compact (16-bit) lists reach kLaneMaxCompact entries and k_normals_long reads 32-bit lists only
static_assert(kLaneMax >= kLaneMaxCompact, "lists up to kLaneMaxCompact must take the lane-per-query chains");

#ifndef PFX_LANE_DENSE_MUL
#define PFX_LANE_DENSE_MUL 2
#endif
constexpr int kLaneMaxDense = PFX_LANE_DENSE_MUL * kLaneMax;

__device__ __forceinline__ void chain_add(float a[9], float x, float y, float z) {
  a[0] = a[0] + x * x;
  a[1] = a[1] + x * y;
  a[2] = a[2] + x * z;
  a[3] = a[3] + y * y;
  a[4] = a[4] + y * z;
  a[5] = a[5] + z * z;
  a[6] = a[6] + x;
  a[7] = a[7] + y;
  a[8] = a[8] + z;
}

__device__ __forceinline__ void store_normal(const GridView& g, int32_t p, const float a[9], int k, float vpx,
                                             float vpy, float vpz, float* nx, float* ny, float* nz, float* curv) {
  float o[4];
  const float4 q = g.sp[p];
  finish_normal(a, k, q.x, q.y, q.z, vpx, vpy, vpz, o);
  const int32_t orig = g.perm[p];
  nx[orig] = o[0];
  ny[orig] = o[1];
  nz[orig] = o[2];
  curv[orig] = o[3];
}

// ---- k_normals_chain: one lane per query, candidate coordinates staged in LDS ----------------
//
// A workgroup takes 256 consecutive queries (cell order: a few z-consecutive cells of one or a
// few grid columns).  Their lists only reference the 3x3x3 blocks of their cells, i.e. runs of
// the grid columns around the query columns.  The workgroup collects those columns (LDS hash),
// takes per column the z range its queries need, and stages the union (contiguous position
// ranges of the cell-sorted packed copy) in LDS once; a per-cell table maps a list entry's run
// to its LDS base.  The nine chains then read neighbour coordinates from LDS (x, y as one ds_read_b64 over the 64 banks, z ds_read_b32) instead
// of 64-address global gathers (the TA/L2 latency that bounded the previous version).
// Fallbacks keep every list exact: union > kStageCap -> the same table with global bases;
// > kMaxCells distinct cells -> per-lane run starts.
constexpr int kMaxCells = 64;
constexpr int kHash = 1024;
constexpr int kStageSmall = 3584;  // SoA floats: 42 KB, three workgroups per CU
constexpr int kStageBig = 12288;   // 144 KB, one workgroup per CU: the dense regions
constexpr int kMaxCols = kMaxCells * 9;
constexpr uint32_t kEmpty = 0xffffffffu;

template <int CAP>
struct ChainLds {
  static_assert(CAP * 3 >= 256 * 9, "lane-mode run tables live in the staging LDS");
  union {
    struct {  // x, y as one 8-byte word (one ds_read_b64 per neighbour over 64 banks) + z
      float2 xy[CAP];
      float z[CAP];
    } c;
    struct {
      uint32_t key[kHash];
      int32_t a[kHash];  // z low, then the run start
      int32_t b[kHash];  // z high, then the LDS base
    } h;
  } u;
  int32_t tbl[kMaxCells * 9];
  int32_t ostart[kMaxCols], olen[kMaxCols], obase[kMaxCols];
  uint32_t ckey[kMaxCells];
  int32_t wsum[4], wocc[4];
};
__device__ __forceinline__ uint32_t col_hash(uint32_t c) { return (c * 2654435761u) >> 22; }  // 10 bits

struct CellXYZ { int32_t x, y, z; };
__device__ __forceinline__ CellXYZ cell_of(const GridView& g, uint32_t key) {
  CellXYZ c;
  c.z = (int32_t)(key % (uint32_t)g.nz);
  const uint32_t xy = key / (uint32_t)g.nz;
  c.y = (int32_t)(xy % (uint32_t)g.ny);
  c.x = (int32_t)(xy / (uint32_t)g.ny);
  return c;
}

// block-wide exclusive scan of v (256 threads); returns the prefix, *total = sum
__device__ __forceinline__ int block_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int x = wsum[w];
    off += w < wv ? x : 0;
    tot += x;
  }
  __syncthreads();  // wsum may be reused by the next scan
  *total = tot;
  return off + inc - v;
}

template <int KB, class At, class Fetch, int NBUF = 2>
__device__ __forceinline__ void run_chain(At at_clamped, int k, Fetch fetch, float a[9]) {
  // Branch-free batches: entry loads use a clamped index and padded terms are exact zeros
  // (accumulators are never -0, so + 0.0f is the identity).  NBUF entry buffers rotate without
  // register copies (a copy of a pending load forces a vmcnt wait), so NBUF - 1 batches of entry
  // loads are always in flight behind the batch being summed.  (Measured and rejected in
  // round 4: 32-bit element offsets, chains 0.50 -> 0.54-0.62 ms; an all-zero coordinate slot
  // fetched by the padded steps instead of three coordinate selects, no change.  Round 5: deeper
  // rotation in the three-workgroups-per-CU kernel and a software pipeline over the LDS rounds,
  // both slower: 0.47 -> 0.50-0.75 ms.)
  const int last = k - 1;
  auto at = [&](int m) { return at_clamped(m < last ? m : last); };
  auto half = [&](uint32_t (&eq)[KB], int m0) {
    float4 c[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) c[b] = fetch(eq[b]);
#pragma unroll
    for (int b = 0; b < KB; ++b) eq[b] = at(m0 + NBUF * KB + b);
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      const bool in = m0 + b < k;
      chain_add(a, in ? c[b].x : 0.f, in ? c[b].y : 0.f, in ? c[b].z : 0.f);
    }
  };
  if constexpr (NBUF == 2) {  // (two named buffers: the round-4 form, kept as it compiles)
    uint32_t eA[KB], eB[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      eA[b] = at(b);
      eB[b] = at(KB + b);
    }
    for (int m0 = 0; m0 < k; m0 += 2 * KB) {
      half(eA, m0);
      half(eB, m0 + KB);  // unconditional (a branch here makes every wait conservative)
    }
  } else {
    uint32_t e[NBUF][KB];
#pragma unroll
    for (int q = 0; q < NBUF; ++q)
#pragma unroll
      for (int b = 0; b < KB; ++b) e[q][b] = at(q * KB + b);
    for (int m0 = 0; m0 < k; m0 += NBUF * KB) {
#pragma unroll
      for (int q = 0; q < NBUF; ++q) half(e[q], m0 + q * KB);
    }
  }
}

#ifdef PFX_SHOT_PROFILE
__device__ unsigned long long g_chain_prof[16];  // [0|8] prologue cycles, [1|9] wave chain cycles,
                                                 // [2|10] sum of wave max k, [3|11] waves, [4|12] WGs,
                                                 // [5|13] sum of the lanes' k
#endif

template <int CAP, bool DEFER>
__device__ __forceinline__ void chain_wg(ChainLds<CAP>& S, const GridView& g, const NbLists& L, int64_t j0,
                                         float vpx, float vpy, float vpz, float* __restrict__ nx,
                                         float* __restrict__ ny, float* __restrict__ nz, float* __restrict__ curv,
                                         int32_t* __restrict__ longq, int* __restrict__ n_long,
                                         int* __restrict__ modes, int64_t* __restrict__ deferq,
                                         const uint8_t* __restrict__ mask, int want, int lane_max) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t j = j0 + tid;
#ifdef PFX_SHOT_PROFILE
  constexpr int PO = CAP == kStageSmall ? 0 : 8;
  const long long pt0 = clock64();
#endif
  const bool valid = j < nq_of(L);
  int32_t p = 0;
  uint32_t key = 0, prev = kEmpty;
  int k = 0;
  bool active = false;  // this pass computes the query (masked passes: mask[caller] == want)
  bool sel = false;     // mask[caller] != 0
  if (valid) {
    p = L.qpos[j];
    key = L.skeys[p];
    k = L.cnt[j];
    if (tid > 0) prev = L.skeys[L.qpos[j - 1]];
    sel = mask && mask[g.perm[p]] != 0;
    active = !mask || want >= 2 || (sel == ((want & 1) != 0));
  }
  if (want >= 2 && mask) {  // workgroup partition: all of a workgroup with any selected query
    if ((__syncthreads_or(sel) != 0) != ((want & 1) != 0)) return;
  }
  if (!__syncthreads_or(active)) return;  // nothing of this pass in the workgroup
  // cell slots: first query of each distinct cell in the workgroup
  const bool first = valid && key != prev;
  const uint64_t fm = __ballot(first);
  if (lane == 0) S.wsum[wv] = __popcll(fm);
  __syncthreads();
  int cbase = 0, ncell = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    cbase += w < wv ? S.wsum[w] : 0;
    ncell += S.wsum[w];
  }
  const int cs = cbase + __popcll(fm & (lanemask_lt() | (1ull << lane))) - 1;
  __syncthreads();
  const bool indexed = ncell <= kMaxCells;
  bool staged = false;
  if (indexed) {
    if (first) S.ckey[cs] = key;
    for (int s = tid; s < kHash; s += 256) {
      S.u.h.key[s] = kEmpty;
      S.u.h.a[s] = 0x7fffffff;
      S.u.h.b[s] = -1;
    }
    __syncthreads();
    // touched columns and the z range each needs; each (cell, run)'s run start is loaded here
    // already (the run table below needs it: one global round less in the prologue)
    constexpr int kIt = (kMaxCells * 9 + 255) / 256;
    int32_t pre_sr[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = tid + 256 * it;
      pre_sr[it] = 0;
      if (i < ncell * 9) {
        const CellXYZ c = cell_of(g, S.ckey[i / 9]);
        const int r = i % 9, X = c.x + r / 3 - 1, Y = c.y + r % 3 - 1;
        if (X >= 0 && X < g.nx && Y >= 0 && Y < g.ny) {
          const uint32_t col = (uint32_t)X * (uint32_t)g.ny + (uint32_t)Y;
          pre_sr[it] = g.cell_start[(int64_t)col * g.nz + (c.z > 0 ? c.z - 1 : 0)];
          uint32_t h = col_hash(col);
          for (;;) {
            const uint32_t old = atomicCAS(&S.u.h.key[h], kEmpty, col);
            if (old == kEmpty || old == col) break;
            h = (h + 1) & (kHash - 1);
          }
          atomicMin(&S.u.h.a[h], c.z > 0 ? c.z - 1 : 0);
          atomicMax(&S.u.h.b[h], c.z + 1 < g.nz ? c.z + 1 : g.nz - 1);
        }
      }
    }
    __syncthreads();
    // position range of every touched column, LDS bases by a block scan
    int st4[4], len4[4], lsum = 0, osum = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int s = tid * 4 + v;
      const uint32_t col = S.u.h.key[s];
      st4[v] = len4[v] = 0;
      if (col != kEmpty) {
        const int64_t c0 = (int64_t)col * g.nz;
        st4[v] = g.cell_start[c0 + S.u.h.a[s]];
        len4[v] = g.cell_start[c0 + S.u.h.b[s] + 1] - st4[v];
      }
      lsum += len4[v];
      osum += len4[v] > 0;
    }
    int total = 0, nocc = 0;
    int lb = block_scan(lsum, S.wsum, &total);
    int ob = block_scan(osum, S.wocc, &nocc);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int s = tid * 4 + v;
      S.u.h.a[s] = st4[v];
      S.u.h.b[s] = lb;
      if (len4[v] > 0) {
        S.ostart[ob] = st4[v];
        S.olen[ob] = len4[v];
        S.obase[ob] = lb;
        ++ob;
      }
      lb += len4[v];
    }
    staged = total <= CAP;
    if (DEFER && !staged) {  // the big-LDS pass takes this workgroup (every thread agrees)
      if (tid == 0) deferq[atomicAdd(&modes[3], 1)] = j0;
      __syncthreads();
      return;
    }
    __syncthreads();
    // run table: list entry (r, off) of a query of cell cs -> tbl[cs * 9 + r] + off
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int i = tid + 256 * it;
      if (i >= ncell * 9) continue;
      const CellXYZ c = cell_of(g, S.ckey[i / 9]);
      const int r = i % 9, X = c.x + r / 3 - 1, Y = c.y + r % 3 - 1;
      int32_t t = 0;
      if (X >= 0 && X < g.nx && Y >= 0 && Y < g.ny) {
        const uint32_t col = (uint32_t)X * (uint32_t)g.ny + (uint32_t)Y;
        const int32_t s_r = pre_sr[it];
        t = s_r;
        if (staged) {
          uint32_t h = col_hash(col);
          while (S.u.h.key[h] != col) h = (h + 1) & (kHash - 1);
          t = S.u.h.b[h] + (s_r - S.u.h.a[h]);
        }
      }
      S.tbl[i] = t;
    }
    __syncthreads();  // the hash is dead from here on: its LDS holds the staged candidates
    if (staged) {
      // flattened over the whole union (runs are short in sparse regions: a loop per run would
      // serialise one global latency per run): element i -> run by binary search over the LDS
      // bases, four elements per thread in flight
      for (int i0 = 0; i0 < total; i0 += 4 * 256) {
        int32_t src[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = i0 + u * 256 + tid;
          int lo = 0, hi = nocc - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (S.obase[mid] <= i) lo = mid;
            else hi = mid - 1;
          }
          src[u] = i < total ? S.ostart[lo] + (i - S.obase[lo]) : -1;
        }
        float4 v[4];  // (the packed copy: one load per point instead of three)
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = g.sp[src[u] < 0 ? 0 : src[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = i0 + u * 256 + tid;
          if (src[u] >= 0) {
            S.u.c.xy[i] = make_float2(v[u].x, v[u].y);
            S.u.c.z[i] = v[u].z;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) atomicAdd(&modes[staged ? 0 : 1], 1);
  } else if (tid == 0) {
    atomicAdd(&modes[2], 1);
  }
  __syncthreads();  // LDS reuse: every thread has passed the shared phases
#ifdef PFX_SHOT_PROFILE
  const long long pt1 = clock64();
  if (tid == 0) {
    atomicAdd(&g_chain_prof[PO + 0], (unsigned long long)(pt1 - pt0));
    atomicAdd(&g_chain_prof[PO + 4], 1ull);
  }
  int wk = (active && k <= lane_max) ? k : 0, wsk = wk;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    wk = max(wk, __shfl_xor(wk, o));
    wsk += __shfl_xor(wsk, o);
  }
  const uint64_t wm = __ballot(active && k == wk);
  const bool rec = wm && lane == __builtin_ctzll(wm);
#endif
  if (!active) return;
  if (k > lane_max) return;  // listed by k_long_lists, chained by k_normals_long
  // the query's list: 32-bit run entries, or 16-bit ones (kLgCompact: the tile kernels' lists of
  // blocks with runs of <= 4096 points).  The two widths take two loops behind a divergent branch:
  // a wave of one width runs one of them (the same instructions per step either way), a mixed
  // wave both in turn, exec-masked (a per-lane select of the width cost 32 spilled VGPRs).
  const int lgr = L.lg[j];
  const bool c16 = (lgr & kLgCompact) != 0;
  const int lg = lgr & 0x7f;
  const int64_t loff = L.off[j];
  const uint32_t* l32 = L.list + loff;
  const uint16_t* l16 = reinterpret_cast<const uint16_t*>(L.list) + loff;
  auto at32 = [&](int m) { return l32[(int64_t)m << lg]; };
  auto at16 = [&](int m) { return (uint32_t)l16[(int64_t)m << lg]; };
  // run entry -> slot of run r's first point + offset (32-bit layout, or 16-bit: r << 12 | off)
  auto slot32 = [](const int32_t* tb, uint32_t e) { return tb[entry_run(e)] + (int32_t)entry_off(e); };
  auto slot16 = [](const int32_t* tb, uint32_t e) { return tb[e >> 12] + (int32_t)(e & 0xfffu); };
  float a[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) a[i] = 0.0f;
  // run the chains with the loop of this wave's list width
  // (round 5, measured: a per-lane width select in one loop for mixed waves of the big kernel,
  // 0.217 -> 0.226 ms; four entry batches in flight there instead of two, no change)
  auto chains = [&](auto fetch32, auto fetch16) {
    if (c16) run_chain<kBatch>(at16, k, fetch16, a);
    else run_chain<kBatch>(at32, k, fetch32, a);
  };
  if (staged) {
    const int32_t* tb = S.tbl + cs * 9;
    const float2* cxy = S.u.c.xy;
    const float* czs = S.u.c.z;
    auto lds = [&](int32_t i) {
      const float2 v = cxy[i];
      return make_float4(v.x, v.y, czs[i], 0.f);
    };
    chains([&](uint32_t e) { return lds(slot32(tb, e)); }, [&](uint32_t e) { return lds(slot16(tb, e)); });
  } else if (indexed) {
    const int32_t* tb = S.tbl + cs * 9;
    const float4* sp = g.sp;
    chains([&](uint32_t e) { return sp[slot32(tb, e)]; }, [&](uint32_t e) { return sp[slot16(tb, e)]; });
  } else if constexpr (CAP != kStageBig) {  // (a deferred workgroup is indexed: never here)
    // too many cells for the shared table: each lane keeps its own nine run starts in the
    // (unused) staging LDS
    int32_t* tb = reinterpret_cast<int32_t*>(S.u.c.xy) + tid * 9;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      int32_t st, len;
      block_run(g, key, r, st, len);
      tb[r] = st;
    }
    const float4* sp = g.sp;
    chains([&](uint32_t e) { return sp[slot32(tb, e)]; }, [&](uint32_t e) { return sp[slot16(tb, e)]; });
  }
  store_normal(g, p, a, k, vpx, vpy, vpz, nx, ny, nz, curv);
#ifdef PFX_SHOT_PROFILE
  if (rec) {
    atomicAdd(&g_chain_prof[PO + 1], (unsigned long long)(clock64() - pt1));
    atomicAdd(&g_chain_prof[PO + 2], (unsigned long long)wk);
    atomicAdd(&g_chain_prof[PO + 3], 1ull);
    atomicAdd(&g_chain_prof[PO + 5], (unsigned long long)wsk);
  }
#endif
}

__global__ void __launch_bounds__(256, 3) k_normals_chain(GridView g, NbLists L, float vpx, float vpy, float vpz,
                                                          float* __restrict__ nx, float* __restrict__ ny,
                                                          float* __restrict__ nz, float* __restrict__ curv,
                                                          int32_t* __restrict__ longq, int* __restrict__ n_long,
                                                          int* __restrict__ modes, int64_t* __restrict__ deferq,
                                                          const uint8_t* __restrict__ mask, int want,
                                                          int lane_max) {
  __shared__ ChainLds<kStageSmall> S;
  chain_wg<kStageSmall, true>(S, g, L, (int64_t)blockIdx.x * 256, vpx, vpy, vpz, nx, ny, nz, curv,
                              longq, n_long, modes, deferq, mask, want, lane_max);
}

// the deferred (dense) workgroups: one 144 KB workgroup per CU, persistent over the queue
__global__ void __launch_bounds__(256, 1) k_normals_chain_big(GridView g, NbLists L, float vpx, float vpy,
                                                              float vpz, float* __restrict__ nx,
                                                              float* __restrict__ ny, float* __restrict__ nz,
                                                              float* __restrict__ curv, int32_t* __restrict__ longq,
                                                              int* __restrict__ n_long, int* __restrict__ modes,
                                                              const int64_t* __restrict__ deferq,
                                                              const uint8_t* __restrict__ mask, int want,
                                                              int lane_max) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  ChainLds<kStageBig>& S = *reinterpret_cast<ChainLds<kStageBig>*>(dyn);
  const int count = modes[3];
  for (int w = blockIdx.x; w < count; w += gridDim.x) {
    __syncthreads();  // the previous workgroup's chains have finished reading the LDS
    chain_wg<kStageBig, false>(S, g, L, deferq[w], vpx, vpy, vpz, nx, ny, nz, curv, longq, n_long, modes, nullptr,
                               mask, want, lane_max);
  }
}

// long lists: nine lanes per query (one chain each), seven queries per wave.  The chains of a
// list are strictly sequential, so the kernel's time is the longest list's chain; a batch of
// global gathers per few steps put one memory latency on that chain every batch.  Here the wave
// gathers kLB (32) steps of its seven lists at a time into LDS (seven coordinate loads per lane,
// issued one batch ahead, with the list entries two batches ahead), and the chains read LDS
// (four steps per ds_read_b128): one latency per 32 steps instead of per 16.
// Persistent waves (grid-stride over groups of seven queries): the queue length is only known
// on the device, and a grid sized for the worst case spends its time dispatching empty waves.
#ifndef PFX_LONG_LB
#define PFX_LONG_LB 64
#endif
// steps per batch (round 6: 64, two 32-step halves per lane -- a batch's gathers are one latency
// on the wave's chain, so twice the steps per batch halves that exposure; 32 before)
constexpr int kPerWave = 7, kLB = PFX_LONG_LB, kLR = kLB / 32;
static_assert(kLB % 32 == 0, "whole 32-step halves");
// workgroups of k_normals_long resident per CU (its launch is sized to them: a persistent grid,
// workgroups beyond them would run as a second round): 124 VGPRs at 32 steps, 154 at 64
constexpr int kLongWgPerCu = kLB <= 32 ? 4 : 3;
#ifndef PFX_BIG_GRID  // workgroups of k_normals_chain_big (static stride over the deferred groups, one per CU resident)
#define PFX_BIG_GRID 256
#endif
#ifndef PFX_LONG_ORDERED  // (A/B: 0 = the pushed long-list queue in the dense schedule too)
#define PFX_LONG_ORDERED 1
#endif
#ifndef PFX_LONG_GRID_MUL  // (A/B: workgroups launched per resident one)
#define PFX_LONG_GRID_MUL 1
#endif
// rows padded by one float4 (a 144-B stride): the 21 rows a chain step reads (7 queries x 3
// planes, one ds_read_b128 per lane at the same step) spread over the LDS banks instead of
// piling onto two bank groups (a 128-B stride: 9.4 conflict cycles per LDS instruction, r03 PMC)
constexpr int kLBPad = kLB + 4;
struct LongLds {
  float c[2][3][kPerWave][kLBPad];  // double-buffered x | y | z per query and step (11 KB)
  int32_t rtab[kPerWave * 9];
};

// NaN (PCL's value for points without a normal: std::numeric_limits<float>::quiet_NaN(),
// 0x7FC00000, the bits finish_normal writes too) in the four output arrays, one launch
__global__ void k_nan_fill4(float* __restrict__ a, float* __restrict__ b, float* __restrict__ c,
                            float* __restrict__ d, int64_t n) {
  const float v = __builtin_nanf("");
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a[i] = v; b[i] = v; c[i] = v; d[i] = v;
  }
}

// NaN (PCL's value for points without a normal) in the four outputs of the points with
// (mask != 0) == want
__global__ void k_nan_fill4_masked(float* __restrict__ a, float* __restrict__ b, float* __restrict__ c,
                                   float* __restrict__ d, int64_t n, const uint8_t* __restrict__ mask, int want) {
  const float v = __builtin_nanf("");
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if ((mask[i] != 0) != (want != 0)) continue;
    a[i] = v; b[i] = v; c[i] = v; d[i] = v;
  }
}

// the lists longer than kLaneMax of this pass (mask[caller] == want), for k_normals_long: pushed
// to longq, or (flags non-null) flagged for an order-preserving compaction
__global__ void __launch_bounds__(256) k_long_lists(GridView g, NbLists L, const uint8_t* __restrict__ mask, int want,
                                                    int lane_max,
                                                    int32_t* __restrict__ longq, int* __restrict__ n_long,
                                                    uint8_t* __restrict__ flags) {
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  bool push = false;
  if (want >= 2 && mask) {  // workgroup partition (blocks of 256 queries, as k_normals_chain's)
    const bool sel = j < nq_of(L) && mask[g.perm[L.qpos[j]]] != 0;
    const bool mine = (__syncthreads_or(sel) != 0) == ((want & 1) != 0);
    push = mine && j < nq_of(L) && L.cnt[j] > lane_max;
  } else if (j < nq_of(L) && L.cnt[j] > lane_max) {
    push = !mask || ((mask[g.perm[L.qpos[j]]] != 0) == (want != 0));
  }
  if (flags) {
    flags[j] = push ? 1 : 0;  // (every slot of the grid: a deferred build's count is an upper bound on the host)
  } else if (push) {
    longq[wave_push_slot(n_long)] = (int32_t)j;
  }
}

__global__ void __launch_bounds__(256) k_normals_long(GridView g, NbLists L, const int32_t* __restrict__ longq,
                                                      const int* __restrict__ n_long, float vpx, float vpy,
                                                      float vpz, float* __restrict__ nx, float* __restrict__ ny,
                                                      float* __restrict__ nz, float* __restrict__ curv) {
  __shared__ LongLds S4[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  LongLds& S = S4[wv];
  const int qi = lane / 9, a = lane - 9 * qi;
  const int count = *n_long;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  auto wsync = [] {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  for (int64_t w = (int64_t)blockIdx.x * 4 + wv; w * kPerWave < count; w += nwaves) {
    const int64_t slot = w * kPerWave + qi;
    const bool active = qi < kPerWave && slot < count;
    int k = 0;
    int32_t j = 0;
    if (active) {
      j = longq[slot];
      k = L.cnt[j];
      int32_t s, len;
      block_run(g, L.skeys[L.qpos[j]], a, s, len);
      S.rtab[9 * qi + a] = s;
    }
    // the group's seven lists (wave-uniform: SGPRs); a batch gathers step (lane & 31) of query
    // 2 * i + (lane >> 5) in slot i, i < 4 (every lane serves up to four queries)
    int kq[kPerWave], lgq[kPerWave];
    int64_t offq[kPerWave];
    int kmax = 0;
#pragma unroll
    for (int i = 0; i < kPerWave; ++i) {
      const int64_t si = w * kPerWave + i;
      const int32_t ji = si < count ? longq[si] : 0;
      kq[i] = __builtin_amdgcn_readfirstlane(si < count ? L.cnt[ji] : 0);
      lgq[i] = __builtin_amdgcn_readfirstlane(si < count ? (int)L.lg[ji] : 0);
      const int64_t o = si < count ? L.off[ji] : 0;
      offq[i] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(o >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)o));
      kmax = max(kmax, kq[i]);
    }
    wsync();  // rtab
    // entry of step m of query qq (clamped: padded steps repeat the last entry, summed as zeros)
    const int half = lane >> 5, st = lane & 31;
    auto pick = [&](const int (&v)[kPerWave], int qq) {
      int r = v[0];
#pragma unroll
      for (int i = 1; i < kPerWave; ++i) r = qq == i ? v[i] : r;
      return r;
    };
    auto entry = [&](int slot, int m) -> uint32_t {
      const int qq = 2 * slot + half;
      const int kk = qq < kPerWave ? pick(kq, qq) : 0;
      int64_t of = offq[0];
#pragma unroll
      for (int i = 1; i < kPerWave; ++i) of = qq == i ? offq[i] : of;
      const int mm = kk > 0 ? min(m, kk - 1) : 0;
      return kk > 0 ? L.list[of + ((int64_t)mm << pick(lgq, qq))] : 0u;
    };
    auto coord = [&](int slot, uint32_t e) -> float4 {
      const int qq = 2 * slot + half;
      const bool ok = qq < kPerWave && pick(kq, qq) > 0;
      return ok ? g.sp[S.rtab[9 * qq + entry_run(e)] + (int32_t)entry_off(e)] : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    constexpr int NS = (kPerWave + 1) / 2;  // slots per lane
    uint32_t e1[NS * kLR], e2[NS * kLR];
    float4 cv[NS * kLR];
    // staged steps past a list's end are exact zeros (acc is never -0: + 0.0f is the identity),
    // so every lane runs whole batches without bounds checks
    auto put = [&](int buf, int m0) {
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int qq = 2 * i + half;
        if (qq < kPerWave) {
#pragma unroll
          for (int h = 0; h < kLR; ++h) {
            const int step = st + 32 * h;
            const bool in = m0 + step < pick(kq, qq);
            S.c[buf][0][qq][step] = in ? cv[i * kLR + h].x : 0.f;
            S.c[buf][1][qq][step] = in ? cv[i * kLR + h].y : 0.f;
            S.c[buf][2][qq][step] = in ? cv[i * kLR + h].z : 0.f;
          }
        }
      }
    };
#pragma unroll
    for (int i = 0; i < NS * kLR; ++i) e1[i] = entry(i / kLR, st + 32 * (i % kLR));
#pragma unroll
    for (int i = 0; i < NS * kLR; ++i) cv[i] = coord(i / kLR, e1[i]);
#pragma unroll
    for (int i = 0; i < NS * kLR; ++i) e1[i] = entry(i / kLR, kLB + st + 32 * (i % kLR));
    put(0, 0);
    wsync();
    // chain term a = u * v over the coordinate planes: x*x x*y x*z y*y y*z z*z x y z
    const int pu = (a == 0 || a == 1 || a == 2 || a == 6) ? 0 : ((a == 3 || a == 4 || a == 7) ? 1 : 2);
    const int pv = (a == 0) ? 0 : ((a == 1 || a == 3) ? 1 : 2);
    const bool linear = a >= 6;
    const int q7 = qi < kPerWave ? qi : 0;
    float acc = 0.0f;
    for (int m0 = 0, buf = 0; m0 < kmax; m0 += kLB, buf ^= 1) {
      const bool more = m0 + kLB < kmax;
      if (more) {
#pragma unroll
        for (int i = 0; i < NS * kLR; ++i) cv[i] = coord(i / kLR, e1[i]);  // batch m0 + kLB
#pragma unroll
        for (int i = 0; i < NS * kLR; ++i) e2[i] = entry(i / kLR, m0 + 2 * kLB + st + 32 * (i % kLR));
      }
      const float4* bu = reinterpret_cast<const float4*>(&S.c[buf][pu][q7][0]);
      const float4* bv = reinterpret_cast<const float4*>(&S.c[buf][pv][q7][0]);
#pragma unroll 1
      for (int t4 = 0; t4 < kLB / 4; t4 += 4) {
        float4 u4[4], v4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          u4[i] = bu[t4 + i];
          v4[i] = bv[t4 + i];
        }
        const float* fu = reinterpret_cast<const float*>(u4);
        const float* fv = reinterpret_cast<const float*>(v4);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc = acc + (linear ? fu[i] : fu[i] * fv[i]);
      }
      if (more) {
        put(buf ^ 1, m0 + kLB);
#pragma unroll
        for (int i = 0; i < NS * kLR; ++i) e1[i] = e2[i];
      }
      wsync();
    }
    float accu[9];
    const int base = 9 * (lane < 63 ? qi : 0);
#pragma unroll
    for (int i = 0; i < 9; ++i) accu[i] = __shfl(acc, base + i);
    if (active && a == 0) store_normal(g, L.qpos[j], accu, k, vpx, vpy, vpz, nx, ny, nz, curv);
    wsync();  // LDS is rewritten by the next group
  }
}

}  // namespace


// pfx_normals_gate_dev: the caller's event is waited for inside build_lists, right before the
// list kernels (after the list set-up)

// The gate is borrowed for one normal-estimation call: whichever way the call ends (no points,
// no list build, an error before the wait), the event is dropped with it, so no later call waits
// on an event the caller may have destroyed.
struct GateScope {
  pfx_ctx* ctx;
  explicit GateScope(pfx_ctx* c) : ctx(c) {}
  ~GateScope() { ctx->lists_gate = nullptr; }
};

void normals_release(pfx_ctx* ctx) {
  delete ctx->normals;
  ctx->normals = nullptr;
}

// Phase 1: grid + FLANN-ordered neighbour lists of every finite point (kept in ctx), outputs
// NaN-filled (non-finite points are not queries: PCL writes NaN).
void normals_lists_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                       float* nx, float* ny, float* nz, float* curv) {
  GateScope gate_scope(ctx);
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (!ctx->normals) ctx->normals = new NormalsState();
  NormalsState& ns = *ctx->normals;
  ns.ready = false;
  ns.pending = false;
  ns.n = n;
  ns.x = x;
  ns.y = y;
  ns.z = z;
  ns.r = r;
  ns.L = NbLists();
  if (n == 0) {
    ns.ready = true;
    return;
  }
  hipStream_t st = ctx->stream;
  TimeScope total(ctx, "normals_lists_phase", true);
  build_grid(ctx, ctx->grid_a, x, y, z, n, r);
  k_nan_fill4<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, st>>>(nx, ny, nz, curv, n);
  check_launch("k_nan_fill4");
  build_lists(ctx, ctx->grid_a, nullptr, r, true, ns.L, "normals", false, 1, false, /*gate=*/true);
  ctx->stats["normals_neighbors"] = ns.L.total;
  ctx->stats["normals_long_neighbors"] = ns.L.long_total;
  ctx->stats["normals_long_queries"] = ns.L.long_nq;
  ctx->stats["normals_queries"] = ns.L.nq;
  ns.ready = true;
}

// Phase 2 on ctx's stream: the ordered covariance chains of the queries whose caller index has
// (mask[i] != 0) == want (every query when mask is null), from the lists held by `owner`
// (which may be another context on the same device: the workspace used here is ctx's own, so
// two passes with complementary masks can run concurrently on two streams).
void normals_chains_dev(pfx_ctx* ctx, pfx_ctx* owner, const uint8_t* mask, int want, const float vp[3], float* nx,
                        float* ny, float* nz, float* curv) {
  PFX_CHECK(owner->normals && owner->normals->ready, "normals: lists not built (call the lists phase first)");
  const NbLists& L = owner->normals->L;
  if (L.nq == 0) return;
  hipStream_t st = ctx->stream;
  const Grid& G = owner->grid_a;
  int32_t* longq = ctx->buf("normals_longq").as<int32_t>(L.nq);
  // [0] long lists, [1..3] chain modes (staged, table, lane), [4] deferred workgroups
  int* n_long = ctx->buf("normals_nlong").as<int>(5);
  PFX_HIP(hipMemsetAsync(n_long, 0, 5 * sizeof(int), st));
  const int64_t nb = ceil_div(L.nq, 256);
  // the long lists first: when they are few (their chains, bound by the longest list, leave the
  // device mostly idle) k_normals_long runs on a side stream concurrently with the short-list
  // chains, which leave them out; when most lists are long (dense clouds) the two kernels would
  // only crowd each other, so it runs after them on the same stream
  // (a deferred build has no count yet: the previous estimation's decision on this context)
  const bool fork = L.nq_dev ? ctx->normals_fork_hint : L.long_nq * 8 <= L.nq;
  if (!L.nq_dev) ctx->normals_fork_hint = fork;
  const int lane_max = fork ? kLaneMax : kLaneMaxDense;
  if (fork || !PFX_LONG_ORDERED) {
    k_long_lists<<<(unsigned)nb, 256, 0, st>>>(view(G), L, mask, want, lane_max, longq, n_long, nullptr);
    check_launch("k_long_lists");
  } else {
    // many long lists (dense clouds): the queue keeps the cell order, so the groups k_normals_long
    // runs at once gather from one compact region (the pushed queue's order is the order the
    // resident workgroups of k_long_lists happened to reach their atomics: its L2 hit rate was
    // 0.745 on the dense variant)
    uint8_t* flags = ctx->buf("normals_longflag").as<uint8_t>(nb * 256);
    k_long_lists<<<(unsigned)nb, 256, 0, st>>>(view(G), L, mask, want, lane_max, longq, n_long, flags);
    check_launch("k_long_lists");
    size_t tb = 0;
    PFX_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<int32_t>(0), flags, longq, n_long,
                            (size_t)L.nq, st));
    void* tmp = ctx->buf("normals_longsel").get(tb + 16);
    PFX_HIP(rocprim::select(tmp, tb, rocprim::counting_iterator<int32_t>(0), flags, longq, n_long, (size_t)L.nq,
                            st));
  }
  // (sized to what is resident at once: waves beyond it would wait for a second round)
  const int64_t lb = std::min<int64_t>(ceil_div(L.nq, 7 * 4), 256 * kLongWgPerCu * PFX_LONG_GRID_MUL);
  if (fork) {
    ctx->ensure_side();
    PFX_HIP(hipEventRecord(ctx->fork_ev[0], st));
    PFX_HIP(hipStreamWaitEvent(ctx->side, ctx->fork_ev[0], 0));
    // persistent: the queue length stays on the device (no host round trip)
    k_normals_long<<<(unsigned)lb, 256, 0, ctx->side>>>(view(G), L, longq, n_long, vp[0], vp[1], vp[2], nx, ny, nz,
                                                        curv);
    check_launch("k_normals_long");
  }
  {
    // natural block order = round-robin over the 8 XCDs: the dense (heavy) workgroups cluster in
    // space, so contiguous per-XCD slices would leave one XCD with ~1.4x the mean work
    int64_t* deferq = ctx->buf("normals_deferq").as<int64_t>(nb);
    {
      TimeScope ts(ctx, "normals_chain");
      k_normals_chain<<<(unsigned)nb, 256, 0, st>>>(view(G), L, vp[0], vp[1], vp[2], nx, ny, nz, curv, longq, n_long,
                                                    n_long + 1, deferq, mask, want, lane_max);
      check_launch("k_normals_chain");
    }
    static std::once_flag attr;  // contexts may run on several host threads
    hipError_t attr_err = hipSuccess;
    std::call_once(attr, [&] {
      attr_err = hipFuncSetAttribute((const void*)k_normals_chain_big, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)sizeof(ChainLds<kStageBig>));
    });
    PFX_HIP(attr_err);
    TimeScope tb(ctx, "normals_chain_big");
    k_normals_chain_big<<<PFX_BIG_GRID, 256, sizeof(ChainLds<kStageBig>), st>>>(view(G), L, vp[0], vp[1], vp[2], nx, ny, nz,
                                                                         curv, longq, n_long, n_long + 1, deferq,
                                                                         mask, want, lane_max);
    check_launch("k_normals_chain_big");
  }
  {
    TimeScope ts(ctx, "normals_long");  // (forked: the join, what the long chains add after the short ones)
    if (fork) {
      PFX_HIP(hipEventRecord(ctx->fork_ev[1], ctx->side));
      PFX_HIP(hipStreamWaitEvent(st, ctx->fork_ev[1], 0));
    } else {
      k_normals_long<<<(unsigned)lb, 256, 0, st>>>(view(G), L, longq, n_long, vp[0], vp[1], vp[2], nx, ny, nz, curv);
      check_launch("k_normals_long");
    }
  }
  if (ctx->timer.enabled && !ctx->timer.stages_only) {  // per-kernel timing (diagnostics, host sync): the chain modes
    int h[5];
    PFX_HIP(hipMemcpyAsync(h, n_long, sizeof(h), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    ctx->stats["normals_long_lists"] = h[0];
    ctx->stats["normals_chain_wg_staged"] = h[1];
    ctx->stats["normals_chain_wg_table"] = h[2];
    ctx->stats["normals_chain_wg_lane"] = h[3];
    ctx->stats["normals_chain_wg_deferred"] = h[4];
  }
#ifdef PFX_SHOT_PROFILE
  {
    unsigned long long pr[16];
    PFX_HIP(hipStreamSynchronize(st));
    PFX_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_chain_prof), sizeof(pr)));
    for (int b = 0; b < 16; b += 8)
      fprintf(stderr, "chain%s: WGs %llu prologue %.0f cyc/WG | waves %llu chain %.0f cyc/wave, max k %.1f/wave, "
              "%.1f cyc/step, mean k %.1f/lane\n", b ? "_big" : "", pr[b + 4], pr[b + 0] / (double)(pr[b + 4] + !pr[b + 4]), pr[b + 3],
              pr[b + 1] / (double)(pr[b + 3] + !pr[b + 3]), pr[b + 2] / (double)(pr[b + 3] + !pr[b + 3]),
              pr[b + 1] / (double)(pr[b + 2] + !pr[b + 2]), pr[b + 5] / 64.0 / (double)(pr[b + 3] + !pr[b + 3]));
    const unsigned long long z[16] = {};
    PFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_prof), z, sizeof(z)));
  }
#endif
}

namespace {

// grid on the hint, NaN fill, list kernels launched without their readback (the lists check
// follows in the caller); false when the speculative form does not apply
bool normals_speculative_lists(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                               float* nx, float* ny, float* nz, float* curv) {
  if (n == 0) return false;
  if (!ctx->normals) ctx->normals = new NormalsState();
  NormalsState& ns = *ctx->normals;
  ns.ready = false;
  ns.pending = false;
  ns.n = n;
  ns.x = x;
  ns.y = y;
  ns.z = z;
  ns.r = r;
  ns.L = NbLists();
  TimeScope phase(ctx, "normals_lists_phase", true);
  // (the grid queued ahead by normals_grid_launch_dev for this cloud and radius, else built here)
  const bool ahead = ns.grid_ahead_gen != 0 && ns.grid_ahead_gen == ctx->grid_a.gen && ns.grid_ahead_x == x &&
                     ns.grid_ahead_y == y && ns.grid_ahead_z == z && ns.grid_ahead_n == n && ns.grid_ahead_r == r;
  ns.grid_ahead_gen = 0;
  if (!ahead) build_grid(ctx, ctx->grid_a, x, y, z, n, r, /*use_hint=*/true);
  k_nan_fill4<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, ctx->stream>>>(nx, ny, nz, curv, n);
  check_launch("k_nan_fill4");
  build_lists(ctx, ctx->grid_a, nullptr, r, true, ns.L, "normals", /*defer=*/true, /*want=*/1, /*compact=*/true,
              /*gate=*/true);
  return true;
}

// the lists check's verdict: statistics, or one exact rerun of lists and chains
bool normals_conclude(pfx_ctx* ctx, bool ok, const float* x, const float* y, const float* z, int64_t n, double r,
                      const float vp[3], float* nx, float* ny, float* nz, float* curv) {
  NormalsState& ns = *ctx->normals;
  ctx->grid_a.oob = nullptr;
  ctx->stats["normals_speculative_reruns"] += ok ? 0 : 1;
  if (ok) {
    ctx->stats["normals_neighbors"] = ns.L.total;
    ctx->stats["normals_long_neighbors"] = ns.L.long_total;
    ctx->stats["normals_long_queries"] = ns.L.long_nq;
    ctx->stats["normals_queries"] = ns.L.nq;
    ctx->normals_fork_hint = ns.L.long_nq * 8 <= ns.L.nq;
    return true;
  }
  normals_lists_dev(ctx, x, y, z, n, r, nx, ny, nz, curv);
  normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
  return false;
}
}  // namespace

// The estimation with one host round trip: the grid on the previous call's widened bounds (no
// bounds readback), then one readback validating the grid and the lists together before the
// chains (a grid whose bounds missed a point, a list buffer that overflowed or the first very long
// lists: the exact two-phase path reruns).  The chains are launched after the check so the host
// returns while they run and the caller's next stage (FPFH) is queued behind them; launching them
// before the check left the host waiting on the chains instead (round 3: 170.6 vs 171.9
// Mpoints/s; the exact bounds readback path: 171.9).  normals_launch_dev + normals_finish_dev
// take the check off the caller's path altogether.
void normals_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                 const float vp[3], float* nx, float* ny, float* nz, float* curv) {
  GateScope gate_scope(ctx);
  TimeScope total(ctx, "normals", true);
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (normals_speculative_lists(ctx, x, y, z, n, r, nx, ny, nz, curv)) {
    NormalsState& ns = *ctx->normals;
    const bool ok = build_lists_check(ctx, ctx->grid_a, ns.L, "normals");
    ns.ready = true;
    if (ok) normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
    normals_conclude(ctx, ok, x, y, z, n, r, vp, nx, ny, nz, curv);
    return;
  }
  normals_lists_dev(ctx, x, y, z, n, r, nx, ny, nz, curv);
  if (n > 0) normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
}

// Launch half of a split estimation: grid, lists and chains are all queued with no host round
// trip (the chains see a zero query count unless the lists are whole, k_defer_gate), so a
// consumer can be queued behind them at once.  normals_finish_dev must follow before the outputs
// are trusted: it validates and, rarely, reruns the exact path (the consumer then reruns too).
void normals_launch_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                        const float vp[3], float* nx, float* ny, float* nz, float* curv) {
  GateScope gate_scope(ctx);
  TimeScope total(ctx, "normals", true);
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (normals_speculative_lists(ctx, x, y, z, n, r, nx, ny, nz, curv)) {
    NormalsState& ns = *ctx->normals;
    ns.ready = true;
    normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
    ns.pending = true;
    ns.vp[0] = vp[0]; ns.vp[1] = vp[1]; ns.vp[2] = vp[2];
    ns.nx = nx; ns.ny = ny; ns.nz = nz; ns.curv = curv;
    return;
  }
  normals_lists_dev(ctx, x, y, z, n, r, nx, ny, nz, curv);
  if (n > 0) normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
}

// true when the launched estimation stood; false when it was rerun (exactly, stream-ordered on
// ctx's stream: whatever consumed the outputs in between must run again)
bool normals_finish_dev(pfx_ctx* ctx) {
  NormalsState* ns = ctx->normals;
  if (!ns || !ns->pending) return true;
  ns->pending = false;
  const bool ok = build_lists_check(ctx, ctx->grid_a, ns->L, "normals");
  return normals_conclude(ctx, ok, ns->x, ns->y, ns->z, ns->n, ns->r, ns->vp, ns->nx, ns->ny, ns->nz, ns->curv);
}

// The speculative grid of the next normals_dev / normals_launch_dev of this cloud and radius,
// queued now (no host wait once a previous build left its bounds hint): the caller can issue it
// ahead of another stream's work and the estimation's list kernels after that work.
void normals_grid_launch_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r) {
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (!ctx->normals) ctx->normals = new NormalsState();
  NormalsState& ns = *ctx->normals;
  ns.grid_ahead_gen = 0;
  if (n == 0) return;
  build_grid(ctx, ctx->grid_a, x, y, z, n, r, /*use_hint=*/true);
  ns.grid_ahead_gen = ctx->grid_a.gen;
  ns.grid_ahead_x = x;
  ns.grid_ahead_y = y;
  ns.grid_ahead_z = z;
  ns.grid_ahead_n = n;
  ns.grid_ahead_r = r;
}

// The grid of a subset estimation built ahead (it needs only the coordinates): the normal-estimation
// stream builds it while the subset mask is still being computed elsewhere.
void normals_prepare_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r) {
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (!ctx->normals) ctx->normals = new NormalsState();
  NormalsState& ns = *ctx->normals;
  ns.ready = false;
  ns.L = NbLists();
  ns.n = n;
  ns.x = x;
  ns.y = y;
  ns.z = z;
  ns.r = r;
  if (n == 0) return;
  TimeScope ts(ctx, "normals_prepare", true);
  build_grid(ctx, ctx->grid_a, x, y, z, n, r);
  ns.grid_gen = ctx->grid_a.gen;
}

// Normal estimation of the points with (mask[i] != 0) == want only (PCL's values, bit for bit;
// the other outputs are left untouched): lists of those points on the full cloud's grid, then
// their chains.  Two calls with want = 1 and 0 give pfx_normals_dev's result, the first one's
// points complete when its stream reaches the end of the call (FPFH's support first, so FPFH can
// start while the rest is estimated).
void normals_subset_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                        const uint8_t* mask, int want, const float vp[3], float* nx, float* ny, float* nz,
                        float* curv) {
  GateScope gate_scope(ctx);
  TimeScope total(ctx, "normals", true);
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  PFX_CHECK(mask != nullptr, "normals subset: null mask");
  if (n == 0) return;
  if (!ctx->normals) ctx->normals = new NormalsState();
  NormalsState& ns = *ctx->normals;
  const bool grid_ok = ns.grid_gen == ctx->grid_a.gen && ns.grid_gen != 0 && ns.x == x && ns.y == y && ns.z == z &&
                       ns.n == n && ns.r == r;
  if (!grid_ok) normals_prepare_dev(ctx, x, y, z, n, r);
  ns.ready = false;
  hipStream_t st = ctx->stream;
  {
    TimeScope phase(ctx, "normals_lists_phase", true);
    k_nan_fill4_masked<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, st>>>(nx, ny, nz, curv, n, mask,
                                                                                           want);
    check_launch("k_nan_fill4_masked");
    build_lists(ctx, ctx->grid_a, mask, r, true, ns.L, "normals", /*defer=*/false, want, /*compact=*/false,
                /*gate=*/true);
  }
  ns.ready = true;
  if (ns.L.nq > 0) normals_chains_dev(ctx, ctx, nullptr, 0, vp, nx, ny, nz, curv);
  ns.ready = false;  // (the lists hold a subset: not the cloud's, nothing may reuse them)
  ctx->stats["normals_queries"] = ns.L.nq;
  ctx->stats["normals_neighbors"] = ns.L.total;
  ctx->stats["normals_long_neighbors"] = ns.L.long_total;
  ctx->stats["normals_long_queries"] = ns.L.long_nq;
}

}  // namespace pfx
