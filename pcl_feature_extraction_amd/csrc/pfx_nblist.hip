// pfx_nblist.hip -- radius-neighbour lists of grid points in FLANN order (see pfx_nblist.h).
//
// Tiles: up to 16 consecutive queries of one grid cell share the 3x3x3 candidate block (9
// contiguous runs of the cell-sorted SoA copy), staged once in LDS.  Each wave owns 4 of the
// tile's queries: it streams the candidates from LDS and keeps hits as u16 candidate indices
// (wave-uniform cursors, no atomics), then orders each list with a wave-local LDS bucket sort on
// d2 (exact (d2, caller index) rank inside a bucket).  The tile's lists are written to HBM
// interleaved (stride 2^lg >= tile size) with one global atomic per tile.
//   sparse tiles: <= 1280 candidates, <= 512 neighbours per query in LDS  (3 workgroups / CU)
//   dense tiles:  <= 8000 candidates read from L2, <= 1024 neighbours per query (2 WG / CU)
// Queries of larger blocks and overflowing lists go to k_nb_query (one 256-thread workgroup per
// query, candidates streamed from L2/HBM, <= 4096 neighbours sorted in LDS); beyond that the
// same kernel runs with its sort arrays in global scratch (<= 262144 neighbours).
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_nblist.h"
#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kQ = 16;  // tile: consecutive queries of one cell
typedef float pf2 __attribute__((ext_vector_type(2)));  // packed f32 pair (v_pk_add_f32 / v_pk_mul_f32)
constexpr int kArena = 16384;   // list entries per arena reservation of a tile workgroup (> a typical tile)
constexpr int kArenaQuery = 16384;  // ... of a per-query workgroup (lists of 1k-4k entries)
constexpr int kTcapSmall = 384, kTcapSparse = 1280, kTcapDense = 8000;
constexpr int kCapQuery = 4096, kBucketsQuery = 1024;
constexpr int kCapMid8 = 8192, kBucketsMid8 = 1024;  // 72 KB of LDS: two workgroups per CU
constexpr int kCapMid = 16384, kBucketsMid = 2048;  // 144 KB of LDS: one workgroup per CU
#ifndef PFX_HUGE_BLOCKS
#define PFX_HUGE_BLOCKS 1024
#endif
// the huge tier: up to kHugeBlocks workgroups with 4 MB of scratch each, allocated on demand for
// as many workgroups as lists (>= 256); 1024 (was 256): dense 10M per-query tiers 449 -> 409 ms
constexpr int kCapHuge = 1 << 18, kBucketsHuge = 4096, kHugeBlocks = PFX_HUGE_BLOCKS;
// threads per workgroup of the per-query tiers (see k_nb_query)
#ifndef PFX_NT_QUERY
#define PFX_NT_QUERY 512
#endif
#ifndef PFX_NT_MID
#define PFX_NT_MID 1024
#endif
#ifndef PFX_NT_MID8
#define PFX_NT_MID8 1024
#endif
#ifndef PFX_Q_PF  // the per-query tiers' record prefetch (A/B)
#define PFX_Q_PF 1
#endif
#ifndef PFX_Q_WPE  // waves per SIMD the 4k tier's registers are held to
#define PFX_Q_WPE 6
#endif
constexpr int kNtQuery = PFX_NT_QUERY, kNtMid8 = PFX_NT_MID8, kNtMid = PFX_NT_MID, kNtHuge = 256;
constexpr int kNCounters = 20;

// The lists of a wide tile are written unsorted to HBM by a test pass and ordered in place by the
// per-query tiers: work items j | kListMode (the tier by k: <= 4096, <= 8192, <= 16384, beyond);
// queue 0 also takes the test-mode items of the lists that overflow a tile kernel.
constexpr int32_t kListMode = 1 << 30;
struct TierQ {
  int32_t* q[4];
  int* n[4];
};
// the per-query tier of a list of k entries (<= 4096, <= 8192, <= 16384, beyond)
__device__ __forceinline__ int query_tier(int k) {
  return k <= kCapQuery ? 0 : (k <= kCapMid8 ? 1 : (k <= kCapMid ? 2 : 3));
}

// Tile record (written by k_tile_class, one per tile, in class order): the 9 candidate runs of
// the tile's 3x3x3 block, its first query (index into qpos) and query count.  A workgroup loads
// the record of its next tile one lane per word while it works on the current one and unpacks it
// with readlane into SGPRs, so a tile starts with no dependent global loads (the old chain
// tiles -> qpos -> skeys -> cell_start was four serial latencies per tile).
constexpr int kRecInts = 24;
constexpr int kRecQ0 = 19, kRecQn = 20;

__device__ __forceinline__ void rec_write(int32_t* __restrict__ rec, const Runs& R, int32_t q0, int qn) {
#pragma unroll
  for (int r = 0; r < 9; ++r) rec[r] = R.start[r];
#pragma unroll
  for (int r = 0; r < 10; ++r) rec[9 + r] = R.pref[r];
  rec[kRecQ0] = q0;
  rec[kRecQn] = qn;
}

// lane l < kRecInts of the calling wave loads word l of record i (0 when !ok)
__device__ __forceinline__ int rec_load(const int32_t* __restrict__ rec_base, int rec_step, int i, bool ok) {
  const int lane = threadIdx.x & 63;
  return (ok && lane < kRecInts) ? rec_base[(int64_t)i * rec_step + lane] : 0;
}

__device__ __forceinline__ void rec_unpack(int v, Runs& R, int32_t& q0, int& qn) {
#pragma unroll
  for (int r = 0; r < 9; ++r) R.start[r] = __builtin_amdgcn_readlane(v, r);
#pragma unroll
  for (int r = 0; r < 10; ++r) R.pref[r] = __builtin_amdgcn_readlane(v, 9 + r);
  q0 = __builtin_amdgcn_readlane(v, kRecQ0);
  qn = __builtin_amdgcn_readlane(v, kRecQn);
}

// Query record (one per query the per-query tiers take, indexed by its query index j, written by
// the tile / wide-tile kernel that queues it): the 9 run starts and 10 prefixes of its block, its
// cell-sorted position and coordinates.  A per-query workgroup then starts with one record load
// (one lane per word, unpacked with readlane) instead of the chain qpos -> skeys -> cell_start
// (three dependent global rounds) plus the coordinate load.
constexpr int kQRecQp = 19, kQRecX = 20;
__device__ __forceinline__ void qrec_write(int32_t* __restrict__ qrec, int64_t j, const Runs& R, int32_t qp, float x,
                                           float y, float z) {
  int4* o = reinterpret_cast<int4*>(qrec + j * kRecInts);
  o[0] = make_int4(R.start[0], R.start[1], R.start[2], R.start[3]);
  o[1] = make_int4(R.start[4], R.start[5], R.start[6], R.start[7]);
  o[2] = make_int4(R.start[8], R.pref[0], R.pref[1], R.pref[2]);
  o[3] = make_int4(R.pref[3], R.pref[4], R.pref[5], R.pref[6]);
  o[4] = make_int4(R.pref[7], R.pref[8], R.pref[9], qp);
  o[5] = make_int4(__float_as_int(x), __float_as_int(y), __float_as_int(z), 0);
}
__device__ __forceinline__ void qrec_unpack(int v, Runs& R, int32_t& qp, float4& q) {
#pragma unroll
  for (int r = 0; r < 9; ++r) R.start[r] = __builtin_amdgcn_readlane(v, r);
#pragma unroll
  for (int r = 0; r < 10; ++r) R.pref[r] = __builtin_amdgcn_readlane(v, 9 + r);
  qp = __builtin_amdgcn_readlane(v, kQRecQp);
  q = make_float4(__int_as_float(__builtin_amdgcn_readlane(v, kQRecX)),
                  __int_as_float(__builtin_amdgcn_readlane(v, kQRecX + 1)),
                  __int_as_float(__builtin_amdgcn_readlane(v, kQRecX + 2)), 0.0f);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// one launch for the list build's set-up: counters and cursors zeroed, and (unmasked builds)
// qpos = 0..n-1 with the query count = the finite points (cell_start[ncells])
__global__ void k_list_init(int32_t* __restrict__ qpos, int64_t n, const int32_t* __restrict__ nq_src,
                            int64_t* __restrict__ d_nq, int* __restrict__ counters, int ncounters,
                            unsigned long long* __restrict__ cursor, TierQ tq, TierQ* __restrict__ tq_dev) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i == 0) *tq_dev = tq;
  if (qpos && i < n) qpos[i] = (int32_t)i;
  if (i < ncounters) counters[i] = 0;
  if (i < 4) cursor[i] = 0ull;
  if (i == 0 && nq_src) *d_nq = (int64_t)*nq_src;
}

// deferred builds: the query count the consumers see is 0 unless the lists are whole (every
// entry inside the list buffer, no query left for the first very-long-list pass, no capacity
// overflow, a speculative grid that held every point): an invalid build is then never read
// (its offsets may point past the buffer) and build_lists_check reruns the exact path
__global__ void k_defer_gate(const int* __restrict__ counters, const unsigned long long* __restrict__ cursor,
                             unsigned long long cap, int have_huge, int ran_mids, const int* __restrict__ oob,
                             const int64_t* __restrict__ d_nq, int64_t* __restrict__ d_nq_eff) {
  if (threadIdx.x != 0) return;
  const bool ok = cursor[0] <= cap && (have_huge || counters[3] == 0) && counters[4] == 0 && (!oob || *oob == 0) &&
                  ((ran_mids & 1) || counters[14] == 0) && ((ran_mids & 2) || counters[12] == 0) &&
                  ((ran_mids & 4) || counters[16] == 0);
  *d_nq_eff = ok ? *d_nq : 0;
}

__global__ void k_mask_flags(const int32_t* __restrict__ perm, const uint32_t* __restrict__ skeys, int64_t n,
                             uint64_t ncells, const uint8_t* __restrict__ mask, int want, uint8_t* __restrict__ flags) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flags[i] = ((uint64_t)skeys[i] < ncells) && ((mask[perm[i]] != 0) == (want != 0));
}

// segment (cell) start of each query position j, as (j if the cell changes at j else 0)
__global__ void k_seg_marks(const int32_t* __restrict__ qpos, const uint32_t* __restrict__ skeys,
                            const int64_t* __restrict__ nq_ptr, int32_t* __restrict__ marks) {
  int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j >= *nq_ptr) return;
  marks[j] = (j == 0 || skeys[qpos[j]] != skeys[qpos[j - 1]]) ? (int32_t)j : 0;
}

__global__ void k_tile_flags(const int32_t* __restrict__ seg, const int64_t* __restrict__ nq_ptr,
                             uint8_t* __restrict__ flags, int64_t n) {
  int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j >= n) return;
  flags[j] = (j < *nq_ptr) && ((j - seg[j]) % kQ == 0);
}

// candidate-block class of a tile: small, sparse, dense or wide.  The tile's record goes to its class's region of
// `recs` (slots reserved with one atomic per wave and class): small at [0, n) upward, wide at
// [0, n) downward from n - 1, sparse at [n, 2n) upward, dense at [n, 2n) downward from 2n - 1
// (each pair shares <= n tiles, so they never meet); a wide tile also gets its work entry.
__global__ void __launch_bounds__(256) k_tile_class(GridView g, const int32_t* __restrict__ qpos,
                                                    const uint32_t* __restrict__ skeys,
                                                    const int64_t* __restrict__ nq_ptr,
                                                    const int32_t* __restrict__ tiles,
                                                    const int64_t* __restrict__ ntiles_ptr,
                                                    int32_t* __restrict__ recs, int64_t n,
                                                    int32_t* __restrict__ wide, int* __restrict__ counts) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t ntiles = *ntiles_ptr;
  const int lane = threadIdx.x & 63;
  int cls = -1, qn = 0;
  int32_t start = 0;
  Runs R;
  if (t < ntiles) {
    start = tiles[t];
    const int64_t next = (t + 1 < ntiles) ? tiles[t + 1] : *nq_ptr;  // tiles never span cells
    qn = (int)(next - start < kQ ? next - start : kQ);
    const int T = block_runs(g, skeys[qpos[start]], R);
    // 3: small tiles (<= kTcapSmall candidates, so no list can exceed them: a low-LDS kernel
    // with more workgroups per CU), 0: sparse, 1: dense, 2: wide (k_nb_wide: any block size)
    cls = T <= kTcapSmall ? 3 : (T <= kTcapSparse ? 0 : (T <= kTcapDense ? 1 : 2));
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint64_t m = __ballot(cls == c);
    if (!m) continue;
    int base = 0;
    const int ci = c == 3 ? 10 : (c == 2 ? 16 : c);
    if (lane == __builtin_ctzll(m)) base = atomicAdd(&counts[ci], __popcll(m));
    base = __shfl(base, __builtin_ctzll(m));
    if (cls == c) {
      const int64_t slot = base + __popcll(m & lanemask_lt());
      // small at [0, n) upward, wide at [0, n) downward from n - 1
      const int64_t at = c == 3 ? slot : (c == 0 ? n + slot : (c == 1 ? 2 * n - 1 - slot : n - 1 - slot));
      rec_write(recs + at * kRecInts, R, start, qn);
      if (c == 2) wide[slot] = (int32_t)at;
    }
  }
}

struct ListOut {
  int64_t* off;
  int32_t* cnt;
  uint8_t* lg;
  uint32_t* list;
  unsigned long long* cursor;  // [0] slots allocated, [1] neighbours, [2] neighbours in long lists, [3] long lists
  unsigned long long cap;
  int compact;  // the tile kernels may write 16-bit entries (pfx_nblist.h kLgCompact)
  int32_t* qrec;  // query records of the lists queued to the per-query tiers (kRecInts per query)
};

// Candidate coordinates of a tile: staged in LDS, or read from the packed grid copy (L2).
struct CandLds {
  const float2* cxy;
  const float* cz;
  __device__ __forceinline__ void get(int t, float& x, float& y, float& z) const {
    const float2 v = cxy[t];
    x = v.x; y = v.y; z = cz[t];
  }
};
struct CandGlobal {
  const float4* sp;
  const Runs* R;
  __device__ __forceinline__ void get(int t, float& x, float& y, float& z) const {
    const float4 c = sp[run_pos(*R, t)];
    x = c.x; y = c.y; z = c.z;
  }
};

#ifdef PFX_SHOT_PROFILE
// phase probes, accumulated in registers and added to the globals once per workgroup / wave at
// the kernel's end (an atomic per probe left global atomics outstanding that the kernel's own
// vmcnt waits then waited for, inflating the very phases they measured)
__device__ unsigned long long g_tile_prof[28];
// per-wave probes (lane 0 of every wave): [class * 4 + i], class 0 small / 1 sparse / 2 dense;
// i = 0 the wave's own sort work, 1 its wait at the barrier after the sort, 2 the staging round
// (sort barrier -> staged registers stored), 3 the list-write loop
__device__ unsigned long long g_tile_prof2[12];
#define TPROF_DECL unsigned long long tacc_[28] = {}, wacc_[12] = {}
#define TPROF_T(v) long long v = (threadIdx.x == 0) ? clock64() : 0
#define TPROF_ADD(i, a, b) tacc_[i] += (unsigned long long)((b) - (a))
#define WPROF_T(v) long long v = ((threadIdx.x & 63) == 0) ? clock64() : 0
#define WPROF_ADD(i, a, b) wacc_[i] += (unsigned long long)((b) - (a))
#define TPROF_FLUSH                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0)                                                                \
      _Pragma("unroll") for (int i_ = 0; i_ < 28; ++i_)                                  \
        if (tacc_[i_]) atomicAdd(&g_tile_prof[i_], tacc_[i_]);                           \
    if ((threadIdx.x & 63) == 0)                                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 12; ++i_)                                  \
        if (wacc_[i_]) atomicAdd(&g_tile_prof2[i_], wacc_[i_]);                          \
  } while (0)
#else
#define TPROF_DECL
#define TPROF_T(v)
#define TPROF_ADD(i, a, b)
#define WPROF_T(v)
#define WPROF_ADD(i, a, b)
#define TPROF_FLUSH
#endif

// wave_sort for k <= 64 * E with every element's (t, d2, bucket, slot) kept in registers
// (element i of a lane is e = lane + 64 i): one LDS round trip per phase instead of one per
// 64 elements, and the candidate coordinates are read once.
template <int NB, int E, class Cand>
__device__ __forceinline__ void wave_sort_regs(uint16_t* L, int k, float qx, float qy, float qz, const Cand& cand,
                                               float bscale, uint32_t* Sd, uint16_t* St, int* bcount, int* bpos,
                                               const GridView& g, const Runs& R, int lane) {
  for (int b = lane; b < NB; b += 64) bcount[b] = 0;
  int t[E], b[E];
  uint32_t d[E];
#pragma unroll
  for (int i = 0; i < E; ++i) t[i] = lane + 64 * i < k ? L[lane + 64 * i] : 0;
  wave_sync();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    float px, py, pz;
    cand.get(t[i], px, py, pz);
    const float d2 = flann_d2(qx, qy, qz, px, py, pz);
    d[i] = __float_as_uint(d2);  // d2 >= +0: bit order == value order
    const int bb = (int)(d2 * bscale);
    b[i] = bb < NB ? bb : NB - 1;
    if (lane + 64 * i < k) atomicAdd(&bcount[b[i]], 1);
  }
  wave_sync();
  {
    constexpr int PER = NB / 64;
    int c[PER], sum = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bcount[lane * PER + v]; sum += c[v]; }
    const int inc = wave_incl_scan(sum);
    int ex = inc - sum;
#pragma unroll
    for (int v = 0; v < PER; ++v) { bpos[lane * PER + v] = ex; ex += c[v]; }
  }
  wave_sync();
  int slot[E];
#pragma unroll
  for (int i = 0; i < E; ++i) slot[i] = lane + 64 * i < k ? atomicAdd(&bpos[b[i]], 1) : 0;
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (lane + 64 * i < k) {
      Sd[slot[i]] = d[i];
      St[slot[i]] = (uint16_t)t[i];
    }
  wave_sync();
  // bucket [st, en): en = bpos after the scatter; rank = keys of the bucket below mine
  int st[E], en[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    en[i] = bpos[b[i]];
    st[i] = en[i] - bcount[b[i]];
  }
  int rank[E];
  bool tie = false;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    uint32_t dv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dv[j] = st[i] + j < en[i] ? Sd[st[i] + j] : 0xffffffffu;
    int r = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r += dv[j] < d[i];
      eq += dv[j] == d[i];
    }
    for (int v = st[i] + 4; v < en[i]; ++v) {
      const uint32_t x = Sd[v];
      r += x < d[i];
      eq += x == d[i];
    }
    rank[i] = r;
    tie |= lane + 64 * i < k && eq > 1;
  }
  if (__builtin_amdgcn_ballot_w64(tie)) {  // equal d2: the caller index decides (FLANN); rare
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (lane + 64 * i >= k) continue;
      const int32_t mine = g.perm[run_pos(R, t[i])];
      for (int v = st[i]; v < en[i]; ++v)
        if (v != slot[i] && Sd[v] == d[i] && g.perm[run_pos(R, St[v])] < mine) ++rank[i];
    }
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (lane + 64 * i < k) L[st[i] + rank[i]] = (uint16_t)t[i];
  wave_sync();
}

// Wave-local bucket sort of one query's list L[0..k) (u16 candidate indices) into FLANN order.
// Sd/St: wave-private scratch (k entries), bcount/bpos: wave-private NB buckets.
template <int NB, class Cand>
__device__ __forceinline__ void wave_sort(uint16_t* L, int k, float qx, float qy, float qz, const Cand& cand,
                                          float bscale, uint32_t* Sd, uint16_t* St, int* bcount, int* bpos,
                                          const GridView& g, const Runs& R, int lane) {
  for (int b = lane; b < NB; b += 64) bcount[b] = 0;
  wave_sync();
  for (int e = lane; e < k; e += 64) {
    const int t = L[e];
    float px, py, pz;
    cand.get(t, px, py, pz);
    const int b = (int)(flann_d2(qx, qy, qz, px, py, pz) * bscale);
    atomicAdd(&bcount[b < NB ? b : NB - 1], 1);
  }
  wave_sync();
  {
    constexpr int PER = NB / 64;
    int c[PER], s = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bcount[lane * PER + v]; s += c[v]; }
    const int inc = wave_incl_scan(s);
    int ex = inc - s;
#pragma unroll
    for (int v = 0; v < PER; ++v) { bpos[lane * PER + v] = ex; ex += c[v]; }
  }
  wave_sync();
  for (int e = lane; e < k; e += 64) {
    const int t = L[e];
    float px, py, pz;
    cand.get(t, px, py, pz);
    const float d2 = flann_d2(qx, qy, qz, px, py, pz);
    int b = (int)(d2 * bscale);
    b = b < NB ? b : NB - 1;
    const int slot = atomicAdd(&bpos[b], 1);
    Sd[slot] = __float_as_uint(d2);  // d2 >= +0: bit order == value order
    St[slot] = (uint16_t)t;
  }
  wave_sync();
  // rank inside the bucket; two elements per lane per round and the first four bucket entries
  // read at once, so the LDS round trips of a round overlap
  auto bucket_rank = [&](int s, uint32_t d, int t, int st, int en) {
    uint32_t dv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dv[i] = st + i < en ? Sd[st + i] : 0xffffffffu;
    int rank = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = st + i;
      if (v < en) {
        if (dv[i] < d) ++rank;
        else if (dv[i] == d && v != s && g.perm[run_pos(R, St[v])] < g.perm[run_pos(R, t)]) ++rank;
      }
    }
    for (int v = st + 4; v < en; ++v) {
      const uint32_t x = Sd[v];
      if (x < d) ++rank;
      else if (x == d && v != s && g.perm[run_pos(R, St[v])] < g.perm[run_pos(R, t)]) ++rank;
    }
    return rank;
  };
  for (int s0 = lane; s0 < k; s0 += 128) {
    const int s1 = s0 + 64;
    const bool h1 = s1 < k;
    const uint32_t d0 = Sd[s0], d1 = h1 ? Sd[s1] : 0u;
    const int t0 = St[s0], t1 = h1 ? St[s1] : 0;
    int b0 = (int)(__uint_as_float(d0) * bscale), b1 = (int)(__uint_as_float(d1) * bscale);
    b0 = b0 < NB ? b0 : NB - 1;
    b1 = b1 < NB ? b1 : NB - 1;
    const int en0 = bpos[b0], c0 = bcount[b0], en1 = bpos[b1], c1 = bcount[b1];
    const int st0 = en0 - c0, st1 = en1 - c1;
    const int r0 = bucket_rank(s0, d0, t0, st0, en0);
    const int r1 = h1 ? bucket_rank(s1, d1, t1, st1, en1) : 0;
    L[st0 + r0] = (uint16_t)t0;
    if (h1) L[st1 + r1] = (uint16_t)t1;
  }
  wave_sync();
}

// k <= 64: one entry per lane, rank = entries with a smaller d2, counted over v_readlane (no
// LDS); only when two entries of the list share a d2 (rare) are the caller indices loaded and
// the (d2, caller index) keys compared
template <class Cand>
__device__ __forceinline__ void wave_rank_sort(uint16_t* L, int k, float qx, float qy, float qz, const Cand& cand,
                                               const GridView& g, const Runs& R, int lane) {
  const bool in = lane < k;
  const int t = in ? L[lane] : 0;
  float px, py, pz;
  cand.get(t, px, py, pz);
  const uint32_t d = in ? __float_as_uint(flann_d2(qx, qy, qz, px, py, pz)) : 0xffffffffu;
  int rank = 0, eq = 0;
  for (int m = 0; m < k; ++m) {
    const uint32_t dm = (uint32_t)__builtin_amdgcn_readlane((int)d, m);
    rank += dm < d ? 1 : 0;
    eq += dm == d ? 1 : 0;
  }
  if (__builtin_amdgcn_ballot_w64(in && eq > 1)) {
    const int32_t id = in ? g.perm[run_pos(R, t)] : 0x7fffffff;
    rank = 0;
    for (int m = 0; m < k; ++m) {
      const uint32_t dm = (uint32_t)__builtin_amdgcn_readlane((int)d, m);
      const int32_t im = __builtin_amdgcn_readlane(id, m);
      rank += (dm < d || (dm == d && im < id)) ? 1 : 0;
    }
  }
  wave_sync();
  if (in) L[rank] = (uint16_t)t;
  wave_sync();
}

template <int NB, class Cand, bool SMALL = false>
__device__ __forceinline__ void sort_list(uint16_t* L, int k, float qx, float qy, float qz, const Cand& cand,
                                          float bscale, uint32_t* Sd, uint16_t* St, int* bcount, int* bpos,
                                          const GridView& g, const Runs& R, int lane) {
  // register tiers in steps of 64-128 elements: the unrolled per-element work of a tier runs for
  // every slot, so a list is sorted by the smallest tier that holds it
  if (k <= 64) wave_rank_sort(L, k, qx, qy, qz, cand, g, R, lane);
  else if (k <= 128) wave_sort_regs<NB, 2>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 192) wave_sort_regs<NB, 3>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 256) wave_sort_regs<NB, 4>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 320) wave_sort_regs<NB, 5>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (SMALL || k <= 384) wave_sort_regs<NB, 6>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 448) wave_sort_regs<NB, 7>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 512) wave_sort_regs<NB, 8>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 640) wave_sort_regs<NB, 10>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 768) wave_sort_regs<NB, 12>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 896) wave_sort_regs<NB, 14>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else if (k <= 1024) wave_sort_regs<NB, 16>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
  else wave_sort<NB>(L, k, qx, qy, qz, cand, bscale, Sd, St, bcount, bpos, g, R, lane);
}

// STAGE: candidates staged in LDS (small and sparse tiles); otherwise read from L2 (dense tiles,
// where staging 8000 candidates would cap the kernel at one workgroup per CU).
// Software pipeline, per tile i (its record unpacked into SGPRs, its candidates and query
// positions already in LDS):
//   [A] load the record of tile i+1 (one lane per word)   [B] test -> barrier
//   [C] sort, one list per wave at a time -> barrier
//   [D] unpack record i+1; issue its candidate + query-position loads into registers; write the
//       lists of tile i to HBM; store the registers to LDS -> barrier
// so the one global-latency round of a tile (staging loads, list stores) is shared.  Tiles come
// from a dynamic queue `chunk` at a time; thread 0 keeps the next chunk's base fetched one chunk
// ahead and publishes it in [D].
// (the kernels get the queues through one pointer to a device copy: eight pointers as kernel
// arguments pushed the tile kernels into spilling scalar registers)
__device__ __forceinline__ void push_sort(const TierQ* tq, int32_t j, int k) {
  const int t = query_tier(k);
  tq->q[t][atomicAdd(tq->n[t], 1)] = j | kListMode;
}

// One pass of a tile's candidates against the wave's queries u (act[u], wave-uniform): hits are
// counted in cursor[u] and, with STORE, written to glist[gb[u] + slot] as run entries (in
// candidate order).  STAGE: the candidates are staged in cxy / cz; otherwise they stream through
// hxy / hz in chunks of kChunkWide (the whole workgroup takes part: barriers inside).
constexpr int kChunkWide = 1024;
template <bool STAGE, int SCAP, bool STORE>
__device__ __forceinline__ void tile_pass(const GridView& g, const Runs& R, int T, const float2* cxy, const float* cz,
                                          float2* hxy, float* hz, const pf2* qxy, const float* qz, const bool* act,
                                          const int64_t* gb, int* cursor, uint32_t* __restrict__ glist, float rr) {
  constexpr int CH = kChunkWide, U = 2, QW = 4;
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int u = 0; u < QW; ++u) cursor[u] = 0;
  // streamed chunks: chunk c + 1's loads are issued right after chunk c is in LDS and land during
  // chunk c's test (round 6: each chunk waited a full L2 round trip before its test)
  float4 cc[STAGE ? 1 : CH / 256];
  if (!STAGE)
#pragma unroll
    for (int u = 0; u < CH / 256; ++u) cc[u] = g.sp[run_pos(R, min(tid + 256 * u, T - 1))];
  for (int c0 = 0; c0 < T; c0 += (STAGE ? T : CH)) {
    const int cend = STAGE ? T : min(T, c0 + CH);
    if (!STAGE) {
      __syncthreads();  // the previous chunk's readers are done
#pragma unroll
      for (int u = 0; u < CH / 256; ++u) {
        hxy[tid + 256 * u] = make_float2(cc[u].x, cc[u].y);
        hz[tid + 256 * u] = cc[u].z;
      }
      __syncthreads();
      if (c0 + CH < T)
#pragma unroll
        for (int u = 0; u < CH / 256; ++u) cc[u] = g.sp[run_pos(R, min(c0 + CH + tid + 256 * u, T - 1))];
    }
    const float2* XYs = STAGE ? cxy : hxy - c0;
    const float* Zs = STAGE ? cz : hz - c0;
    for (int t0 = c0; t0 < cend; t0 += 64 * U) {
      pf2 pxy[U];
      float pz[U], rrv[U];
#pragma unroll
      for (int v = 0; v < U; ++v) {
        const int t = t0 + 64 * v + lane;
        const int tr = STAGE ? min(t, SCAP - 1) : t;  // (chunks: CH is a multiple of 64 U)
        const float2 xy = XYs[tr];
        pxy[v] = pf2{xy.x, xy.y};
        pz[v] = Zs[tr];
        rrv[v] = t < cend ? rr : -1.0f;
      }
#pragma unroll
      for (int v = 0; v < U; ++v) {
        const int t = t0 + 64 * v + lane;
#pragma unroll
        for (int u = 0; u < QW; ++u) {
          if (!act[u]) continue;  // wave-uniform
          const pf2 dxy = qxy[u] - pxy[v];
          const pf2 sq = dxy * dxy;
          const float dz = qz[u] - pz[v];
          const bool hit = (sq.x + sq.y) + dz * dz < rrv[v];
          const uint64_t m = __builtin_amdgcn_ballot_w64(hit);
          if (STORE && hit) {
            const int slot = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)cursor[u]));
            glist[gb[u] + slot] = run_entry(R, t);
          }
          cursor[u] += __popcll(m);
        }
      }
    }
  }
}

template <int TCAP, bool STAGE>
struct Stager {
  static constexpr int PT = STAGE ? (TCAP + 255) / 256 : 0;
  float x[PT > 0 ? PT : 1], y[PT > 0 ? PT : 1], z[PT > 0 ? PT : 1];
  int32_t qp;
  __device__ __forceinline__ void load(const GridView& g, const int32_t* __restrict__ qpos, const Runs& R,
                                       int32_t start, int qn, bool ok) {
    // branch-free: every load is issued (clamped index, one address computation), so all of
    // them are in flight at once
    const int tid = threadIdx.x;
    const int T = ok ? R.pref[9] : 0;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int tc = max(0, min(tid + 256 * u, T - 1));
      const float4 c = g.sp[run_pos(R, tc)];
      x[u] = c.x; y[u] = c.y; z[u] = c.z;
    }
    qp = qpos[start + (tid < qn ? tid : 0)];
  }
  // unconditional (slots >= T get don't-care values; the arrays hold PT * 256): a conditional
  // store lets the compiler sink each load into its own branch and wait for it there
  __device__ __forceinline__ void store(float2* cxy, float* cz, int32_t* s_qp, int qn) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int t = tid + 256 * u;
      cxy[t] = make_float2(x[u], y[u]);
      cz[t] = z[u];
    }
    if (tid < qn) s_qp[tid] = qp;
  }
};

template <int LCAP, int NB, int TCAP, bool STAGE>
__global__ void __launch_bounds__(256, TCAP <= kTcapSmall ? 4 : (STAGE ? 3 : 2)) k_nb_tile(GridView g, const int32_t* __restrict__ qpos,
                                                 const int32_t* __restrict__ rec_base, int rec_step,
                                                 const int* __restrict__ ntiles_ptr,
                                                 float rr, float bscale, int sorted, ListOut out,
                                                 const TierQ* __restrict__ tq,
                                                 int* __restrict__ next_tile, int chunk) {
  constexpr int Q = kQ, QW = Q / 4;  // queries per tile / per wave
  constexpr int U = 2;               // candidates per lane in flight in the test loop
  constexpr int SCAP = STAGE ? Stager<TCAP, STAGE>::PT * 256 : 1;
  __shared__ float2 cxy[SCAP];
  __shared__ float cz[SCAP];
  // dense tiles: the test loop reads candidates from LDS chunks of CH staged by the whole
  // workgroup (one latency round and one run search per candidate, not per wave and candidate)
  constexpr int CH = STAGE ? 1 : 1024;
  __shared__ float2 hxy[CH];
  __shared__ float hz[CH];
  // the tile's lists (+2: odd dword row stride, no bank conflicts), then the test's trash slots
  // (a miss stores its candidate to its lane's slot: the test loop has no branch)
  __shared__ uint16_t lists_flat[Q * (LCAP + 2) + 4 * 64];
  uint16_t(*lists)[LCAP + 2] = reinterpret_cast<uint16_t(*)[LCAP + 2]>(lists_flat);
  __shared__ uint32_t sd[4][LCAP];
  __shared__ uint16_t stt[4][LCAP];
  __shared__ int bcount[4][NB], bpos[4][NB];
  __shared__ int s_k[Q];
  __shared__ int32_t s_qp[Q];
  __shared__ unsigned long long s_base;
  __shared__ int s_chunk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): per-query branches are scalar
  const uint32_t trash_at = (uint32_t)(Q * (LCAP + 2) + 64 * wv + lane);
  const uint32_t wrow = (uint32_t)(wv * (LCAP + 2));  // the wave's first list row (its queries: wv + 4 u)
  const int ntiles = *ntiles_ptr;
  TPROF_DECL;
  unsigned long long wg_total = 0, arena_base = 0, arena_left = 0;  // thread 0's
  int next_chunk = 0;                                                // thread 0's
  if (tid == 0) {
    s_chunk = atomicAdd(next_tile, chunk);
    next_chunk = atomicAdd(next_tile, chunk);
  }
  __syncthreads();
  int i = __builtin_amdgcn_readfirstlane(s_chunk), i_end = i + chunk;
  Runs R;
  int32_t start = 0;
  int qn = 0;
  {
    const int v = rec_load(rec_base, rec_step, i, i < ntiles);
    rec_unpack(v, R, start, qn);
    Stager<TCAP, STAGE> sg;
    sg.load(g, qpos, R, start, qn, R.pref[9] <= TCAP);
    __syncthreads();  // s_chunk read by every thread before it is republished
    if (i + 1 == i_end && tid == 0) {
      s_chunk = next_chunk;
      next_chunk = atomicAdd(next_tile, chunk);
    }
    sg.store(cxy, cz, s_qp, qn);
    __syncthreads();
  }
  while (i < ntiles) {
    TPROF_T(p0);
    const int T = R.pref[9];
    const bool ok = T <= TCAP;  // always true after k_tile_class; keep the kernel safe regardless
    // [A] the next tile and its record
    int ni = i + 1;
    if (ni == i_end) {
      ni = __builtin_amdgcn_readfirstlane(s_chunk);
      i_end = ni + chunk;
    }
    const int recv = rec_load(rec_base, rec_step, ni, ni < ntiles);
    // [B] test
    pf2 qxy[QW];
    float qz[QW];
    int cursor[QW];
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const int j = wv + 4 * u;
      cursor[u] = 0;
      qxy[u] = pf2{0.f, 0.f};
      qz[u] = 0.f;
      if (j < qn) {
        const int32_t p = s_qp[j];
        if (STAGE) {  // a query lies in its own cell, i.e. in run 4 of its block
          const int t = R.pref[4] + (p - R.start[4]);
          const float2 v = cxy[t];
          qxy[u] = pf2{v.x, v.y};
          qz[u] = cz[t];
        } else {
          const float4 c = g.sp[p];
          qxy[u] = pf2{c.x, c.y};
          qz[u] = c.z;
        }
      }
    }
    for (int c0 = 0; ok && c0 < T; c0 += (STAGE ? T : CH)) {  // one pass for staged tiles
      const int cend = STAGE ? T : min(T, c0 + CH);
      if (!STAGE) {
        constexpr int CPT = CH >= 256 ? CH / 256 : 1;
        float4 cc[CPT];
#pragma unroll
        for (int u = 0; u < CPT; ++u) cc[u] = g.sp[run_pos(R, min(c0 + tid + 256 * u, T - 1))];
        __syncthreads();  // the previous chunk's readers are done
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
          hxy[tid + 256 * u] = make_float2(cc[u].x, cc[u].y);
          hz[tid + 256 * u] = cc[u].z;
        }
        __syncthreads();
      }
      const float2* XYs = STAGE ? cxy : hxy - c0;
      const float* Zs = STAGE ? cz : hz - c0;
      // Branch-free test (round 4): candidate reads are unconditional (index clamped into the
      // staging array), a slot past the block gets the threshold -1 (never a hit), and every lane
      // stores -- a hit to its compacted slot, a miss to its own trash slot -- through one
      // v_cndmask of the two element offsets; FLANN's d2 = (dx^2 + dy^2) + dz^2 (dx = q - p; the
      // 0 + dx^2 of L2_Simple is exact) with x, y on packed f32.  The branchy form compiled into
      // ~30 instructions and two exec-mask branches per candidate and query.
      for (int t0 = c0; t0 < cend; t0 += 64 * U) {
        pf2 pxy[U];
        float pz[U], rrv[U];
#pragma unroll
        for (int v = 0; v < U; ++v) {
          const int t = t0 + 64 * v + lane;
          const int tr = STAGE ? min(t, SCAP - 1) : t;  // (dense chunks: t - c0 < CH always)
          const float2 xy = XYs[tr];
          pxy[v] = pf2{xy.x, xy.y};
          pz[v] = Zs[tr];
          rrv[v] = t < cend ? rr : -1.0f;
        }
#pragma unroll
        for (int v = 0; v < U; ++v) {
          const int t = t0 + 64 * v + lane;
#pragma unroll
          for (int u = 0; u < QW; ++u) {
            const int j = wv + 4 * u;
            if (j >= qn) continue;  // wave-uniform
            const pf2 dxy = qxy[u] - pxy[v];
            const pf2 sq = dxy * dxy;
            const float dz = qz[u] - pz[v];
            const bool hit = (sq.x + sq.y) + dz * dz < rrv[v];
            const uint64_t m = __builtin_amdgcn_ballot_w64(hit);
            const int slot = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)cursor[u]));
            // (an overflowing list -- it goes to the per-query path -- keeps writing its row's pad
            // slot).  The select as bit arithmetic: a plain ?: let the compiler sink the slot
            // computation into an exec-masked if/else around every store.
            const uint32_t hit_at = (uint32_t)(min(slot, LCAP) + wrow) + (uint32_t)(4 * u * (LCAP + 2));
            const uint32_t sel = 0u - (uint32_t)hit;
            lists_flat[trash_at ^ ((trash_at ^ hit_at) & sel)] = (uint16_t)t;
            cursor[u] += __popcll(m);
          }
        }
      }
    }
    // tile layout in HBM: the lists of the tile's qn queries interleaved with stride 2^lg >= qn
    // (entry m of query j at base + (m << lg) + j), so lane-per-query consumers read coalesced
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < QW; ++u)
        if (wv + 4 * u < qn) {
          const int kq = ok ? cursor[u] : LCAP + 1;
          s_k[wv + 4 * u] = kq;
          // an overflowing list goes to the per-query kernel: its record, from the owner wave
          if (kq > LCAP) qrec_write(out.qrec, start + wv + 4 * u, R, s_qp[wv + 4 * u], qxy[u].x, qxy[u].y, qz[u]);
        }
    }
    __syncthreads();
    TPROF_T(p1);
    TPROF_ADD(TCAP <= kTcapSmall ? 17 : (STAGE ? 1 : 5), p0, p1);
    // [C] list slots, sort
    WPROF_T(ws0);
    [[maybe_unused]] constexpr int kWp0 = TCAP <= kTcapSmall ? 0 : (STAGE ? 4 : 8);
    int lg = 0;
    while ((1 << lg) < qn) ++lg;
    // 16-bit entries when every run of the block fits their 12-bit offset (the list bytes the
    // chains stream from HBM halve)
    bool c16 = out.compact != 0;
#pragma unroll
    for (int r = 0; r < 9; ++r) c16 = c16 && R.pref[r + 1] - R.pref[r] <= kCompactRun;
    int maxk = 0;
    for (int j = 0; j < qn; ++j) {
      const int k = s_k[j];
      maxk = (k <= LCAP && k > maxk) ? k : maxk;
    }
    if (tid == 0)
      for (int j = 0; j < qn; ++j) wg_total += s_k[j] <= LCAP ? (unsigned long long)s_k[j] : 0ull;
    // list slots come from a per-workgroup arena reserved kArena entries at a time (one cursor
    // atomic per arena, not per tile); unused arena tails are never read (compact: two entries per
    // 32-bit slot).  The reservation is issued here and its result read in [D], after the sort:
    // the atomic's round trip (same-address, every workgroup) used to stall the whole workgroup
    // at [D]'s barrier (round 6; the file is built without the atomic optimizer, which reads an
    // atomic's result at once to spread it over the lanes)
    const unsigned long long need = c16 ? (((unsigned long long)maxk << lg) + 1) >> 1 : (unsigned long long)maxk << lg;
    unsigned long long arena_new = 0, arena_res = 0;  // thread 0's
    if (tid == 0 && need > arena_left) {
      arena_res = need > (unsigned long long)kArena ? need : (unsigned long long)kArena;
      arena_new = atomicAdd(out.cursor, arena_res);
    }
    if (tid < qn) {
      const int k = s_k[tid];
      if (k <= LCAP) {
        out.cnt[start + tid] = k;
        out.lg[start + tid] = (uint8_t)(lg | (c16 ? kLgCompact : 0));
      } else {
        // the per-query kernel (test + sort): measured against a second tile pass writing these
        // lists unsorted for a sort-only per-query pass, that pass cost more (room: dense tiles
        // +0.22 ms against 0.07 saved; dense variant: no change)
        // (the tier that holds k: a dense tile's 4k-8k lists no longer pass through the 4k tier's
        // test first)
        const int t = ok ? query_tier(k) : 0;
        if (t == 0) tq->q[0][wave_push_slot(tq->n[0])] = start + tid;
        else tq->q[t][atomicAdd(tq->n[t], 1)] = start + tid;
      }
    }
    if (sorted) {
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const int j = wv + 4 * u;
        const int k = cursor[u];
        if (ok && j < qn && k <= LCAP && k > 1) {  // wave-uniform
          if (STAGE) {
            const CandLds cand{cxy, cz};
            sort_list<NB, CandLds, (TCAP <= kTcapSmall)>(lists[j], k, qxy[u].x, qxy[u].y, qz[u], cand, bscale, sd[wv],
                                                         stt[wv], bcount[wv], bpos[wv], g, R, lane);
          } else {
            const CandGlobal cand{g.sp, &R};
            sort_list<NB>(lists[j], k, qxy[u].x, qxy[u].y, qz[u], cand, bscale, sd[wv], stt[wv], bcount[wv], bpos[wv],
                          g, R, lane);
          }
        }
      }
    }
    WPROF_T(ws1);
    WPROF_ADD(kWp0 + 0, ws0, ws1);
    __syncthreads();
    TPROF_T(p2);
    TPROF_ADD(TCAP <= kTcapSmall ? 18 : (STAGE ? 2 : 6), p1, p2);
    WPROF_T(ws2);
    [[maybe_unused]] constexpr int kWp = TCAP <= kTcapSmall ? 0 : (STAGE ? 4 : 8);
    WPROF_ADD(kWp + 1, ws1, ws2);
    // [D] one latency round: the next tile's staging loads, the list-slot reservation and the
    // queue fetch; their results land in LDS, then this tile's lists are written (stores in
    // flight until the next tile's round)
    Runs Rn;
    int32_t start_n;
    int qn_n;
    rec_unpack(recv, Rn, start_n, qn_n);
    const bool ok_n = ni < ntiles && Rn.pref[9] <= TCAP;
    Stager<TCAP, STAGE> sg;
    if (ni < ntiles) sg.load(g, qpos, Rn, start_n, qn_n, ok_n);
    if (tid == 0) {
      if (ni + 1 == i_end) {  // publish the next chunk (fetched one chunk ago), fetch the one after
        s_chunk = next_chunk;
        next_chunk = atomicAdd(next_tile, chunk);  // (read a chunk later)
      }
      if (arena_res) {  // the reservation issued in [C]
        arena_base = arena_new;
        arena_left = arena_res;
      }
      s_base = arena_base;
      arena_base += need;
      arena_left -= need;
    }
    if (ni < ntiles) sg.store(cxy, cz, s_qp, qn_n);
    WPROF_T(ws3);
    WPROF_ADD(kWp + 2, ws2, ws3);
    __syncthreads();
    WPROF_T(ws4);
    const int64_t base = (int64_t)s_base;
    // (compact: offsets count 16-bit entries)
    if (tid < qn && s_k[tid] <= LCAP) out.off[start + tid] = (c16 ? 2 * base : base) + tid;
    // coalesced write of the interleaved block (padding slots are left unwritten)
    const int total = maxk << lg;
    if (c16) {
      // two entries per 32-bit store (entries 2w, 2w + 1 of the block; padding halves are 0)
      const int words = (total + 1) >> 1;
      if ((unsigned long long)(base + words) <= out.cap) {
        for (int w = tid; w < words; w += 256) {
          uint32_t pair = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e = 2 * w + h;
            const int m = e >> lg, j = e & ((1 << lg) - 1);
            const int k = j < qn ? s_k[j] : 0;
            if (e < total && m < k && k <= LCAP) pair |= (uint32_t)run_entry16(R, lists[j][m]) << (16 * h);
          }
          out.list[base + w] = pair;
        }
      }
    } else if ((unsigned long long)(base + total) <= out.cap) {
      for (int e = tid; e < total; e += 256) {
        const int m = e >> lg, j = e & ((1 << lg) - 1);
        if (j < qn) {
          const int k = s_k[j];
          if (m < k && k <= LCAP) out.list[base + e] = run_entry(R, lists[j][m]);
        }
      }
    }
    WPROF_T(ws5);
    WPROF_ADD(kWp + 3, ws4, ws5);
    __syncthreads();  // lists and s_k read before the next tile's test overwrites them
    TPROF_T(p3);
    TPROF_ADD(TCAP <= kTcapSmall ? 19 : (STAGE ? 3 : 7), p2, p3);
    i = ni;
    R = Rn;
    start = start_n;
    qn = qn_n;
  }
  if (tid == 0 && wg_total) atomicAdd(out.cursor + 1, wg_total);
  TPROF_FLUSH;
}

// ---- wide tiles (round 4) ----------------------------------------------------------------
// Every query of a tile whose 3x3x3 block has T > 8000 candidates (k_tile_class): one
// workgroup per tile (dynamic queue) streams the block through LDS in chunks shared by the
// tile's (up to 16) queries -- the per-query kernel read the block once per query, with a run
// search per candidate -- in a count pass and a pass writing the hits unsorted to their slots in
// HBM; the per-query tiers then order each list in place (kListMode work items, no test).
__global__ void __launch_bounds__(256) k_nb_wide(GridView g, const int32_t* __restrict__ qpos,
                                                 const int32_t* __restrict__ recs, const int32_t* __restrict__ work,
                                                 const int* __restrict__ n_ptr, float rr, int sorted, ListOut out,
                                                 const TierQ* __restrict__ tq, int* __restrict__ next_work) {
  constexpr int QW = 4;
  __shared__ float2 hxy[kChunkWide];
  __shared__ float hz[kChunkWide];
  __shared__ int s_k[kQ];
  __shared__ int32_t s_qp[kQ];
  __shared__ int s_w;
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int count = *n_ptr;
  if (count == 0) return;  // (the room has no wide tiles: an empty launch costs only its dispatch)
  // thread 0's: list slots from a per-workgroup arena, totals added once per workgroup
  unsigned long long wg_total = 0, wg_long = 0, wg_long_n = 0, arena_base = 0, arena_left = 0;
  for (;;) {
    if (tid == 0) s_w = atomicAdd(next_work, 1);
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(s_w);
    __syncthreads();
    if (w >= count) break;
    Runs R;
    int32_t start;
    int qn;
    rec_unpack(rec_load(recs, kRecInts, work[w], true), R, start, qn);
    const int T = R.pref[9];
    if (tid < qn) s_qp[tid] = qpos[start + tid];
    __syncthreads();
    pf2 qxy[QW];
    float qz[QW];
    bool act[QW];
    int cursor[QW];
    int64_t gb[QW];
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const int j = wv + 4 * u;
      act[u] = j < qn;
      qxy[u] = pf2{0.f, 0.f};
      qz[u] = 0.f;
      gb[u] = 0;
      if (act[u]) {
        const float4 c = g.sp[s_qp[j]];
        qxy[u] = pf2{c.x, c.y};
        qz[u] = c.z;
      }
    }
    tile_pass<false, 1, false>(g, R, T, nullptr, nullptr, hxy, hz, qxy, qz, act, gb, cursor, nullptr, rr);
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < QW; ++u)
        if (act[u]) {
          s_k[wv + 4 * u] = cursor[u];
          qrec_write(out.qrec, start + wv + 4 * u, R, s_qp[wv + 4 * u], qxy[u].x, qxy[u].y, qz[u]);
        }
    }
    __syncthreads();
    int need = 0;
    for (int j = 0; j < qn; ++j) need += s_k[j];
    need = __builtin_amdgcn_readfirstlane(need);
    if (tid == 0) {
      if ((unsigned long long)need > arena_left) {
        const unsigned long long res = need > kArenaQuery ? (unsigned long long)need : (unsigned long long)kArenaQuery;
        arena_base = atomicAdd(out.cursor, res);
        arena_left = res;
      }
      s_base = arena_base;
      arena_base += need;
      arena_left -= need;
      wg_total += need;
      for (int j = 0; j < qn; ++j)
        if (s_k[j] > kLongList) {
          wg_long += (unsigned long long)s_k[j];
          ++wg_long_n;
        }
    }
    __syncthreads();
    const int64_t base = (int64_t)s_base;
    const bool fits = (unsigned long long)(base + need) <= out.cap;
    if (fits) {
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        int pre = 0;
        for (int j = 0; j < wv + 4 * u && j < qn; ++j) pre += s_k[j];
        gb[u] = base + pre;
      }
      tile_pass<false, 1, true>(g, R, T, nullptr, nullptr, hxy, hz, qxy, qz, act, gb, cursor, out.list, rr);
    }
    if (tid < qn) {
      int pre = 0;
      for (int j = 0; j < tid; ++j) pre += s_k[j];
      const int k = s_k[tid];
      out.off[start + tid] = base + pre;
      out.cnt[start + tid] = k;
      out.lg[start + tid] = 0;
      if (fits && sorted && k > 1) push_sort(tq, start + tid, k);
    }
    __syncthreads();  // s_k / s_qp are rewritten by the next tile
  }
  if (tid == 0) {
    if (wg_total) atomicAdd(out.cursor + 1, wg_total);
    if (wg_long_n) {
      atomicAdd(out.cursor + 2, wg_long);
      atomicAdd(out.cursor + 3, wg_long_n);
    }
  }
}

// One workgroup of NT threads per query: candidates streamed from L2/HBM, the list bucket-sorted
// in LDS (GLOBAL = false) or in a per-workgroup global scratch slice (GLOBAL = true).
// A test-mode list longer than CAP goes straight to the tier that holds it (`tq`: its length is
// known once it has been counted), or raises err when tq == nullptr.
// list entry of grid position p: (run << 28) | offset in the run
__device__ __forceinline__ uint32_t pos_entry(const Runs& R, int32_t p) {
  uint32_t e = 0;
#pragma unroll
  for (int r = 0; r < 9; ++r)
    if (p >= R.start[r] && p < R.start[r] + (R.pref[r + 1] - R.pref[r])) e = ((uint32_t)r << 28) | (uint32_t)(p - R.start[r]);
  return e;
}

__device__ __forceinline__ uint32_t pos_entry16(const Runs& R, int32_t p) {
  const uint32_t e = pos_entry(R, p);
  return ((e >> 28) << 12) | (e & 0xfffu);
}

// exclusive scan of NB bucket counts into bpos by all NT threads (NB / NT consecutive buckets
// each: a one-wave scan of 16-64 buckets per lane read them at a lane stride of 16-64 words,
// 16-64-way LDS bank conflicts)
template <int NB, int NT>
__device__ __forceinline__ void bucket_scan(const int* bcount, int* bpos, int* wsum) {
  constexpr int PER = NB >= NT ? NB / NT : 1;
  const int tid = threadIdx.x;
  const bool in = tid * PER < NB;
  int c[PER];
  int s = 0;
#pragma unroll
  for (int v = 0; v < PER; ++v) {
    c[v] = in ? bcount[tid * PER + v] : 0;
    s += c[v];
  }
  const int inc = wave_incl_scan(s);
  if ((tid & 63) == 63) wsum[tid >> 6] = inc;
  __syncthreads();
  int ex = inc - s;
  for (int w = 0; w < (tid >> 6); ++w) ex += wsum[w];
  if (in) {
#pragma unroll
    for (int v = 0; v < PER; ++v) {
      bpos[tid * PER + v] = ex;
      ex += c[v];
    }
  }
}

// the GLOBAL tier's rank pass reads the bucket-ordered d2 bits through LDS windows of this many
// (16 KB: with its one bucket array, 16 KB, the tier keeps four workgroups per CU)
constexpr int kRankWindow = 4096;

// NT (round 6): 512 threads for the 4k tier, 1024 for the 8k and 16k tiers -- their LDS, not their
// registers, caps the workgroups per CU (4 / 2 / 1), so a wider workgroup shortens each list's
// chain of dependent latency rounds at the same LDS (the 16k tier ran one wave per SIMD).
// GLOBAL (the > 16k tier): one bucket array (counts, scanned in place to starts, advanced by the
// scatter to ends: a bucket is [end of b - 1, end of b)), eight entries per thread in flight in
// the passes over the scratch, the rank pass through LDS windows
// WPE: the waves per SIMD the tier's LDS allows (the register budget the compiler is held to)
template <int CAP, int NB, bool GLOBAL, int NT, int WPE>
__global__ void __launch_bounds__(NT, WPE) k_nb_query(GridView g, const int32_t* __restrict__ work,
                                                 const int* __restrict__ n_ptr,
                                                 float rr, float bscale, int sorted, ListOut out,
                                                 const TierQ* __restrict__ tq,
                                                 int* __restrict__ err, uint32_t* __restrict__ scratch,
                                                 int* __restrict__ next_work) {
  static_assert(NT % 256 == 0 && CAP % NT == 0, "whole rounds of NT entries");
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ int bcount[NB], bpos[GLOBAL ? 1 : NB];
  __shared__ uint32_t wd[GLOBAL ? kRankWindow : 1];  // GLOBAL: the rank pass's window of d2 bits
  constexpr int UL = GLOBAL ? 8 : 4;  // entries / candidates per thread in flight
  __shared__ int wsum[NT / 64];
  __shared__ int s_count;
  __shared__ unsigned long long s_base;
  uint32_t* base_arr = GLOBAL ? scratch + (size_t)blockIdx.x * 4 * CAP : smem;
  uint32_t* hits = base_arr;        // positions, then the sorted list
  uint32_t* hd = base_arr + CAP;    // d2 bits of hits
  uint32_t* sdv = base_arr + 2 * CAP;  // (GLOBAL: bucket-ordered copies)
  uint32_t* spv = base_arr + 3 * CAP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int count = *n_ptr;
  if (count == 0) return;  // an empty tier costs only its dispatch (the queue head stays 0)
  __shared__ int s_w, s_wn;
  // thread 0's: list slots from a per-workgroup arena and the totals added once per workgroup
  // (one same-address atomic per query made the cursors the bottleneck of this kernel)
  unsigned long long wg_total = 0, wg_long = 0, wg_long_n = 0, arena_base = 0, arena_left = 0;
  TPROF_DECL;
  // Work items are fetched two ahead by thread 0 (w1: the next item, w2: the one after), so each
  // item's work index is loaded at the top of the item before it and its record after that item's
  // first phase: an item starts with its record in registers (round 6: it used to start with the
  // chain queue atomic -> work[] -> record, three dependent round trips)
  int w1 = 0, w2 = 0;
  if (tid == 0) {
    w1 = atomicAdd(next_work, 1);
    w2 = w1 < count ? atomicAdd(next_work, 1) : count;
  }
  int32_t jw_pf = 0;   // the next item's work entry
  int rec_pf = 0;      // and its record word (lane l < kRecInts of each wave: word l)
  bool have_pf = false;
  for (;;) {  // dynamic queue: list lengths (and costs) differ by orders of magnitude
    if (tid == 0) {
      s_w = w1;
      s_wn = w2;
      w1 = w2;
      if (w2 < count) w2 = atomicAdd(next_work, 1);
    }
    __syncthreads();
    const int w = s_w, wn = s_wn;
    __syncthreads();
    if (w >= count) break;
    int32_t jw;
    int recv;
    if (PFX_Q_PF && have_pf) {
      jw = jw_pf;
      recv = rec_pf;
    } else {
      jw = work[w];
      recv = lane < kRecInts ? out.qrec[(int64_t)(jw & (kListMode - 1)) * kRecInts + lane] : 0;
    }
    const bool pf = PFX_Q_PF && wn < count;
    const int32_t jn = pf ? work[wn] : 0;  // (its record load is issued after the first phase)
    const bool from_list = (jw & kListMode) != 0;  // the list is in place, unsorted: sort only
    const int32_t j = jw & (kListMode - 1);
    // the query's record (its block: the runs its list entries refer to)
    Runs R;
    int32_t qp;
    float4 q;
    qrec_unpack(recv, R, qp, q);
    if (tid == 0) s_count = 0;
    for (int b = tid; b < NB; b += NT) bcount[b] = 0;
    __syncthreads();
    TPROF_T(q0);
    if (from_list) {
      // entries -> positions and d2, four per thread in flight (a list past the buffer's end is
      // left alone: the build reruns with a larger buffer)
      const int kl = out.cnt[j];
      const int64_t lo = out.off[j];
      const int kk = (unsigned long long)(lo + kl) <= out.cap && kl <= CAP ? kl : 0;
      if (tid == 0) {
        s_count = kk;
        s_base = (unsigned long long)lo;
        if (kl > CAP) atomicMax(err, kl);
      }
      for (int e0 = tid; e0 < kk; e0 += UL * NT) {
        int32_t pos[UL];
        float4 c[UL];
#pragma unroll
        for (int u = 0; u < UL; ++u) {
          const uint32_t en = out.list[lo + min(e0 + NT * u, kk - 1)];
          const int r = entry_run(en);
          int32_t st = R.start[0];
#pragma unroll
          for (int v = 1; v < 9; ++v) st = r == v ? R.start[v] : st;
          pos[u] = st + (int32_t)entry_off(en);
          c[u] = g.sp[pos[u]];
        }
#pragma unroll
        for (int u = 0; u < UL; ++u) {
          const int e = e0 + NT * u;
          if (e < kk) {
            const float d2 = flann_d2(q.x, q.y, q.z, c[u].x, c[u].y, c[u].z);
            hits[e] = (uint32_t)pos[u];
            hd[e] = __float_as_uint(d2);
            const int b = (int)(d2 * bscale);
            if (sorted) atomicAdd(&bcount[b < NB ? b : NB - 1], 1);
          }
        }
      }
    }
    for (int t0 = 0; !from_list && t0 < R.pref[9]; t0 += UL * NT) {  // UL candidates per thread in flight
      float4 c[UL];
      int32_t pos[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const int t = t0 + u * NT + tid;
        pos[u] = t < R.pref[9] ? run_pos(R, t) : -1;
        c[u] = g.sp[pos[u] < 0 ? 0 : pos[u]];
      }
      // one slot reservation per wave and round (the four ballots' total) instead of one per
      // ballot, and the sort's bucket counts taken here instead of in a pass over the hits
      float d2[UL];
      uint64_t m[UL];
      int tot = 0;
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        d2[u] = flann_d2(q.x, q.y, q.z, c[u].x, c[u].y, c[u].z);
        m[u] = __ballot(pos[u] >= 0 && d2[u] < rr);
        tot += __popcll(m[u]);
      }
      int base = 0;
      if (lane == 0 && tot) base = atomicAdd(&s_count, tot);
      base = __shfl(base, 0);
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        if ((m[u] >> lane) & 1) {
          const int slot = base + __popcll(m[u] & lanemask_lt());
          if (slot < CAP) {
            hits[slot] = (uint32_t)pos[u];
            hd[slot] = __float_as_uint(d2[u]);
            const int b = (int)(d2[u] * bscale);
            if (sorted) atomicAdd(&bcount[b < NB ? b : NB - 1], 1);
          }
        }
        base += __popcll(m[u]);
      }
    }
    __syncthreads();
    // the next item's record (its work entry has arrived with this item's loads)
    rec_pf = pf && lane < kRecInts ? out.qrec[(int64_t)(jn & (kListMode - 1)) * kRecInts + lane] : 0;
    jw_pf = jn;
    have_pf = pf;
    TPROF_T(q1);
    if (!GLOBAL && CAP == kCapQuery) { TPROF_ADD(20, q0, q1); }
    const int k = s_count;
    if (k > CAP) {
      if (tid == 0) {
        if (tq) {
          const int t = query_tier(k);
          tq->q[t][atomicAdd(tq->n[t], 1)] = j;
        } else {
          atomicMax(err, k);
        }
      }
      __syncthreads();
      continue;
    }
    // compact (16-bit) output: a compact build, runs of <= 4096 points, and a list the lane-per-query
    // chains read (<= kLaneMaxCompact: k_normals_long reads 32-bit lists only)
    bool c16 = out.compact != 0 && k <= kLaneMaxCompact;
#pragma unroll
    for (int r = 0; r < 9; ++r) c16 = c16 && R.pref[r + 1] - R.pref[r] <= kCompactRun;
    if (tid == 0 && from_list && c16) {  // sorted in place: the same slots, as 16-bit entries
      out.off[j] = 2 * (int64_t)s_base;
      out.lg[j] = kLgCompact;
    }
    // list slots from the workgroup's arena: a refill's atomic is issued here and its result read
    // by commit() after the sort's scatter (its round trip overlaps the scan and the scatter)
    const unsigned long long need = c16 ? ((unsigned long long)k + 1) >> 1 : (unsigned long long)k;
    unsigned long long arena_new = 0, arena_res = 0;  // thread 0's
    if (tid == 0 && !from_list && need > arena_left) {
      arena_res = need > (unsigned long long)kArenaQuery ? need : (unsigned long long)kArenaQuery;
      arena_new = atomicAdd(out.cursor, arena_res);
    }
    auto commit = [&]() {  // thread 0, before the barrier that precedes the list write
      if (tid == 0 && !from_list) {
        if (arena_res) {
          arena_base = arena_new;
          arena_left = arena_res;
        }
        s_base = arena_base;
        arena_base += need;
        arena_left -= need;
        wg_total += (unsigned long long)k;  // (neighbours, not list words)
        if (k > kLongList) {
          wg_long += (unsigned long long)k;
          ++wg_long_n;
        }
        out.off[j] = c16 ? 2 * (int64_t)s_base : (int64_t)s_base;
        out.cnt[j] = k;
        out.lg[j] = c16 ? kLgCompact : 0;
      }
    };
    // the entry at bucket-order slot s of position p goes to list slot st + rank
    auto put = [&](int64_t off, int slot, uint32_t p) {
      if (c16) reinterpret_cast<uint16_t*>(out.list)[2 * off + slot] = (uint16_t)pos_entry16(R, (int32_t)p);
      else out.list[off + slot] = pos_entry(R, (int32_t)p);
    };
    auto bucket_of = [&](uint32_t d) {
      const int b = (int)(__uint_as_float(d) * bscale);
      return b < NB ? b : NB - 1;
    };
    if (sorted && k > 1) {  // (the bucket counts were taken with the hits)
      bucket_scan<NB, NT>(bcount, GLOBAL ? bcount : bpos, wsum);
      __syncthreads();
      TPROF_T(q1s);
      if (!GLOBAL && CAP == kCapQuery) { TPROF_ADD(24, q1, q1s); TPROF_ADD(27, 0, (long long)from_list); }
      if constexpr (!GLOBAL) {
        // bucket scatter in place through registers (8 B of LDS per entry)
        constexpr int PT = CAP / NT;
        uint32_t rp[PT], rd[PT];
#pragma unroll
        for (int u = 0; u < PT; ++u) {
          const int e = tid + u * NT;
          rp[u] = e < k ? hits[e] : 0u;
          rd[u] = e < k ? hd[e] : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PT; ++u) {
          if (tid + u * NT < k) {
            const int slot = atomicAdd(&bpos[bucket_of(rd[u])], 1);
            hd[slot] = rd[u];
            hits[slot] = rp[u];
          }
        }
        commit();
        __syncthreads();
        TPROF_T(q1c);
        if (CAP == kCapQuery) { TPROF_ADD(25, q1s, q1c); }
        const int64_t off = (int64_t)s_base;
        // (a compact list occupies (k + 1) / 2 words: the words its slot reservation counted)
        const bool fits = (unsigned long long)(off + (c16 ? (k + 1) / 2 : k)) <= out.cap;
        // exact (d2, caller index) rank inside the bucket, written straight to the list
        // (round 6: the bucket's first four entries read together -- buckets hold ~2-4 -- the rest
        // one by one; it read every mate in turn, one dependent LDS round trip each)
        for (int s = tid; s < k; s += NT) {
          const uint32_t d = hd[s], p = hits[s];
          const int b = bucket_of(d);
          const int en = bpos[b], st = en - bcount[b];
          uint32_t dv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) dv[j] = st + j < en ? hd[st + j] : 0xffffffffu;  // (never < or == d)
          int rank = 0;
          bool tie = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            rank += dv[j] < d ? 1 : 0;
            tie |= dv[j] == d && st + j != s;
          }
          for (int v = st + 4; v < en; ++v) {
            const uint32_t x = hd[v];
            rank += x < d ? 1 : 0;
            tie |= x == d && v != s;
          }
          if (tie) {  // equal d2: the caller index decides (FLANN); rare
            const int32_t mine = g.perm[p];
            for (int v = st; v < en; ++v)
              if (v != s && hd[v] == d && g.perm[hits[v]] < mine) ++rank;
          }
          if (fits) put(off, st + rank, p);
        }
        __syncthreads();
        TPROF_T(q2);
        if (CAP == kCapQuery) {
          TPROF_ADD(21, q1, q2); TPROF_ADD(22, 0, (long long)k); TPROF_ADD(23, 0, (long long)R.pref[9]);
          TPROF_ADD(26, q1c, q2);
        }
        continue;
      } else {
        // scatter to bucket order (scratch), UL entries per thread in flight; bcount holds the
        // bucket starts, advanced to the ends
        for (int e0 = tid; e0 < k; e0 += UL * NT) {
          uint32_t dd[UL], pp[UL];
#pragma unroll
          for (int u = 0; u < UL; ++u) {
            const int e = min(e0 + u * NT, k - 1);
            dd[u] = hd[e];
            pp[u] = hits[e];
          }
#pragma unroll
          for (int u = 0; u < UL; ++u) {
            if (e0 + u * NT < k) {
              const int slot = atomicAdd(&bcount[bucket_of(dd[u])], 1);
              sdv[slot] = dd[u];
              spv[slot] = pp[u];
            }
          }
        }
        commit();
        __syncthreads();
        const int64_t off = (int64_t)s_base;
        const bool fits = (unsigned long long)(off + (c16 ? (k + 1) / 2 : k)) <= out.cap;
        // rank pass in windows of kRankWindow bucket-order entries staged in LDS (it read every
        // bucket mate from the scratch: one dependent L2 round trip per mate); a bucket that
        // straddles the window reads its mates from the scratch
        for (int w0 = 0; w0 < k; w0 += kRankWindow) {
          const int wn = min(kRankWindow, k - w0);
          constexpr int WPT = kRankWindow / NT;
          uint32_t wv_[WPT];
#pragma unroll
          for (int u = 0; u < WPT; ++u) wv_[u] = sdv[w0 + min(tid + u * NT, wn - 1)];
#pragma unroll
          for (int u = 0; u < WPT; ++u) wd[tid + u * NT] = wv_[u];
          __syncthreads();
          for (int s = w0 + tid; s < w0 + wn; s += NT) {
            const uint32_t p = spv[s];
            const uint32_t d = wd[s - w0];
            const int b = bucket_of(d);
            const int en = bcount[b], st = b ? bcount[b - 1] : 0;
            int rank = 0;
            bool tie = false;
            if (st >= w0 && en <= w0 + wn) {
              uint32_t dv[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) dv[j] = st + j < en ? wd[st + j - w0] : 0xffffffffu;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                rank += dv[j] < d ? 1 : 0;
                tie |= dv[j] == d && st + j != s;
              }
              for (int v = st + 4; v < en; ++v) {
                const uint32_t x = wd[v - w0];
                rank += x < d ? 1 : 0;
                tie |= x == d && v != s;
              }
            } else {
              for (int v = st; v < en; ++v) {
                const uint32_t dv = sdv[v];
                rank += dv < d ? 1 : 0;
                tie |= dv == d && v != s;
              }
            }
            if (tie) {  // equal d2: the caller index decides (FLANN); rare
              const int32_t mine = g.perm[p];
              for (int v = st; v < en; ++v)
                if (v != s && sdv[v] == d && g.perm[spv[v]] < mine) ++rank;
            }
            if (fits) put(off, st + rank, p);
          }
          __syncthreads();  // the window is rewritten by the next one
        }
        continue;
      }
    }
    commit();
    __syncthreads();
    const int64_t off = (int64_t)s_base;
    if ((unsigned long long)(off + (c16 ? (k + 1) / 2 : k)) <= out.cap)
      for (int m = tid; m < k; m += NT) put(off, m, hits[m]);
    __syncthreads();
  }
  if (tid == 0) {
    if (wg_total) atomicAdd(out.cursor + 1, wg_total);
    if (wg_long_n) {
      atomicAdd(out.cursor + 2, wg_long);
      atomicAdd(out.cursor + 3, wg_long_n);
    }
  }
  TPROF_FLUSH;
}

std::string bname(const char* tag, const char* what) { return std::string(tag) + "_" + what; }

// the pinned readback block of a list build
struct ListsRb {
  int cnt[kNCounters];
  int oob;
  int pad;
  unsigned long long cur[4];
  int64_t nq;
};

}  // namespace

// The 4k-8k and 8k-16k per-query tiers need 72 / 144 KB of LDS per workgroup, so even an empty
// launch waits until whole CUs are free of the concurrent NARF stream's workgroups (150-200 us on
// the headline's critical path, whose lists never reach these tiers).  A tier is launched while
// one of the last 16 builds of this (context, tag) had work for it (always on the first build);
// a skipped tier that turns out to have work is launched after the readback (or, for a deferred
// build, the lists are rebuilt exactly), so results never depend on the hint.
static bool mid_tier_wanted(pfx_ctx* ctx, const char* tag, const char* which) {
  const auto it = ctx->stats.find(std::string(tag) + which);
  return it == ctx->stats.end() || it->second > 0;
}
static void note_mid_tiers(pfx_ctx* ctx, const char* tag, const int* h_cnt) {
  static const char* const keys[3] = {"_hint_mid8", "_hint_mid", "_hint_wide"};
  for (int t = 0; t < 3; ++t) {
    const std::string key = std::string(tag) + keys[t];
    const int work = h_cnt[t == 0 ? 14 : (t == 1 ? 12 : 16)];
    int64_t& v = ctx->stats[key];
    v = work > 0 ? 16 : std::max<int64_t>(0, v - 1);
  }
}

bool build_lists_check(pfx_ctx* ctx, const Grid& G, NbLists& out, const char* tag) {
  hipStream_t st = ctx->stream;
  auto B = [&](const char* what) -> DevBuf& { return ctx->bufs[bname(tag, what)]; };
  ListsRb* rb = ctx->readback<ListsRb>();
  PFX_HIP(hipMemcpyAsync(rb->cnt, B("counters").ptr, sizeof(rb->cnt), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(rb->cur, B("cursor").ptr, sizeof(rb->cur), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(&rb->nq, B("nq").ptr, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  rb->oob = 0;
  if (G.oob) PFX_HIP(hipMemcpyAsync(&rb->oob, G.oob, sizeof(int), hipMemcpyDeviceToHost, st));
  ctx->sync_spin(st);
  const int* h_cnt = rb->cnt;
  const unsigned long long* h_cur = rb->cur;
  const DevBuf& lb = B("list");
  if (rb->oob > 0) return false;                                    // speculative grid too small
  if (h_cur[0] > lb.bytes / sizeof(uint32_t)) return false;         // list buffer too small
  if (!B("scratch").ptr && h_cnt[3] > 0) return false;              // first very long lists
  const int ran = (int)ctx->stats[std::string(tag) + "_ran_mid_tiers"];
  note_mid_tiers(ctx, tag, h_cnt);
  if ((!(ran & 1) && h_cnt[14] > 0) || (!(ran & 2) && h_cnt[12] > 0) || (!(ran & 4) && h_cnt[16] > 0))
    return false;  // a skipped tier had work
  if (h_cnt[4] > 0)
    throw Error(PFX_ERR_CAPACITY, std::string(tag) + ": a query has " + std::to_string(h_cnt[4]) +
                                      " neighbours (> " + std::to_string(kCapHuge) + " supported)");
  out.nq = rb->nq;
  out.nq_dev = nullptr;
  out.total = (int64_t)h_cur[1];
  out.long_total = (int64_t)h_cur[2];
  out.long_nq = (int64_t)h_cur[3];
  out.slots = (int64_t)h_cur[0];
  ctx->stats[std::string(tag) + "_tiles_sparse"] = h_cnt[0];
  ctx->stats[std::string(tag) + "_tiles_dense"] = h_cnt[1];
  ctx->stats[std::string(tag) + "_single"] = h_cnt[2];
  ctx->stats[std::string(tag) + "_huge"] = h_cnt[3];
  ctx->stats[std::string(tag) + "_mid"] = h_cnt[12];
  ctx->stats[std::string(tag) + "_wide"] = h_cnt[16];
  ctx->stats[std::string(tag) + "_slots"] = (int64_t)h_cur[0];
  ctx->stats[std::string(tag) + "_list_words"] = (int64_t)(lb.bytes / sizeof(uint32_t));
  return true;
}

void build_lists(pfx_ctx* ctx, const Grid& G, const uint8_t* mask, double radius, bool sorted, NbLists& out,
                 const char* tag, bool defer, int want, bool compact, bool gate) {
  hipStream_t st = ctx->stream;
  const int64_t n = G.n;
  GridView g = view(G);
  const float rr = (float)(radius * radius);
  out = NbLists();
  if (n == 0) return;
  if (n >= (int64_t(1) << 28))
    throw Error(PFX_ERR_CAPACITY, std::string(tag) + ": neighbour lists support < 2^28 points");
  auto B = [&](const char* what) -> DevBuf& { return ctx->bufs[bname(tag, what)]; };
  int32_t* qpos = B("qpos").as<int32_t>(n);
  int64_t* d_nq = B("nq").as<int64_t>(1);
  uint8_t* flags = B("flags").as<uint8_t>(n);
  int32_t* seg = B("seg").as<int32_t>(n);
  int32_t* tiles = B("tiles").as<int32_t>(n);
  int64_t* d_ntiles = B("ntiles").as<int64_t>(1);
  // tile records: small at [0, n), sparse at [n, 2n) upward, dense at [n, 2n) downward
  int32_t* recs = B("recs").as<int32_t>((size_t)2 * n * kRecInts);
  int32_t* single = B("single").as<int32_t>(n);
  int32_t* huge = B("huge").as<int32_t>(n);
  int64_t* off = B("off").as<int64_t>(n);
  int32_t* cnt = B("cnt").as<int32_t>(n);
  uint8_t* lgs = B("lg").as<uint8_t>(n);
  // counters: 0 sparse tiles, 1 dense tiles, 2 per-query work, 3 huge work, 4 max k over cap,
  // 5 / 7 sparse / dense tile queue heads, 6 unused, 8 / 9 per-query / huge work queue heads,
  // 10 small tiles, 11 their queue head,
  // 12 mid work (lists of 8k-16k entries), 13 its queue head, 14 mid8 work (4k-8k), 15 its head,
  // 16 wide-tile work (queued by the classifier), 17 its queue head
  int* counters = B("counters").as<int>(kNCounters);
  int32_t* wq = B("wide").as<int32_t>((size_t)n);  // wide-tile work: record indices
  int32_t* mid = B("mid").as<int32_t>(n);
  int32_t* mid8 = B("mid8").as<int32_t>(n);
  int32_t* qrec = B("qrec").as<int32_t>((size_t)n * kRecInts);
  unsigned long long* cursor = B("cursor").as<unsigned long long>(4);
  size_t t1 = 0, t2 = 0, t3 = 0;
  PFX_HIP(rocprim::select(nullptr, t1, rocprim::counting_iterator<int32_t>(0), flags, qpos, d_nq, (size_t)n, st));
  PFX_HIP(rocprim::inclusive_scan(nullptr, t2, seg, seg, (size_t)n, rocprim::maximum<int32_t>(), st));
  PFX_HIP(rocprim::select(nullptr, t3, rocprim::counting_iterator<int32_t>(0), flags, tiles, d_ntiles, (size_t)n,
                          st));
  void* tmp = B("tmp").get(std::max(t1, std::max(t2, t3)) + 16);
  const unsigned nb = (unsigned)ceil_div(n, 256);
  unsigned long long* cursor0 = B("cursor").as<unsigned long long>(4);
  // sort-only work (kListMode) of the lists the tile kernels write unsorted, by length; the
  // kernels read the queues from a device copy written by k_list_init
  constexpr bool use_mid8 = true;  // the 4k-8k tier (round 3; without it those lists take the 16k tier)
  const TierQ tq{{single, use_mid8 ? mid8 : mid, mid, huge},
                 {counters + 2, counters + (use_mid8 ? 14 : 12), counters + 12, counters + 3}};
  TierQ* tq_dev = static_cast<TierQ*>(B("tierq").get(sizeof(TierQ)));
  {
    TimeScope ts(ctx, std::string(tag) + "_tiles");
    if (mask) {
      k_list_init<<<1, 256, 0, st>>>(nullptr, 0, nullptr, d_nq, counters, kNCounters, cursor0, tq, tq_dev);
      k_mask_flags<<<nb, 256, 0, st>>>(G.perm, G.skeys, n, (uint64_t)G.ncells, mask, want, flags);
      PFX_HIP(rocprim::select(tmp, t1, rocprim::counting_iterator<int32_t>(0), flags, qpos, d_nq, (size_t)n, st));
    } else {
      // every finite point, in cell order: sorted positions [0, cell_start[ncells])
      k_list_init<<<nb, 256, 0, st>>>(qpos, n, G.cell_start + G.ncells, d_nq, counters, kNCounters, cursor0, tq,
                                      tq_dev);
    }
    k_seg_marks<<<nb, 256, 0, st>>>(qpos, G.skeys, d_nq, seg);
    PFX_HIP(rocprim::inclusive_scan(tmp, t2, seg, seg, (size_t)n, rocprim::maximum<int32_t>(), st));
    k_tile_flags<<<nb, 256, 0, st>>>(seg, d_nq, flags, n);
    PFX_HIP(rocprim::select(tmp, t3, rocprim::counting_iterator<int32_t>(0), flags, tiles, d_ntiles, (size_t)n, st));
    k_tile_class<<<nb, 256, 0, st>>>(g, qpos, G.skeys, d_nq, tiles, d_ntiles, recs, n, wq, counters);
    check_launch("nblist tiles");
  }
  const size_t lds_q = sizeof(uint32_t) * 2 * kCapQuery;
  PFX_HIP(hipFuncSetAttribute((const void*)k_nb_query<kCapQuery, kBucketsQuery, false, kNtQuery, PFX_Q_WPE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_q));
  const size_t lds_m8 = sizeof(uint32_t) * 2 * kCapMid8;
  PFX_HIP(hipFuncSetAttribute((const void*)k_nb_query<kCapMid8, kBucketsMid8, false, kNtMid8, kNtMid8 / 128>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_m8));
  const size_t lds_m = sizeof(uint32_t) * 2 * kCapMid;
  PFX_HIP(hipFuncSetAttribute((const void*)k_nb_query<kCapMid, kBucketsMid, false, kNtMid, kNtMid / 256>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_m));
  DevBuf& lb = B("list");
  if (!lb.ptr) {
    // (PFX_LIST_WORDS: the first buffer's size in 32-bit words, for tests of the capacity guards
    // and the regrow path; the buffer grows as needed either way)
    size_t words = 64 * (size_t)(n + 1);
    if (const char* e = std::getenv("PFX_LIST_WORDS")) words = std::max<size_t>(256, std::strtoull(e, nullptr, 10));
    lb.get(sizeof(uint32_t) * words);
  }
  const int isort = sorted ? 1 : 0;
  // tiles per queue fetch, per class: many cheap small tiles amortise the queue atomic over 4,
  // the heavy sparse / dense tiles balance better with 2 / 1 at ~1M queries (sweep S/P/D on the
  // 1M-pt room, configs[1] and Harris3D: 4/4/4 162.7, 31.7, 230.4; 4/2/2 166.0, 33.2, 230.3;
  // 4/2/1 166.6, 34.9, 229.6; 2/2/2 166.5, 33.5, 208.4 Mpoints/s), while the 10M-pt dense
  // variant, with ~10x the heavy tiles per workgroup, wants 4 again (P/D 2/1 8.83, 2/2 9.11,
  // 2/4 9.22, 4/4 9.25 Mpoints/s): the heavy classes take n / 2M tiles per fetch, clamped to
  // [2, 4] / [1, 4]
  const int heavy = (int)std::min<int64_t>(4, n >> 21);
  const int ch_small = 4, ch_sparse = std::max(2, heavy), ch_dense = std::max(1, heavy);
  for (int attempt = 0; attempt < 3; ++attempt) {
    ListOut lo{off, cnt, lgs, static_cast<uint32_t*>(lb.ptr), cursor, lb.bytes / sizeof(uint32_t), compact ? 1 : 0, qrec};
    if (attempt) {  // (the first attempt's cursors were zeroed by k_list_init)
      PFX_HIP(hipMemsetAsync(cursor, 0, 4 * sizeof(unsigned long long), st));
      PFX_HIP(hipMemsetAsync(counters + 2, 0, sizeof(int), st));  // per-query work
      PFX_HIP(hipMemsetAsync(counters + 3, 0, 3 * sizeof(int), st));  // huge, max k, sparse queue
      PFX_HIP(hipMemsetAsync(counters + 7, 0, 3 * sizeof(int), st));  // dense, query, huge queues
      PFX_HIP(hipMemsetAsync(counters + 11, 0, 5 * sizeof(int), st));  // small queue, mid / mid8 work + queues
      PFX_HIP(hipMemsetAsync(counters + 17, 0, sizeof(int), st));  // wide queue (its work: the classifier's)
    }
    // one synchronisation per call: counters, cursors and the query count in one pinned block
    ListsRb* rb = ctx->readback<ListsRb>();
    auto read_back = [&] {
      PFX_HIP(hipMemcpyAsync(rb->cnt, counters, sizeof(rb->cnt), hipMemcpyDeviceToHost, st));
      PFX_HIP(hipMemcpyAsync(rb->cur, cursor, sizeof(rb->cur), hipMemcpyDeviceToHost, st));
      PFX_HIP(hipMemcpyAsync(&rb->nq, d_nq, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      ctx->sync_spin(st);
    };
    DevBuf& hs = B("scratch");
    auto launch_mid8 = [&] {
      k_nb_query<kCapMid8, kBucketsMid8, false, kNtMid8, kNtMid8 / 128><<<256 * 2, kNtMid8, lds_m8, st>>>(
          g, mid8, counters + 14, rr, (float)kBucketsMid8 / rr, isort, lo, tq_dev, counters + 4, nullptr,
          counters + 15);
      check_launch("nblist 8k lists");
    };
    auto launch_mid = [&] {
      k_nb_query<kCapMid, kBucketsMid, false, kNtMid, kNtMid / 256><<<256, kNtMid, lds_m, st>>>(
          g, mid, counters + 12, rr, (float)kBucketsMid / rr, isort, lo, tq_dev, counters + 4, nullptr,
          counters + 13);
      check_launch("nblist 16k lists");
    };
    // (see mid_tier_wanted; a rerun launches every tier)
    // (bit 4: the wide-tile kernel -- an empty launch of it also waits for whole CUs beside NARF)
    const int ran_mids = attempt ? 7 : ((use_mid8 && mid_tier_wanted(ctx, tag, "_hint_mid8") ? 1 : 0) |
                                        (mid_tier_wanted(ctx, tag, "_hint_mid") ? 2 : 0) | (use_mid8 ? 0 : 1) |
                                        (mid_tier_wanted(ctx, tag, "_hint_wide") ? 4 : 0));
    ctx->stats[std::string(tag) + "_ran_mid_tiers"] = ran_mids;
    // one 4 MB scratch slice per workgroup of the persistent huge tier: as many workgroups as
    // slices (sized from the queue length the first time it was seen, 256 to kHugeBlocks: a
    // context holds 1-4 GB only when that many lists above 16k entries exist)
    const size_t huge_slice = sizeof(uint32_t) * 4 * (size_t)kCapHuge;
    auto huge_blocks = [&] { return (unsigned)std::min<size_t>(kHugeBlocks, hs.bytes / huge_slice); };
    auto huge_alloc = [&](int count) {
      hs.get(huge_slice * (size_t)std::min(kHugeBlocks, std::max(256, count)));
    };
    auto launch_huge = [&] {
      k_nb_query<kCapHuge, kBucketsHuge, true, kNtHuge, 4><<<huge_blocks(), kNtHuge, 0, st>>>(
          g, huge, counters + 3, rr, (float)kBucketsHuge / rr, isort, lo, nullptr, counters + 4,
          static_cast<uint32_t*>(hs.ptr), counters + 9);
      check_launch("nblist huge lists");
    };
    if (gate && ctx->lists_gate) {  // pfx_normals_gate_dev: the caller's event, once, right before the list kernels
      // (after the list set-up above, which therefore overlaps the gated stage)
      PFX_HIP(hipStreamWaitEvent(st, ctx->lists_gate, 0));
      ctx->lists_gate = nullptr;
    }
    {
      TimeScope ts(ctx, std::string(tag) + "_lists");
      {
        TimeScope t0(ctx, std::string(tag) + "_lists_small");
        k_nb_tile<kTcapSmall, 256, kTcapSmall, true><<<256 * 4 * 2, 256, 0, st>>>(
            g, qpos, recs, kRecInts, counters + 10, rr, 256.0f / rr, isort, lo, tq_dev, counters + 11,
            ch_small);
      }
      {
        TimeScope t1(ctx, std::string(tag) + "_lists_sparse");
        k_nb_tile<512, 256, kTcapSparse, true><<<256 * 3 * 4, 256, 0, st>>>(
            g, qpos, recs + (size_t)n * kRecInts, kRecInts, counters + 0, rr, 256.0f / rr, isort, lo, tq_dev, counters + 5,
            ch_sparse);
      }
      {
        TimeScope t2(ctx, std::string(tag) + "_lists_dense");
        k_nb_tile<1024, 256, kTcapDense, false><<<256 * 2 * 4, 256, 0, st>>>(
            g, qpos, recs + (size_t)(2 * n - 1) * kRecInts, -kRecInts, counters + 1, rr, 256.0f / rr, isort, lo, tq_dev,
            counters + 7, ch_dense);
      }
      {
        TimeScope t4(ctx, std::string(tag) + "_lists_wide");
        if (ran_mids & 4) {
          k_nb_wide<<<256 * 4, 256, 0, st>>>(g, qpos, recs, wq, counters + 16, rr, isort, lo, tq_dev, counters + 17);
          check_launch("nblist wide tiles");
        }
      }
      {
        TimeScope t3(ctx, std::string(tag) + "_lists_query");
        k_nb_query<kCapQuery, kBucketsQuery, false, kNtQuery, PFX_Q_WPE><<<256 * 4, kNtQuery, lds_q, st>>>(
            g, single, counters + 2, rr, (float)kBucketsQuery / rr, isort, lo, tq_dev, counters + 4, nullptr,
            counters + 8);
        // lists of 4k-8k entries (dense clouds: ~14 % of the 10M-pt room's queries, 31 % of its
        // entries) in two 72 KB workgroups per CU instead of the 16k tier's one (10M-pt dense
        // variant: per-query lists 750 -> 650 ms, 1066 -> 968 ms per step; PFX_LIST_MID8=0 turns
        // it off); the count stays on the device
        if (use_mid8 && (ran_mids & 1)) launch_mid8();
        // lists of up to 16k entries, one 144 KB workgroup per CU
        if (ran_mids & 2) launch_mid();
        // beyond 16k entries: once the scratch exists the launch is unconditional (count on the
        // device); the first time, the readback below decides
        if (hs.ptr) launch_huge();
      }
      check_launch("nblist lists");
    }
    if (defer && attempt == 0) {  // consumers are launched before the readback (build_lists_check)
      int64_t* d_nq_eff = B("nq_eff").as<int64_t>(1);
      k_defer_gate<<<1, 64, 0, st>>>(counters, cursor, lo.cap, hs.ptr ? 1 : 0, ran_mids, G.oob, d_nq, d_nq_eff);
      check_launch("k_defer_gate");
      out.nq = n;
      out.nq_dev = d_nq_eff;
      out.qpos = qpos;
      out.off = off;
      out.cnt = cnt;
      out.lg = lgs;
      out.list = lo.list;
      out.compact = compact;
      out.list_cap = (int64_t)lo.cap;
      out.skeys = G.skeys;
      return;
    }
    read_back();
    if (!(ran_mids & 4) && rb->cnt[16] > 0) {  // skipped wide tiles had work: rerun with every tier
      note_mid_tiers(ctx, tag, rb->cnt);
      ++ctx->stats[std::string(tag) + "_wide_reruns"];
      continue;
    }
    if ((!(ran_mids & 1) && rb->cnt[14] > 0) || (!(ran_mids & 2) && rb->cnt[12] > 0)) {
      // a skipped per-query tier had work: run it and the tiers after it.  A launch that drained
      // its queue left the head at count + gridDim (every workgroup's last fetch overshoots), so
      // the head of each tier that already ran is first set back to the count it drained: the
      // relaunch then takes exactly the entries the catch-up launches append
      if (ran_mids & 2) PFX_HIP(hipMemcpyAsync(counters + 13, counters + 12, sizeof(int), hipMemcpyDeviceToDevice, st));
      if (hs.ptr) PFX_HIP(hipMemcpyAsync(counters + 9, counters + 3, sizeof(int), hipMemcpyDeviceToDevice, st));
      if (!(ran_mids & 1) && rb->cnt[14] > 0) launch_mid8();
      launch_mid();
      if (hs.ptr) launch_huge();
      read_back();
      ++ctx->stats[std::string(tag) + "_tier_catchups"];
    }
    note_mid_tiers(ctx, tag, rb->cnt);
    if (!hs.ptr && rb->cnt[3] > 0) {  // very long lists, first time: allocate the scratch and sort them
      huge_alloc(rb->cnt[3]);
      launch_huge();
      read_back();
    } else if (hs.ptr && rb->cnt[3] > (int)huge_blocks() && huge_blocks() < (unsigned)kHugeBlocks) {
      // more such lists than workgroups: more slices for the next build (this one has finished:
      // the readback synchronised)
      hs.release();
      huge_alloc(rb->cnt[3]);
    }
    int* h_cnt = rb->cnt;
    unsigned long long* h_cur = rb->cur;
    const int64_t h_nq = rb->nq;
    if (h_cnt[4] > 0)
      throw Error(PFX_ERR_CAPACITY, std::string(tag) + ": a query has " + std::to_string(h_cnt[4]) +
                                        " neighbours (> " + std::to_string(kCapHuge) + " supported)");
    if (h_cur[0] > lo.cap) {  // list buffer too small: grow (no copy needed) and rebuild once
      // The slot demand of a run is the entries + interleave padding (fixed by the input) + the
      // unused arena tails (scheduling-dependent, at most one arena per launched workgroup), so
      // this run's demand plus the tail bound always fits the rebuild.
      const size_t tails = (size_t)(256 * 4 * 2 + 256 * 3 * 4 + 256 * 2 * 4) * kArena +
                           (size_t)(256 * 4 + 256 * 4 + 256 * 2 + 256 + kHugeBlocks) * kArenaQuery;
      lb.release();
      lb.get(sizeof(uint32_t) * ((size_t)h_cur[0] + tails + ((size_t)1 << 20)));
      continue;
    }
    out.nq = h_nq;
    out.total = (int64_t)h_cur[1];
    out.long_total = (int64_t)h_cur[2];
    out.long_nq = (int64_t)h_cur[3];
    out.slots = (int64_t)h_cur[0];
    out.qpos = qpos;
    out.off = off;
    out.cnt = cnt;
    out.lg = lgs;
    out.list = lo.list;
    out.compact = compact;
    out.list_cap = (int64_t)lo.cap;
    out.skeys = G.skeys;
    ctx->stats[std::string(tag) + "_tiles_sparse"] = h_cnt[0];
    ctx->stats[std::string(tag) + "_tiles_dense"] = h_cnt[1];
    ctx->stats[std::string(tag) + "_single"] = h_cnt[2];
    ctx->stats[std::string(tag) + "_huge"] = h_cnt[3];
    ctx->stats[std::string(tag) + "_mid"] = h_cnt[12];
    ctx->stats[std::string(tag) + "_wide"] = h_cnt[16];
    ctx->stats[std::string(tag) + "_mid8"] = h_cnt[14];
    ctx->stats[std::string(tag) + "_slots"] = (int64_t)h_cur[0];  // list words reserved (entries + padding + arena tails)
    ctx->stats[std::string(tag) + "_list_words"] = (int64_t)lo.cap;
#ifdef PFX_SHOT_PROFILE
    {
      unsigned long long pr[28];
      PFX_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_tile_prof), sizeof(pr)));
      fprintf(stderr, "%s wave_sort cycles (wave 0): count %llu scan %llu scatter %llu rank %llu\n", tag, pr[8],
              pr[9], pr[10], pr[11]);
      fprintf(stderr, "%s tile cycles: sparse stage %llu test %llu sort %llu write %llu | dense - %llu test %llu "
              "sort %llu write %llu | small - %llu test %llu sort %llu write %llu (cumulative)\n", tag, pr[0], pr[1], pr[2],
              pr[3], pr[4], pr[5], pr[6], pr[7], pr[16], pr[17], pr[18], pr[19]);
      fprintf(stderr, "%s query cycles: test %llu sort+write %llu | entries %llu candidates %llu\n", tag, pr[20],
              pr[21], pr[22], pr[23]);
      fprintf(stderr, "%s query 4k-tier phases: scan %llu scatter %llu rank+write %llu | list-mode items %llu\n", tag,
              pr[24], pr[25], pr[26], pr[27]);
      unsigned long long pw[12];
      PFX_HIP(hipMemcpyFromSymbol(pw, HIP_SYMBOL(g_tile_prof2), sizeof(pw)));
      fprintf(stderr, "%s wave cycles (sum over waves): small sort %llu sortwait %llu staging %llu listwrite %llu | "
              "sparse %llu %llu %llu %llu | dense %llu %llu %llu %llu\n", tag, pw[0], pw[1], pw[2], pw[3], pw[4], pw[5],
              pw[6], pw[7], pw[8], pw[9], pw[10], pw[11]);
      static const unsigned long long zw[12] = {};
      PFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tile_prof2), zw, sizeof(zw)));
      static const unsigned long long zero[24] = {};
      PFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tile_prof), zero, sizeof(zero)));
    }
#endif
    return;
  }
  throw Error(PFX_ERR_DEVICE, std::string(tag) + ": neighbour-list buffer growth failed");
}

}  // namespace pfx
