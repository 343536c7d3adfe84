// pfx_neighbors.h -- device-side radius search on the uniform grid (pfx_grid.hip), producing
// FLANN's result: every p with ((0+dx^2)+dy^2)+dz^2 < (float)(r*r), dx = q - p,
// ordered by the 64-bit key (float_bits(d2) << 32) | caller_index  ==  (d2, index) ascending.
#pragma once
#include "pfx_device_math.h"
#include "pfx_internal.h"

namespace pfx {

__device__ __forceinline__ uint64_t nb_key(float d2, int32_t idx) {
  return ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)idx;
}
__device__ __forceinline__ float key_d2(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
__device__ __forceinline__ int32_t key_idx(uint64_t k) { return (int32_t)(uint32_t)(k & 0xffffffffu); }

// a wave-uniform float kept in an SGPR (the compiler cannot prove values loaded through LDS or
// indexed by threadIdx >> 6 uniform)
__device__ __forceinline__ float uniformf(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Inclusive prefix sum over the 64 lanes of a wave on DPP row shifts and row broadcasts (round 6):
// no LDS traffic -- __shfl_up is a ds_bpermute, so the six steps of a shuffle scan were six
// dependent LDS-pipe latencies in the middle of every list sort.  Every lane must be active.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8 (rows of 16 scanned)
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// slot for each calling lane in an array filled through `counter`: one atomic per wave, not per
// lane (same-address atomics serialise at the L2)
__device__ __forceinline__ int wave_push_slot(int* counter) {
  const uint64_t m = __ballot(1);
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  return base + __popcll(m & lanemask_lt());
}

// XCD-aware block remap: blocks b and b+8 share an XCD (observed round-robin placement);
// give each XCD a contiguous slice of the (spatially sorted) work so its L2 sees one region.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nblocks) {
  if (nblocks < 8 || (nblocks & 7)) return b;
  return (b & 7) * (nblocks >> 3) + (b >> 3);
}

// The 9 candidate runs (3 contiguous z-cells each) of the 3x3x3 block around a query.
struct Runs {
  int32_t start[9];
  int32_t pref[10];  // exclusive prefix of run lengths, pref[9] = total candidates
};

__device__ __forceinline__ void query_runs(const GridView& g, float qx, float qy, float qz, Runs& R) {
  int64_t cx = (int64_t)floor(((double)qx - g.ox) * g.inv);
  int64_t cy = (int64_t)floor(((double)qy - g.oy) * g.inv);
  int64_t cz = (int64_t)floor(((double)qz - g.oz) * g.inv);
  bool finite = isfinite(qx) && isfinite(qy) && isfinite(qz);
  cx = cx < -2 ? -2 : (cx > g.nx + 1 ? g.nx + 1 : cx);
  cy = cy < -2 ? -2 : (cy > g.ny + 1 ? g.ny + 1 : cy);
  cz = cz < -2 ? -2 : (cz > g.nz + 1 ? g.nz + 1 : cz);
  int64_t z0 = cz - 1 < 0 ? 0 : cz - 1;
  int64_t z1 = cz + 1 >= g.nz ? g.nz - 1 : cz + 1;
  // branch-free: all 18 cell_start loads issued together (clamped to a valid address, results
  // selected), not one dependent round trip per run behind a branch
  const bool zok = finite && z0 <= z1;
  int32_t acc = 0;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int64_t ix = cx + (r / 3) - 1, iy = cy + (r % 3) - 1;
    const bool ok = zok && ix >= 0 && ix < g.nx && iy >= 0 && iy < g.ny;
    const int64_t base = ok ? (ix * g.ny + iy) * g.nz : 0;
    const int32_t a = g.cell_start[base + (ok ? z0 : 0)];
    const int32_t b = g.cell_start[base + (ok ? z1 + 1 : 0)];
    R.start[r] = ok ? a : 0;
    R.pref[r] = acc;
    acc += ok ? b - a : 0;
  }
  R.pref[9] = acc;
}

// Run r of the block of grid cell `key` (the cell a grid point lies in): start position and length.
__device__ __forceinline__ void block_run(const GridView& g, uint32_t key, int r, int32_t& s, int32_t& len) {
  const int64_t iz = key % g.nz, iy = (key / g.nz) % g.ny, ix = key / ((uint64_t)g.nz * g.ny);
  const int64_t bx = ix + (r / 3) - 1, by = iy + (r % 3) - 1;
  const int64_t z0 = iz - 1 < 0 ? 0 : iz - 1, z1 = iz + 1 >= g.nz ? g.nz - 1 : iz + 1;
  // branch-free (clamped address, selected result): block_runs' loads are issued together
  const bool ok = bx >= 0 && bx < g.nx && by >= 0 && by < g.ny;
  const int64_t base = ok ? (bx * g.ny + by) * g.nz : 0;
  const int32_t a = g.cell_start[base + (ok ? z0 : 0)];
  const int32_t b = g.cell_start[base + (ok ? z1 + 1 : 0)];
  s = ok ? a : 0;
  len = ok ? b - a : 0;
}

__device__ __forceinline__ int block_runs(const GridView& g, uint32_t key, Runs& R) {
  int acc = 0;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    block_run(g, key, r, s, len);
    R.start[r] = s;
    R.pref[r] = acc;
    acc += len;
  }
  R.pref[9] = acc;
  return acc;
}

// position of candidate t of the block: t + (start[r] - pref[r]) for its run r -- one compare and
// one select per run boundary (the differences are per-block scalars when R is uniform)
__device__ __forceinline__ int32_t run_pos(const Runs& R, int32_t t) {
  int32_t d = R.start[0] - R.pref[0];
#pragma unroll
  for (int r = 1; r < 9; ++r) d = t >= R.pref[r] ? R.start[r] - R.pref[r] : d;
  return t + d;
}

// run entry (pfx_nblist.h) of candidate t of the block: (run << 28) | offset within the run,
// = t + ((r << 28) - pref[r]) in wrapping u32 (the offset is < 2^28)
__device__ __forceinline__ uint32_t run_entry(const Runs& R, int32_t t) {
  uint32_t d = 0u - (uint32_t)R.pref[0];
#pragma unroll
  for (int r = 1; r < 9; ++r) d = t >= R.pref[r] ? ((uint32_t)r << 28) - (uint32_t)R.pref[r] : d;
  return (uint32_t)t + d;
}

// compact (16-bit) run entry: (r << 12) | off, for blocks whose runs hold <= kCompactRun points
constexpr int kCompactRun = 4096;
__device__ __forceinline__ uint16_t run_entry16(const Runs& R, int32_t t) {
  uint32_t d = 0u - (uint32_t)R.pref[0];
#pragma unroll
  for (int r = 1; r < 9; ++r) d = t >= R.pref[r] ? ((uint32_t)r << 12) - (uint32_t)R.pref[r] : d;
  return (uint16_t)((uint32_t)t + d);
}

// Gather the neighbours of q into keys[0..min(k,cap)) (unsorted); returns k (may exceed cap).
// Executed by every thread of the block (nthreads = blockDim.x, a multiple of 64); uses
// `s_count` (LDS int) for the cross-wave compaction cursor.
__device__ __forceinline__ int gather_keys(const GridView& g, float qx, float qy, float qz, float rr,
                                           uint64_t* keys, int cap, int* s_count) {
  Runs R;
  query_runs(g, qx, qy, qz, R);
  const int tid = threadIdx.x, nth = blockDim.x;
  if (tid == 0) *s_count = 0;
  __syncthreads();
  const int32_t T = R.pref[9];
  // four candidates per thread in flight (branch-free: clamped positions, unconditional loads) and
  // one compaction cursor reservation per wave and round: a dependent global round trip per
  // candidate batch instead of per candidate (SHOT's sorted search scans ~5k candidates a query)
  constexpr int U = 4;
  for (int32_t t0 = 0; t0 < T; t0 += U * nth) {
    int32_t p[U];
    float4 c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t t = t0 + u * nth + tid;
      p[u] = t < T ? run_pos(R, t) : -1;
      c[u] = g.sp[p[u] < 0 ? 0 : p[u]];
    }
    int32_t id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) id[u] = g.perm[p[u] < 0 ? 0 : p[u]];
    float d2[U];
    uint64_t m[U];
    int tot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d2[u] = flann_d2(qx, qy, qz, c[u].x, c[u].y, c[u].z);
      m[u] = __ballot(p[u] >= 0 && d2[u] < rr);
      tot += __popcll(m[u]);
    }
    int base = 0;
    if ((tid & 63) == 0 && tot) base = atomicAdd(s_count, tot);
    base = __shfl(base, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((m[u] >> (tid & 63)) & 1) {
        const int pos = base + __popcll(m[u] & lanemask_lt());
        if (pos < cap) keys[pos] = nb_key(d2[u], id[u]);
      }
      base += __popcll(m[u]);
    }
  }
  __syncthreads();
  int k = *s_count;
  __syncthreads();  // every thread has read the cursor before the next call resets it
  return k;
}

// In-place ascending bitonic sort of keys[0..P), P a power of two >= 2 (pad with ~0ull).
__device__ __forceinline__ void bitonic_sort(uint64_t* keys, int P) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (P >> 1); i += nth) {
        int lo = ((i / stride) * stride << 1) + (i & (stride - 1));
        int hi = lo + stride;
        bool asc = (lo & size) == 0;
        uint64_t a = keys[lo], b = keys[hi];
        if ((a > b) == asc) { keys[lo] = b; keys[hi] = a; }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int next_pow2(int k) {
  int P = 2;
  while (P < k) P <<= 1;
  return P;
}

// gather + pad + sort; returns k.  keys must hold cap entries (cap a power of two).
__device__ __forceinline__ int sorted_neighbors(const GridView& g, float qx, float qy, float qz,
                                                float rr, uint64_t* keys, int cap, int* s_count) {
  int k = gather_keys(g, qx, qy, qz, rr, keys, cap, s_count);
  if (k > cap) return k;
  int P = next_pow2(k);
  for (int i = k + threadIdx.x; i < P; i += blockDim.x) keys[i] = ~0ull;
  __syncthreads();
  bitonic_sort(keys, P);
  return k;
}

// ---- bucketed sort: FLANN order without a bitonic network ----
// d2 -> bucket is monotone (one multiplication by a positive constant, then floor), so bucket
// order is d2 order; inside a bucket every key's final slot is its exact rank among the bucket's
// keys (keys are unique: the index breaks ties).  Neighbours of a surface point spread evenly
// over d2 (area grows with d2), so buckets hold a handful of keys; a bucket above kMaxBucket
// makes the caller fall back to the bitonic sort.  NT threads (a multiple of 64), NT buckets.
constexpr int kSortBuckets = 256;
constexpr int kMaxBucket = 96;

template <int NT = kSortBuckets>
struct BucketLdsT {
  int off[NT + 1];
  int cur[NT];
  int wsum[NT / 64];
  int maxn;
};
using BucketLds = BucketLdsT<kSortBuckets>;

__device__ __forceinline__ int d2_bucket(float d2, float inv, int nb) {
  const int b = (int)(d2 * inv);
  return b < nb - 1 ? b : nb - 1;
}

// gather (as gather_keys) + sort into keys[0..k); tmp: cap more keys.  Requires blockDim.x == NT.
// Returns k (> cap: nothing sorted, as sorted_neighbors).
template <int NT = kSortBuckets>
__device__ __forceinline__ int sorted_neighbors_bucketed(const GridView& g, float qx, float qy, float qz,
                                                         float rr, uint64_t* keys, uint64_t* tmp, int cap,
                                                         int* s_count, BucketLdsT<NT>& B) {
  const int tid = threadIdx.x, lane = tid & 63;
  const float inv = (float)NT / rr;
  B.off[tid] = 0;  // counts first
  if (tid == 0) B.maxn = 0;
  const int k = gather_keys(g, qx, qy, qz, rr, keys, cap, s_count);  // (its barriers order the zeroing)
  if (k > cap) return k;
  for (int i = tid; i < k; i += NT) atomicAdd(&B.off[d2_bucket(key_d2(keys[i]), inv, NT)], 1);
  __syncthreads();
  const int c = B.off[tid];
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) B.wsum[tid >> 6] = incl;
  atomicMax(&B.maxn, c);
  __syncthreads();
  int base = 0;
  for (int w = 0; w < (tid >> 6); ++w) base += B.wsum[w];
  const int ex = base + incl - c;
  __syncthreads();  // every count read before the offsets overwrite them
  B.off[tid] = ex;
  B.cur[tid] = ex;
  if (tid == 0) B.off[NT] = k;
  const bool fallback = B.maxn > kMaxBucket;
  __syncthreads();
  if (fallback) {
    const int P = next_pow2(k);
    for (int i = k + tid; i < P; i += NT) keys[i] = ~0ull;
    __syncthreads();
    bitonic_sort(keys, P);
    return k;
  }
  for (int i = tid; i < k; i += NT) {
    const uint64_t key = keys[i];
    tmp[atomicAdd(&B.cur[d2_bucket(key_d2(key), inv, NT)], 1)] = key;
  }
  __syncthreads();
  for (int i = tid; i < k; i += NT) {
    const uint64_t key = tmp[i];
    const int b = d2_bucket(key_d2(key), inv, NT);
    const int o = B.off[b], e = B.off[b + 1];
    int r = 0;
    for (int j = o; j < e; ++j) r += tmp[j] < key;
    keys[o + r] = key;
  }
  __syncthreads();
  return k;
}

}  // namespace pfx
