// pfx_normals.hip -- NormalEstimationOMP<PointXYZRGB,Normal> (tools.h:22-32) on gfx950.
//
// Per query point q:
//   N(q)  = radius-r neighbours in FLANN order (d2, index)
//   accu  = sequential float sums {x^2, xy, xz, y^2, yz, z^2, x, y, z} in that order
//   C     = accu/|N| - mean mean^T;  (lambda, n) = pcl::eigen33(C);  curvature = |lambda/tr C|
//   flip n towards the viewpoint;  |N| < 3 -> NaN
//
// Paths (all bit-identical; they differ only in where the neighbour list lives):
//   k_normals_tile<16,512>   tiles of <= 16 points of a cell whose 27-cell block has <= 1280
//                            points (pfx_normals_tile.h) -- the bulk of every cloud;
//   k_normals_tile<8,1024>   denser blocks (<= 3072 candidates);
//   k_normals_medium         one wave per remaining query, <= 2048 neighbours;
//   k_normals_query          one workgroup per query, <= 16384 neighbours (bitonic in LDS).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_normals_tile.h"

namespace pfx {
namespace {

constexpr int kTileQ = 16;        // queries per tile (tile starts every kTileQ points of a cell)
constexpr int kCapQuery = 16384;  // fallback kernel: neighbours sorted in LDS
constexpr int kChunk = 1024;      // fallback kernel: coordinates staged per chunk
constexpr int kTcapSparse = 1280, kTcapDense = 3072;

// tile starts: the first point of a cell and every kTileQ-th point after it
__global__ void k_tile_flags(const uint32_t* __restrict__ skeys, const int32_t* __restrict__ cell_start,
                             int64_t n, uint64_t ncells, uint8_t* __restrict__ flags) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t key = skeys[i];
  uint8_t f = 0;
  if ((uint64_t)key < ncells) {  // finite point
    int64_t first = cell_start[key];
    f = ((i - first) % kTileQ) == 0;
  }
  flags[i] = f;
}

// split tiles by candidate-block size: sparse (16-query tiles), dense (two 8-query tiles),
// huge (every query to the per-query path)
__global__ void k_tile_class(GridView g, const uint32_t* __restrict__ skeys, const int32_t* __restrict__ tiles,
                             const int64_t* __restrict__ ntiles, int32_t* __restrict__ sparse,
                             int32_t* __restrict__ dense, int32_t* __restrict__ huge, int* __restrict__ counts) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int)*ntiles) return;
  const int32_t start = tiles[t];
  const uint32_t key = skeys[start];
  int T = 0;
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    cell_runs(g, key, r, s, len);
    T += len;
  }
  const int qn = min(kTileQ, g.cell_start[key + 1] - start);
  if (T <= kTcapSparse) {
    sparse[atomicAdd(&counts[0], 1)] = start;
  } else if (T <= kTcapDense) {
    const int d = atomicAdd(&counts[1], 2);
    dense[d] = start;
    dense[d + 1] = qn > 8 ? start + 8 : -1;
  } else {
    const int h = atomicAdd(&counts[2], qn);
    for (int j = 0; j < qn; ++j) huge[h + j] = start + j;
  }
}

constexpr int kCapMedium = 2048;
constexpr int kBucketsMedium = 512;

__global__ void __launch_bounds__(64) k_normals_medium(GridView g, const int32_t* __restrict__ list,
                                                       const int* __restrict__ count_ptr,
                                                       float rr, float bscale, float vpx, float vpy, float vpz,
                                                       float* __restrict__ nx, float* __restrict__ ny,
                                                       float* __restrict__ nz, float* __restrict__ curv,
                                                       int32_t* __restrict__ overflow, int* __restrict__ n_overflow,
                                                       unsigned long long* __restrict__ total_nb) {
  __shared__ uint32_t nb[kCapMedium];
  __shared__ uint32_t tmp_d2[kCapMedium], tmp_pos[kCapMedium];
  __shared__ int bcount[kBucketsMedium], bstart[kBucketsMedium], bfill[kBucketsMedium];
  __shared__ int s_count;
  const int lane = threadIdx.x;
  const int count = *count_ptr;
  for (int w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t i = list[w];
    const float qx = g.sx[i], qy = g.sy[i], qz = g.sz[i];
    Runs R;
    query_runs(g, qx, qy, qz, R);
    if (lane == 0) s_count = 0;
    for (int b = lane; b < kBucketsMedium; b += 64) { bcount[b] = 0; bfill[b] = 0; }
    __syncthreads();
    for (int t0 = 0; t0 < R.pref[9]; t0 += 64) {
      const int t = t0 + lane;
      bool hit = false;
      int32_t pos = 0;
      if (t < R.pref[9]) {
        pos = run_pos(R, t);
        hit = flann_d2(qx, qy, qz, g.sx[pos], g.sy[pos], g.sz[pos]) < rr;
      }
      const uint64_t m = __ballot(hit);
      const int base = s_count;
      if (hit) {
        const int slot = base + __popcll(m & lanemask_lt());
        if (slot < kCapMedium) nb[slot] = (uint32_t)pos;
      }
      __syncthreads();
      if (lane == 0) s_count = base + __popcll(m);
      __syncthreads();
    }
    const int k = s_count;
    if (k > kCapMedium) {
      if (lane == 0) overflow[atomicAdd(n_overflow, 1)] = (int32_t)i;
      __syncthreads();
      continue;
    }
    for (int e = lane; e < k; e += 64) {
      const uint32_t p = nb[e];
      int b = (int)(flann_d2(qx, qy, qz, g.sx[p], g.sy[p], g.sz[p]) * bscale);
      atomicAdd(&bcount[b < kBucketsMedium ? b : kBucketsMedium - 1], 1);
    }
    __syncthreads();
    {
      int c[8], s = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) { c[u] = bcount[lane * 8 + u]; s += c[u]; }
      int inc = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        int v = __shfl_up(inc, off);
        if (lane >= off) inc += v;
      }
      int ex = inc - s;
#pragma unroll
      for (int u = 0; u < 8; ++u) { bstart[lane * 8 + u] = ex; ex += c[u]; }
    }
    __syncthreads();
    for (int e = lane; e < k; e += 64) {
      const uint32_t p = nb[e];
      const float d2 = flann_d2(qx, qy, qz, g.sx[p], g.sy[p], g.sz[p]);
      int b = (int)(d2 * bscale);
      b = b < kBucketsMedium ? b : kBucketsMedium - 1;
      const int slot = bstart[b] + atomicAdd(&bfill[b], 1);
      tmp_d2[slot] = __float_as_uint(d2);
      tmp_pos[slot] = p;
    }
    __syncthreads();
    for (int s = lane; s < k; s += 64) {
      const uint32_t d2 = tmp_d2[s], p = tmp_pos[s];
      int b = (int)(__uint_as_float(d2) * bscale);
      b = b < kBucketsMedium ? b : kBucketsMedium - 1;
      const int st = bstart[b], en = st + bcount[b];
      int rank = 0;
      for (int u = st; u < en; ++u) {
        const uint32_t du = tmp_d2[u];
        if (du < d2) ++rank;
        else if (du == d2 && u != s && g.perm[tmp_pos[u]] < g.perm[p]) ++rank;
      }
      nb[st + rank] = p;
    }
    __syncthreads();
    float acc = 0.0f;
    if (lane < 9) {
#pragma unroll 4
      for (int m = 0; m < k; ++m) {
        const uint32_t p = nb[m];
        acc = acc + chain_term(lane, g.sx[p], g.sy[p], g.sz[p]);
      }
    }
    float accu[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) accu[a] = __shfl(acc, a);
    if (lane == 0) {
      float o[4];
      finish_normal(accu, k, qx, qy, qz, vpx, vpy, vpz, o);
      const int32_t orig = g.perm[i];
      nx[orig] = o[0]; ny[orig] = o[1]; nz[orig] = o[2]; curv[orig] = o[3];
      atomicAdd(total_nb, (unsigned long long)k);
    }
    __syncthreads();
  }
}

// fallback: one 256-thread workgroup per query (neighbour counts > kCapMedium)
__global__ void __launch_bounds__(256) k_normals_query(GridView g, const int32_t* __restrict__ list,
                                                       const int* __restrict__ count_ptr,
                                                       float rr, float vpx, float vpy, float vpz,
                                                       float* __restrict__ nx, float* __restrict__ ny,
                                                       float* __restrict__ nz, float* __restrict__ curv,
                                                       int* __restrict__ err,
                                                       unsigned long long* __restrict__ total_nb) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_big[];
  float4* pts = reinterpret_cast<float4*>(keys_big + kCapQuery);
  __shared__ int s_count;
  const int count = *count_ptr;
  for (int w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t i = list[w];
    const float qx = g.sx[i], qy = g.sy[i], qz = g.sz[i];
    const int32_t orig = g.perm[i];
    const int k = sorted_neighbors(g, qx, qy, qz, rr, keys_big, kCapQuery, &s_count);
    if (k > kCapQuery) {
      if (threadIdx.x == 0) atomicMax(err, k);
      continue;
    }
    float acc = 0.0f;
    for (int c0 = 0; c0 < k; c0 += kChunk) {
      const int m = min(kChunk, k - c0);
      for (int j = threadIdx.x; j < m; j += blockDim.x) {
        const int32_t idx = key_idx(keys_big[c0 + j]);
        pts[j] = make_float4(g.ux[idx], g.uy[idx], g.uz[idx], 0.0f);
      }
      __syncthreads();
      if (threadIdx.x < 9) {
        const int a = threadIdx.x;
        for (int j = 0; j < m; ++j) {
          const float4 p = pts[j];
          acc = acc + chain_term(a, p.x, p.y, p.z);
        }
      }
      __syncthreads();
    }
    float accu[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) accu[a] = __shfl(acc, a);
    if (threadIdx.x == 0) {
      float o[4];
      finish_normal(accu, k, qx, qy, qz, vpx, vpy, vpz, o);
      nx[orig] = o[0]; ny[orig] = o[1]; nz[orig] = o[2]; curv[orig] = o[3];
      atomicAdd(total_nb, (unsigned long long)k);
    }
    __syncthreads();
  }
}

}  // namespace


void normals_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                 const float vp[3], float* nx, float* ny, float* nz, float* curv) {
  PFX_CHECK(r > 0.0, "normals: radius must be > 0");
  PFX_CHECK(n >= 0, "normals: negative point count");
  if (n == 0) return;
  hipStream_t st = ctx->stream;
  build_grid(ctx, ctx->grid_a, x, y, z, n, r);
  const Grid& G = ctx->grid_a;
  GridView g = view(G);
  const float rr = (float)(r * r);
  // non-finite points (key == ncells) are not queries of any tile: NaN outputs (PCL: NaN)
  PFX_HIP(hipMemsetAsync(nx, 0xff, sizeof(float) * n, st));
  PFX_HIP(hipMemsetAsync(ny, 0xff, sizeof(float) * n, st));
  PFX_HIP(hipMemsetAsync(nz, 0xff, sizeof(float) * n, st));
  PFX_HIP(hipMemsetAsync(curv, 0xff, sizeof(float) * n, st));
  uint8_t* flags = ctx->buf("nrm_tile_flags").as<uint8_t>(n);
  int32_t* tiles = ctx->buf("nrm_tiles").as<int32_t>(n);
  int32_t* sparse = ctx->buf("nrm_sparse").as<int32_t>(n);
  int32_t* dense = ctx->buf("nrm_dense").as<int32_t>(2 * n + 2);
  int32_t* medium = ctx->buf("nrm_medium").as<int32_t>(n);
  int32_t* big = ctx->buf("nrm_big").as<int32_t>(n);
  int64_t* d_ntiles = ctx->buf("nrm_ntiles").as<int64_t>(1);
  size_t tmp_bytes = 0;
  PFX_HIP(rocprim::select(nullptr, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, tiles, d_ntiles,
                          (size_t)n, st));
  void* tmp = ctx->buf("nrm_tmp").get(tmp_bytes + 16);
  // counters: 0 sparse tiles, 1 dense half-tiles, 2 medium queries, 3 big queries, 4 max k over cap
  int* counters = ctx->buf("nrm_counters").as<int>(8);
  unsigned long long* total = ctx->buf("nrm_total").as<unsigned long long>(1);
  PFX_HIP(hipMemsetAsync(counters, 0, 8 * sizeof(int), st));
  PFX_HIP(hipMemsetAsync(total, 0, sizeof(unsigned long long), st));
  {
    TimeScope ts(ctx, "normals_tiles");
    k_tile_flags<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(G.skeys, G.cell_start, n, (uint64_t)G.ncells, flags);
    check_launch("k_tile_flags");
    PFX_HIP(rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, tiles, d_ntiles,
                            (size_t)n, st));
    k_tile_class<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(g, G.skeys, tiles, d_ntiles, sparse, dense, medium,
                                                             counters);
    check_launch("k_tile_class");
  }
  {
    // every launch below sizes its loop from a device-side count: no host round trip in between
    TimeScope ts(ctx, "normals");
    k_normals_tile<16, 512, 256, kTcapSparse><<<256 * 3 * 4, 256, 0, st>>>(
        g, G.skeys, sparse, counters + 0, rr, 256.0f / rr, vp[0], vp[1], vp[2], nx, ny, nz, curv, medium,
        counters + 2, total);
    check_launch("k_normals_tile<16>");
    k_normals_tile<8, 1024, 256, kTcapDense><<<256 * 2 * 2, 256, 0, st>>>(
        g, G.skeys, dense, counters + 1, rr, 256.0f / rr, vp[0], vp[1], vp[2], nx, ny, nz, curv, medium,
        counters + 2, total);
    check_launch("k_normals_tile<8>");
    k_normals_medium<<<256 * 4, 64, 0, st>>>(g, medium, counters + 2, rr, (float)kBucketsMedium / rr, vp[0], vp[1],
                                             vp[2], nx, ny, nz, curv, big, counters + 3, total);
    check_launch("k_normals_medium");
    const size_t lds = sizeof(uint64_t) * kCapQuery + sizeof(float4) * kChunk;
    PFX_HIP(hipFuncSetAttribute((const void*)k_normals_query, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_normals_query<<<256, 256, lds, st>>>(g, big, counters + 3, rr, vp[0], vp[1], vp[2], nx, ny, nz, curv,
                                           counters + 4, total);
    check_launch("k_normals_query");
  }
  int h_counters[8];
  unsigned long long h_total = 0;
  PFX_HIP(hipMemcpyAsync(h_counters, counters, sizeof(h_counters), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(&h_total, total, sizeof(h_total), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (h_counters[4] > 0)
    throw Error(PFX_ERR_CAPACITY, "normals: a query has " + std::to_string(h_counters[4]) + " neighbours (> " +
                                      std::to_string(kCapQuery) + " supported)");
  ctx->stats["normals_neighbors"] = (int64_t)h_total;
  ctx->stats["normals_tiles_sparse"] = h_counters[0];
  ctx->stats["normals_tiles_dense"] = h_counters[1];
  ctx->stats["normals_medium"] = h_counters[2];
  ctx->stats["normals_overflow"] = h_counters[3];
}

}  // namespace pfx
