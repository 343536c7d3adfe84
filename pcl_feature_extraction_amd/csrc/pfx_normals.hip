// pfx_normals.hip -- NormalEstimationOMP<PointXYZRGB,Normal> (tools.h:22-32) on gfx950.
//
// Per query point q:
//   N(q)  = radius-r neighbours in FLANN order (d2, index)          [gather + LDS sort]
//   accu  = sequential float sums {x^2, xy, xz, y^2, yz, z^2, x, y, z} in that order
//   C     = accu/|N| - mean mean^T;  (lambda, n) = pcl::eigen33(C);  curvature = |lambda/tr C|
//   flip n towards the viewpoint;  |N| < 3 -> NaN
// The 9 accumulation chains are strictly sequential (bit-exact with PCL's float rounding), so
// they run one chain per lane (lanes 0..8) over the sorted neighbour list staged in LDS as
// float4; the rest of the wave does the gather and the bitonic sort.
//
// HBM layout: inputs x/y/z (caller order) are read once into the grid's cell-sorted SoA copy;
// the neighbour gather reads the sorted copy through contiguous per-run loads (the 3x3 column
// block of cells = 9 runs), outputs are written in caller order (nx/ny/nz/curvature SoA).
#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kCapMain = 1024;   // neighbours handled in LDS by the main kernel
constexpr int kCapBig = 16384;   // overflow kernel (one 256-thread block per query)

// 9 ordered accumulation chains; lane a < 9 owns accu[a].  pts: sorted neighbour xyz.
__device__ __forceinline__ float chain_sum(int a, const float4* pts, int k) {
  float acc = 0.0f;
  for (int j = 0; j < k; ++j) {
    float4 p = pts[j];
    float u = (a == 0 || a == 1 || a == 2 || a == 6) ? p.x : ((a == 3 || a == 4 || a == 7) ? p.y : p.z);
    float v = (a == 0) ? p.x : ((a == 1 || a == 3) ? p.y : p.z);
    float t = (a < 6) ? u * v : u;
    acc = acc + t;
  }
  return acc;
}

__device__ __forceinline__ void finish_normal(const float accu_in[9], int k, float px, float py, float pz,
                                              float vpx, float vpy, float vpz, float out[4]) {
  if (k < 3) {
    out[0] = out[1] = out[2] = out[3] = __builtin_nanf("");
    return;
  }
  float a[9];
  const float cnt = (float)k;
#pragma unroll
  for (int i = 0; i < 9; ++i) a[i] = accu_in[i] / cnt;
  Sym3 C;
  C.a00 = a[0] - a[6] * a[6];
  C.a01 = a[1] - a[6] * a[7];
  C.a02 = a[2] - a[6] * a[8];
  C.a11 = a[3] - a[7] * a[7];
  C.a12 = a[4] - a[7] * a[8];
  C.a22 = a[5] - a[8] * a[8];
  C.a10 = C.a01; C.a20 = C.a02; C.a21 = C.a12;
  float lambda;
  f3 n;
  eigen33_min(C, lambda, n);
  float eig_sum = C.a00 + C.a11 + C.a22;
  float curv = (eig_sum != 0.0f) ? fabsf(lambda / eig_sum) : 0.0f;
  float ax = vpx - px, ay = vpy - py, az = vpz - pz;
  float cos_theta = (ax * n.x + ay * n.y) + az * n.z;
  if (cos_theta < 0.0f) { n.x *= -1.0f; n.y *= -1.0f; n.z *= -1.0f; }
  out[0] = n.x; out[1] = n.y; out[2] = n.z; out[3] = curv;
}

__global__ void __launch_bounds__(64) k_normals_main(GridView g, int64_t n, float rr, float vpx, float vpy,
                                                     float vpz, float* __restrict__ nx, float* __restrict__ ny,
                                                     float* __restrict__ nz, float* __restrict__ curv,
                                                     int32_t* __restrict__ overflow, int* __restrict__ n_overflow,
                                                     unsigned long long* __restrict__ total_nb) {
  __shared__ uint64_t keys[kCapMain];
  __shared__ float4 pts[kCapMain];
  __shared__ int s_count;
  const int lane = threadIdx.x;
  unsigned long long my_total = 0;
  const int64_t vb = xcd_block(blockIdx.x, gridDim.x);
  for (int64_t i = vb; i < n; i += gridDim.x) {
    // query = i-th point in cell order (spatially coherent across neighbouring blocks)
    const float qx = g.sx[i], qy = g.sy[i], qz = g.sz[i];
    const int32_t orig = g.perm[i];
    int k = sorted_neighbors(g, qx, qy, qz, rr, keys, kCapMain, &s_count);
    if (k > kCapMain) {
      if (lane == 0) overflow[atomicAdd(n_overflow, 1)] = (int32_t)i;
      continue;
    }
    my_total += (unsigned long long)k;
    // stage the sorted neighbours' coordinates (the key's index addresses the caller arrays)
    for (int j = lane; j < k; j += 64) {
      int32_t idx = key_idx(keys[j]);
      pts[j] = make_float4(g.ux[idx], g.uy[idx], g.uz[idx], 0.0f);
    }
    __syncthreads();
    float acc = 0.0f;
    if (lane < 9) acc = chain_sum(lane, pts, k);
    float accu[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) accu[a] = __shfl(acc, a);
    if (lane == 0) {
      float o[4];
      finish_normal(accu, k, qx, qy, qz, vpx, vpy, vpz, o);
      nx[orig] = o[0]; ny[orig] = o[1]; nz[orig] = o[2]; curv[orig] = o[3];
    }
    __syncthreads();
  }
  if (lane == 0 && my_total) atomicAdd(total_nb, my_total);
}

__global__ void __launch_bounds__(256) k_normals_big(GridView g, const int32_t* __restrict__ list, int count,
                                                     float rr, float vpx, float vpy, float vpz,
                                                     float* __restrict__ nx, float* __restrict__ ny,
                                                     float* __restrict__ nz, float* __restrict__ curv,
                                                     int* __restrict__ err, unsigned long long* __restrict__ total_nb) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_big[];
  __shared__ int s_count;
  for (int w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t i = list[w];
    const float qx = g.sx[i], qy = g.sy[i], qz = g.sz[i];
    const int32_t orig = g.perm[i];
    int k = sorted_neighbors(g, qx, qy, qz, rr, keys_big, kCapBig, &s_count);
    if (k > kCapBig) {
      if (threadIdx.x == 0) atomicMax(err, k);
      continue;
    }
    float acc = 0.0f;
    if (threadIdx.x < 9) {
      const int a = threadIdx.x;
      for (int j = 0; j < k; ++j) {
        int32_t idx = key_idx(keys_big[j]);
        float px = g.ux[idx], py = g.uy[idx], pz = g.uz[idx];
        float u = (a == 0 || a == 1 || a == 2 || a == 6) ? px : ((a == 3 || a == 4 || a == 7) ? py : pz);
        float v = (a == 0) ? px : ((a == 1 || a == 3) ? py : pz);
        float t = (a < 6) ? u * v : u;
        acc = acc + t;
      }
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
  GridView g = view(ctx->grid_a);
  const float rr = (float)(r * r);
  int32_t* overflow = ctx->buf("nrm_overflow").as<int32_t>(n);
  int* counters = ctx->buf("nrm_counters").as<int>(4);
  unsigned long long* total = ctx->buf("nrm_total").as<unsigned long long>(1);
  PFX_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(int), st));
  PFX_HIP(hipMemsetAsync(total, 0, sizeof(unsigned long long), st));
  {
    TimeScope ts(ctx, "normals");
    int blocks = (int)std::min<int64_t>(n, 256 * 8);
    blocks = std::max(8, blocks & ~7);
    k_normals_main<<<blocks, 64, 0, st>>>(g, n, rr, vp[0], vp[1], vp[2], nx, ny, nz, curv, overflow,
                                          counters, total);
    check_launch("k_normals_main");
  }
  int h_counters[4];
  PFX_HIP(hipMemcpyAsync(h_counters, counters, sizeof(h_counters), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (h_counters[0] > 0) {
    TimeScope ts(ctx, "normals_big");
    size_t lds = sizeof(uint64_t) * kCapBig;
    PFX_HIP(hipFuncSetAttribute((const void*)k_normals_big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_normals_big<<<std::min(h_counters[0], 2048), 256, lds, st>>>(g, overflow, h_counters[0], rr, vp[0], vp[1],
                                                                   vp[2], nx, ny, nz, curv, counters + 1, total);
    check_launch("k_normals_big");
    PFX_HIP(hipMemcpyAsync(h_counters, counters, sizeof(h_counters), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    if (h_counters[1] > 0)
      throw Error(PFX_ERR_CAPACITY, "normals: a query has " + std::to_string(h_counters[1]) +
                                        " neighbours (> " + std::to_string(kCapBig) + " supported)");
  }
  unsigned long long h_total = 0;
  PFX_HIP(hipMemcpy(&h_total, total, sizeof(h_total), hipMemcpyDeviceToHost));
  ctx->stats["normals_neighbors"] = (int64_t)h_total;
  ctx->stats["normals_overflow"] = h_counters[0];
}

}  // namespace pfx
