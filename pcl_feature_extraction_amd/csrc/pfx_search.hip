// pfx_search.hip -- search::KdTree<PointXYZRGB>::radiusSearch (FLANN) for arbitrary
// query points: counts + the first `cap` neighbours in (d2, index) order.
#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kCapSearch = 16384;

__global__ void __launch_bounds__(256) k_radius_search(GridView g, const float* __restrict__ qx,
                                                       const float* __restrict__ qy, const float* __restrict__ qz,
                                                       int64_t nq, float rr, int64_t* __restrict__ counts,
                                                       int32_t* __restrict__ idx, float* __restrict__ d2,
                                                       int64_t cap) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_s[];
  __shared__ int s_count;
  for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
    int k;
    if (idx) {
      k = sorted_neighbors(g, qx[q], qy[q], qz[q], rr, keys_s, kCapSearch, &s_count);
      if (k <= kCapSearch) {
        int64_t m = k < cap ? k : cap;
        for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
          uint64_t key = keys_s[j];
          idx[q * cap + j] = key_idx(key);
          d2[q * cap + j] = key_d2(key);
        }
      } else if (threadIdx.x == 0) {
        k = -k;  // too many to order in LDS: report as negative count
      }
    } else {
      k = gather_keys(g, qx[q], qy[q], qz[q], rr, keys_s, 0, &s_count);
    }
    if (threadIdx.x == 0) counts[q] = k;
    __syncthreads();
  }
}

}  // namespace

void radius_search_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                       const float* qx, const float* qy, const float* qz, int64_t nq, double r,
                       int64_t* d_counts, int32_t* d_idx, float* d_d2, int64_t cap) {
  PFX_CHECK(r > 0.0, "radius_search: radius must be > 0");
  if (nq == 0) return;
  if (n == 0) {
    PFX_HIP(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * nq, ctx->stream));
    return;
  }
  build_grid(ctx, ctx->grid_b, x, y, z, n, r);
  GridView g = view(ctx->grid_b);
  const float rr = (float)(r * r);
  size_t lds = d_idx ? sizeof(uint64_t) * kCapSearch : 0;
  if (lds) PFX_HIP(hipFuncSetAttribute((const void*)k_radius_search, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  TimeScope ts(ctx, "radius_search");
  int blocks = (int)std::min<int64_t>(nq, 4096);
  k_radius_search<<<blocks, 256, lds, ctx->stream>>>(g, qx, qy, qz, nq, rr, d_counts, d_idx, d_d2, cap);
  check_launch("k_radius_search");
}

}  // namespace pfx
