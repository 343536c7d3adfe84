// pfx_search.hip -- search::KdTree<PointXYZRGB>::radiusSearch (FLANN) for arbitrary
// query points: counts + the first `cap` neighbours in (d2, index) order.
#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kCapSearch = 16384;         // lists ordered in LDS
constexpr int kOvfBlocks = 16;            // workgroups of the global-scratch pass
constexpr int64_t kCapGlobal = 1 << 22;   // lists ordered in global scratch (PCL: unbounded)

// GLOBAL = false: one workgroup per query, the list ordered in LDS; a query with more than
// kCapSearch neighbours is pushed to `ovf`.  GLOBAL = true: the overflow queries, the list
// ordered in a per-workgroup global scratch slice of gcap keys (the count is read on the
// device, so no host round trip decides whether this pass has work).
template <bool GLOBAL>
__global__ void __launch_bounds__(256) k_radius_search(GridView g, const float* __restrict__ qx,
                                                       const float* __restrict__ qy, const float* __restrict__ qz,
                                                       int64_t nq, float rr, int64_t* __restrict__ counts,
                                                       int32_t* __restrict__ idx, float* __restrict__ d2,
                                                       int64_t cap, int32_t* __restrict__ ovf, int* __restrict__ n_ovf,
                                                       uint64_t* __restrict__ scratch, int64_t gcap) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_s[];
  __shared__ int s_count;
  uint64_t* keys = GLOBAL ? scratch + (size_t)blockIdx.x * gcap : keys_s;
  const int kcap = GLOBAL ? (int)gcap : kCapSearch;
  const int64_t count = GLOBAL ? (int64_t)*n_ovf : nq;
  for (int64_t w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t q = GLOBAL ? (int64_t)ovf[w] : w;
    int k;
    if (idx) {
      k = sorted_neighbors(g, qx[q], qy[q], qz[q], rr, keys, kcap, &s_count);
      if (k <= kcap) {
        int64_t m = k < cap ? k : cap;
        for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
          uint64_t key = keys[j];
          idx[q * cap + j] = key_idx(key);
          d2[q * cap + j] = key_d2(key);
        }
      } else if (threadIdx.x == 0) {
        if (!GLOBAL && ovf) ovf[atomicAdd(n_ovf, 1)] = (int32_t)q;  // ordered by the global pass
        else k = -k;  // beyond kCapGlobal: reported as a negative count
      }
    } else {
      k = gather_keys(g, qx[q], qy[q], qz[q], rr, keys, 0, &s_count);
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
  if (lds) PFX_HIP(hipFuncSetAttribute((const void*)k_radius_search<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // a list can only outgrow the LDS when the cloud has more than kCapSearch points
  const bool overflow_pass = d_idx && n > kCapSearch;
  int32_t* ovf = nullptr;
  int* n_ovf = nullptr;
  uint64_t* scratch = nullptr;
  int64_t gcap = 0;
  if (overflow_pass) {
    gcap = std::min<int64_t>(kCapGlobal, (int64_t)1 << (64 - __builtin_clzll((unsigned long long)n - 1)));
    ovf = ctx->buf("search_ovf").as<int32_t>(nq);
    n_ovf = ctx->buf("search_novf").as<int>(1);
    scratch = ctx->buf("search_scratch").as<uint64_t>((size_t)kOvfBlocks * gcap);
    PFX_HIP(hipMemsetAsync(n_ovf, 0, sizeof(int), ctx->stream));
  }
  TimeScope ts(ctx, "radius_search");
  int blocks = (int)std::min<int64_t>(nq, 4096);
  k_radius_search<false><<<blocks, 256, lds, ctx->stream>>>(g, qx, qy, qz, nq, rr, d_counts, d_idx, d_d2, cap, ovf,
                                                             n_ovf, nullptr, 0);
  if (overflow_pass)
    k_radius_search<true><<<kOvfBlocks, 256, 0, ctx->stream>>>(g, qx, qy, qz, nq, rr, d_counts, d_idx, d_d2, cap,
                                                                ovf, n_ovf, scratch, gcap);
  check_launch("k_radius_search");
}

}  // namespace pfx
