// pfx_fpfh.hip -- FPFHEstimation<PointXYZRGB,Normal,FPFHSignature33> (evaluation.cpp:593-612,
// features.h:175-196) on gfx950.  SURVEY A.3.
//
//   S        = union of the radius-r neighbourhoods of the queries (or every surface point
//              when input == surface, PCL's special case)            k_fpfh_mark + select
//   SPFH(p)  = 3 x 11 bins of the pair features (p, q), q in N(p)\{p}: each hit adds the same
//              float hist_incr = 100/(|N(p)|-1); the float value of a bin therefore depends
//              only on its hit count c (c sequential adds), so bins are counted with LDS
//              atomics (order-free) and materialised by c ordered adds      k_fpfh_spfh
//   FPFH(q)  = sum over N(q) in FLANN order, skipping d2 == 0, of SPFH(nbr) / d2 (float per bin,
//              double per 11-bin block), then each block scaled to 100      k_fpfh_weight
// SPFH rows are stored by caller index (n_surface x 33 floats, row-major) -- only rows in S
// are written/read.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kBins = 11;
constexpr int kDesc = 33;
constexpr int kCapW = 2048;     // sorted-neighbour capacity of the weighting kernel (LDS)
constexpr int kCapWBig = 16384; // overflow weighting kernel

// PCL 1.7 `acos (fabs (a1)) > acos (fabs (a2))` (double acos, correctly rounded by glibc):
// acos is strictly decreasing and distinct floats >= 2^-26 map to distinct rounded values, so
// the test is |a1| < |a2|; below 2^-26 acos(x) rounds as H + (L - x), pi/2 = H + L.
__device__ __forceinline__ bool acos_greater(float a1, float a2) {
  float x1 = fabsf(a1), x2 = fabsf(a2);
  if (x1 >= 1.4901161e-08f || x2 >= 1.4901161e-08f) return x1 < x2;
  const double H = 1.5707963267948966, L = 6.123233995736766e-17;
  return (H + (L - (double)x1)) > (H + (L - (double)x2));
}

// pcl::computePairFeatures (features/src/pfh.cpp), Vector4f maps with w = 0
__device__ __forceinline__ void pair_features(f3 p1, f3 n1, f3 p2, f3 n2, float& f1, float& f2, float& f3o) {
  f3 dp = sub3(p2, p1);
  float f4 = sqrtf(sqn4(dp));
  if (f4 == 0.0f) { f1 = f2 = f3o = 0.0f; return; }
  f3 n1c = n1, n2c = n2;
  float angle1 = dot4(n1c, dp) / f4;
  float angle2 = dot4(n2c, dp) / f4;
  if (acos_greater(angle1, angle2)) {
    n1c = n2; n2c = n1;
    dp = scale3(dp, -1.0f);
    f3o = -angle2;
  } else {
    f3o = angle1;
  }
  f3 v = cross3(dp, n1c);
  float v_norm = sqrtf(sqn4(v));
  if (v_norm == 0.0f) { f1 = f2 = f3o = 0.0f; return; }
  v = div3(v, v_norm);
  f3 w = cross3(n1c, v);
  f2 = dot4(v, n2c);
  f1 = atan2f_cr(dot4(w, n2c), dot4(n1c, n2c));
}

__device__ __forceinline__ int bin_of(double v) {
  if (!(v == v)) return 0;  // static_cast<int>(NaN) == INT_MIN on x86 -> clamped to 0
  double f = floor(v);
  int h = (f >= 2147483647.0 || f < -2147483648.0) ? (int)0x80000000 : (int)f;
  return h < 0 ? 0 : (h >= kBins ? kBins - 1 : h);
}

__global__ void __launch_bounds__(256) k_fpfh_mark(GridView g, const float* __restrict__ qx,
                                                   const float* __restrict__ qy, const float* __restrict__ qz,
                                                   int64_t nq, float rr, uint8_t* __restrict__ flags) {
  for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
    Runs R;
    float x = qx[q], y = qy[q], z = qz[q];
    query_runs(g, x, y, z, R);
    for (int32_t t = threadIdx.x; t < R.pref[9]; t += blockDim.x) {
      int32_t p = run_pos(R, t);
      if (flann_d2(x, y, z, g.sx[p], g.sy[p], g.sz[p]) < rr) flags[g.perm[p]] = 1;
    }
  }
}

// one 64-thread block per S point
__global__ void __launch_bounds__(64) k_fpfh_spfh(GridView g, const float* __restrict__ nxs,
                                                  const float* __restrict__ nys, const float* __restrict__ nzs,
                                                  const int32_t* __restrict__ list, int64_t count, float rr,
                                                  float* __restrict__ spfh) {
  __shared__ int hist[kDesc];
  const int lane = threadIdx.x;
  const float d_pi = 1.0f / (2.0f * 3.14159265358979323846f);
  const int64_t vb = xcd_block(blockIdx.x, gridDim.x);
  for (int64_t w = vb; w < count; w += gridDim.x) {
    const int32_t p = list ? list[w] : (int32_t)w;
    if (lane < kDesc) hist[lane] = 0;
    __syncthreads();
    const f3 pp = mk3(g.ux[p], g.uy[p], g.uz[p]);
    const f3 pn = mk3(nxs[p], nys[p], nzs[p]);
    Runs R;
    query_runs(g, pp.x, pp.y, pp.z, R);
    int my_k = 0;
    for (int32_t t = lane; t < R.pref[9]; t += 64) {
      int32_t s = run_pos(R, t);
      float d2 = flann_d2(pp.x, pp.y, pp.z, g.sx[s], g.sy[s], g.sz[s]);
      if (!(d2 < rr)) continue;
      ++my_k;
      int32_t q = g.perm[s];
      if (q == p) continue;
      float f1, f2, f3v;
      pair_features(pp, pn, mk3(g.sx[s], g.sy[s], g.sz[s]), mk3(nxs[q], nys[q], nzs[q]), f1, f2, f3v);
      int h1 = bin_of((double)kBins * (((double)f1 + 3.14159265358979323846) * (double)d_pi));
      int h2 = bin_of((double)kBins * (((double)f2 + 1.0) * 0.5));
      int h3 = bin_of((double)kBins * (((double)f3v + 1.0) * 0.5));
      atomicAdd(&hist[h1], 1);
      atomicAdd(&hist[kBins + h2], 1);
      atomicAdd(&hist[2 * kBins + h3], 1);
    }
    // wave reduction of the neighbour count
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) my_k += __shfl_xor(my_k, off);
    __syncthreads();
    if (lane < kDesc) {
      const int c = hist[lane];
      const float incr = 100.0f / (float)(my_k - 1);
      float v = 0.0f;
      for (int j = 0; j < c; ++j) v = v + incr;
      spfh[(int64_t)p * kDesc + lane] = v;
    }
    __syncthreads();
  }
}

// weighting: one block per query (64 threads: lanes 0..32 own a bin, 33..35 the block sums)
template <int CAP>
__device__ __forceinline__ void weight_one(const uint64_t* keys, int k, const float* __restrict__ spfh,
                                           float* __restrict__ out_row) {
  const int lane = threadIdx.x;
  float fh = 0.0f;
  double sum = 0.0;
  if (lane < kDesc) {
    for (int j = 0; j < k; ++j) {
      uint64_t key = keys[j];
      float d2 = key_d2(key);
      if (d2 == 0.0f) continue;
      float w = 1.0f / d2;
      float val = spfh[(int64_t)key_idx(key) * kDesc + lane] * w;
      fh = fh + val;
    }
  } else if (lane < kDesc + 3) {
    const int blk = lane - kDesc;
    for (int j = 0; j < k; ++j) {
      uint64_t key = keys[j];
      float d2 = key_d2(key);
      if (d2 == 0.0f) continue;
      float w = 1.0f / d2;
      const float* row = spfh + (int64_t)key_idx(key) * kDesc + blk * kBins;
#pragma unroll
      for (int b = 0; b < kBins; ++b) {
        float val = row[b] * w;
        sum = sum + (double)val;
      }
    }
    if (sum != 0.0) sum = 100.0 / sum;
  }
  double s0 = __shfl(sum, kDesc + 0), s1 = __shfl(sum, kDesc + 1), s2 = __shfl(sum, kDesc + 2);
  if (lane < kDesc) {
    double s = lane < kBins ? s0 : (lane < 2 * kBins ? s1 : s2);
    out_row[lane] = fh * (float)s;
  }
}

__global__ void __launch_bounds__(64) k_fpfh_weight(GridView g, const float* __restrict__ qx,
                                                    const float* __restrict__ qy, const float* __restrict__ qz,
                                                    int64_t nq, float rr, const float* __restrict__ spfh,
                                                    float* __restrict__ out, int32_t* __restrict__ overflow,
                                                    int* __restrict__ n_overflow) {
  __shared__ uint64_t keys[kCapW];
  __shared__ int s_count;
  const int64_t vb = xcd_block(blockIdx.x, gridDim.x);
  for (int64_t q = vb; q < nq; q += gridDim.x) {
    int k = sorted_neighbors(g, qx[q], qy[q], qz[q], rr, keys, kCapW, &s_count);
    if (k > kCapW) {
      if (threadIdx.x == 0) overflow[atomicAdd(n_overflow, 1)] = (int32_t)q;
      continue;
    }
    if (k == 0) {
      if (threadIdx.x < kDesc) out[q * kDesc + threadIdx.x] = __builtin_nanf("");
    } else {
      weight_one<kCapW>(keys, k, spfh, out + q * kDesc);
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(64) k_fpfh_weight_big(GridView g, const float* __restrict__ qx,
                                                        const float* __restrict__ qy, const float* __restrict__ qz,
                                                        const int32_t* __restrict__ list, int count, float rr,
                                                        const float* __restrict__ spfh, float* __restrict__ out,
                                                        int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_big[];
  __shared__ int s_count;
  for (int w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t q = list[w];
    int k = sorted_neighbors(g, qx[q], qy[q], qz[q], rr, keys_big, kCapWBig, &s_count);
    if (k > kCapWBig) {
      if (threadIdx.x == 0) atomicMax(err, k);
      continue;
    }
    weight_one<kCapWBig>(keys_big, k, spfh, out + q * kDesc);
    __syncthreads();
  }
}

}  // namespace

void fpfh_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
              const float* sny, const float* snz, int64_t ns, const float* qx, const float* qy, const float* qz,
              int64_t nq, int same, double r, float* out) {
  PFX_CHECK(r > 0.0, "fpfh: radius must be > 0");
  if (nq == 0) return;
  hipStream_t st = ctx->stream;
  if (ns == 0) {
    // no surface: every query has an empty neighbourhood -> NaN rows (PCL fills NaN)
    std::vector<float> nanrow((size_t)nq * kDesc, __builtin_nanf(""));
    PFX_HIP(hipMemcpyAsync(out, nanrow.data(), sizeof(float) * nanrow.size(), hipMemcpyHostToDevice, st));
    PFX_HIP(hipStreamSynchronize(st));
    return;
  }
  build_grid(ctx, ctx->grid_b, sx, sy, sz, ns, r);
  GridView g = view(ctx->grid_b);
  const float rr = (float)(r * r);
  float* spfh = ctx->buf("fpfh_spfh").as<float>(ns * kDesc);
  int32_t* list = nullptr;
  int64_t count = ns;
  if (!same) {
    uint8_t* flags = ctx->buf("fpfh_flags").as<uint8_t>(ns);
    list = ctx->buf("fpfh_list").as<int32_t>(ns);
    int64_t* d_sel = ctx->buf("fpfh_nsel").as<int64_t>(1);
    size_t tmp_bytes = 0;
    PFX_HIP(rocprim::select(nullptr, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, list, d_sel,
                            (size_t)ns, st));
    void* tmp = ctx->buf("fpfh_tmp").get(tmp_bytes + 16);
    PFX_HIP(hipMemsetAsync(flags, 0, ns, st));
    {
      TimeScope ts(ctx, "fpfh_mark");
      k_fpfh_mark<<<(unsigned)std::min<int64_t>(nq, 8192), 256, 0, st>>>(g, qx, qy, qz, nq, rr, flags);
      check_launch("k_fpfh_mark");
    }
    PFX_HIP(rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, list, d_sel,
                            (size_t)ns, st));
    PFX_HIP(hipMemcpyAsync(&count, d_sel, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
  }
  ctx->stats["fpfh_spfh_points"] = count;
  if (count > 0) {
    TimeScope ts(ctx, "fpfh_spfh");
    int blocks = (int)std::min<int64_t>(count, 256 * 16);
    blocks = std::max(8, blocks & ~7);
    k_fpfh_spfh<<<blocks, 64, 0, st>>>(g, snx, sny, snz, list, count, rr, spfh);
    check_launch("k_fpfh_spfh");
  }
  int* counters = ctx->buf("fpfh_counters").as<int>(4);
  int32_t* overflow = ctx->buf("fpfh_overflow").as<int32_t>(nq);
  PFX_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(int), st));
  {
    TimeScope ts(ctx, "fpfh_weight");
    int blocks = (int)std::min<int64_t>(nq, 256 * 12);
    blocks = std::max(8, blocks & ~7);
    k_fpfh_weight<<<blocks, 64, 0, st>>>(g, qx, qy, qz, nq, rr, spfh, out, overflow, counters);
    check_launch("k_fpfh_weight");
  }
  int h[4];
  PFX_HIP(hipMemcpyAsync(h, counters, sizeof(h), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (h[0] > 0) {
    size_t lds = sizeof(uint64_t) * kCapWBig;
    PFX_HIP(hipFuncSetAttribute((const void*)k_fpfh_weight_big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    TimeScope ts(ctx, "fpfh_weight_big");
    k_fpfh_weight_big<<<std::min(h[0], 2048), 64, lds, st>>>(g, qx, qy, qz, overflow, h[0], rr, spfh, out,
                                                              counters + 1);
    check_launch("k_fpfh_weight_big");
    PFX_HIP(hipMemcpyAsync(h, counters, sizeof(h), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    if (h[1] > 0)
      throw Error(PFX_ERR_CAPACITY, "fpfh: a query has " + std::to_string(h[1]) + " neighbours (> " +
                                        std::to_string(kCapWBig) + " supported)");
  }
}

}  // namespace pfx
