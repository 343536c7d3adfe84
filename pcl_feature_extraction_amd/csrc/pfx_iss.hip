// pfx_iss.hip -- the reference's active-list ISS keypoints:
//
//   Keypoints::computeCloudResolution            keypoints.h:401-428
//     mean over the finite points of sqrtf(d2 of the 2nd nearest point), the 1st being the
//     point itself (FLANN kNN, k = 2), summed in double in index order
//   Keypoints::compute, ISS branch                keypoints.h:177-189
//     pcl::ISSKeypoint3D (PCL 1.7 iss_3d.hpp): salient radius 6 res, non-max radius 4 res,
//     min neighbours 5, thresholds 0.975 / 0.975, sorted search::KdTree, no border radius
//
// Design (MI355X): three uniform grids, no kd-tree.
//   resolution: lane per point scans the 3x3x3 block of a grid of cell h; the 2nd-NN d2 is
//     certified when <= h^2 (every point closer than the cell edge lies in the block), the rest
//     go to a queue that is retried on a grid of 2h and finally scanned exhaustively by one
//     workgroup each.  The double sum is formed exactly: every term is a float, so all are
//     multiples of 2^L (L = ulp exponent of the smallest non-zero term); when the integer sum
//     in units of 2^L stays below 2^53, every partial sum of PCL's sequential loop is exact and
//     equals the order-free integer sum.  Otherwise one workgroup runs the sequential loop.
//   scatter: FLANN-ordered lists at the salient radius (pfx_nblist), lane per query, the six
//     distinct double covariance chains in list order, then Eigen 3.2.0's
//     SelfAdjointEigenSolver<Matrix3d> restated per lane (tridiagonalisation + implicit QR).
//   non-max suppression: lane per point on the non-max grid, third values gathered in that
//     grid's order so candidate reads are contiguous; keypoints compacted in index order.
#include <cstring>
#include <algorithm>
#include <cmath>
#include <rocprim/rocprim.hpp>

#include "pfx_internal.h"
#include "pfx_nblist.h"
#include "pfx_neighbors.h"

namespace pfx {

struct KeypointState {
  Grid res, sal, nms;
  NbLists L;
};

void keypoints_release(pfx_ctx* ctx) {
  if (!ctx->kp) return;
  ctx->kp->res.release();
  ctx->kp->sal.release();
  ctx->kp->nms.release();
  delete ctx->kp;
  ctx->kp = nullptr;
}

namespace {

constexpr int kBruteMax = 1024;  // failed queries scanned exhaustively (one workgroup each)

__device__ __forceinline__ void top2(float d, float& b1, float& b2) {  // the two smallest d2
  b2 = fminf(b2, fmaxf(b1, d));
  b1 = fminf(b1, d);
}

__device__ __forceinline__ int32_t grid_nfinite(const GridView& g) {
  return g.cell_start[(int64_t)g.nx * g.ny * g.nz];  // non-finite points sort behind every cell
}

// 2nd-nearest d2 of each query from its 3x3x3 block (queue == nullptr: every finite point, in
// cell order); certified values -> term[i] = sqrtf(d2), the others -> failq
__global__ void __launch_bounds__(256) k_nn2(GridView g, const int32_t* __restrict__ queue,
                                             const int* __restrict__ n_queue, float hh, float* __restrict__ term,
                                             int32_t* __restrict__ failq, int* __restrict__ n_fail) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int32_t i;
  float qx, qy, qz;
  if (queue) {
    if (t >= *n_queue) return;
    i = queue[t];
    qx = g.ux[i];
    qy = g.uy[i];
    qz = g.uz[i];
  } else {
    if (t >= grid_nfinite(g)) return;
    const float4 c = g.sp[t];
    i = g.perm[t];
    qx = c.x;
    qy = c.y;
    qz = c.z;
  }
  Runs R;
  query_runs(g, qx, qy, qz, R);
  float b1 = INFINITY, b2 = INFINITY;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int32_t s = R.start[r], e = s + (R.pref[r + 1] - R.pref[r]);
#pragma unroll 2
    for (int32_t p = s; p < e; ++p) {
      const float4 c = g.sp[p];
      top2(flann_d2(qx, qy, qz, c.x, c.y, c.z), b1, b2);
    }
  }
  if (b2 <= hh)
    term[i] = sqrtf(b2);
  else
    failq[atomicAdd(n_fail, 1)] = i;
}

// exhaustive 2nd-nearest of the queued points: one workgroup per query over every finite point
__global__ void __launch_bounds__(256) k_nn2_brute(GridView g, const int32_t* __restrict__ queue,
                                                   const int* __restrict__ n_queue, float* __restrict__ term) {
  __shared__ float s1[4], s2[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nq = *n_queue;
  const int32_t nf = grid_nfinite(g);
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int32_t i = queue[q];
    const float qx = g.ux[i], qy = g.uy[i], qz = g.uz[i];
    float b1 = INFINITY, b2 = INFINITY;
    for (int32_t p = tid; p < nf; p += 256) {
      const float4 c = g.sp[p];
      top2(flann_d2(qx, qy, qz, c.x, c.y, c.z), b1, b2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float o1 = __shfl_xor(b1, o), o2 = __shfl_xor(b2, o);
      const float n2 = fminf(fmaxf(b1, o1), fminf(b2, o2));
      b1 = fminf(b1, o1);
      b2 = n2;
    }
    if (lane == 0) {
      s1[wv] = b1;
      s2[wv] = b2;
    }
    __syncthreads();
    if (tid == 0) {
      float a1 = s1[0], a2 = s2[0];
      for (int w = 1; w < 4; ++w) {
        const float n2 = fminf(fmaxf(a1, s1[w]), fminf(a2, s2[w]));
        a1 = fminf(a1, s1[w]);
        a2 = n2;
      }
      term[i] = a2 < INFINITY ? sqrtf(a2) : __int_as_float(0x7fc00000);  // nres < 2: no term
    }
    __syncthreads();
  }
}

// [0] count, [1] min positive term bits, [2] max term bits, [3] term of a magnitude the fixed
// point sum cannot hold, [4..5] u64 integer sum in units of 2^L, [6..7] double approximate sum
struct ResAcc {
  unsigned long long count;
  unsigned int minbits, maxbits, overflow, pad;
  unsigned long long isum;
  double dsum;
};

__device__ __forceinline__ int term_ulp_exp(unsigned int bits) {  // exponent of the ulp of a float
  return (int)((bits >> 23) & 0xff) - 127 - 23;
}

__global__ void __launch_bounds__(256) k_res_stats(const float* __restrict__ term, int64_t n, ResAcc* acc) {
  unsigned long long cnt = 0;
  unsigned int mn = 0xffffffffu, mx = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float t = term[i];
    if (isnan(t)) continue;
    ++cnt;
    const unsigned int b = __float_as_uint(t);
    if (t > 0.0f) mn = min(mn, b);
    mx = max(mx, b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    mn = min(mn, (unsigned int)__shfl_xor((int)mn, o));
    mx = max(mx, (unsigned int)__shfl_xor((int)mx, o));
  }
  if ((threadIdx.x & 63) == 0) {
    if (cnt) atomicAdd(&acc->count, cnt);
    atomicMin(&acc->minbits, mn);
    atomicMax(&acc->maxbits, mx);
  }
}

__global__ void __launch_bounds__(256) k_res_fixed(const float* __restrict__ term, int64_t n, ResAcc* acc) {
  const unsigned int mn = acc->minbits;
  const int L = mn == 0xffffffffu ? 0 : term_ulp_exp(mn);
  unsigned long long is = 0;
  double ds = 0.0;
  unsigned int ovf = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float t = term[i];
    if (!(t > 0.0f)) continue;  // NaN (no term) and zeros add nothing
    const int sh = (int)((__float_as_uint(t) >> 23) & 0xff) - 127 - 23 - L;  // t = m * 2^(L + sh)
    if (sh > 39) {
      ovf = 1;
      continue;
    }
    const unsigned long long m = (unsigned long long)((__float_as_uint(t) & 0x7fffffu) | 0x800000u);
    is += m << sh;
    ds += (double)t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    is += __shfl_xor(is, o);
    ds += __shfl_xor(ds, o);
    ovf |= __shfl_xor(ovf, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&acc->isum, is);
    atomicAdd(&acc->dsum, ds);
    if (ovf) atomicOr(&acc->overflow, 1u);
  }
}

// PCL's loop verbatim: one workgroup, terms staged through LDS, one lane adds in index order
__global__ void __launch_bounds__(256) k_res_sequential(const float* __restrict__ term, int64_t n,
                                                        double* __restrict__ out) {
  __shared__ float s[4096];
  double sum = 0.0;
  for (int64_t b = 0; b < n; b += 4096) {
    for (int k = threadIdx.x; k < 4096; k += 256) s[k] = b + k < n ? term[b + k] : __int_as_float(0x7fc00000);
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll 16
      for (int k = 0; k < 4096; ++k) {
        const float t = s[k];
        if (!isnan(t)) sum += (double)t;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sum;
}

// ---- Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d>, eigenvalues (ascending) ----------------
__device__ __forceinline__ double hypot_e(double x, double y) {  // internal::hypot_impl
  const double ax = fabs(x), ay = fabs(y);
  const double p = ax > ay ? ax : ay;
  if (p == 0.0) return 0.0;
  const double q = ax > ay ? ay : ax;
  const double qp = q / p;
  return p * sqrt(1.0 + qp * qp);
}

__device__ __forceinline__ void make_givens(double p, double q, double& c, double& s) {
  if (q == 0.0) {
    c = p < 0.0 ? -1.0 : 1.0;
    s = 0.0;
  } else if (p == 0.0) {
    c = 0.0;
    s = q < 0.0 ? 1.0 : -1.0;
  } else if (fabs(p) > fabs(q)) {
    const double t = q / p;
    double u = sqrt(1.0 + t * t);
    if (p < 0.0) u = -u;
    c = 1.0 / u;
    s = -t * c;
  } else {
    const double t = p / q;
    double u = sqrt(1.0 + t * t);
    if (q < 0.0) u = -u;
    s = -1.0 / u;
    c = -t * s;
  }
}

// one implicit QR step on the unreduced block [start, end] of a 3x3 tridiagonal
__device__ void qr_step(double d[3], double e[2], int start, int end) {
  const double td = (d[end - 1] - d[end]) * 0.5;
  const double ee = e[end - 1];
  double mu = d[end];
  if (td == 0.0) {
    mu -= fabs(ee);
  } else {
    const double e2 = ee * ee;
    const double h = hypot_e(td, ee);
    if (e2 == 0.0)
      mu -= (ee / (td + (td > 0.0 ? 1.0 : -1.0))) * (ee / h);
    else
      mu -= e2 / (td + (td > 0.0 ? h : -h));
  }
  double x = d[start] - mu;
  double z = e[start];
  for (int k = start; k < end; ++k) {
    double c, s;
    make_givens(x, z, c, s);
    const double sdk = s * d[k] + c * e[k];
    const double dkp1 = s * e[k] + c * d[k + 1];
    d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
    d[k + 1] = s * sdk + c * dkp1;
    e[k] = c * sdk - s * dkp1;
    if (k > start) e[k - 1] = c * e[k - 1] - s * z;
    x = e[k];
    if (k < end - 1) {
      z = -s * e[k + 1];
      e[k + 1] = c * e[k + 1];
    }
  }
}

// lower triangle a00, a10, a11, a20, a21, a22 of a symmetric matrix -> ev ascending
__device__ void eigen_selfadjoint3(double a00, double a10, double a11, double a20, double a21, double a22,
                                   double ev[3]) {
  double scale = fmax(fmax(fmax(fabs(a00), fabs(a10)), fmax(fabs(a11), fabs(a20))), fmax(fabs(a21), fabs(a22)));
  if (scale == 0.0) scale = 1.0;
  a00 /= scale;
  a10 /= scale;
  a11 /= scale;
  a20 /= scale;
  a21 /= scale;
  a22 /= scale;
  double d[3], e[2];
  d[0] = a00;
  const double v1norm2 = a20 * a20;
  if (v1norm2 == 0.0) {
    d[1] = a11;
    d[2] = a22;
    e[0] = a10;
    e[1] = a21;
  } else {
    const double beta = sqrt(a10 * a10 + v1norm2);
    const double inv_beta = 1.0 / beta;
    const double m01 = a10 * inv_beta;
    const double m02 = a20 * inv_beta;
    const double q = 2.0 * m01 * a21 + m02 * (a22 - a11);
    d[1] = a11 + m02 * q;
    d[2] = a22 - m02 * q;
    e[0] = beta;
    e[1] = a21 - m01 * q;
  }
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (fabs(e[i]) <= (fabs(d[i]) + fabs(d[i + 1])) * 1e-12) e[i] = 0.0;
    while (end > 0 && e[end - 1] == 0.0) end--;
    if (end <= 0) break;
    if (++iter > 90) break;
    start = end - 1;
    while (start > 0 && e[start - 1] != 0.0) start--;
    qr_step(d, e, start, end);
  }
  if (iter <= 90) {
    for (int i = 0; i < 2; ++i) {
      int k = i;
      for (int j = i + 1; j < 3; ++j)
        if (d[j] < d[k]) k = j;
      if (k != i) {
        const double t = d[i];
        d[i] = d[k];
        d[k] = t;
      }
    }
  }
  ev[0] = d[0] * scale;
  ev[1] = d[1] * scale;
  ev[2] = d[2] * scale;
}

// ISSKeypoint3D::getScatterMatrix + the eigenvalue tests, lane per query, from FLANN-ordered
// lists: the six distinct double chains cov[a*3+b] += (p_a - c_a) * (p_b - c_b) in list order
__global__ void __launch_bounds__(256) k_iss_scatter(GridView g, NbLists L, int min_nb, double g21, double g32,
                                                     double* __restrict__ third) {
  __shared__ int32_t s_rt[9 * 256];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  if (j >= L.nq) return;  // no barriers below
  const int32_t p = L.qpos[j];
  const int32_t i = g.perm[p];
  const float4 cq = g.sp[p];
  const int k = L.cnt[j];
  double c00 = 0.0, c01 = 0.0, c02 = 0.0, c11 = 0.0, c12 = 0.0, c22 = 0.0;
  if (k >= min_nb) {
    const uint32_t key = L.skeys[p];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      int32_t s, len;
      block_run(g, key, r, s, len);
      s_rt[r * 256 + tid] = s;
    }
    const uint32_t* lst = L.list + L.off[j];
    const int lg = L.lg[j];
    const double cx = cq.x, cy = cq.y, cz = cq.z;
    constexpr int kB = 8;
    const int last = k - 1;  // branch-free batches: clamped loads, exact-zero padded terms
    for (int m0 = 0; m0 < k; m0 += kB) {
      float4 v[kB];
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const int m = m0 + b < last ? m0 + b : last;
        const uint32_t e = lst[(int64_t)m << lg];
        v[b] = g.sp[s_rt[entry_run(e) * 256 + tid] + (int32_t)entry_off(e)];
      }
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const bool in = m0 + b < k;
        const double dx = (double)v[b].x - cx, dy = (double)v[b].y - cy, dz = (double)v[b].z - cz;
        c00 = c00 + (in ? dx * dx : 0.0);
        c01 = c01 + (in ? dx * dy : 0.0);
        c02 = c02 + (in ? dx * dz : 0.0);
        c11 = c11 + (in ? dy * dy : 0.0);
        c12 = c12 + (in ? dy * dz : 0.0);
        c22 = c22 + (in ? dz * dz : 0.0);
      }
    }
  }
  double ev[3];
  eigen_selfadjoint3(c00, c01, c11, c02, c12, c22, ev);
  const double e1 = ev[2], e2 = ev[1], e3 = ev[0];
  double t = 0.0;
  if (isfinite(e1) && isfinite(e2) && isfinite(e3) && !(e3 < 0.0) && e2 / e1 < g21 && e3 / e2 < g32) t = e3;
  third[i] = t;
}

__global__ void __launch_bounds__(256) k_gather_third(GridView g, const double* __restrict__ third,
                                                      double* __restrict__ tn) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= grid_nfinite(g)) return;
  tn[p] = third[g.perm[p]];
}

// non-maximum suppression on the non-max grid (third values in its sorted order)
__global__ void __launch_bounds__(256) k_iss_nms(GridView g, const double* __restrict__ tn, float rr, int min_nb,
                                                 uint8_t* __restrict__ flag) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= grid_nfinite(g)) return;
  const double t = tn[p];
  if (!(t > 0.0)) return;
  const float4 q = g.sp[p];
  Runs R;
  query_runs(g, q.x, q.y, q.z, R);
  int cnt = 0;
  bool ok = true;
#pragma unroll 1
  for (int r = 0; r < 9 && ok; ++r) {
    const int32_t s = R.start[r], e = s + (R.pref[r + 1] - R.pref[r]);
    for (int32_t c = s; c < e; ++c) {
      const float4 v = g.sp[c];
      if (flann_d2(q.x, q.y, q.z, v.x, v.y, v.z) < rr) {
        ++cnt;
        if (t < tn[c]) {
          ok = false;
          break;
        }
      }
    }
  }
  if (ok && cnt >= min_nb) flag[g.perm[p]] = 1;
}

}  // namespace

double cloud_resolution_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n) {
  PFX_CHECK(n >= 0, "cloud_resolution: negative point count");
  if (n == 0) return 0.0;
  if (!ctx->kp) ctx->kp = new KeypointState();
  Grid& G = ctx->kp->res;
  hipStream_t st = ctx->stream;
  TimeScope total(ctx, "resolution");
  float* term = ctx->buf("res_term").as<float>(n);
  int32_t* qa = ctx->buf("res_qa").as<int32_t>(n);
  int32_t* qb = ctx->buf("res_qb").as<int32_t>(n);
  int* nq = ctx->buf("res_nq").as<int>(2);  // [0] current queue length, [1] failures
  PFX_HIP(hipMemsetAsync(term, 0xff, sizeof(float) * n, st));  // NaN: no term
  // first cell: any cell gives the exact answer; half the mean spacing of the bounding volume
  // puts a few tens of points in the block of a point on a scanned surface
  double lo[3], hi[3];
  points_bbox(ctx, G, x, y, z, n, lo, hi);
  double ext = 0.0, vol = 1.0;
  for (int d = 0; d < 3; ++d) ext = std::max(ext, hi[d] - lo[d]);
  for (int d = 0; d < 3; ++d) vol *= std::max(hi[d] - lo[d], ext * 1e-3);
  double h = ext > 0.0 ? 0.5 * std::cbrt(vol / (double)n) : 1.0;
  int64_t nfin = -1;
  int rounds = 0, brute = 0;
  const int32_t* queue = nullptr;
  int32_t* fail = qa;
  int h_fail = 0;
  for (;; ++rounds) {
    build_grid(ctx, G, x, y, z, n, h);
    if (nfin < 0) {
      int32_t nf = 0;
      PFX_HIP(hipMemcpyAsync(&nf, G.cell_start + G.ncells, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      PFX_HIP(hipStreamSynchronize(st));
      nfin = nf;
    }
    PFX_HIP(hipMemsetAsync(nq + 1, 0, sizeof(int), st));
    const int64_t work = queue ? h_fail : nfin;
    if (work > 0) {
      TimeScope ts(ctx, "resolution_nn2");
      k_nn2<<<(unsigned)ceil_div(work, 256), 256, 0, st>>>(view(G), queue, nq, (float)(h * h), term, fail, nq + 1);
      check_launch("k_nn2");
    }
    PFX_HIP(hipMemcpyAsync(&h_fail, nq + 1, sizeof(int), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    if (h_fail == 0) break;
    PFX_HIP(hipMemcpyAsync(nq, nq + 1, sizeof(int), hipMemcpyDeviceToDevice, st));
    if (h_fail <= kBruteMax || rounds >= 8) {
      brute = h_fail;
      TimeScope ts(ctx, "resolution_brute");
      k_nn2_brute<<<(unsigned)std::min(h_fail, 1024), 256, 0, st>>>(view(G), fail, nq, term);
      check_launch("k_nn2_brute");
      break;
    }
    queue = fail;
    fail = fail == qa ? qb : qa;
    h *= 2.0;
  }
  ResAcc* acc = ctx->buf("res_acc").as<ResAcc>(1);
  ResAcc init{};
  init.minbits = 0xffffffffu;
  PFX_HIP(hipMemcpyAsync(acc, &init, sizeof(init), hipMemcpyHostToDevice, st));
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n, 256), 1024);
  k_res_stats<<<blocks, 256, 0, st>>>(term, n, acc);
  k_res_fixed<<<blocks, 256, 0, st>>>(term, n, acc);
  check_launch("k_res_sum");
  ResAcc h_acc;
  PFX_HIP(hipMemcpyAsync(&h_acc, acc, sizeof(h_acc), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  double sum = 0.0;
  const int L = h_acc.minbits == 0xffffffffu ? 0 : (int)((h_acc.minbits >> 23) & 0xff) - 150;
  const bool exact = !h_acc.overflow && h_acc.dsum < std::ldexp(1.0, L + 62) && h_acc.isum < (1ull << 53);
  if (exact) {
    sum = std::ldexp((double)h_acc.isum, L);
  } else {
    double* d = ctx->buf("res_seq").as<double>(1);
    k_res_sequential<<<1, 256, 0, st>>>(term, n, d);
    check_launch("k_res_sequential");
    PFX_HIP(hipMemcpyAsync(&sum, d, sizeof(double), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
  }
  ctx->stats["resolution_rounds"] = rounds + 1;
  ctx->stats["resolution_brute"] = brute;
  ctx->stats["resolution_exact_sum"] = exact ? 1 : 0;
  ctx->stats["resolution_points"] = (int64_t)h_acc.count;
  return h_acc.count ? sum / (double)(int64_t)h_acc.count : 0.0;
}

int64_t iss_keypoints_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double salient,
                          double non_max, int min_nb, double g21, double g32, int32_t* out, int64_t cap,
                          double* third_out) {
  PFX_CHECK(n >= 0, "iss: negative point count");
  if (!ctx->kp) ctx->kp = new KeypointState();
  KeypointState& K = *ctx->kp;
  hipStream_t st = ctx->stream;
  if (n == 0) return 0;
  TimeScope total(ctx, "iss");
  double* third = third_out ? third_out : ctx->buf("iss_third").as<double>(n);
  PFX_HIP(hipMemsetAsync(third, 0, sizeof(double) * n, st));
  build_grid(ctx, K.sal, x, y, z, n, salient);
  build_lists(ctx, K.sal, nullptr, salient, true, K.L, "iss");
  if (K.L.nq > 0) {
    TimeScope ts(ctx, "iss_scatter");
    k_iss_scatter<<<(unsigned)ceil_div(K.L.nq, 256), 256, 0, st>>>(view(K.sal), K.L, min_nb, g21, g32, third);
    check_launch("k_iss_scatter");
  }
  ctx->stats["iss_neighbors"] = K.L.total;
  build_grid(ctx, K.nms, x, y, z, n, non_max);
  double* tn = ctx->buf("iss_tn").as<double>(n);
  uint8_t* flag = ctx->buf("iss_flag").as<uint8_t>(n);
  PFX_HIP(hipMemsetAsync(flag, 0, n, st));
  {
    TimeScope ts(ctx, "iss_nms");
    const unsigned nb = (unsigned)ceil_div(n, 256);
    k_gather_third<<<nb, 256, 0, st>>>(view(K.nms), third, tn);
    k_iss_nms<<<nb, 256, 0, st>>>(view(K.nms), tn, (float)(non_max * non_max), min_nb, flag);
    check_launch("k_iss_nms");
  }
  int32_t* sel = ctx->buf("iss_sel").as<int32_t>(n);
  int64_t* d_cnt = ctx->buf("iss_cnt").as<int64_t>(1);
  size_t tb = 0;
  PFX_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<int32_t>(0), flag, sel, d_cnt, (size_t)n, st));
  void* tmp = ctx->buf("iss_tmp").get(tb + 16);
  PFX_HIP(rocprim::select(tmp, tb, rocprim::counting_iterator<int32_t>(0), flag, sel, d_cnt, (size_t)n, st));
  int64_t k = 0;
  PFX_HIP(hipMemcpyAsync(&k, d_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (k <= cap && k > 0) PFX_HIP(hipMemcpyAsync(out, sel, sizeof(int32_t) * k, hipMemcpyDeviceToDevice, st));
  return k;
}

}  // namespace pfx
