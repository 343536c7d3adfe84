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
//   scatter: lane per point over its 3x3x3 block of the salient grid, the six distinct double
//     covariance chains in scan order -- exact, hence equal to PCL's FLANN-order sums, whenever
//     every partial sum is provably exact (k_iss_cov); the rest (coordinates near 0) sorted per
//     wave into FLANN order (k_iss_ordered) or, beyond 512 neighbours, from FLANN-ordered lists
//     (pfx_nblist).  Then Eigen 3.2.0's SelfAdjointEigenSolver<Matrix3d> restated per lane
//     (tridiagonalisation + implicit QR).
//   non-max suppression: lane per point on the non-max grid, third values gathered in that
//     grid's order so candidate reads are contiguous; keypoints compacted in index order.
#include <cstring>
#include <algorithm>
#include <cmath>
#include <rocprim/rocprim.hpp>

#include "pfx_eigen3.h"
#include "pfx_internal.h"
#include "pfx_nblist.h"
#include "pfx_neighbors.h"
#include "pfx_wave_sort.h"

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

// exhaustive 2nd-nearest of the queued points: kParts workgroups per query, each over a slice
// of every finite point, then one lane per query merges the slices
constexpr int kParts = 64;

__device__ __forceinline__ void top2_merge(float& a1, float& a2, float b1, float b2) {
  const float n2 = fminf(fmaxf(a1, b1), fminf(a2, b2));
  a1 = fminf(a1, b1);
  a2 = n2;
}

__global__ void __launch_bounds__(256) k_nn2_brute(GridView g, const int32_t* __restrict__ queue,
                                                   float2* __restrict__ part) {
  __shared__ float s1[4], s2[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q = blockIdx.x / kParts, pt = blockIdx.x % kParts;
  const int32_t nf = grid_nfinite(g);
  const int32_t chunk = (nf + kParts - 1) / kParts, p0 = pt * chunk, p1 = min(nf, p0 + chunk);
  const int32_t i = queue[q];
  const float qx = g.ux[i], qy = g.uy[i], qz = g.uz[i];
  float b1 = INFINITY, b2 = INFINITY;
  for (int32_t p = p0 + tid; p < p1; p += 256) {
    const float4 c = g.sp[p];
    top2(flann_d2(qx, qy, qz, c.x, c.y, c.z), b1, b2);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) top2_merge(b1, b2, __shfl_xor(b1, o), __shfl_xor(b2, o));
  if (lane == 0) {
    s1[wv] = b1;
    s2[wv] = b2;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) top2_merge(b1, b2, s1[w], s2[w]);
    part[blockIdx.x] = make_float2(b1, b2);
  }
}

__global__ void __launch_bounds__(64) k_nn2_brute_merge(const int32_t* __restrict__ queue, int nq,
                                                        const float2* __restrict__ part, float* __restrict__ term) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= nq) return;
  float b1 = INFINITY, b2 = INFINITY;
  for (int k = 0; k < kParts; ++k) {
    const float2 v = part[q * kParts + k];
    top2_merge(b1, b2, v.x, v.y);
  }
  term[queue[q]] = b2 < INFINITY ? sqrtf(b2) : __int_as_float(0x7fc00000);  // nres < 2: no term
}

// Exact sum of the terms.  Per block: count, smallest positive term (its ulp exponent L_b) and
// the integer sum in units of 2^L_b; the final pass rescales every block to the global L.
struct ResPart {
  unsigned long long count, isum;
  double dsum;
  unsigned int minbits, overflow;
};
struct ResAcc {
  unsigned long long count, isum;
  double dsum;
  int L, exact;
};

__device__ __forceinline__ int ulp_exp(unsigned int bits) {  // exponent of the ulp of a normal float
  return (int)((bits >> 23) & 0xff) - 150;
}

__global__ void __launch_bounds__(256) k_res_partial(const float* __restrict__ term, int64_t n,
                                                     ResPart* __restrict__ part) {
  __shared__ unsigned long long s_c[4], s_i[4];
  __shared__ double s_d[4];
  __shared__ unsigned int s_m[4], s_o[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t stride = (int64_t)gridDim.x * 256;
  unsigned long long cnt = 0;
  unsigned int mn = 0xffffffffu;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < n; i += stride) {
    const float t = term[i];
    if (isnan(t)) continue;
    ++cnt;
    if (t > 0.0f) mn = min(mn, __float_as_uint(t));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    mn = min(mn, (unsigned int)__shfl_xor((int)mn, o));
  }
  if (lane == 0) {
    s_c[wv] = cnt;
    s_m[wv] = mn;
  }
  __syncthreads();
  mn = min(min(s_m[0], s_m[1]), min(s_m[2], s_m[3]));
  const int L = mn == 0xffffffffu ? 0 : ulp_exp(mn);
  unsigned long long is = 0;
  double ds = 0.0;
  unsigned int ovf = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < n; i += stride) {
    const float t = term[i];
    if (!(t > 0.0f)) continue;  // NaN (no term) and zeros add nothing
    const unsigned int b = __float_as_uint(t);
    const int sh = ulp_exp(b) - L;  // t = m * 2^(L + sh)
    if (sh > 39) {
      ovf = 1;
      continue;
    }
    is += (unsigned long long)((b & 0x7fffffu) | 0x800000u) << sh;
    ds += (double)t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    is += __shfl_xor(is, o);
    ds += __shfl_xor(ds, o);
    ovf |= __shfl_xor(ovf, o);
  }
  if (lane == 0) {
    s_i[wv] = is;
    s_d[wv] = ds;
    s_o[wv] = ovf;
  }
  __syncthreads();
  if (tid == 0) {
    ResPart r;
    r.count = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    r.isum = s_i[0] + s_i[1] + s_i[2] + s_i[3];  // < 2^63 each: a wrap shows in dsum below
    r.dsum = (s_d[0] + s_d[1]) + (s_d[2] + s_d[3]);
    r.minbits = mn;
    r.overflow = s_o[0] | s_o[1] | s_o[2] | s_o[3];
    part[blockIdx.x] = r;
  }
}

// one wave: global L = min over blocks, then every block sum rescaled to 2^L (exactness checked)
__global__ void __launch_bounds__(64) k_res_final(const ResPart* __restrict__ part, int nb, ResAcc* __restrict__ acc) {
  const int lane = threadIdx.x;
  unsigned int mn = 0xffffffffu;
  for (int b = lane; b < nb; b += 64) mn = min(mn, part[b].minbits);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned int)__shfl_xor((int)mn, o));
  const int L = mn == 0xffffffffu ? 0 : ulp_exp(mn);
  unsigned long long cnt = 0, is = 0;
  double ds = 0.0;
  int bad = 0;
  for (int b = lane; b < nb; b += 64) {
    const ResPart r = part[b];
    cnt += r.count;
    ds += r.dsum;
    if (r.overflow) bad = 1;
    if (r.isum == 0) continue;
    const int sh = ulp_exp(r.minbits) - L;
    // the block sum in units of 2^L must stay below 2^53 (and its own sum must not have wrapped)
    if (r.dsum >= ldexp(1.0, ulp_exp(r.minbits) + 62) || sh > 52 || r.isum >= (1ull << (53 - sh))) {
      bad = 1;
      continue;
    }
    is += r.isum << sh;  // < 2^53 per block, <= 16 blocks per lane: no wrap
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    is += __shfl_xor(is, o);
    ds += __shfl_xor(ds, o);
    bad |= __shfl_xor(bad, o);
  }
  if (lane == 0) {
    acc->count = cnt;
    acc->isum = is;
    acc->dsum = ds;
    acc->L = L;
    acc->exact = (!bad && is < (1ull << 53)) ? 1 : 0;
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

// Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d> eigenvalues: pfx_eigen3.h

__device__ __forceinline__ double iss_third(double c00, double c01, double c02, double c11, double c12, double c22,
                                            double g21, double g32) {
  double ev[3];
  eigen_selfadjoint3<false>(c00, c01, c11, c02, c12, c22, ev, nullptr);
  const double e1 = ev[2], e2 = ev[1], e3 = ev[0];
  if (isfinite(e1) && isfinite(e2) && isfinite(e3) && !(e3 < 0.0) && e2 / e1 < g21 && e3 / e2 < g32) return e3;
  return 0.0;
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
  third[i] = iss_third(c00, c01, c02, c11, c12, c22, g21, g32);
}

// ISSKeypoint3D::getScatterMatrix without neighbour lists: lane per finite point of the salient
// grid, the block scanned in grid order.  PCL adds the terms (p_a - c_a)(p_b - c_b) in FLANN
// order; every coordinate difference is a multiple of 2^(E - 23) (E = the smallest float
// exponent among the coordinates involved), so every term is a multiple of 2^L, L = 2E - 46,
// and with sum |term| <= k r^2 < 2^(L + 53) every partial sum in ANY order is exact: the scan
// order gives PCL's result bit for bit.  Points that miss the bound (coordinates near 0) are
// queued (oq) for k_iss_ordered.  part[block] = neighbours found (statistics).
__global__ void __launch_bounds__(256) k_iss_cov(GridView g, float rr, int min_nb, double g21, double g32,
                                                 double* __restrict__ third, int32_t* __restrict__ oq,
                                                 int* __restrict__ n_mask, unsigned int* __restrict__ part) {
  __shared__ unsigned int s_cnt[4];
  const int tid = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * 256 + tid;
  unsigned int cnt = 0;
  if (p < grid_nfinite(g)) {
    const float4 q = g.sp[p];
    const int32_t i = g.perm[p];
    const double qx = q.x, qy = q.y, qz = q.z;
    Runs R;
    query_runs(g, q.x, q.y, q.z, R);
    double c00 = 0.0, c01 = 0.0, c02 = 0.0, c11 = 0.0, c12 = 0.0, c22 = 0.0;
    unsigned int ex = (__float_as_uint(q.x) >> 23) & 0xffu, ey = (__float_as_uint(q.y) >> 23) & 0xffu,
                 ez = (__float_as_uint(q.z) >> 23) & 0xffu;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int32_t s = R.start[r], e = s + (R.pref[r + 1] - R.pref[r]);
      for (int32_t c = s; c < e; ++c) {
        const float4 v = g.sp[c];
        if (flann_d2(q.x, q.y, q.z, v.x, v.y, v.z) < rr) {
          ++cnt;
          const double dx = (double)v.x - qx, dy = (double)v.y - qy, dz = (double)v.z - qz;
          c00 += dx * dx;
          c01 += dx * dy;
          c02 += dx * dz;
          c11 += dy * dy;
          c12 += dy * dz;
          c22 += dz * dz;
          ex = min(ex, (__float_as_uint(v.x) >> 23) & 0xffu);
          ey = min(ey, (__float_as_uint(v.y) >> 23) & 0xffu);
          ez = min(ez, (__float_as_uint(v.z) >> 23) & 0xffu);
        }
      }
    }
    double t = 0.0;  // fewer than min_nb neighbours: PCL's zero matrix, NaN ratios, no value
    if ((int)cnt >= min_nb) {
      // per axis a: the differences are multiples of 2^(E_a - 23); chain (a, a) is exact when
      // sum dx_a^2 < 2^(2 E_a + 7), and then chain (a, b) too (Cauchy-Schwarz)
      const bool ok = c00 * 1.000001 < ldexp(1.0, 2 * ((int)ex - 127) + 7) &&
                      c11 * 1.000001 < ldexp(1.0, 2 * ((int)ey - 127) + 7) &&
                      c22 * 1.000001 < ldexp(1.0, 2 * ((int)ez - 127) + 7);
      if (ok) {
        t = iss_third(c00, c01, c02, c11, c12, c22, g21, g32);
      } else {
        oq[wave_push_slot(n_mask)] = (int32_t)p;
      }
    }
    third[i] = t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) part[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// The queued points in PCL's order: one wave per point gathers its salient neighbours as
// (d2, index) keys into LDS, bitonic-sorts them (= FLANN's sorted result), stages their
// coordinates, and one lane runs the sequential double chains.  More than kOrdCap neighbours:
// the point is masked for the list path (pfx_nblist).
constexpr int kOrdCap = kWaveSortCap;

__global__ void __launch_bounds__(256) k_iss_ordered(GridView g, const int32_t* __restrict__ oq,
                                                     int* __restrict__ n_oq, float rr, int min_nb, double g21,
                                                     double g32, double* __restrict__ third,
                                                     uint8_t* __restrict__ mask, int* __restrict__ n_over) {
  __shared__ uint64_t s_key[4][kOrdCap];
  __shared__ float s_c[4][3][kOrdCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int count = n_oq[0];
  uint64_t* key = s_key[wv];
  for (;;) {  // dynamic queue: the cost per point varies with the local density
    int w = 0;
    if (lane == 0) w = atomicAdd(n_oq + 4, 1);
    w = __shfl(w, 0);
    if (w >= count) break;
    const int32_t p = oq[w];
    const float4 q = g.sp[p];
    const int32_t i = g.perm[p];
    Runs R;
    query_runs(g, q.x, q.y, q.z, R);
    const int32_t T = R.pref[9];
    int k = 0;
    for (int32_t t0 = 0; t0 < T; t0 += 64) {
      const int32_t t = t0 + lane;
      bool hit = false;
      uint64_t kv = 0;
      if (t < T) {
        const int32_t pos = run_pos(R, t);
        const float4 v = g.sp[pos];
        const float d2 = flann_d2(q.x, q.y, q.z, v.x, v.y, v.z);
        hit = d2 < rr;
        kv = nb_key(d2, g.perm[pos]);
      }
      const uint64_t m = __ballot(hit);
      const int slot = k + __popcll(m & lanemask_lt());
      if (hit && slot < kOrdCap) key[slot] = kv;
      k += __popcll(m);
    }
    if (k > kOrdCap) {
      if (lane == 0) {
        mask[i] = 1;
        atomicAdd(n_over, 1);
      }
      continue;
    }
    wave_sort_keys(key, k, lane);  // = FLANN's sorted result
    for (int m = lane; m < k; m += 64) {
      const int32_t j = key_idx(key[m]);
      s_c[wv][0][m] = g.ux[j];
      s_c[wv][1][m] = g.uy[j];
      s_c[wv][2][m] = g.uz[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      const double qx = q.x, qy = q.y, qz = q.z;
      double c00 = 0.0, c01 = 0.0, c02 = 0.0, c11 = 0.0, c12 = 0.0, c22 = 0.0;
      for (int m = 0; m < k; ++m) {
        const double dx = (double)s_c[wv][0][m] - qx, dy = (double)s_c[wv][1][m] - qy, dz = (double)s_c[wv][2][m] - qz;
        c00 += dx * dx;
        c01 += dx * dy;
        c02 += dx * dz;
        c11 += dy * dy;
        c12 += dy * dz;
        c22 += dz * dz;
      }
      third[i] = k >= min_nb ? iss_third(c00, c01, c02, c11, c12, c22, g21, g32) : 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the LDS regions are rewritten by the next point
  }
}

__global__ void __launch_bounds__(256) k_sum_u32(const unsigned int* __restrict__ v, int64_t n,
                                                 unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s[4];
  unsigned long long a = 0;
  for (int64_t i = threadIdx.x; i < n; i += 256) a += v[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) *out = s[0] + s[1] + s[2] + s[3];
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
  TimeScope total(ctx, "resolution", true);
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
      float2* part = ctx->buf("res_brute").as<float2>((size_t)h_fail * kParts);
      k_nn2_brute<<<(unsigned)(h_fail * kParts), 256, 0, st>>>(view(G), fail, part);
      k_nn2_brute_merge<<<(unsigned)ceil_div(h_fail, 64), 64, 0, st>>>(fail, h_fail, part, term);
      check_launch("k_nn2_brute");
      break;
    }
    queue = fail;
    fail = fail == qa ? qb : qa;
    h *= 2.0;
  }
  const int nblk = (int)std::min<int64_t>(ceil_div(n, 256), 1024);
  ResPart* part = ctx->buf("res_part").as<ResPart>(nblk);
  ResAcc* acc = ctx->buf("res_acc").as<ResAcc>(1);
  {
    TimeScope ts(ctx, "resolution_sum");
    k_res_partial<<<nblk, 256, 0, st>>>(term, n, part);
    k_res_final<<<1, 64, 0, st>>>(part, nblk, acc);
    check_launch("k_res_sum");
  }
  ResAcc h_acc;
  PFX_HIP(hipMemcpyAsync(&h_acc, acc, sizeof(h_acc), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  double sum = 0.0;
  const bool exact = h_acc.exact != 0;
  if (exact) {
    sum = std::ldexp((double)h_acc.isum, h_acc.L);
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
  TimeScope total(ctx, "iss", true);
  double* third = third_out ? third_out : ctx->buf("iss_third").as<double>(n);
  PFX_HIP(hipMemsetAsync(third, 0, sizeof(double) * n, st));
  build_grid(ctx, K.sal, x, y, z, n, salient);
  const unsigned nb = (unsigned)ceil_div(n, 256);
  uint8_t* mask = ctx->buf("iss_mask").as<uint8_t>(n);
  int32_t* oq = ctx->buf("iss_oq").as<int32_t>(n);
  // [0] queued for the ordered scatter, [1] of those beyond kOrdCap, [2..3] u64 neighbour count,
  // [4] queue head of k_iss_ordered
  int* n_mask = ctx->buf("iss_nmask").as<int>(6);
  unsigned int* part = ctx->buf("iss_part").as<unsigned int>(nb);
  PFX_HIP(hipMemsetAsync(n_mask, 0, 6 * sizeof(int), st));
  {
    TimeScope ts(ctx, "iss_scatter");
    k_iss_cov<<<nb, 256, 0, st>>>(view(K.sal), (float)(salient * salient), min_nb, g21, g32, third, oq, n_mask,
                                  part);
    k_sum_u32<<<1, 256, 0, st>>>(part, nb, reinterpret_cast<unsigned long long*>(n_mask + 2));
    check_launch("k_iss_cov");
  }
  {
    TimeScope ts(ctx, "iss_ordered");
    PFX_HIP(hipMemsetAsync(mask, 0, n, st));
    // persistent: the queue length stays on the device
    k_iss_ordered<<<1024, 256, 0, st>>>(view(K.sal), oq, n_mask, (float)(salient * salient), min_nb, g21, g32,
                                        third, mask, n_mask + 1);
    check_launch("k_iss_ordered");
  }
  int h_nm[4];
  PFX_HIP(hipMemcpyAsync(h_nm, n_mask, sizeof(h_nm), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  int64_t nbrs = 0;
  std::memcpy(&nbrs, h_nm + 2, sizeof(nbrs));
  ctx->stats["iss_neighbors"] = nbrs;
  ctx->stats["iss_ordered"] = h_nm[0];
  ctx->stats["iss_ordered_lists"] = h_nm[1];
  if (h_nm[1] > 0) {  // ordered points with more than kOrdCap neighbours: masked FLANN-ordered lists
    TimeScope ts(ctx, "iss_ordered_lists");
    build_lists(ctx, K.sal, mask, salient, true, K.L, "iss");
    if (K.L.nq > 0) {
      k_iss_scatter<<<(unsigned)ceil_div(K.L.nq, 256), 256, 0, st>>>(view(K.sal), K.L, min_nb, g21, g32, third);
      check_launch("k_iss_scatter");
    }
  }
  build_grid(ctx, K.nms, x, y, z, n, non_max);
  double* tn = ctx->buf("iss_tn").as<double>(n);
  uint8_t* flag = ctx->buf("iss_flag").as<uint8_t>(n);
  PFX_HIP(hipMemsetAsync(flag, 0, n, st));
  {
    TimeScope ts(ctx, "iss_nms");
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
