// pfx_shot.hip -- SHOTEstimationOMP<PointXYZRGB,Normal,SHOT352> (evaluation.cpp:766-785 via
// Features<T>::compute, features.h:175-196) on gfx950.  SURVEY A.7.
//
// One 256-thread workgroup per query:
//   1. radius neighbours in FLANN order (bitonic sort of (d2, caller index) keys in LDS);
//   2. SHOTLocalReferenceFrameEstimation::getLocalRF: the weighted double covariance is a set of
//      strictly ordered double chains (one lane per matrix entry + one for the weight sum) over
//      LDS-staged neighbour chunks; Eigen 3.2.0's SelfAdjointEigenSolver<Matrix3d> with
//      eigenvectors (pfx_eigen3.h, the oracle's operation sequence); sign disambiguation counts
//      reduced over the block;
//   3. SHOT: every neighbour's (up to) five interpolated bin updates are computed in parallel and
//      applied per bin in PCL's sequential order (each wave owns a quarter of the bins; lanes
//      that collide on a bin are serialised lowest-first); normalizeHistogram by one lane (double accumulation, as PCL).
// Descriptors and reference frames are bit-exact against the restatement.
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_eigen3.h"
#include "pfx_neighbors.h"

namespace pfx {
namespace {

#ifdef PFX_SHOT_PROFILE
// phase cycles (thread 0 of each workgroup): [7] sequential normalisations, [8] normalisation
// cycles; k_shot_lrf: [10] search + sort, [11] records, [12] LRF chains, [13] queries
__device__ unsigned long long g_shot_prof[16];
#define SPROF_T(v) long long v = (threadIdx.x == 0) ? clock64() : 0
#define SPROF_ADD(i, a, b) if (threadIdx.x == 0) atomicAdd(&g_shot_prof[i], (unsigned long long)((b) - (a)))
#else
#define SPROF_T(v)
#define SPROF_ADD(i, a, b)
#endif

#ifndef PFX_SHOT_GRID_MUL  // (A/B: the split kernels' grids, x this)
#define PFX_SHOT_GRID_MUL 4
#endif
constexpr int kCapSmall = 2048;  // sorted-neighbour capacity of the first pass (LDS keys, 5 WG/CU)
constexpr int kCap = 16384;      // second pass for the longer lists (1 WG/CU)
constexpr int kChunk = 256;   // neighbours staged per chunk
constexpr int kLen = 352, kBins = 10;
constexpr double kRad45 = 0.78539816339744830961566084581988;
constexpr double kRad90 = 1.5707963267948966192313216916398;
constexpr double kRad135 = 2.3561944901923449288469825374596;
constexpr double kRadPi78 = 2.7488935718910690836548129603691;

// the five (bin, value) updates of one neighbour (SHOTEstimation::interpolateSingleChannel with
// the bin distance of createBinDistanceShape); bin -1 = no update.  Order = PCL's order.
__device__ __forceinline__ void shot_updates(f3 delta, double distance, double binDist, f3 fx, f3 fy, f3 fz,
                                             double radius, int bins[5], float vals[5]) {
  for (int s = 0; s < 5; ++s) bins[s] = -1;
  const double radius3_4 = (radius * 3) / 4, radius1_4 = radius / 4, radius1_2 = radius / 2;
  double xIn = dot4(delta, fx), yIn = dot4(delta, fy), zIn = dot4(delta, fz);
  if (fabs(yIn) < 1E-30) yIn = 0;
  if (fabs(xIn) < 1E-30) xIn = 0;
  if (fabs(zIn) < 1E-30) zIn = 0;
  const int bit4 = ((yIn > 0) || ((yIn == 0.0) && (xIn < 0))) ? 1 : 0;
  const int bit3 = ((xIn > 0) || ((xIn == 0.0) && (yIn > 0))) ? !bit4 : bit4;
  int desc_index = ((bit4 << 3) + (bit3 << 2)) << 1;
  if ((xIn * yIn > 0) || (xIn == 0.0))
    desc_index += (fabs(xIn) >= fabs(yIn)) ? 0 : 4;
  else
    desc_index += (fabs(xIn) > fabs(yIn)) ? 4 : 0;
  desc_index += zIn > 0 ? 1 : 0;
  desc_index += (distance > radius1_2) ? 2 : 0;
  const int step_index = (int)floor(binDist + 0.5);
  const int volume_index = desc_index * (kBins + 1);
  binDist -= step_index;
  double intWeight = (1 - fabs(binDist));
  if (binDist > 0) {
    bins[0] = volume_index + ((step_index + 1) % kBins);
    vals[0] = (float)binDist;
  } else {
    bins[0] = volume_index + ((step_index - 1 + kBins) % kBins);
    vals[0] = -(float)binDist;
  }
  if (distance > radius1_2) {
    const double rd = (distance - radius3_4) / radius1_2;
    if (distance > radius3_4) {
      intWeight += 1 - rd;
    } else {
      intWeight += 1 + rd;
      bins[1] = (desc_index - 2) * (kBins + 1) + step_index;
      vals[1] = -(float)rd;
    }
  } else {
    const double rd = (distance - radius1_4) / radius1_2;
    if (distance < radius1_4) {
      intWeight += 1 + rd;
    } else {
      intWeight += 1 - rd;
      bins[1] = (desc_index + 2) * (kBins + 1) + step_index;
      vals[1] = (float)rd;
    }
  }
  double ic = zIn / distance;
  if (ic < -1.0) ic = -1.0;
  if (ic > 1.0) ic = 1.0;
  const double incl = acos(ic);
  if (incl > kRad90 || (fabs(incl - kRad90) < 1e-30 && zIn <= 0)) {
    const double idist = (incl - kRad135) / kRad90;
    if (incl > kRad135) {
      intWeight += 1 - idist;
    } else {
      intWeight += 1 + idist;
      bins[2] = (desc_index + 1) * (kBins + 1) + step_index;
      vals[2] = -(float)idist;
    }
  } else {
    const double idist = (incl - kRad45) / kRad90;
    if (incl < kRad45) {
      intWeight += 1 + idist;
    } else {
      intWeight += 1 - idist;
      bins[2] = (desc_index - 1) * (kBins + 1) + step_index;
      vals[2] = (float)idist;
    }
  }
  if (yIn != 0.0 || xIn != 0.0) {
    const double azimuth = atan2(yIn, xIn);
    const int sel = desc_index >> 2;
    double ad = (azimuth - (-kRadPi78 + kRad45 * sel)) / kRad45;
    ad = fmax(-0.5, fmin(ad, 0.5));
    if (ad > 0) {
      intWeight += 1 - ad;
      bins[3] = ((desc_index + 4) % 32) * (kBins + 1) + step_index;
      vals[3] = (float)ad;
    } else {
      intWeight += 1 + ad;
      bins[3] = ((desc_index - 4 + 32) % 32) * (kBins + 1) + step_index;
      vals[3] = -(float)ad;
    }
  }
  bins[4] = volume_index + step_index;
  vals[4] = (float)intWeight;
}


// the seven distinct LRF chains: cov (0,0) (0,1) (0,2) (1,1) (1,2) (2,2) and the weight sum
constexpr int kChains = 7;
constexpr int kMaskWords = kChunk / 64;

struct ShotLds {
  union {
    double lrf[kChains][kChunk];  // per-neighbour chain terms of one chunk (0 for invalid ones)
    struct {
      uint64_t mask[kMaskWords][kLen];  // which neighbours of the chunk hit each bin (word-major:
                                        // the bin owners' reads are lane-consecutive)
      int off[kLen + 1];                // bucket offsets (exclusive scan of the hit counts)
      int seg[8];                       // the counts' scan: totals of the 64-bin segments
      uint32_t pw[kLen];                // per bin: hits from waves < 1, < 2, < 3 (a byte each)
      float val[5 * kChunk];            // the chunk's update values bucketed by bin, neighbour order
    } upd;
    alignas(16) float hist[kLen];  // the finished histogram (written once the chunks are binned)
  };
  double cov[10];
  double axes[6];  // v1 (x axis), v3 (z axis)
  int lrf_l[4];    // normalisation: per-wave smallest lsb exponent and largest square
  float lrf_m[4];
  float rf[9];
  int n_invalid, zero_prefix, plusT, plusN, ok;
};

// ---- the phases of one query, shared by the fused and the split kernels ----

// A query's neighbour j for the frame and the histogram: its offset from the query (the float
// subtraction PCL's `delta` is) with its d2, and its normal.  NbKeys: from the FLANN keys and the
// caller-order arrays (the fused kernel); NbRecs: from the records k_shot_lrf writes (one float4
// of offset + d2 and one of normal per neighbour, two planes of kCapSmall per query), so the
// split kernels read a neighbour with one coalesced load instead of a key, then its point.
struct NbKeys {
  const uint64_t* keys;
  const float *ux, *uy, *uz, *nx, *ny, *nz;
  float cx, cy, cz;
  __device__ __forceinline__ float4 pt(int j) const {
    const uint64_t key = keys[j];
    const int32_t p = key_idx(key);
    return make_float4(ux[p] - cx, uy[p] - cy, uz[p] - cz, key_d2(key));
  }
  __device__ __forceinline__ float3 nrm(int j) const {
    const int32_t p = key_idx(keys[j]);
    return make_float3(nx[p], ny[p], nz[p]);
  }
};
struct NbRecs {
  const float4* __restrict__ pts;   // {dx, dy, dz, d2}
  const float4* __restrict__ nrms;  // {nx, ny, nz, 0}
  __device__ __forceinline__ float4 pt(int j) const { return pts[j]; }
  __device__ __forceinline__ float3 nrm(int j) const {
    const float4 v = nrms[j];
    return make_float3(v.x, v.y, v.z);
  }
};
// (a copy of the query: a zero offset -- a difference of finite floats is zero only when they are
// equal)
__device__ __forceinline__ bool nb_self(const float4& c) { return c.x == 0.0f && c.y == 0.0f && c.z == 0.0f; }

// SHOTLocalReferenceFrameEstimation's weighted double covariance over keys[0..k): S.cov (3x3
// row-major + the weight sum at [9]), S.n_invalid (copies of the query), S.zero_prefix.
// Every thread forms its neighbour's chain terms dist * (v_a * v_b) and dist exactly as the
// reference loop does; lanes 0..6 then add them in neighbour order (the only sequential part).
// An invalid neighbour (a copy of the query) contributes +0.0, which leaves a chain unchanged.
template <class Lds, class Src>
__device__ __forceinline__ void shot_lrf(Lds& S, double (*lrf)[kChunk], const Src& src, int k, double radius) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    S.n_invalid = 0; S.zero_prefix = 0; S.plusT = 0; S.plusN = 0;
  }
  double acc = 0.0;
  // the next chunk's neighbour is loaded while lanes 0..6 sum the current one
  float4 c_n = tid < k ? src.pt(tid) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c0 = 0; c0 < k; c0 += kChunk) {
    const int m = min(kChunk, k - c0);
    const float4 c = c_n;
    if (c0 + kChunk + tid < k) c_n = src.pt(c0 + kChunk + tid);
    __syncthreads();
    if (tid < m) {
      const bool valid = !nb_self(c);
      const double vx = (double)c.x, vy = (double)c.y, vz = (double)c.z;
      const double dist = radius - sqrt((double)c.w);
      lrf[0][tid] = valid ? dist * (vx * vx) : 0.0;
      lrf[1][tid] = valid ? dist * (vx * vy) : 0.0;
      lrf[2][tid] = valid ? dist * (vx * vz) : 0.0;
      lrf[3][tid] = valid ? dist * (vy * vy) : 0.0;
      lrf[4][tid] = valid ? dist * (vy * vz) : 0.0;
      lrf[5][tid] = valid ? dist * (vz * vz) : 0.0;
      lrf[6][tid] = valid ? dist : 0.0;
      if (!valid) atomicAdd(&S.n_invalid, 1);
      if (c.w == 0.0f) atomicAdd(&S.zero_prefix, 1);
    }
    __syncthreads();
    if (tid < kChains) {  // (32 terms loaded per round: one LDS latency per 32 dependent adds)
      const double* row = lrf[tid];
      int t = 0;
      for (; t + 32 <= m; t += 32) {
        double2 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const double2*>(row + t + 2 * u);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc = acc + v[u].x;
          acc = acc + v[u].y;
        }
      }
      for (; t < m; ++t) acc = acc + row[t];
    }
  }
  __syncthreads();
  if (tid < kChains) {  // chain -> cov[3a + b] (v_a v_b == v_b v_a exactly), cov[9] = weight sum
    constexpr int kSlot[kChains][2] = {{0, 0}, {1, 3}, {2, 6}, {4, 4}, {5, 7}, {8, 8}, {9, 9}};
    S.cov[kSlot[tid][0]] = acc;
    S.cov[kSlot[tid][1]] = acc;
  }
  __syncthreads();
}

// `cov_m /= sum` (Eigen 3.2: times the reciprocal), SelfAdjointEigenSolver<Matrix3d>: axes = the
// x (largest) and z (smallest) eigenvectors; false when the frame is undefined (PCL: NaN rows)
__device__ __forceinline__ bool shot_eigen(const double cov[10], int valid, double axes[6]) {
  if (valid < 5) return false;
  double ev[3], V[3][3];
  const double inv = 1.0 / cov[9];
  eigen_selfadjoint3<true>(cov[0] * inv, cov[3] * inv, cov[4] * inv, cov[6] * inv, cov[7] * inv, cov[8] * inv, ev,
                           V);
  if (!(isfinite(ev[0]) && isfinite(ev[1]) && isfinite(ev[2]))) return false;
  for (int i = 0; i < 3; ++i) { axes[i] = V[2][i]; axes[3 + i] = V[0][i]; }
  return true;
}

// sign disambiguation of S.axes over the valid neighbours, then S.rf (x, y = z cross x, z)
template <class Lds, class Src>
__device__ __forceinline__ void shot_frame(Lds& S, const Src& src, int k, int valid) {
  const int tid = threadIdx.x, lane = tid & 63;
  {
    const double v1x = S.axes[0], v1y = S.axes[1], v1z = S.axes[2];
    const double v3x = S.axes[3], v3y = S.axes[4], v3z = S.axes[5];
    int cT = 0, cN = 0;
    for (int j0 = tid; j0 < k; j0 += 4 * 256) {  // (four neighbours per thread in flight)
      float4 c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + 256 * u;
        c[u] = src.pt(j < k ? j : j0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j0 + 256 * u >= k || nb_self(c[u])) continue;
        const double vx = (double)c[u].x, vy = (double)c[u].y, vz = (double)c[u].z;
        if (((vx * v1x + vy * v1y) + vz * v1z) + 0.0 >= 0) ++cT;
        if (((vx * v3x + vy * v3y) + vz * v3z) + 0.0 >= 0) ++cN;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { cT += __shfl_xor(cT, o); cN += __shfl_xor(cN, o); }
    if (lane == 0) { atomicAdd(&S.plusT, cT); atomicAdd(&S.plusN, cN); }
  }
  __syncthreads();
  if (tid == 0) {
    double ax[2][3] = {{S.axes[0], S.axes[1], S.axes[2]}, {S.axes[3], S.axes[4], S.axes[5]}};
    const int counts[2] = {S.plusT, S.plusN};
    // the valid neighbours in order: the d2 == 0 prefix holds every invalid one
    const int zp = S.zero_prefix;
    int valid_in_prefix = 0;
    for (int j = 0; j < zp; ++j)
      if (!nb_self(src.pt(j))) ++valid_in_prefix;
    for (int w = 0; w < 2; ++w) {
      int plus = 2 * counts[w] - valid;
      if (plus == 0) {
        const int median = valid / 2;
        for (int i = -2; i <= 2; ++i) {
          const int ne = median - i;
          int j;
          if (ne < valid_in_prefix) {
            int seen = -1;
            for (j = 0; j < zp; ++j)
              if (!nb_self(src.pt(j)) && ++seen == ne) break;
          } else {
            j = zp + (ne - valid_in_prefix);
          }
          const float4 c = src.pt(j);
          const double vx = (double)c.x, vy = (double)c.y, vz = (double)c.z;
          if (((vx * ax[w][0] + vy * ax[w][1]) + vz * ax[w][2]) + 0.0 > 0) ++plus;
        }
        if (plus < 3)
          for (int c = 0; c < 3; ++c) ax[w][c] *= -1;
      } else if (plus < 0) {
        for (int c = 0; c < 3; ++c) ax[w][c] *= -1;
      }
    }
    const f3 x = mk3((float)ax[0][0], (float)ax[0][1], (float)ax[0][2]);
    const f3 z = mk3((float)ax[1][0], (float)ax[1][1], (float)ax[1][2]);
    const f3 y = cross3(z, x);
    S.rf[0] = x.x; S.rf[1] = x.y; S.rf[2] = x.z;
    S.rf[3] = y.x; S.rf[4] = y.y; S.rf[5] = y.z;
    S.rf[6] = z.x; S.rf[7] = z.y; S.rf[8] = z.z;
  }
}

// exponent of the least significant set bit of a finite nonzero float
__device__ __forceinline__ int lsb_exp_f(float v) {
  const uint32_t b = __float_as_uint(v);
  const int e = (int)((b >> 23) & 0xff);
  const uint32_t m = b & 0x7fffffu;
  const uint32_t full = e ? (m | 0x800000u) : m;
  return (e ? e : 1) - 150 + __builtin_ctz(full);
}

// The histogram's per-chunk binning.  Each neighbour adds to at most one bin per update statement
// (its <= 5 bins are distinct), so PCL's sequential order restricted to one bin is neighbour
// order.  Per chunk of m neighbours (one per thread): hit masks per bin -> counts -> offsets ->
// every update written to its bin's bucket at its rank among the bin's hits (a stable counting
// sort) -> each bin's owner (thread j: bins j and j + 256) adds its bucket in order.  The masks
// must be zero on entry (they are left zero).
__device__ __forceinline__ void hist_chunk(ShotLds& S, int m, const int bins[5], const float vals[5], float& h0,
                                           float& h1) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int b0 = tid, b1 = tid + 256;
  SPROF_T(h0t);
  if (tid < m) {
    const uint64_t bit = 1ull << (tid & 63);
#pragma unroll
    for (int s = 0; s < 5; ++s)
      if (bins[s] >= 0) atomicOr(reinterpret_cast<unsigned long long*>(&S.upd.mask[tid >> 6][bins[s]]), bit);
  }
  __syncthreads();
  SPROF_T(h1t);
  SPROF_ADD(0, h0t, h1t);
  // hit counts -> exclusive offsets: thread t counts its bins t and t + 256 (the bins it sums
  // below), wave scans, the eight segment totals through LDS
  static_assert(kMaskWords == 4, "one byte per lower wave");
  int c0 = 0, c1 = 0;
  {
    uint32_t pw = 0;
#pragma unroll
    for (int w = 0; w < kMaskWords; ++w) {
      c0 += __popcll(S.upd.mask[w][b0]);
      if (w < kMaskWords - 1) pw |= (uint32_t)c0 << (8 * w);
    }
    S.upd.pw[b0] = pw;
  }
  if (b1 < kLen) {
    uint32_t pw = 0;
#pragma unroll
    for (int w = 0; w < kMaskWords; ++w) {
      c1 += __popcll(S.upd.mask[w][b1]);
      if (w < kMaskWords - 1) pw |= (uint32_t)c1 << (8 * w);
    }
    S.upd.pw[b1] = pw;
  }
  int i0 = c0, i1 = c1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y0 = __shfl_up(i0, o), y1 = __shfl_up(i1, o);
    if (lane >= o) { i0 += y0; i1 += y1; }
  }
  const int wv = tid >> 6;
  if (lane == 63) { S.upd.seg[wv] = i0; S.upd.seg[4 + wv] = i1; }
  __syncthreads();
  {
    int p0 = 0, p1 = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int s0 = S.upd.seg[v], s1 = S.upd.seg[4 + v];
      p1 += s0;
      if (v < wv) { p0 += s0; p1 += s1; }
    }
    S.upd.off[b0] = p0 + i0 - c0;
    if (b1 < kLen) S.upd.off[b1] = p1 + i1 - c1;
  }
  __syncthreads();
  SPROF_T(h2t);
  SPROF_ADD(1, h1t, h2t);
  if (tid < m) {  // scatter: rank = hits of the bin from lower neighbours of the chunk
    const int wq = tid >> 6;
    const uint64_t below = lanemask_lt();
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int bb = bins[s];
      if (bb < 0) continue;
      int r = __popcll(S.upd.mask[wq][bb] & below);
      if (wq) r += (int)((S.upd.pw[bb] >> (8 * (wq - 1))) & 0xffu);
      S.upd.val[S.upd.off[bb] + r] = vals[s];
    }
  }
  __syncthreads();
  SPROF_T(h3t);
  SPROF_ADD(2, h2t, h3t);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int b = o ? b1 : b0;
    if (b < kLen) {
      const int cnt = o ? c1 : c0;
#pragma unroll
      for (int w = 0; w < kMaskWords; ++w) S.upd.mask[w][b] = 0;  // ready for the next chunk
      const float* v = S.upd.val + S.upd.off[b];
      float h = o ? h1 : h0;
      int i = 0;
      for (; i + 4 <= cnt; i += 4) {
        const float a0 = v[i], a1 = v[i + 1], a2 = v[i + 2], a3 = v[i + 3];
        h = h + a0; h = h + a1; h = h + a2; h = h + a3;
      }
      for (; i < cnt; ++i) h = h + v[i];
      if (o) h1 = h; else h0 = h;
    }
  }
  __syncthreads();
  SPROF_T(h4t);
  SPROF_ADD(3, h3t, h4t);
}

__device__ __forceinline__ void hist_clear(ShotLds& S) {
  for (int i = threadIdx.x; i < kLen; i += 256)
    for (int w = 0; w < kMaskWords; ++w) S.upd.mask[w][i] = 0;
  __syncthreads();
}

// normalizeHistogram and the outputs (rfo: the frame rows, nullable)
__device__ __forceinline__ void hist_finish(ShotLds& S, float h0, float h1, float* __restrict__ d,
                                            float* __restrict__ rfo) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int b0 = tid, b1 = tid + 256;
  SPROF_T(pe0);
  S.hist[b0] = h0;
  if (b1 < kLen) S.hist[b1] = h1;
  __syncthreads();
  // normalizeHistogram: acc_norm += shot[j] * shot[j] (float squares, double sum, in bin order).
  // The squares are multiples of 2^L (L the smallest least-significant-bit exponent among the
  // nonzero ones) and non-negative, so when 352 x the largest stays below 2^(L + 53) every
  // partial sum is exact and any order gives PCL's value: a parallel sum; otherwise one lane
  // runs the sequential loop.
  {
    float sq[2] = {h0 * h0, b1 < kLen ? h1 * h1 : 0.0f};
    double part = (double)sq[0] + (double)sq[1];
    float mx = fmaxf(sq[0], sq[1]);
    int L = 1 << 20;
    for (int o = 0; o < 2; ++o)
      if (sq[o] != 0.0f && isfinite(sq[o])) L = min(L, lsb_exp_f(sq[o]));
      else if (!(sq[o] == 0.0f)) L = -(1 << 20);  // non-finite: the sequential loop decides
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      part += __shfl_xor(part, o);
      mx = fmaxf(mx, __shfl_xor(mx, o));
      L = min(L, __shfl_xor(L, o));
    }
    if (lane == 0) {
      S.axes[tid >> 6] = part;  // (axes are dead here: four wave partials)
      S.lrf_l[tid >> 6] = L;
      S.lrf_m[tid >> 6] = mx;
    }
    __syncthreads();
    if (tid == 0) {
      const double tot = (S.axes[0] + S.axes[1]) + (S.axes[2] + S.axes[3]);
      const int Lm = min(min(S.lrf_l[0], S.lrf_l[1]), min(S.lrf_l[2], S.lrf_l[3]));
      const float mm = fmaxf(fmaxf(S.lrf_m[0], S.lrf_m[1]), fmaxf(S.lrf_m[2], S.lrf_m[3]));
      double acc_norm;
      if (mm == 0.0f) {
        acc_norm = 0.0;
      } else if (Lm > -(1 << 19) && (double)mm * kLen < ldexp(1.0, Lm + 53)) {
        acc_norm = tot;
      } else {
        acc_norm = 0;
        // (PCL's order; the squares read 16 at a time, so only the additions are sequential)
        for (int j = 0; j < kLen; j += 16) {
          float4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(S.hist + j + 4 * u);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            acc_norm += v[u].x * v[u].x;
            acc_norm += v[u].y * v[u].y;
            acc_norm += v[u].z * v[u].z;
            acc_norm += v[u].w * v[u].w;
          }
        }
#ifdef PFX_SHOT_PROFILE
        atomicAdd(&g_shot_prof[7], 1ull);
#endif
      }
      S.cov[0] = sqrt(acc_norm);
    }
    __syncthreads();
  }
  SPROF_T(pe1);
  SPROF_ADD(8, pe0, pe1);
  const float nrm = (float)S.cov[0];
  for (int i = tid; i < kLen; i += 256) d[i] = S.hist[i] / nrm;
  if (rfo && tid < 9) rfo[tid] = S.rf[tid];
  __syncthreads();
}

// a neighbour's (<= 5) histogram updates from the frame S.rf (fx, fy, fz)
__device__ __forceinline__ void nb_updates(const float4& c, const float3& nv, const f3& fx, const f3& fy,
                                           const f3& fz, double radius, int bins[5], float vals[5]) {
#pragma unroll
  for (int s = 0; s < 5; ++s) bins[s] = -1;
  const double distance = sqrt((double)c.w);
  if (isfinite(nv.x) && isfinite(nv.y) && isfinite(nv.z) && !(fabs(distance - 0.0) < 1E-15)) {
    double cosd = dot4(mk3(nv.x, nv.y, nv.z), fz);
    if (cosd > 1.0) cosd = 1.0;
    if (cosd < -1.0) cosd = -1.0;
    const double binDist = ((1.0 + cosd) * kBins) / 2;
    shot_updates(mk3(c.x, c.y, c.z), distance, binDist, fx, fy, fz, radius, bins, vals);
  }
}

// the SHOT histogram from S.rf, normalizeHistogram, outputs (the fused kernel: updates computed
// chunk by chunk)
template <class Src>
__device__ __forceinline__ void shot_hist(ShotLds& S, const Src& src, int k, double radius, float* __restrict__ d,
                                          float* __restrict__ rfo) {
  const int tid = threadIdx.x;
  float h0 = 0.0f, h1 = 0.0f;
  hist_clear(S);
  const f3 fx = mk3(S.rf[0], S.rf[1], S.rf[2]), fy = mk3(S.rf[3], S.rf[4], S.rf[5]),
           fz = mk3(S.rf[6], S.rf[7], S.rf[8]);
  for (int c0 = 0; c0 < k; c0 += kChunk) {
    const int m = min(kChunk, k - c0);
    int bins[5];
    float vals[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) bins[s] = -1;
    if (tid < m) nb_updates(src.pt(c0 + tid), src.nrm(c0 + tid), fx, fy, fz, radius, bins, vals);
    hist_chunk(S, m, bins, vals, h0, h1);
  }
  hist_finish(S, h0, h1, d, rfo);
}

// the split kernels' update records: one 32-B record per neighbour, {bin0 | bin1 << 16,
// bin2 | bin3 << 16, bin4 (low half), val0} + {val1, val2, val3, val4} (bins as int16, -1: none)
__device__ __forceinline__ void upd_pack(const int bins[5], const float vals[5], uint4& a, float4& b) {
  auto h = [](int v) { return (uint32_t)(uint16_t)(int16_t)v; };
  a = make_uint4(h(bins[0]) | (h(bins[1]) << 16), h(bins[2]) | (h(bins[3]) << 16), h(bins[4]),
                 __float_as_uint(vals[0]));
  b = make_float4(vals[1], vals[2], vals[3], vals[4]);
}
__device__ __forceinline__ void upd_unpack(const uint4& a, const float4& b, int bins[5], float vals[5]) {
  auto s = [](uint32_t v) { return (int)(int16_t)(uint16_t)v; };
  bins[0] = s(a.x); bins[1] = s(a.x >> 16); bins[2] = s(a.y); bins[3] = s(a.y >> 16); bins[4] = s(a.z);
  vals[0] = __uint_as_float(a.w); vals[1] = b.x; vals[2] = b.y; vals[3] = b.z; vals[4] = b.w;
}

__device__ __forceinline__ void shot_nan(float* __restrict__ d, float* __restrict__ rfo) {
  for (int i = threadIdx.x; i < kLen; i += 256) d[i] = __builtin_nanf("");
  if (threadIdx.x < 9) rfo[threadIdx.x] = __builtin_nanf("");
}

// Fused form (the lists longer than the split path's capacity): every phase of a query in one
// workgroup.  CAP: LDS key capacity.  `list` (nullable): query subset with its device-side
// count; queries with more than CAP neighbours go to `over` (or raise err when over == nullptr).
template <int CAP>
__global__ void __launch_bounds__(256) k_shot(GridView g, const float* __restrict__ nx,
                                              const float* __restrict__ ny, const float* __restrict__ nz,
                                              const float* __restrict__ qx, const float* __restrict__ qy,
                                              const float* __restrict__ qz, int64_t nq,
                                              const int32_t* __restrict__ list, const int* __restrict__ n_list,
                                              int32_t* __restrict__ over, int* __restrict__ n_over,
                                              double radius, float* __restrict__ desc, float* __restrict__ rf_out,
                                              int* __restrict__ err, unsigned long long* __restrict__ nbr) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];  // CAP (+ CAP sort scratch, first pass)
  __shared__ ShotLds S;
  __shared__ BucketLds SB;
  __shared__ int s_count;
  const int tid = threadIdx.x;
  const float rr = (float)(radius * radius);
  const int64_t count = list ? (int64_t)*n_list : nq;
  for (int64_t w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t q = list ? (int64_t)list[w] : w;
    float* d = desc + q * kLen;
    float* rfo = rf_out + q * 9;
    const float cx = qx[q], cy = qy[q], cz = qz[q];
    if (!(isfinite(cx) && isfinite(cy) && isfinite(cz))) {
      shot_nan(d, rfo);
      continue;
    }
    const int k = CAP == kCapSmall
                      ? sorted_neighbors_bucketed(g, cx, cy, cz, rr, keys, keys + CAP, CAP, &s_count, SB)
                      : sorted_neighbors(g, cx, cy, cz, rr, keys, CAP, &s_count);
    if (k > CAP) {
      if (tid == 0) {
        if (over) over[atomicAdd(n_over, 1)] = (int32_t)q;
        else atomicMax(err, k);
      }
      continue;
    }
    if (tid == 0) atomicAdd(nbr, (unsigned long long)k);
    const NbKeys src{keys, g.ux, g.uy, g.uz, nx, ny, nz, cx, cy, cz};
    shot_lrf(S, S.lrf, src, k, radius);
    const int valid = k - S.n_invalid;
    if (tid == 0) {
      double cov[10], axes[6];
      for (int i = 0; i < 10; ++i) cov[i] = S.cov[i];
      S.ok = shot_eigen(cov, valid, axes) ? 1 : 0;
      for (int i = 0; i < 6; ++i) S.axes[i] = axes[i];
    }
    __syncthreads();
    if (!S.ok) {
      shot_nan(d, rfo);
      continue;
    }
    shot_frame(S, src, k, valid);
    shot_hist(S, src, k, radius, d, rfo);
  }
}

// the split kernels' views of the surface: caller index -> cell-sorted position, and the normals
// in cell order.  Two coalesced-read passes (the inverse permutation, then each caller-order
// normal written to its cell position) instead of one pass gathering three 4-byte normal
// components through the permutation (283 MB fetched per 1M points: a cache line per component).
// (round 5: the records gathered from caller-order packed copies instead -- one global round,
// not two -- measured 0.92 -> 0.97 ms: the cell-sorted gathers' locality wins)
__global__ void k_shot_ipos(const int32_t* __restrict__ perm, int64_t n, int32_t* __restrict__ ipos) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) ipos[perm[i]] = (int32_t)i;
}
__global__ void k_shot_prep(const int32_t* __restrict__ ipos, int64_t n, const float* __restrict__ nx,
                            const float* __restrict__ ny, const float* __restrict__ nz, float4* __restrict__ snp) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) snp[ipos[i]] = make_float4(nx[i], ny[i], nz[i], 0.0f);
}

// ---- split form: the single-lane eigen solve off the workgroups' critical path ----
// Per query state between the three kernels.  status: 0 frame pending / defined, 1 done (NaN
// written: non-finite query or no frame), 2 over the split capacity (the fused kernel's).
struct ShotQuery {
  double cov[10];
  double axes[6];
  int k, n_invalid, zero_prefix, status;
};

// the LDS of the LRF phase alone (kernel A; its chain terms live in the sort's scratch half of
// the keys, free once the keys are sorted: 34 KB a workgroup, four per CU)
struct LrfLds {
  double cov[10];
  int n_invalid, zero_prefix, plusT, plusN;
};

// A: sort + LRF covariance; the neighbour records (NbRecs: offset + d2, normal) kept in global
// memory for C (two planes of kCapSmall float4 per query)
__global__ void __launch_bounds__(256) k_shot_lrf(GridView g, const float* __restrict__ qx,
                                                  const float* __restrict__ qy, const float* __restrict__ qz,
                                                  int64_t base, int64_t nq, int32_t* __restrict__ over,
                                                  int* __restrict__ n_over,
                                                  double radius, float* __restrict__ desc, float* __restrict__ rf_out,
                                                  float4* __restrict__ grec, ShotQuery* __restrict__ sq,
                                                  const int32_t* __restrict__ ipos, const float4* __restrict__ snp,
                                                  unsigned long long* __restrict__ nbr,
                                                  const int32_t* __restrict__ order) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];  // kCapSmall + kCapSmall scratch
  __shared__ LrfLds S;
  __shared__ BucketLds SB;
  __shared__ int s_count;
  const int tid = threadIdx.x;
  const float rr = (float)(radius * radius);
  // the queries in cell order (`order`, round 6), each XCD a contiguous eighth of them (blocks b
  // and b + 8 share an XCD): neighbouring queries' candidate blocks then come from the same L2
  // instead of each query scanning its r-block from HBM (r05: 2.0 GB fetched for 0.24 GB of
  // algorithmic bytes)
  int64_t l0 = blockIdx.x, lend = nq, lstep = gridDim.x;
  if (order && (gridDim.x & 7) == 0) {
    const int64_t per = (nq + 7) >> 3;
    l0 = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    lend = min(nq, (int64_t)((blockIdx.x & 7) + 1) * per);
    lstep = gridDim.x >> 3;
  }
  for (int64_t l = l0; l < lend; l += lstep) {  // l: index in the batch, q: caller's
    const int64_t q = order ? order[base + l] : base + l;
    const float cx = qx[q], cy = qy[q], cz = qz[q];
    if (!(isfinite(cx) && isfinite(cy) && isfinite(cz))) {
      shot_nan(desc + q * kLen, rf_out + q * 9);
      if (tid == 0) sq[l].status = 1;
      continue;
    }
    SPROF_T(l0);
    const int k = sorted_neighbors_bucketed(g, cx, cy, cz, rr, keys, keys + kCapSmall, kCapSmall, &s_count, SB);
    if (k > kCapSmall) {
      if (tid == 0) {
        over[atomicAdd(n_over, 1)] = (int32_t)q;
        sq[l].status = 2;
      }
      continue;
    }
    if (tid == 0) atomicAdd(nbr, (unsigned long long)k);
    SPROF_T(l1);
    SPROF_ADD(10, l0, l1);
    SPROF_ADD(13, 0, 1);
    // the keys (d2, caller index) in FLANN order -> the neighbour records, same order (read back
    // by this thread in shot_lrf, and by the frame and histogram kernel)
    // (four neighbours per thread in flight: two dependent global rounds for the whole list)
    float4* rp = grec + l * 2 * kCapSmall;
    for (int i0 = tid; i0 < k; i0 += 4 * 256) {
      uint64_t key[4];
      int32_t pos[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        key[u] = keys[min(i0 + 256 * u, k - 1)];
        pos[u] = ipos[key_idx(key[u])];
      }
      float4 c[4], nv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[u] = g.sp[pos[u]];
        nv[u] = snp[pos[u]];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 256 * u;
        if (i < k) {
          rp[i] = make_float4(c[u].x - cx, c[u].y - cy, c[u].z - cz, key_d2(key[u]));
          rp[kCapSmall + i] = make_float4(nv[u].x, nv[u].y, nv[u].z, 0.0f);
        }
      }
    }
    __syncthreads();
    SPROF_T(l2);
    SPROF_ADD(11, l1, l2);
    static_assert(sizeof(double) * kChains * kChunk <= sizeof(uint64_t) * kCapSmall, "chain terms fit the sort scratch");
    shot_lrf(S, reinterpret_cast<double(*)[kChunk]>(keys + kCapSmall), NbRecs{rp, rp + kCapSmall}, k, radius);
    SPROF_T(l3);
    SPROF_ADD(12, l2, l3);
    if (tid < 10) sq[l].cov[tid] = S.cov[tid];
    if (tid == 0) {
      sq[l].k = k;
      sq[l].n_invalid = S.n_invalid;
      sq[l].zero_prefix = S.zero_prefix;
      sq[l].status = 0;
    }
    __syncthreads();
  }
}

// B: one lane per query, SelfAdjointEigenSolver<Matrix3d>
__global__ void __launch_bounds__(64) k_shot_eigen(ShotQuery* __restrict__ sq, int64_t nq) {
  const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (q >= nq || sq[q].status != 0) return;
  double cov[10], axes[6];
  for (int i = 0; i < 10; ++i) cov[i] = sq[q].cov[i];
  if (shot_eigen(cov, sq[q].k - sq[q].n_invalid, axes)) {
    for (int i = 0; i < 6; ++i) sq[q].axes[i] = axes[i];
  } else {
    sq[q].status = 3;  // no frame: NaN rows (written by C)
  }
}

// C: sign disambiguation and the histogram updates of every neighbour, written as records (the
// double-precision interpolation of shot_updates, ~170 VGPRs: three workgroups per CU, with no
// barrier between a workgroup's neighbours)
struct FrameLds {
  double axes[6];
  float rf[9];
  int zero_prefix, plusT, plusN;
};
#ifndef PFX_SHOT_HIST_WG
#define PFX_SHOT_HIST_WG 3
#endif
__global__ void __launch_bounds__(256, PFX_SHOT_HIST_WG) k_shot_frame(int64_t base, int64_t nq, double radius,
                                                                       float* __restrict__ desc,
                                                                       float* __restrict__ rf_out,
                                                                       const float4* __restrict__ grec,
                                                                       const ShotQuery* __restrict__ sq,
                                                                       uint4* __restrict__ upd,
                                                                       const int32_t* __restrict__ order) {
  __shared__ FrameLds S;
  const int tid = threadIdx.x;
  for (int64_t l = blockIdx.x; l < nq; l += gridDim.x) {
    const int64_t q = order ? order[base + l] : base + l;
    const int status = sq[l].status;
    if (status == 1 || status == 2) continue;
    float* rfo = rf_out + q * 9;
    if (status == 3) {
      shot_nan(desc + q * kLen, rfo);
      continue;
    }
    const int k = sq[l].k;
    const NbRecs src{grec + l * 2 * kCapSmall, grec + l * 2 * kCapSmall + kCapSmall};
    if (tid < 6) S.axes[tid] = sq[l].axes[tid];
    if (tid == 0) {
      S.zero_prefix = sq[l].zero_prefix;
      S.plusT = 0;
      S.plusN = 0;
    }
    __syncthreads();
    SPROF_T(f0t);
    shot_frame(S, src, k, k - sq[l].n_invalid);
    __syncthreads();
    SPROF_T(f1t);
    SPROF_ADD(6, f0t, f1t);
    if (tid < 9) rfo[tid] = S.rf[tid];
    const f3 fx = mk3(S.rf[0], S.rf[1], S.rf[2]), fy = mk3(S.rf[3], S.rf[4], S.rf[5]),
             fz = mk3(S.rf[6], S.rf[7], S.rf[8]);
    uint4* u = upd + l * 2 * kCapSmall;
    for (int j = tid; j < k; j += 256) {
      int bins[5];
      float vals[5];
      nb_updates(src.pt(j), src.nrm(j), fx, fy, fz, radius, bins, vals);
      uint4 a;
      float4 b;
      upd_pack(bins, vals, a, b);
      u[2 * j] = a;
      reinterpret_cast<float4*>(u)[2 * j + 1] = b;
    }
    __syncthreads();  // S is rewritten by the next query
    SPROF_T(f2t);
    SPROF_ADD(9, f1t, f2t);
    SPROF_ADD(14, 0, 1);
  }
}

// D: the histogram from the update records, normalisation, descriptor (no double-precision
// interpolation here: a light kernel, many workgroups per CU)
#ifndef PFX_SHOT_ACCUM_WG
#define PFX_SHOT_ACCUM_WG 8
#endif
__global__ void __launch_bounds__(256, PFX_SHOT_ACCUM_WG) k_shot_accum(int64_t base, int64_t nq, float* __restrict__ desc,
                                                    const uint4* __restrict__ upd,
                                                    const ShotQuery* __restrict__ sq,
                                                    const int32_t* __restrict__ order) {
  __shared__ ShotLds S;
  const int tid = threadIdx.x;
  for (int64_t l = blockIdx.x; l < nq; l += gridDim.x) {
    if (sq[l].status != 0) continue;
    const int k = sq[l].k;
    SPROF_T(a0t);
    const uint4* u = upd + l * 2 * kCapSmall;
    float h0 = 0.0f, h1 = 0.0f;
    hist_clear(S);
    // the next chunk's records are loaded while this one is binned
    uint4 a_n = make_uint4(0, 0, 0, 0);
    float4 b_n = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < k) {
      a_n = u[2 * tid];
      b_n = reinterpret_cast<const float4*>(u)[2 * tid + 1];
    }
    for (int c0 = 0; c0 < k; c0 += kChunk) {
      const int m = min(kChunk, k - c0);
      const uint4 a = a_n;
      const float4 b = b_n;
      if (c0 + kChunk + tid < k) {
        a_n = u[2 * (c0 + kChunk + tid)];
        b_n = reinterpret_cast<const float4*>(u)[2 * (c0 + kChunk + tid) + 1];
      }
      int bins[5];
      float vals[5];
      upd_unpack(a, b, bins, vals);
      if (tid >= m) {
#pragma unroll
        for (int s = 0; s < 5; ++s) bins[s] = -1;
      }
      hist_chunk(S, m, bins, vals, h0, h1);
    }
    hist_finish(S, h0, h1, desc + (order ? (int64_t)order[base + l] : base + l) * kLen, nullptr);
    SPROF_T(a1t);
    SPROF_ADD(4, a0t, a1t);
    SPROF_ADD(5, 0, 1);
  }
}

// cell key of each query on the surface grid (clamped into it; non-finite: past the last cell),
// for the cell-ordered processing of k_shot_lrf
__global__ void __launch_bounds__(256) k_shot_qkeys(GridView g, const float* __restrict__ qx,
                                                    const float* __restrict__ qy, const float* __restrict__ qz,
                                                    int64_t nq, uint32_t* __restrict__ keys,
                                                    int32_t* __restrict__ vals) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float px = qx[i], py = qy[i], pz = qz[i];
  uint32_t key = (uint32_t)((int64_t)g.nx * g.ny * g.nz);
  if (isfinite(px) && isfinite(py) && isfinite(pz)) {
    int64_t ix = (int64_t)floor(((double)px - g.ox) * g.inv);
    int64_t iy = (int64_t)floor(((double)py - g.oy) * g.inv);
    int64_t iz = (int64_t)floor(((double)pz - g.oz) * g.inv);
    ix = ix < 0 ? 0 : (ix >= g.nx ? g.nx - 1 : ix);
    iy = iy < 0 ? 0 : (iy >= g.ny ? g.ny - 1 : iy);
    iz = iz < 0 ? 0 : (iz >= g.nz ? g.nz - 1 : iz);
    key = (uint32_t)((ix * g.ny + iy) * g.nz + iz);
  }
  keys[i] = key;
  vals[i] = (int32_t)i;
}

}  // namespace

// PFX_SHOT_ORDER=0: the split kernels take the queries in caller order (A/B)
static bool shot_cell_order() {
  static const bool on = [] {
    const char* e = getenv("PFX_SHOT_ORDER");
    return !(e && e[0] == '0');
  }();
  return on;
}

void shot_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx, const float* sny,
              const float* snz, int64_t ns, const float* qx, const float* qy, const float* qz, int64_t nq, double r,
              float* desc, float* rf) {
  PFX_CHECK(r > 0.0, "shot: radius must be > 0");
  if (nq == 0) return;
  hipStream_t st = ctx->stream;
  if (ns == 0) {
    std::vector<float> nanv((size_t)nq * kLen, __builtin_nanf(""));
    PFX_HIP(hipMemcpyAsync(desc, nanv.data(), sizeof(float) * nq * kLen, hipMemcpyHostToDevice, st));
    PFX_HIP(hipMemcpyAsync(rf, nanv.data(), sizeof(float) * nq * 9, hipMemcpyHostToDevice, st));
    PFX_HIP(hipStreamSynchronize(st));
    return;
  }
  // the surface grid prepared ahead (pfx_fpfh_prepare_dev: coordinates only, e.g. while the normals
  // are estimated on another stream), else built here
  const bool grid_ready = ctx->prep_x == sx && ctx->prep_n == ns && ctx->prep_r == r;
  if (grid_ready) fpfh_validate_grid(ctx);  // (a speculative prepared grid: exact after this)
  ctx->prep_x = nullptr;  // one-shot
  ctx->prep_n = -1;
  ctx->prep_qx = nullptr;
  ctx->prep_nq = -1;
  if (!grid_ready) build_grid(ctx, ctx->grid_b, sx, sy, sz, ns, r);
  GridView g = view(ctx->grid_b);
  int* err = ctx->buf("shot_err").as<int>(4);
  unsigned long long* nbr = reinterpret_cast<unsigned long long*>(err + 2);
  PFX_HIP(hipMemsetAsync(err, 0, 4 * sizeof(int), st));
  {
    TimeScope ts(ctx, "shot", true);
    int32_t* over = ctx->buf("shot_over").as<int32_t>(nq);
    int* n_over = err + 1;
    const size_t lds_s = 2 * sizeof(uint64_t) * kCapSmall, lds = sizeof(uint64_t) * kCap;
    PFX_HIP(hipFuncSetAttribute((const void*)k_shot<kCap>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    // lists <= kCapSmall: the split kernels in batches of kSplitBatch queries (sort + LRF
    // covariance per workgroup, the eigen solve one lane per query, frame + histogram per
    // workgroup; round 3: 1.93 -> 1.25 ms against every phase in one workgroup per query)
    {
      constexpr int64_t kSplitBatch = 16384;
      const int64_t bq = std::min<int64_t>(nq, kSplitBatch);
      float4* grec = ctx->buf("shot_recs").as<float4>((size_t)bq * 2 * kCapSmall);
      ShotQuery* sq = ctx->buf("shot_q").as<ShotQuery>((size_t)bq);
      uint4* upd = ctx->buf("shot_upd").as<uint4>((size_t)bq * 2 * kCapSmall);
      int32_t* ipos = ctx->buf("shot_ipos").as<int32_t>(ns);
      float4* snp = ctx->buf("shot_snp").as<float4>(ns);
      k_shot_ipos<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(ctx->grid_b.perm, ns, ipos);
      k_shot_prep<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(ipos, ns, snx, sny, snz, snp);
      // the queries in cell order (results are per query: the order changes no value)
      int32_t* order = nullptr;
      if (shot_cell_order()) {
        const Grid& G = ctx->grid_b;
        int bits = 1;
        while ((int64_t(1) << bits) <= G.ncells) ++bits;
        uint32_t* qk = ctx->buf("shot_qkeys").as<uint32_t>((size_t)nq);
        uint32_t* qk2 = ctx->buf("shot_qkeys2").as<uint32_t>((size_t)nq);
        int32_t* qv = ctx->buf("shot_qvals").as<int32_t>((size_t)nq);
        order = ctx->buf("shot_order").as<int32_t>((size_t)nq);
        size_t tb = 0;
        PFX_HIP(rocprim::radix_sort_pairs(nullptr, tb, qk, qk2, qv, order, (size_t)nq, 0, bits, st));
        void* tmp = ctx->buf("shot_sort_tmp").get(tb + 16);
        k_shot_qkeys<<<(unsigned)ceil_div(nq, 256), 256, 0, st>>>(g, qx, qy, qz, nq, qk, qv);
        PFX_HIP(rocprim::radix_sort_pairs(tmp, tb, qk, qk2, qv, order, (size_t)nq, 0, bits, st));
      }
      for (int64_t q0 = 0; q0 < nq; q0 += kSplitBatch) {
        const int64_t m = std::min<int64_t>(kSplitBatch, nq - q0);
        // (a multiple of 8: k_shot_lrf's per-XCD ranges)
        const unsigned bl = (unsigned)(ceil_div(std::min<int64_t>(m, 256 * 10 * PFX_SHOT_GRID_MUL), 8) * 8);
        k_shot_lrf<<<bl, 256, lds_s, st>>>(g, qx, qy, qz, q0, m, over, n_over, r, desc, rf, grec, sq, ipos, snp, nbr,
                                           order);
        k_shot_eigen<<<(unsigned)ceil_div(m, 64), 64, 0, st>>>(sq, m);
        k_shot_frame<<<(unsigned)std::min<int64_t>(m, 256 * 16 * PFX_SHOT_GRID_MUL), 256, 0, st>>>(q0, m, r, desc, rf,
                                                                                                  grec, sq, upd, order);
        k_shot_accum<<<(unsigned)std::min<int64_t>(m, 256 * 16 * PFX_SHOT_GRID_MUL), 256, 0, st>>>(q0, m, desc, upd, sq,
                                                                                                  order);
      }
    }
    // longer lists: grid sized for the worst case, the count stays on the device
    k_shot<kCap><<<(unsigned)std::min<int64_t>(nq, 256 * 2), 256, lds, st>>>(
        g, snx, sny, snz, qx, qy, qz, nq, over, n_over, nullptr, nullptr, r, desc, rf, err, nbr);
    check_launch("k_shot");
  }
  int h = 0;
  unsigned long long h_nbr = 0;
  PFX_HIP(hipMemcpyAsync(&h, err, sizeof(int), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(&h_nbr, nbr, sizeof(h_nbr), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  ctx->stats["shot_neighbors"] = (int64_t)h_nbr;
#ifdef PFX_SHOT_PROFILE
  {
    unsigned long long pr[16];
    PFX_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_shot_prof), sizeof(pr)));
    const double nq_ = (double)(pr[13] + !pr[13]);
    fprintf(stderr, "shot_accum normalisation %.0f cycles/query (%llu sequential)\n", pr[8] / nq_, pr[7]);
    const double na = (double)(pr[5] + !pr[5]), nf = (double)(pr[14] + !pr[14]);
    fprintf(stderr, "shot_accum cycles/query %.0f: masks %.0f counts %.0f scatter %.0f sums %.0f (%llu queries)\n",
            pr[4] / na, pr[0] / na, pr[1] / na, pr[2] / na, pr[3] / na, pr[5]);
    fprintf(stderr, "shot_frame cycles/query: frame %.0f updates %.0f\n", pr[6] / nf, pr[9] / nf);
    fprintf(stderr, "shot_lrf cycles/query: search+sort %.0f records %.0f chains %.0f\n", pr[10] / (double)(pr[13] + !pr[13]),
            pr[11] / (double)(pr[13] + !pr[13]), pr[12] / (double)(pr[13] + !pr[13]));
    const unsigned long long z[16] = {};
    PFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_shot_prof), z, sizeof(z)));
  }
#endif
  if (h > 0)
    throw Error(PFX_ERR_CAPACITY, "shot: a query has " + std::to_string(h) + " neighbours (> " +
                                      std::to_string(kCap) + " supported)");
}

}  // namespace pfx
