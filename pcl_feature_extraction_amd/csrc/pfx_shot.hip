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
#include "pfx_eigen3.h"
#include "pfx_neighbors.h"

namespace pfx {
namespace {

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

#ifdef PFX_SHOT_PROFILE
__device__ unsigned long long g_shot_prof[8];
#define PROF_T(v) long long v = (tid == 0) ? clock64() : 0
#define PROF_ADD(i, a, b) if (tid == 0) atomicAdd(&g_shot_prof[i], (unsigned long long)((b) - (a)))
#else
#define PROF_T(v)
#define PROF_ADD(i, a, b)
#endif

// the seven distinct LRF chains: cov (0,0) (0,1) (0,2) (1,1) (1,2) (2,2) and the weight sum
constexpr int kChains = 7;
constexpr int kMaskWords = kChunk / 64;

struct ShotLds {
  union {
    double lrf[kChains][kChunk];  // per-neighbour chain terms of one chunk (0 for invalid ones)
    struct {
      uint64_t mask[kLen][kMaskWords];  // which neighbours of the chunk hit each bin
      int off[kLen + 1];                // bucket offsets (exclusive scan of the hit counts)
      float val[5 * kChunk];            // the chunk's update values bucketed by bin, neighbour order
    } upd;
  };
  float hist[kLen];
  double cov[10];
  double axes[6];  // v1 (x axis), v3 (z axis)
  float rf[9];
  int n_invalid, zero_prefix, plusT, plusN, ok;
};

// CAP: LDS key capacity.  `list` (nullable): query subset with its device-side count; queries
// with more than CAP neighbours go to `over` (or raise err when over == nullptr).
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
  const int tid = threadIdx.x, lane = tid & 63;
  const float rr = (float)(radius * radius);
  const int64_t count = list ? (int64_t)*n_list : nq;
  for (int64_t w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t q = list ? (int64_t)list[w] : w;
    float* d = desc + q * kLen;
    float* rfo = rf_out + q * 9;
    const float cx = qx[q], cy = qy[q], cz = qz[q];
    if (!(isfinite(cx) && isfinite(cy) && isfinite(cz))) {
      for (int i = tid; i < kLen; i += 256) d[i] = __builtin_nanf("");
      if (tid < 9) rfo[tid] = __builtin_nanf("");
      continue;
    }
    PROF_T(t0);
    const int k = CAP == kCapSmall
                      ? sorted_neighbors_bucketed(g, cx, cy, cz, rr, keys, keys + CAP, CAP, &s_count, SB)
                      : sorted_neighbors(g, cx, cy, cz, rr, keys, CAP, &s_count);
    PROF_T(t1);
    PROF_ADD(0, t0, t1);
    if (k > CAP) {
      if (tid == 0) {
        if (over) over[atomicAdd(n_over, 1)] = (int32_t)q;
        else atomicMax(err, k);
      }
      continue;
    }
    if (tid == 0) {
      S.n_invalid = 0; S.zero_prefix = 0; S.plusT = 0; S.plusN = 0;
      atomicAdd(nbr, (unsigned long long)k);
    }
    // ---- local reference frame: ordered double covariance ----
    // Every thread forms its neighbour's chain terms dist * (v_a * v_b) and dist exactly as the
    // reference loop does; lanes 0..6 then add them in neighbour order (the only sequential part).
    // An invalid neighbour (a copy of the query) contributes +0.0, which leaves a chain unchanged.
    double acc = 0.0;
    for (int c0 = 0; c0 < k; c0 += kChunk) {
      const int m = min(kChunk, k - c0);
      __syncthreads();
      if (tid < m) {
        const uint64_t key = keys[c0 + tid];
        const int32_t p = key_idx(key);
        const float px = g.ux[p], py = g.uy[p], pz = g.uz[p];
        const bool valid = !(px == cx && py == cy && pz == cz);
        const double vx = (double)(px - cx), vy = (double)(py - cy), vz = (double)(pz - cz);
        const double dist = radius - sqrt((double)key_d2(key));
        S.lrf[0][tid] = valid ? dist * (vx * vx) : 0.0;
        S.lrf[1][tid] = valid ? dist * (vx * vy) : 0.0;
        S.lrf[2][tid] = valid ? dist * (vx * vz) : 0.0;
        S.lrf[3][tid] = valid ? dist * (vy * vy) : 0.0;
        S.lrf[4][tid] = valid ? dist * (vy * vz) : 0.0;
        S.lrf[5][tid] = valid ? dist * (vz * vz) : 0.0;
        S.lrf[6][tid] = valid ? dist : 0.0;
        if (!valid) atomicAdd(&S.n_invalid, 1);
        if (key_d2(key) == 0.0f) atomicAdd(&S.zero_prefix, 1);
      }
      __syncthreads();
      if (tid < kChains) {
        const double* row = S.lrf[tid];
        int t = 0;
        for (; t + 8 <= m; t += 8) {
          const double2 a = *reinterpret_cast<const double2*>(row + t);
          const double2 b = *reinterpret_cast<const double2*>(row + t + 2);
          const double2 c = *reinterpret_cast<const double2*>(row + t + 4);
          const double2 e = *reinterpret_cast<const double2*>(row + t + 6);
          acc = acc + a.x; acc = acc + a.y; acc = acc + b.x; acc = acc + b.y;
          acc = acc + c.x; acc = acc + c.y; acc = acc + e.x; acc = acc + e.y;
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
    PROF_T(t2);
    PROF_ADD(1, t1, t2);
    const int valid = k - S.n_invalid;
    if (tid == 0) {
      S.ok = 0;
      if (valid >= 5) {
        // `cov_m /= sum` (Eigen 3.2: times the reciprocal), SelfAdjointEigenSolver<Matrix3d>
        double ev[3], V[3][3];
        const double inv = 1.0 / S.cov[9];
        eigen_selfadjoint3<true>(S.cov[0] * inv, S.cov[3] * inv, S.cov[4] * inv, S.cov[6] * inv, S.cov[7] * inv,
                                 S.cov[8] * inv, ev, V);
        if (isfinite(ev[0]) && isfinite(ev[1]) && isfinite(ev[2])) {
          S.ok = 1;
          for (int i = 0; i < 3; ++i) { S.axes[i] = V[2][i]; S.axes[3 + i] = V[0][i]; }
        }
      }
    }
    __syncthreads();
    if (!S.ok) {
      for (int i = tid; i < kLen; i += 256) d[i] = __builtin_nanf("");
      if (tid < 9) rfo[tid] = __builtin_nanf("");
      continue;
    }
    // sign disambiguation: counts of non-negative projections over the valid neighbours
    {
      const double v1x = S.axes[0], v1y = S.axes[1], v1z = S.axes[2];
      const double v3x = S.axes[3], v3y = S.axes[4], v3z = S.axes[5];
      int cT = 0, cN = 0;
      for (int j = tid; j < k; j += 256) {
        const int32_t p = key_idx(keys[j]);
        const float px = g.ux[p], py = g.uy[p], pz = g.uz[p];
        if (px == cx && py == cy && pz == cz) continue;
        const double vx = (double)(px - cx), vy = (double)(py - cy), vz = (double)(pz - cz);
        if (((vx * v1x + vy * v1y) + vz * v1z) + 0.0 >= 0) ++cT;
        if (((vx * v3x + vy * v3y) + vz * v3z) + 0.0 >= 0) ++cN;
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
      for (int j = 0; j < zp; ++j) {
        const int32_t p = key_idx(keys[j]);
        if (!(g.ux[p] == cx && g.uy[p] == cy && g.uz[p] == cz)) ++valid_in_prefix;
      }
      for (int w = 0; w < 2; ++w) {
        int plus = 2 * counts[w] - valid;
        if (plus == 0) {
          const int median = valid / 2;
          for (int i = -2; i <= 2; ++i) {
            const int ne = median - i;
            int j;
            if (ne < valid_in_prefix) {
              int seen = -1;
              for (j = 0; j < zp; ++j) {
                const int32_t p = key_idx(keys[j]);
                if (!(g.ux[p] == cx && g.uy[p] == cy && g.uz[p] == cz) && ++seen == ne) break;
              }
            } else {
              j = zp + (ne - valid_in_prefix);
            }
            const int32_t p = key_idx(keys[j]);
            const double vx = (double)(g.ux[p] - cx), vy = (double)(g.uy[p] - cy), vz = (double)(g.uz[p] - cz);
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
    // Bin ownership for the histogram: thread j accumulates bins j and j + 256 in registers.
    const int b0 = tid, b1 = tid + 256;
    float h0 = 0.0f, h1 = 0.0f;
    for (int i = tid; i < kLen; i += 256)
      for (int w = 0; w < kMaskWords; ++w) S.upd.mask[i][w] = 0;
    __syncthreads();
    PROF_T(t3);
    PROF_ADD(2, t2, t3);
    const f3 fx = mk3(S.rf[0], S.rf[1], S.rf[2]), fy = mk3(S.rf[3], S.rf[4], S.rf[5]),
             fz = mk3(S.rf[6], S.rf[7], S.rf[8]);
    // ---- SHOT histogram ----
    // Each neighbour adds to at most one bin per update statement (its <= 5 bins are distinct),
    // so PCL's sequential order restricted to one bin is neighbour order.  Per chunk: hit masks
    // per bin -> counts -> offsets -> every update written to its bin's bucket at its rank among
    // the bin's hits (a stable counting sort) -> each bin's owner adds its bucket in order.
    for (int c0 = 0; c0 < k; c0 += kChunk) {
      const int m = min(kChunk, k - c0);
      PROF_T(t4);
      int bins[5];
      float vals[5];
#pragma unroll
      for (int s = 0; s < 5; ++s) bins[s] = -1;
      if (tid < m) {
        const uint64_t key = keys[c0 + tid];
        const int32_t p = key_idx(key);
        const float pnx = nx[p], pny = ny[p], pnz = nz[p];
        const double distance = sqrt((double)key_d2(key));
        if (isfinite(pnx) && isfinite(pny) && isfinite(pnz) && !(fabs(distance - 0.0) < 1E-15)) {
          double cosd = dot4(mk3(pnx, pny, pnz), fz);
          if (cosd > 1.0) cosd = 1.0;
          if (cosd < -1.0) cosd = -1.0;
          const double binDist = ((1.0 + cosd) * kBins) / 2;
          const f3 delta = mk3(g.ux[p] - cx, g.uy[p] - cy, g.uz[p] - cz);
          shot_updates(delta, distance, binDist, fx, fy, fz, radius, bins, vals);
        }
        const uint64_t bit = 1ull << (tid & 63);
#pragma unroll
        for (int s = 0; s < 5; ++s)
          if (bins[s] >= 0) atomicOr(reinterpret_cast<unsigned long long*>(&S.upd.mask[bins[s]][tid >> 6]), bit);
      }
      __syncthreads();
      PROF_T(t5);
      PROF_ADD(3, t4, t5);
      // hit counts -> exclusive offsets (wave 0: 6 bins per lane, then a wave scan)
      if (tid < 64) {
        int c[6], tot = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int bb = tid * 6 + i;
          c[i] = 0;
          if (bb < kLen)
            for (int w = 0; w < kMaskWords; ++w) c[i] += __popcll(S.upd.mask[bb][w]);
          tot += c[i];
        }
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(incl, o);
          if (lane >= o) incl += y;
        }
        int run = incl - tot;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int bb = tid * 6 + i;
          if (bb < kLen) S.upd.off[bb] = run;
          run += c[i];
        }
      }
      __syncthreads();
      if (tid < m) {  // scatter: rank = hits of the bin from lower neighbours of the chunk
        const int wq = tid >> 6;
        const uint64_t below = lanemask_lt();
#pragma unroll
        for (int s = 0; s < 5; ++s) {
          const int bb = bins[s];
          if (bb < 0) continue;
          int r = __popcll(S.upd.mask[bb][wq] & below);
          for (int w = 0; w < wq; ++w) r += __popcll(S.upd.mask[bb][w]);
          S.upd.val[S.upd.off[bb] + r] = vals[s];
        }
      }
      __syncthreads();
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        const int b = o ? b1 : b0;
        if (b < kLen) {
          int cnt = 0;
          for (int w = 0; w < kMaskWords; ++w) {
            cnt += __popcll(S.upd.mask[b][w]);
            S.upd.mask[b][w] = 0;  // ready for the next chunk
          }
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
      PROF_T(t6);
      PROF_ADD(4, t5, t6);
    }
    S.hist[b0] = h0;
    if (b1 < kLen) S.hist[b1] = h1;
    __syncthreads();
    PROF_T(t7);
    if (tid == 0) {  // normalizeHistogram
      double acc_norm = 0;
      for (int j = 0; j < kLen; ++j) acc_norm += S.hist[j] * S.hist[j];
      S.cov[0] = sqrt(acc_norm);
    }
    __syncthreads();
    const float nrm = (float)S.cov[0];
    for (int i = tid; i < kLen; i += 256) d[i] = S.hist[i] / nrm;
    if (tid < 9) rfo[tid] = S.rf[tid];
    __syncthreads();
    PROF_T(t8);
    PROF_ADD(5, t7, t8);
  }
}

}  // namespace

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
  ctx->prep_x = nullptr;  // grid_b is rebuilt: a pending pfx_fpfh_prepare_dev no longer holds
  ctx->prep_n = -1;
  build_grid(ctx, ctx->grid_b, sx, sy, sz, ns, r);
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
    const unsigned blocks = (unsigned)std::min<int64_t>(nq, 256 * 10);
    k_shot<kCapSmall><<<blocks, 256, lds_s, st>>>(g, snx, sny, snz, qx, qy, qz, nq, nullptr, nullptr, over, n_over,
                                                   r, desc, rf, err, nbr);
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
    unsigned long long pr[8];
    PFX_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_shot_prof), sizeof(pr)));
    fprintf(stderr, "shot phase cycles (summed over queries): sort %llu lrf %llu frame %llu hist %llu apply %llu out %llu\n",
            pr[0], pr[1], pr[2], pr[3], pr[4], pr[5]);
  }
#endif
  if (h > 0)
    throw Error(PFX_ERR_CAPACITY, "shot: a query has " + std::to_string(h) + " neighbours (> " +
                                      std::to_string(kCap) + " supported)");
}

}  // namespace pfx
