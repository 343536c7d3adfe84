// pfx_ransac.hip -- the reference's RANSAC correspondence rejection:
//
//   Features<T>::filterCorrespondences             features.h:282-297
//     registration::CorrespondenceRejectorSampleConsensus<PointXYZRGB>: inlier threshold 0.015,
//     1000 iterations, then getBestTransformation()
//
// PCL's RANSAC draws its samples from a fixed-seed mt19937 (seed 12345) through a persistent
// partial shuffle, independently of the models' scores, so the whole sample sequence is known
// before any model is scored.  The host replays that integer sequence (with PCL's sample test),
// the GPU scores every hypothesis at once -- one workgroup per model: Umeyama on the 3 pairs
// (double, one lane), then the inlier count over all correspondences -- and the host replays
// PCL's adaptive stopping rule (k = log(0.01) / log(1 - w^3)) over the scores in order.
// Arithmetic restated in oracle/or_ransac.cpp (the same operations, so the models, counts and
// kept correspondences agree exactly; parity vs PCL unpinned there).
#include <cmath>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>
#include <vector>
#include <rocprim/rocprim.hpp>

#include "pfx_device_math.h"
#include "pfx_internal.h"

namespace pfx {
namespace {

// one-sided Jacobi SVD of a 3x3 (row-major) in double: A = U diag(d) V^T, d descending >= 0,
// U and V orthonormal (U completed by cross products where d is 0)
__device__ void svd3(const double A[9], double U[9], double d[3], double V[9]) {
  double B[9];
  for (int i = 0; i < 9; ++i) B[i] = A[i];
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double alpha = 0.0, beta = 0.0, gamma = 0.0;
        for (int i = 0; i < 3; ++i) {
          alpha += B[3 * i + p] * B[3 * i + p];
          beta += B[3 * i + q] * B[3 * i + q];
          gamma += B[3 * i + p] * B[3 * i + q];
        }
        if (gamma == 0.0 || fabs(gamma) <= 1e-15 * sqrt(alpha * beta)) continue;
        rotated = true;
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < 3; ++i) {
          const double bp = B[3 * i + p], bq = B[3 * i + q];
          B[3 * i + p] = c * bp - s * bq;
          B[3 * i + q] = s * bp + c * bq;
          const double vp = V[3 * i + p], vq = V[3 * i + q];
          V[3 * i + p] = c * vp - s * vq;
          V[3 * i + q] = s * vp + c * vq;
        }
      }
    if (!rotated) break;
  }
  for (int j = 0; j < 3; ++j)
    d[j] = sqrt(B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j]);
  // sort descending (columns of B and V follow)
  for (int i = 0; i < 2; ++i) {
    int k = i;
    for (int j = i + 1; j < 3; ++j)
      if (d[j] > d[k]) k = j;
    if (k != i) {
      double tmp = d[i];
      d[i] = d[k];
      d[k] = tmp;
      for (int r = 0; r < 3; ++r) {
        tmp = B[3 * r + i]; B[3 * r + i] = B[3 * r + k]; B[3 * r + k] = tmp;
        tmp = V[3 * r + i]; V[3 * r + i] = V[3 * r + k]; V[3 * r + k] = tmp;
      }
    }
  }
  // U columns: B columns / d; zero singular values completed to an orthonormal basis
  for (int j = 0; j < 3; ++j)
    for (int r = 0; r < 3; ++r) U[3 * r + j] = d[j] > 0.0 ? B[3 * r + j] / d[j] : 0.0;
  if (!(d[1] > 0.0)) {  // rank <= 1: any unit vector orthogonal to u0
    const double ux = U[0], uy = U[3], uz = U[6];
    double a[3] = {0.0, 0.0, 0.0};
    const double ax = fabs(ux), ay = fabs(uy), az = fabs(uz);
    if (ax <= ay && ax <= az) a[0] = 1.0; else if (ay <= az) a[1] = 1.0; else a[2] = 1.0;
    double v[3] = {uy * a[2] - uz * a[1], uz * a[0] - ux * a[2], ux * a[1] - uy * a[0]};
    const double nv = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (nv > 0.0) for (int r = 0; r < 3; ++r) U[3 * r + 1] = v[r] / nv;
    if (!(d[0] > 0.0)) { U[0] = 1.0; U[3] = 0.0; U[6] = 0.0; U[1] = 0.0; U[4] = 1.0; U[7] = 0.0; }
  }
  if (!(d[2] > 0.0)) {  // u2 = u0 x u1
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
  }
}

__device__ double det3(const double M[9]) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// pcl::umeyama (Eigen Umeyama, no scaling) for the 3 point pairs; out: row-major float 4x4
__device__ void umeyama3(const double src[3][3], const double dst[3][3], float T[16]) {
  const double one_over_n = 1.0 / 3.0;
  double sm[3], dm[3];
  for (int r = 0; r < 3; ++r) {
    sm[r] = ((src[r][0] + src[r][1]) + src[r][2]) * one_over_n;
    dm[r] = ((dst[r][0] + dst[r][1]) + dst[r][2]) * one_over_n;
  }
  double sd[3][3], dd[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      sd[r][c] = src[r][c] - sm[r];
      dd[r][c] = dst[r][c] - dm[r];
    }
  double sigma[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double acc = (one_over_n * dd[i][0]) * sd[j][0];
      acc += (one_over_n * dd[i][1]) * sd[j][1];
      acc += (one_over_n * dd[i][2]) * sd[j][2];
      sigma[3 * i + j] = acc;
    }
  double U[9], d[3], V[9];
  svd3(sigma, U, d, V);
  double S[3] = {1.0, 1.0, 1.0};
  if (det3(sigma) < 0.0) S[2] = -1.0;
  int rank = 0;
  for (int i = 0; i < 3; ++i)
    if (!(fabs(d[i]) <= fabs(d[0]) * 1e-12)) ++rank;
  double R[9];
  double Sd[3] = {S[0], S[1], S[2]};
  if (rank == 2) {
    if (det3(U) * det3(V) > 0.0) {
      Sd[0] = Sd[1] = Sd[2] = 1.0;
    } else {
      Sd[0] = S[0]; Sd[1] = S[1]; Sd[2] = -1.0;
    }
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double acc = (U[3 * i] * Sd[0]) * V[3 * j];
      acc += (U[3 * i + 1] * Sd[1]) * V[3 * j + 1];
      acc += (U[3 * i + 2] * Sd[2]) * V[3 * j + 2];
      R[3 * i + j] = acc;
    }
  double t[3];
  for (int i = 0; i < 3; ++i) {
    double acc = R[3 * i] * sm[0];
    acc += R[3 * i + 1] * sm[1];
    acc += R[3 * i + 2] * sm[2];
    t[i] = dm[i] - acc;
  }
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) T[4 * i + j] = (float)R[3 * i + j];
    T[4 * i + 3] = (float)t[i];
  }
  T[12] = T[13] = T[14] = 0.0f;
  T[15] = 1.0f;
}

// SampleConsensusModelRegistration::countWithinDistance's test for one pair
__device__ __forceinline__ bool within(const float T[16], const float* sx, const float* sy, const float* sz, int s, const float* tx,
                   const float* ty, const float* tz, int t, double thresh2) {
  const float x = sx[s], y = sy[s], z = sz[s];
  float p[4];
  for (int r = 0; r < 4; ++r) p[r] = ((T[4 * r] * x + T[4 * r + 1] * y) + T[4 * r + 2] * z) + T[4 * r + 3] * 1.0f;
  const float d0 = p[0] - tx[t], d1 = p[1] - ty[t], d2 = p[2] - tz[t], d3 = p[3] - 1.0f;
  const float sq = (d0 * d0 + d2 * d2) + (d1 * d1 + d3 * d3);  // Vector4f squaredNorm (SSE)
  return (double)sq < thresh2;
}


// SampleConsensusModelRegistration::computeSampleDistanceThreshold(cloud, indices): float
// covariance of the source keypoints in index order (computeMeanAndCovarianceMatrix), pcl::eigen33
// values, (sum of square roots / 3)^2 in double -- one lane
__global__ void k_ransac_threshold(const float* __restrict__ x, const float* __restrict__ y,
                                   const float* __restrict__ z, const int32_t* __restrict__ idx, int64_t n,
                                   double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; ++i) {
    const float px = x[idx[i]], py = y[idx[i]], pz = z[idx[i]];
    a[0] += px * px; a[1] += px * py; a[2] += px * pz;
    a[3] += py * py; a[4] += py * pz; a[5] += pz * pz;
    a[6] += px; a[7] += py; a[8] += pz;
  }
  const float inv = 1.0f / (float)n;  // computeMeanAndCovarianceMatrix `accu /= n` (Eigen 3.2)
  for (int k = 0; k < 9; ++k) a[k] *= inv;
  const float c00 = a[0] - a[6] * a[6], c01 = a[1] - a[6] * a[7], c02 = a[2] - a[6] * a[8];
  const float c11 = a[3] - a[7] * a[7], c12 = a[4] - a[7] * a[8], c22 = a[5] - a[8] * a[8];
  float scale = fmaxf(fmaxf(fmaxf(fabsf(c00), fabsf(c01)), fmaxf(fabsf(c02), fabsf(c11))),
                      fmaxf(fabsf(c12), fabsf(c22)));  // max |entry| of the symmetric matrix
  if (scale <= 1.17549435e-38f) scale = 1.0f;
  float ev[3];
  computeRoots(c00 / scale, c01 / scale, c02 / scale, c11 / scale, c12 / scale, c22 / scale, ev);
  for (int k = 0; k < 3; ++k) ev[k] *= scale;
  // `eigen_values.array ().sqrt ().sum ()` on a Vector3f: Redux.h's unrolled x + (y + z)
  const float ssum = sqrtf(ev[0]) + (sqrtf(ev[1]) + sqrtf(ev[2]));
  const double t = (double)ssum / 3.0;
  *out = t * t;
}

// one workgroup per hypothesis h: model from the 3 sampled pairs, inliers over all pairs
__global__ void __launch_bounds__(256) k_ransac_models(const float* __restrict__ sx, const float* __restrict__ sy,
                                                       const float* __restrict__ sz, const float* __restrict__ tx,
                                                       const float* __restrict__ ty, const float* __restrict__ tz,
                                                       const int32_t* __restrict__ query,
                                                       const int32_t* __restrict__ match, int64_t n,
                                                       const int32_t* __restrict__ samples, double thresh2,
                                                       float* __restrict__ models, int* __restrict__ counts) {
  __shared__ float sT[16];
  __shared__ int s_cnt[4];
  const int h = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    double src[3][3], dst[3][3];
    for (int c = 0; c < 3; ++c) {
      const int s = samples[6 * h + 2 * c], t = samples[6 * h + 2 * c + 1];
      src[0][c] = sx[s]; src[1][c] = sy[s]; src[2][c] = sz[s];
      dst[0][c] = tx[t]; dst[1][c] = ty[t]; dst[2][c] = tz[t];
    }
    float T[16];
    umeyama3(src, dst, T);
    for (int k = 0; k < 16; ++k) {
      sT[k] = T[k];
      models[16 * h + k] = T[k];
    }
  }
  __syncthreads();
  float T[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) T[k] = sT[k];
  int cnt = 0;
  for (int64_t i = tid; i < n; i += 256)
    cnt += within(T, sx, sy, sz, query[i], tx, ty, tz, match[i], thresh2) ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) counts[h] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

__global__ void k_ransac_select(const float* __restrict__ sx, const float* __restrict__ sy,
                                const float* __restrict__ sz, const float* __restrict__ tx,
                                const float* __restrict__ ty, const float* __restrict__ tz,
                                const int32_t* __restrict__ query, const int32_t* __restrict__ match, int64_t n,
                                const float* __restrict__ model, double thresh2, uint8_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float T[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) T[k] = model[k];
  flag[i] = within(T, sx, sy, sz, query[i], tx, ty, tz, match[i], thresh2) ? 1 : 0;
}

}  // namespace

// returns the number of kept correspondences (positions into keep_out, host), T row-major
int64_t ransac_rejector(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                        const float* tx, const float* ty, const float* tz, int64_t nt, const int32_t* query,
                        const int32_t* match, int64_t n, double threshold, int max_iterations, int32_t* keep_out,
                        float* T_out, int64_t* iters_out) {
  for (int i = 0; i < 16; ++i) T_out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  if (iters_out) *iters_out = 0;
  auto keep_all = [&]() {
    for (int64_t i = 0; i < n; ++i) keep_out[i] = (int32_t)i;
    return n;
  };
  if (n < 3) return keep_all();
  for (int64_t i = 0; i < n; ++i)
    if (query[i] < 0 || query[i] >= ns || match[i] < 0 || match[i] >= nt)
      throw Error(PFX_ERR_INVALID, "ransac: correspondence index out of range");
  hipStream_t st = ctx->stream;
  TimeScope total(ctx, "ransac", true);
  auto up = [&](const char* name, const void* h, size_t bytes) {
    void* d = ctx->buf(name).get(bytes + 16);
    PFX_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
    return d;
  };
  const float* dsx = static_cast<const float*>(up("rs_sx", sx, sizeof(float) * ns));
  const float* dsy = static_cast<const float*>(up("rs_sy", sy, sizeof(float) * ns));
  const float* dsz = static_cast<const float*>(up("rs_sz", sz, sizeof(float) * ns));
  const float* dtx = static_cast<const float*>(up("rs_tx", tx, sizeof(float) * nt));
  const float* dty = static_cast<const float*>(up("rs_ty", ty, sizeof(float) * nt));
  const float* dtz = static_cast<const float*>(up("rs_tz", tz, sizeof(float) * nt));
  const int32_t* dq = static_cast<const int32_t*>(up("rs_q", query, sizeof(int32_t) * n));
  const int32_t* dm = static_cast<const int32_t*>(up("rs_m", match, sizeof(int32_t) * n));
  double* dthr = ctx->buf("rs_thr").as<double>(1);
  k_ransac_threshold<<<1, 64, 0, st>>>(dsx, dsy, dsz, dq, n, dthr);
  check_launch("k_ransac_threshold");
  double sample_thresh = 0.0;
  PFX_HIP(hipMemcpyAsync(&sample_thresh, dthr, sizeof(double), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  // PCL's sample sequence: partial Fisher-Yates swaps of the persistent index vector with
  // rnd() = mt19937(12345) >> 1 (boost::uniform_int<>(0, INT_MAX)), each sample re-drawn until
  // its three source points are pairwise farther apart than sqrt(sample_thresh) (<= 1000 draws)
  std::unordered_map<int, int> corr_of;
  for (int64_t i = 0; i < n; ++i) corr_of[query[i]] = match[i];
  std::vector<int> shuffled(query, query + n);
  std::mt19937 rng(12345u);
  const int nh_max = max_iterations + 1;
  std::vector<int32_t> samples;
  samples.reserve((size_t)nh_max * 6);
  int nh = 0;
  for (; nh < nh_max; ++nh) {
    int s[3];
    bool good = false;
    for (int check = 0; check < 1000 && !good; ++check) {
      for (int i = 0; i < 3; ++i) std::swap(shuffled[i], shuffled[i + ((int)(rng() >> 1) % (int)(n - i))]);
      for (int i = 0; i < 3; ++i) s[i] = shuffled[i];
      auto sq = [&](int a, int b) {
        const float dx = sx[b] - sx[a], dy = sy[b] - sy[a], dz = sz[b] - sz[a];
        return dx * dx + dy * dy + dz * dz;
      };
      good = sq(s[0], s[1]) > sample_thresh && sq(s[0], s[2]) > sample_thresh && sq(s[1], s[2]) > sample_thresh;
    }
    if (!good) break;  // PCL stops at the first sample it cannot draw
    for (int c = 0; c < 3; ++c) {
      samples.push_back(s[c]);
      samples.push_back(corr_of[s[c]]);
    }
  }
  if (nh == 0) return keep_all();
  int32_t* dsamp = static_cast<int32_t*>(up("rs_samples", samples.data(), sizeof(int32_t) * samples.size()));
  float* dmodels = ctx->buf("rs_models").as<float>(16 * (size_t)nh);
  int* dcounts = ctx->buf("rs_counts").as<int>(nh);
  const double thresh2 = threshold * threshold;
  {
    TimeScope ts(ctx, "ransac_models");
    k_ransac_models<<<nh, 256, 0, st>>>(dsx, dsy, dsz, dtx, dty, dtz, dq, dm, n, dsamp, thresh2, dmodels, dcounts);
    check_launch("k_ransac_models");
  }
  std::vector<int> counts((size_t)nh);
  PFX_HIP(hipMemcpyAsync(counts.data(), dcounts, sizeof(int) * nh, hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  // RandomSampleConsensus::computeModel's loop over the scores, in order
  const double log_probability = std::log(1.0 - 0.99), one_over_indices = 1.0 / (double)n;
  int best_count = -std::numeric_limits<int>::max(), best = -1, iterations = 0;
  double k = 1.0;
  while (iterations < k && iterations < nh) {
    const int c = counts[(size_t)iterations];
    if (c > best_count) {
      best_count = c;
      best = iterations;
      const double w = (double)best_count * one_over_indices;
      double p = 1.0 - std::pow(w, 3.0);
      p = std::max(std::numeric_limits<double>::epsilon(), p);
      p = std::min(1.0 - std::numeric_limits<double>::epsilon(), p);
      k = log_probability / std::log(p);
    }
    ++iterations;
    if (iterations > max_iterations) break;
  }
  if (iters_out) *iters_out = iterations;
  ctx->stats["ransac_models_scored"] = nh;
  if (best < 0) return keep_all();
  uint8_t* flag = ctx->buf("rs_flag").as<uint8_t>(n);
  k_ransac_select<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(dsx, dsy, dsz, dtx, dty, dtz, dq, dm, n,
                                                             dmodels + 16 * (size_t)best, thresh2, flag);
  check_launch("k_ransac_select");
  int32_t* sel = ctx->buf("rs_sel").as<int32_t>(n);
  int64_t* dk = ctx->buf("rs_k").as<int64_t>(1);
  size_t tb = 0;
  PFX_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<int32_t>(0), flag, sel, dk, (size_t)n, st));
  void* tmp = ctx->buf("rs_tmp").get(tb + 16);
  PFX_HIP(rocprim::select(tmp, tb, rocprim::counting_iterator<int32_t>(0), flag, sel, dk, (size_t)n, st));
  int64_t kept = 0;
  float Tb[16];
  PFX_HIP(hipMemcpyAsync(&kept, dk, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(Tb, dmodels + 16 * (size_t)best, sizeof(Tb), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (kept < 3) return keep_all();
  PFX_HIP(hipMemcpyAsync(keep_out, sel, sizeof(int32_t) * kept, hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  std::memcpy(T_out, Tb, sizeof(Tb));
  return kept;
}

}  // namespace pfx
