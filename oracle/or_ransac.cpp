// =====================================================================================
//  oracle/or_ransac.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of the reference's RANSAC correspondence rejection:
//    Features<T>::filterCorrespondences   include/pcl_feature_extraction/features.h:282-297
//      registration::CorrespondenceRejectorSampleConsensus<PointXYZRGB>, inlier threshold
//      0.015, 1000 iterations, refine off (PCL 1.7 default), then getBestTransformation().
//  PCL 1.7 pieces restated (correspondence_rejection_sample_consensus.hpp, ransac.hpp,
//  sac_model.h, sac_model_registration.{h,hpp}, common/centroid.hpp, common/eigen.hpp,
//  Eigen's Umeyama as pcl::umeyama):
//    * model over the source keypoints of the correspondences (indices = index_query, target
//      indices = index_match); sample = 3 indices drawn by partial Fisher-Yates swaps of a
//      persistent shuffled index vector with rnd() = boost::uniform_int<>(0, INT_MAX) over
//      boost::mt19937 seeded 12345 (== mt19937() >> 1); isSampleGood: the three pairwise
//      squared distances > sample_dist_thresh_ = (sum sqrt(eigen33 values of the indices'
//      covariance) / 3)^2; up to 1000 draws per sample;
//    * model: Umeyama (no scaling) in double on the 3 pairs, cast to float;
//    * inliers: |T p_src - p_tgt|^2 < threshold^2 (Matrix4f * Vector4f, SSE squaredNorm);
//    * RANSAC: best = strictly more inliers; k = log(1 - 0.99) / log(1 - w^3), w = inliers / n;
//      loop while iterations < k, stop after max_iterations + 1 models;
//    * result: the correspondences whose source index is an inlier of the best model, in input
//      order; fewer than 3 inliers or no model -> the input unchanged and the identity.
//  Restatement choices (unpinned): the 3x3 SVD inside Umeyama is a one-sided Jacobi SVD in
//  double (Eigen's JacobiSVD reaches the same rotation up to rounding, which the float cast
//  absorbs except in rare cases); Eigen redux orders as in or_common.h.
// =====================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>
#include <vector>

#include "or_common.h"

using orc::i64;

namespace {

// one-sided Jacobi SVD of a 3x3 (row-major) in double: A = U diag(d) V^T, d descending >= 0,
// U and V orthonormal (U completed by cross products where d is 0)
void svd3(const double A[9], double U[9], double d[3], double V[9]) {
  double B[9];
  std::memcpy(B, A, sizeof(B));
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
        if (gamma == 0.0 || std::fabs(gamma) <= 1e-15 * std::sqrt(alpha * beta)) continue;
        rotated = true;
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
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
    d[j] = std::sqrt(B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j]);
  // sort descending (columns of B and V follow)
  for (int i = 0; i < 2; ++i) {
    int k = i;
    for (int j = i + 1; j < 3; ++j)
      if (d[j] > d[k]) k = j;
    if (k != i) {
      std::swap(d[i], d[k]);
      for (int r = 0; r < 3; ++r) {
        std::swap(B[3 * r + i], B[3 * r + k]);
        std::swap(V[3 * r + i], V[3 * r + k]);
      }
    }
  }
  // U columns: B columns / d; zero singular values completed to an orthonormal basis
  for (int j = 0; j < 3; ++j)
    for (int r = 0; r < 3; ++r) U[3 * r + j] = d[j] > 0.0 ? B[3 * r + j] / d[j] : 0.0;
  if (!(d[1] > 0.0)) {  // rank <= 1: any unit vector orthogonal to u0
    const double ux = U[0], uy = U[3], uz = U[6];
    double a[3] = {0.0, 0.0, 0.0};
    const double ax = std::fabs(ux), ay = std::fabs(uy), az = std::fabs(uz);
    if (ax <= ay && ax <= az) a[0] = 1.0; else if (ay <= az) a[1] = 1.0; else a[2] = 1.0;
    double v[3] = {uy * a[2] - uz * a[1], uz * a[0] - ux * a[2], ux * a[1] - uy * a[0]};
    const double nv = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (nv > 0.0) for (int r = 0; r < 3; ++r) U[3 * r + 1] = v[r] / nv;
    if (!(d[0] > 0.0)) { U[0] = 1.0; U[3] = 0.0; U[6] = 0.0; U[1] = 0.0; U[4] = 1.0; U[7] = 0.0; }
  }
  if (!(d[2] > 0.0)) {  // u2 = u0 x u1
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
  }
}

double det3(const double M[9]) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// pcl::umeyama (Eigen Umeyama, no scaling) for the 3 point pairs; out: row-major float 4x4
void umeyama3(const double src[3][3], const double dst[3][3], float T[16]) {
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
    if (!(std::fabs(d[i]) <= std::fabs(d[0]) * 1e-12)) ++rank;
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
inline bool within(const float T[16], const float* sx, const float* sy, const float* sz, int s, const float* tx,
                   const float* ty, const float* tz, int t, double thresh2) {
  const float x = sx[s], y = sy[s], z = sz[s];
  float p[4];
  for (int r = 0; r < 4; ++r) p[r] = ((T[4 * r] * x + T[4 * r + 1] * y) + T[4 * r + 2] * z) + T[4 * r + 3] * 1.0f;
  const float d0 = p[0] - tx[t], d1 = p[1] - ty[t], d2 = p[2] - tz[t], d3 = p[3] - 1.0f;
  const float sq = (d0 * d0 + d2 * d2) + (d1 * d1 + d3 * d3);  // Vector4f squaredNorm (SSE)
  return (double)sq < thresh2;
}

}  // namespace

extern "C" {

// sample_dist_thresh_ of SampleConsensusModelRegistration (for the tests)
double orc_ransac_sample_threshold(const float* x, const float* y, const float* z, const int32_t* idx, i64 n) {
  float accu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (i64 i = 0; i < n; ++i) {
    const float px = x[idx[i]], py = y[idx[i]], pz = z[idx[i]];
    accu[0] += px * px; accu[1] += px * py; accu[2] += px * pz;
    accu[3] += py * py; accu[4] += py * pz; accu[5] += pz * pz;
    accu[6] += px; accu[7] += py; accu[8] += pz;
  }
  const float inv = 1.0f / (float)n;  // computeMeanAndCovarianceMatrix: `accu /= n` (Eigen 3.2)
  for (int k = 0; k < 9; ++k) accu[k] *= inv;
  float C[3][3];
  C[0][0] = accu[0] - accu[6] * accu[6];
  C[0][1] = accu[1] - accu[6] * accu[7];
  C[0][2] = accu[2] - accu[6] * accu[8];
  C[1][1] = accu[3] - accu[7] * accu[7];
  C[1][2] = accu[4] - accu[7] * accu[8];
  C[2][2] = accu[5] - accu[8] * accu[8];
  C[1][0] = C[0][1]; C[2][0] = C[0][2]; C[2][1] = C[1][2];
  // pcl::eigen33 (mat, evals): scale, computeRoots, rescale
  float scale = 0.0f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(C[i][j]));
  if (scale <= std::numeric_limits<float>::min()) scale = 1.0f;
  float Sm[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Sm[i][j] = C[i][j] / scale;
  float ev[3];
  orc::computeRoots(Sm, ev);
  for (int k = 0; k < 3; ++k) ev[k] *= scale;
  // `eigen_values.array ().sqrt ().sum ()` on a Vector3f: Redux.h's unrolled x + (y + z)
  const float ssum = std::sqrt(ev[0]) + (std::sqrt(ev[1]) + std::sqrt(ev[2]));
  double t = (double)ssum / 3.0;
  return t * t;
}

// Features::filterCorrespondences: keep[0..*n_keep) = positions (in the input correspondence
// order) of the remaining correspondences, T = getBestTransformation() (row-major), *iters the
// number of models RANSAC evaluated.  Returns 0.
int orc_ransac_rejector(const float* sx, const float* sy, const float* sz, i64 ns, const float* tx, const float* ty,
                        const float* tz, i64 nt, const int32_t* query, const int32_t* match, i64 n, double threshold,
                        int max_iterations, int32_t* keep, i64* n_keep, float* T, i64* iters) {
  (void)ns;
  (void)nt;
  for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  *iters = 0;
  auto keep_all = [&]() {
    for (i64 i = 0; i < n; ++i) keep[i] = (int32_t)i;
    *n_keep = n;
  };
  if (n < 3) {  // getSamples: fewer indices than the sample size -> no model
    keep_all();
    return 0;
  }
  const double sample_thresh = orc_ransac_sample_threshold(sx, sy, sz, query, n);
  std::unordered_map<int, int> corr_of;  // source index -> target index (setInputTarget)
  for (i64 i = 0; i < n; ++i) corr_of[query[i]] = match[i];
  std::vector<int> shuffled(query, query + n);
  std::mt19937 rng(12345u);
  auto rnd = [&]() { return (int)(rng() >> 1); };  // boost::uniform_int<>(0, INT_MAX)
  const double thresh2 = threshold * threshold;
  const double log_probability = std::log(1.0 - 0.99);
  const double one_over_indices = 1.0 / (double)n;
  int best_count = -std::numeric_limits<int>::max();
  float bestT[16];
  bool have = false;
  double k = 1.0;
  int iterations = 0;
  while (iterations < k) {
    // getSamples (up to 1000 draws for a good sample)
    int sample[3];
    bool good = false;
    for (int check = 0; check < 1000 && !good; ++check) {
      for (int i = 0; i < 3; ++i) std::swap(shuffled[i], shuffled[i + (rnd() % (int)(n - i))]);
      for (int i = 0; i < 3; ++i) sample[i] = shuffled[i];
      auto sq = [&](int a, int b) {
        const float dx = sx[b] - sx[a], dy = sy[b] - sy[a], dz = sz[b] - sz[a];
        return dx * dx + dy * dy + dz * dz;
      };
      good = sq(sample[0], sample[1]) > sample_thresh && sq(sample[0], sample[2]) > sample_thresh &&
             sq(sample[1], sample[2]) > sample_thresh;
    }
    if (!good) break;  // selection.empty(): PCL_ERROR and stop
    double src[3][3], dst[3][3];
    for (int c = 0; c < 3; ++c) {
      const int s = sample[c], t = corr_of[s];
      src[0][c] = sx[s]; src[1][c] = sy[s]; src[2][c] = sz[s];
      dst[0][c] = tx[t]; dst[1][c] = ty[t]; dst[2][c] = tz[t];
    }
    float M[16];
    umeyama3(src, dst, M);
    int cnt = 0;
    for (i64 i = 0; i < n; ++i)
      if (within(M, sx, sy, sz, query[i], tx, ty, tz, match[i], thresh2)) ++cnt;
    if (cnt > best_count) {
      best_count = cnt;
      std::memcpy(bestT, M, sizeof(bestT));
      have = true;
      const double w = (double)best_count * one_over_indices;
      double p_no_outliers = 1.0 - std::pow(w, 3.0);
      p_no_outliers = std::max(std::numeric_limits<double>::epsilon(), p_no_outliers);
      p_no_outliers = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no_outliers);
      k = log_probability / std::log(p_no_outliers);
    }
    ++iterations;
    if (iterations > max_iterations) break;
  }
  *iters = iterations;
  if (!have) {
    keep_all();
    return 0;
  }
  // selectWithinDistance -> inliers (source indices) -> their correspondences, input order
  i64 m = 0;
  for (i64 i = 0; i < n; ++i)
    if (within(bestT, sx, sy, sz, query[i], tx, ty, tz, match[i], thresh2)) keep[m++] = (int32_t)i;
  if (m < 3) {
    keep_all();
    return 0;
  }
  *n_keep = m;
  std::memcpy(T, bestT, sizeof(bestT));
  return 0;
}

}  // extern "C"
