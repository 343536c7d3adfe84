// =====================================================================================
//  oracle/or_features.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of the PCL 1.7 calls on the reference's descriptor path:
//    * search::KdTree::radiusSearch (FLANN)           used at features.h:192, tools.h:29
//    * NormalEstimationOMP<PointXYZRGB,Normal>        tools.h:22-32
//    * FPFHEstimation<PointXYZRGB,Normal,FPFH33>      evaluation.cpp:593-612
//  Exposed through a C ABI for ctypes (tests/, bench.py cpu_baseline only).
// =====================================================================================
#include <set>
#include "or_common.h"
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace orc;

namespace {

// pcl::computeMeanAndCovarianceMatrix (common/impl/centroid.hpp, dense branch) followed by
// pcl::solvePlaneParameters (features/impl/feature.hpp) and flipNormalTowardsViewpoint.
void pointNormal(const float* x, const float* y, const float* z, const std::vector<int>& nb,
                 float px, float py, float pz, float vpx, float vpy, float vpz, float out[4]) {
  if (nb.size() < 3) {
    out[0] = out[1] = out[2] = out[3] = kNaN;
    return;
  }
  float accu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t i = 0; i < nb.size(); ++i) {
    const int p = nb[i];
    accu[0] += x[p] * x[p];
    accu[1] += x[p] * y[p];
    accu[2] += x[p] * z[p];
    accu[3] += y[p] * y[p];
    accu[4] += y[p] * z[p];
    accu[5] += z[p] * z[p];
    accu[6] += x[p];
    accu[7] += y[p];
    accu[8] += z[p];
  }
  // `accu /= static_cast<Scalar> (point_count)`: Eigen 3.2 multiplies by the reciprocal
  const float inv = 1.0f / (float)nb.size();
  for (int i = 0; i < 9; ++i) accu[i] *= inv;
  float C[3][3];
  C[0][0] = accu[0] - accu[6] * accu[6];
  C[0][1] = accu[1] - accu[6] * accu[7];
  C[0][2] = accu[2] - accu[6] * accu[8];
  C[1][1] = accu[3] - accu[7] * accu[7];
  C[1][2] = accu[4] - accu[7] * accu[8];
  C[2][2] = accu[5] - accu[8] * accu[8];
  C[1][0] = C[0][1]; C[2][0] = C[0][2]; C[2][1] = C[1][2];
  float lambda;
  V3 n;
  eigen33_min(C, lambda, n);
  float eig_sum = C[0][0] + C[1][1] + C[2][2];
  float curv = (eig_sum != 0.0f) ? std::fabs(lambda / eig_sum) : 0.0f;
  // flipNormalTowardsViewpoint (features/normal_3d.h)
  float ax = vpx - px, ay = vpy - py, az = vpz - pz;
  float cos_theta = ax * n.x + ay * n.y + az * n.z;
  if (cos_theta < 0.0f) { n.x *= -1.0f; n.y *= -1.0f; n.z *= -1.0f; }
  out[0] = n.x; out[1] = n.y; out[2] = n.z; out[3] = curv;
}

// pcl::computePairFeatures (features/src/pfh.cpp) on Vector4f maps (w forced to 0)
void pairFeatures(V3 p1, V3 n1, V3 p2, V3 n2, float& f1, float& f2, float& f3, float& f4) {
  V3 dp = sub(p2, p1);
  f4 = std::sqrt(sqn4(dp));
  if (f4 == 0.0f) { f1 = f2 = f3 = f4 = 0.0f; return; }
  V3 n1c = n1, n2c = n2;
  float angle1 = dot4(n1c, dp) / f4;
  float angle2 = dot4(n2c, dp) / f4;
  // `acos (fabs (angle))` resolves to ::acos(double) in PCL 1.7's pfh.cpp
  if (std::acos(std::fabs((double)angle1)) > std::acos(std::fabs((double)angle2))) {
    n1c = n2; n2c = n1;
    dp = mul(dp, -1.0f);
    f3 = -angle2;
  } else {
    f3 = angle1;
  }
  V3 v = cross(dp, n1c);
  float v_norm = std::sqrt(sqn4(v));
  if (v_norm == 0.0f) { f1 = f2 = f3 = f4 = 0.0f; return; }
  v = mul(v, 1.0f / v_norm);  // `v /= v_norm` (Eigen 3.2: times the reciprocal)
  V3 w = cross(n1c, v);
  f2 = dot4(v, n2c);
  f1 = atan2f_glibc(dot4(w, n2c), dot4(n1c, n2c));
}

inline int clampBin(double v, int nbins) {
  // static_cast<int>(floor(v)); x86 cvttsd2si gives INT_MIN for NaN -> clamped to 0
  if (!(v == v)) return 0;
  double f = std::floor(v);
  int h = (f >= 2147483647.0 || f < -2147483648.0) ? INT32_MIN : (int)f;
  if (h < 0) h = 0;
  if (h >= nbins) h = nbins - 1;
  return h;
}

}  // namespace

extern "C" {

int orc_version() { return 1; }

// PCL 1.7 computeMeanAndCovarianceMatrix (dense branch) over cloud[idx[0..n)]: the covariance
// entries (c00, c01, c02, c11, c12, c22) as pointNormal forms them (tests: the Eigen 3.2
// reciprocal form of `accu /= n`)
void orc_point_covariance(const float* x, const float* y, const float* z, const int32_t* idx, i64 n, float* out6) {
  float accu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (i64 i = 0; i < n; ++i) {
    const int p = idx[i];
    accu[0] += x[p] * x[p]; accu[1] += x[p] * y[p]; accu[2] += x[p] * z[p];
    accu[3] += y[p] * y[p]; accu[4] += y[p] * z[p]; accu[5] += z[p] * z[p];
    accu[6] += x[p]; accu[7] += y[p]; accu[8] += z[p];
  }
  const float inv = 1.0f / (float)n;
  for (int i = 0; i < 9; ++i) accu[i] *= inv;
  out6[0] = accu[0] - accu[6] * accu[6]; out6[1] = accu[1] - accu[6] * accu[7];
  out6[2] = accu[2] - accu[6] * accu[8]; out6[3] = accu[3] - accu[7] * accu[7];
  out6[4] = accu[4] - accu[7] * accu[8]; out6[5] = accu[5] - accu[8] * accu[8];
}

// Pins the glibc float restatements of or_common.h against the host libm (tests only):
// which = 0: atan2f on n pairs (even i: uniform in [-1, 1]^2, odd i: random bit patterns),
// which = 1: acosf on every stride-th float of [-1, 1] (stride = n).  Returns the number of
// results whose bits differ (NaN == NaN).
i64 orc_libm_mismatches(int which, i64 n, uint64_t seed) {
  uint64_t s = seed ? seed : 88172645463325252ull;
  auto next = [&s]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  auto uni = [&]() { return (float)((double)(next() >> 11) / 9007199254740992.0 * 2.0 - 1.0); };
  i64 bad = 0;
  if (which == 0) {
    for (i64 i = 0; i < n; ++i) {
      float y, x;
      if (i % 2 == 0) { y = uni(); x = uni(); }
      else { y = w2f((int32_t)next()); x = w2f((int32_t)next()); }
      const float a = ::atan2f(y, x), b = atan2f_glibc(y, x);
      if (f2w(a) != f2w(b) && !(a != a && b != b)) ++bad;
    }
  } else {
    const int64_t stride = n > 0 ? n : 1;
    for (int sg = 0; sg < 2; ++sg)
      for (int64_t u = 0; u <= 0x3f800000; u += stride) {
        const float x = w2f((int32_t)((uint32_t)u | (sg ? 0x80000000u : 0u)));
        const float a = ::acosf(x), b = acosf_glibc(x);
        if (f2w(a) != f2w(b) && !(a != a && b != b)) ++bad;
      }
  }
  return bad;
}

// Radius search (FLANN order).  counts[nq]; if idx != NULL, writes up to cap entries per
// query row-major (row stride = cap) of indices and squared distances.
int orc_radius_search(const float* x, const float* y, const float* z, i64 n, const float* qx,
                      const float* qy, const float* qz, i64 nq, double r, i64* counts, int* idx,
                      float* d2, i64 cap) {
  NeighborGrid g;
  g.build(x, y, z, n, r);
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 q = 0; q < nq; ++q) {
      g.radius(qx[q], qy[q], qz[q], r, nb, dd);
      counts[q] = (i64)nb.size();
      if (idx) {
        i64 m = std::min<i64>((i64)nb.size(), cap);
        for (i64 j = 0; j < m; ++j) { idx[q * cap + j] = nb[(size_t)j]; d2[q * cap + j] = dd[(size_t)j]; }
      }
    }
  }
  return 0;
}

// NormalEstimationOMP::computeFeature, input == surface == cloud, viewpoint (vpx,vpy,vpz)
int orc_normals(const float* x, const float* y, const float* z, i64 n, double r, float vpx,
                float vpy, float vpz, float* nx, float* ny, float* nz, float* curv, int nthreads) {
  NeighborGrid g;
  g.build(x, y, z, n, r);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 i = 0; i < n; ++i) {
      g.radius(x[i], y[i], z[i], r, nb, dd);
      float o[4];
      pointNormal(x, y, z, nb, x[i], y[i], z[i], vpx, vpy, vpz, o);
      nx[i] = o[0]; ny[i] = o[1]; nz[i] = o[2]; curv[i] = o[3];
    }
  }
  return 0;
}

// FPFHEstimation::computeFeature (non-OMP class: single-threaded, evaluation.cpp:597).
// same_as_surface != 0 reproduces PCL's "input_ == surface_ and all indices" branch.
// spfh_rows_out (optional, |S| x 33) and n_spfh_out expose the SPFH table for debugging.
int orc_fpfh(const float* sx, const float* sy, const float* sz, const float* snx, const float* sny,
             const float* snz, i64 n_surf, const float* qx, const float* qy, const float* qz, i64 nq,
             int same_as_surface, double r, float* out, int nthreads) {
  const int B = 11, NB = 33;
  NeighborGrid g;
  g.build(sx, sy, sz, n_surf, r);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  // ---- computeSPFHSignatures: the set S (std::set => ascending) ----
  std::vector<int> spfh_indices;
  if (same_as_surface) {
    spfh_indices.resize((size_t)n_surf);
    for (i64 i = 0; i < n_surf; ++i) spfh_indices[(size_t)i] = (int)i;
  } else {
    std::vector<char> in_s((size_t)n_surf, 0);
    std::vector<int> nb;
    std::vector<float> dd;
    for (i64 q = 0; q < nq; ++q) {
      g.radius(qx[q], qy[q], qz[q], r, nb, dd);
      for (size_t j = 0; j < nb.size(); ++j) in_s[(size_t)nb[j]] = 1;
    }
    for (i64 i = 0; i < n_surf; ++i)
      if (in_s[(size_t)i]) spfh_indices.push_back((int)i);
  }
  const size_t S = spfh_indices.size();
  std::vector<float> hist(S * NB, 0.0f);
  std::vector<int> lookup((size_t)n_surf, 0);
  const float d_pi = 1.0f / (2.0f * (float)M_PI);
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 64)
    for (i64 row = 0; row < (i64)S; ++row) {
      const int p = spfh_indices[(size_t)row];
      g.radius(sx[p], sy[p], sz[p], r, nb, dd);
      lookup[(size_t)p] = (int)row;
      if (nb.empty()) continue;
      // computePointSPFHSignature
      float hist_incr = 100.0f / (float)(nb.size() - 1);
      float* h = &hist[(size_t)row * NB];
      V3 pp = v3(sx[p], sy[p], sz[p]), pn = v3(snx[p], sny[p], snz[p]);
      for (size_t j = 0; j < nb.size(); ++j) {
        const int q = nb[j];
        if (q == p) continue;
        float f1, f2, f3, f4;
        pairFeatures(pp, pn, v3(sx[q], sy[q], sz[q]), v3(snx[q], sny[q], snz[q]), f1, f2, f3, f4);
        int h1 = clampBin((double)B * (((double)f1 + M_PI) * (double)d_pi), B);
        int h2 = clampBin((double)B * (((double)f2 + 1.0) * 0.5), B);
        int h3 = clampBin((double)B * (((double)f3 + 1.0) * 0.5), B);
        h[h1] += hist_incr;
        h[B + h2] += hist_incr;
        h[2 * B + h3] += hist_incr;
      }
    }
  }
  // ---- weightPointSPFHSignature per query ----
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 64)
    for (i64 q = 0; q < nq; ++q) {
      float* o = out + q * NB;
      g.radius(qx[q], qy[q], qz[q], r, nb, dd);
      if (nb.empty()) {
        for (int b = 0; b < NB; ++b) o[b] = kNaN;
        continue;
      }
      double sum_f1 = 0.0, sum_f2 = 0.0, sum_f3 = 0.0;
      float fh[33];
      for (int b = 0; b < NB; ++b) fh[b] = 0.0f;
      for (size_t j = 0; j < nb.size(); ++j) {
        if (dd[j] == 0.0f) continue;
        float weight = 1.0f / dd[j];
        const float* h = &hist[(size_t)lookup[(size_t)nb[j]] * NB];
        for (int b = 0; b < B; ++b) { float v = h[b] * weight; sum_f1 += v; fh[b] += v; }
        for (int b = 0; b < B; ++b) { float v = h[B + b] * weight; sum_f2 += v; fh[B + b] += v; }
        for (int b = 0; b < B; ++b) { float v = h[2 * B + b] * weight; sum_f3 += v; fh[2 * B + b] += v; }
      }
      if (sum_f1 != 0) sum_f1 = 100.0 / sum_f1;
      if (sum_f2 != 0) sum_f2 = 100.0 / sum_f2;
      if (sum_f3 != 0) sum_f3 = 100.0 / sum_f3;
      for (int b = 0; b < B; ++b) fh[b] *= (float)sum_f1;
      for (int b = 0; b < B; ++b) fh[B + b] *= (float)sum_f2;
      for (int b = 0; b < B; ++b) fh[2 * B + b] *= (float)sum_f3;
      for (int b = 0; b < NB; ++b) o[b] = fh[b];
    }
  }
  return (int)S;
}

}  // extern "C"
