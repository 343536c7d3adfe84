// =====================================================================================
//  oracle/or_common.h  --  TEST INFRASTRUCTURE ONLY (never linked into the product)
//
//  CPU restatement of the PCL 1.7.x arithmetic that srv/pcl_feature_extraction's hot
//  path calls into.  PCL/Eigen/FLANN are third-party, unpinned
//  (CMakeLists.txt:16,19 `find_package(Eigen|PCL REQUIRED)`, no version) and absent from
//  /root/reference, and the reference holds no tests or golden vectors for this path:
//
//      *** parity vs real PCL is UNPINNED ***
//
//  The restatement is pinned only by analytic known-answer tests (tests/test_oracle.py) and the regression
//  fixtures tests/golden/oracle_small.npz
//  and is the checker the HIP product is compared against.
//
//  Floating-point contract (every oracle TU is built with -O2 -ffp-contract=off, x86-64
//  SSE2, no -march): IEEE binary32/64, left-to-right evaluation, no FMA.  Eigen 3.2
//  evaluation orders are restated explicitly:
//    * fixed-size 3-vectors (not vectorised):    dot/squaredNorm = (x + y) + z
//    * aligned 4-vectors (SSE2 packet predux):   dot/squaredNorm = (x + z) + (y + w)
//  Transcendentals: the float functions PCL calls (atan2f/cosf/sinf/acosf) are restated
//  as the correctly rounded value, computed through glibc's double routine and rounded
//  once.  glibc's own fdlibm-derived atan2f differs from that by <=1 ulp on a fraction
//  of inputs; that part of the "vs PCL" parity is unpinned as well.
// =====================================================================================
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#include <algorithm>

namespace orc {

typedef int64_t i64;

static const float kNaN = std::numeric_limits<float>::quiet_NaN();

// ---- correctly rounded float transcendentals ----------------------------------------
inline float atan2f_cr(float y, float x) { return (float)std::atan2((double)y, (double)x); }
inline float cosf_cr(float t) { return (float)std::cos((double)t); }
inline float sinf_cr(float t) { return (float)std::sin((double)t); }
inline float acosf_cr(float t) { return (float)std::acos((double)t); }
// powf(x, 3) / powf(x, 2) as used by RangeImageBorderExtractor / NarfKeypoint
inline float pow3f_cr(float x) { double d = (double)x; return (float)(d * d * d); }

// ---- small vector algebra with Eigen 3.2 evaluation order ---------------------------
struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
// Vector3f (unvectorised): ((a0 b0 + a1 b1) + a2 b2)
inline float dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float sqn3(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
// Vector4f with w == 0 (SSE2 predux): ((a0 b0 + a2 b2) + (a1 b1 + 0))
inline float dot4(V3 a, V3 b) { return (a.x * b.x + a.z * b.z) + (a.y * b.y + 0.0f); }
inline float sqn4(V3 a) { return (a.x * a.x + a.z * a.z) + (a.y * a.y + 0.0f); }
inline V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Eigen normalized(): v / sqrt(squaredNorm)
inline V3 normalized3(V3 a) { return divs(a, std::sqrt(sqn3(a))); }

// ---- pcl::computeRoots / computeRoots2 (common/impl/eigen.hpp, float) ---------------
inline void computeRoots2(float b, float c, float roots[3]) {
  roots[0] = 0.0f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);  // Scalar (b * b - 4.0 * c)
  if (d < 0.0f) d = 0.0f;
  float sd = std::sqrt(d);
  roots[2] = 0.5f * (b + sd);
  roots[1] = 0.5f * (b - sd);
}

// m: row-major 3x3 (only m[0][0..2], m[1][1..2], m[2][2] are read, as in PCL)
inline void computeRoots(const float m[3][3], float roots[3]) {
  float c0 = m[0][0] * m[1][1] * m[2][2] + 2.0f * m[0][1] * m[0][2] * m[1][2] -
             m[0][0] * m[1][2] * m[1][2] - m[1][1] * m[0][2] * m[0][2] -
             m[2][2] * m[0][1] * m[0][1];
  float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] +
             m[1][1] * m[2][2] - m[1][2] * m[1][2];
  float c2 = m[0][0] + m[1][1] + m[2][2];
  if (std::fabs((double)c0) < (double)FLT_EPSILON) {
    computeRoots2(c2, c1, roots);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = std::sqrt(3.0f);
  float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.0f) a_over_3 = 0.0f;
  float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.0f) q = 0.0f;
  float rho = std::sqrt(-a_over_3);
  float theta = atan2f_cr(std::sqrt(-q), half_b) * s_inv3;
  float cos_theta = cosf_cr(theta);
  float sin_theta = sinf_cr(theta);
  roots[0] = c2_over_3 + 2.0f * rho * cos_theta;
  roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
  roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
  if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
  if (roots[1] >= roots[2]) {
    std::swap(roots[1], roots[2]);
    if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
  }
  if (roots[0] <= 0.0f) computeRoots2(c2, c1, roots);
}

inline void scaleMatrix(const float mat[3][3], float sm[3][3], float& scale) {
  scale = 0.0f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(mat[i][j]));
  if (scale <= FLT_MIN) scale = 1.0f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) sm[i][j] = mat[i][j] / scale;
}

// Pick the longest of the three row cross products of (sm - lambda I), normalised.
inline V3 nullVector(const float sm[3][3], float lambda, float* picked_len = 0) {
  float t[3][3];
  std::memcpy(t, sm, sizeof(t));
  t[0][0] -= lambda; t[1][1] -= lambda; t[2][2] -= lambda;
  V3 r0 = v3(t[0][0], t[0][1], t[0][2]), r1 = v3(t[1][0], t[1][1], t[1][2]),
     r2 = v3(t[2][0], t[2][1], t[2][2]);
  V3 vec1 = cross(r0, r1), vec2 = cross(r0, r2), vec3 = cross(r1, r2);
  float len1 = sqn3(vec1), len2 = sqn3(vec2), len3 = sqn3(vec3);
  if (len1 >= len2 && len1 >= len3) { if (picked_len) *picked_len = len1; return divs(vec1, std::sqrt(len1)); }
  if (len2 >= len1 && len2 >= len3) { if (picked_len) *picked_len = len2; return divs(vec2, std::sqrt(len2)); }
  if (picked_len) *picked_len = len3;
  return divs(vec3, std::sqrt(len3));
}

// pcl::eigen33 (mat, eigenvalue, eigenvector): smallest eigenpair (common/impl/eigen.hpp)
inline void eigen33_min(const float mat[3][3], float& eigenvalue, V3& eigenvector) {
  float sm[3][3], scale;
  scaleMatrix(mat, sm, scale);
  float ev[3];
  computeRoots(sm, ev);
  eigenvalue = ev[0] * scale;
  eigenvector = nullVector(sm, ev[0]);
}

// Eigen unitOrthogonal() for a 3-vector (Eigen/src/Geometry/OrthoMethods.h)
inline V3 unitOrthogonal(V3 s) {
  const float prec = 1e-5f;  // NumTraits<float>::dummy_precision()
  bool x_small = std::fabs(s.x) <= std::fabs(s.z) * prec;
  bool y_small = std::fabs(s.y) <= std::fabs(s.z) * prec;
  if (!x_small || !y_small) {
    float invnm = 1.0f / std::sqrt(s.x * s.x + s.y * s.y);
    return v3(-s.y * invnm, s.x * invnm, 0.0f);
  }
  float invnm = 1.0f / std::sqrt(s.y * s.y + s.z * s.z);
  return v3(0.0f, -s.z * invnm, s.y * invnm);
}

// pcl::eigen33 (mat, evecs, evals): all eigenpairs, evecs[k] = column k (ascending evals)
inline void eigen33_full(const float mat[3][3], V3 evecs[3], float evals[3]) {
  float sm[3][3], scale;
  scaleMatrix(mat, sm, scale);
  computeRoots(sm, evals);
  const float eps = FLT_EPSILON;
  if ((evals[2] - evals[0]) <= eps) {
    evecs[0] = v3(1, 0, 0); evecs[1] = v3(0, 1, 0); evecs[2] = v3(0, 0, 1);
  } else if ((evals[1] - evals[0]) <= eps) {
    evecs[2] = nullVector(sm, evals[2]);
    evecs[1] = unitOrthogonal(evecs[2]);
    evecs[0] = cross(evecs[1], evecs[2]);
  } else if ((evals[2] - evals[1]) <= eps) {
    evecs[0] = nullVector(sm, evals[0]);
    evecs[1] = unitOrthogonal(evecs[0]);
    evecs[2] = cross(evecs[0], evecs[1]);
  } else {
    float mmax[3];
    unsigned min_el = 2, max_el = 2;
    evecs[2] = nullVector(sm, evals[2], &mmax[2]);
    float l1;
    evecs[1] = nullVector(sm, evals[1], &l1);
    mmax[1] = l1;
    min_el = l1 <= mmax[min_el] ? 1 : min_el;
    max_el = l1 > mmax[max_el] ? 1 : max_el;
    // third block: PCL 1.7 compares len3 of the evals(0) block for every branch
    float t[3][3];
    std::memcpy(t, sm, sizeof(t));
    t[0][0] -= evals[0]; t[1][1] -= evals[0]; t[2][2] -= evals[0];
    V3 r0 = v3(t[0][0], t[0][1], t[0][2]), r1 = v3(t[1][0], t[1][1], t[1][2]),
       r2 = v3(t[2][0], t[2][1], t[2][2]);
    V3 vec1 = cross(r0, r1), vec2 = cross(r0, r2), vec3 = cross(r1, r2);
    float len1 = sqn3(vec1), len2 = sqn3(vec2), len3 = sqn3(vec3);
    if (len1 >= len2 && len1 >= len3) { mmax[0] = len1; evecs[0] = divs(vec1, std::sqrt(len1)); }
    else if (len2 >= len1 && len2 >= len3) { mmax[0] = len2; evecs[0] = divs(vec2, std::sqrt(len2)); }
    else { mmax[0] = len3; evecs[0] = divs(vec3, std::sqrt(len3)); }
    min_el = len3 <= mmax[min_el] ? 0 : min_el;
    max_el = len3 > mmax[max_el] ? 0 : max_el;
    unsigned mid_el = 3 - min_el - max_el;
    evecs[min_el] = normalized3(cross(evecs[(min_el + 1) % 3], evecs[(min_el + 2) % 3]));
    evecs[mid_el] = normalized3(cross(evecs[(mid_el + 1) % 3], evecs[(mid_el + 2) % 3]));
  }
  evals[0] *= scale; evals[1] *= scale; evals[2] *= scale;
}

// ---- exact radius search with FLANN result order -------------------------------------
// FLANN KDTreeSingleIndex + RadiusResultSet: d2 = ((0+dx^2)+dy^2)+dz^2 with
// dx = q - p in float, inclusion d2 < (float)(r*r) (strict), result sorted by (d2, index).
// Restated with a uniform grid (cell >= r): the candidate set is a superset, the test and
// the order are FLANN's.
struct NeighborGrid {
  const float *x, *y, *z;
  i64 n;
  double cell, inv, ox, oy, oz;
  std::vector<i64> order;                      // point indices sorted by cell key
  std::vector<uint64_t> keys;                  // unique occupied cell keys (ascending)
  std::vector<i64> start, end;                 // ranges into order[]
  static const i64 OFF = (1 << 20);

  static uint64_t pack(i64 ix, i64 iy, i64 iz) {
    return ((uint64_t)(ix + OFF) << 42) | ((uint64_t)(iy + OFF) << 21) | (uint64_t)(iz + OFF);
  }
  void cellOf(float px, float py, float pz, i64& ix, i64& iy, i64& iz) const {
    ix = (i64)std::floor(((double)px - ox) * inv);
    iy = (i64)std::floor(((double)py - oy) * inv);
    iz = (i64)std::floor(((double)pz - oz) * inv);
  }
  void build(const float* x_, const float* y_, const float* z_, i64 n_, double r) {
    x = x_; y = y_; z = z_; n = n_;
    cell = r > 0 ? r : 1.0;
    inv = 1.0 / cell;
    // non-finite points are not indexed (PCL's kd-tree skips them)
    ox = oy = oz = 0.0;
    bool first = true;
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x[i], y[i], z[i])) continue;
      if (first) { ox = x[i]; oy = y[i]; oz = z[i]; first = false; }
      ox = std::min(ox, (double)x[i]); oy = std::min(oy, (double)y[i]); oz = std::min(oz, (double)z[i]);
    }
    std::vector<std::pair<uint64_t, i64> > kv;
    kv.reserve((size_t)n);
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x[i], y[i], z[i])) continue;
      i64 ix, iy, iz;
      cellOf(x[i], y[i], z[i], ix, iy, iz);
      kv.push_back(std::make_pair(pack(ix, iy, iz), i));
    }
    std::sort(kv.begin(), kv.end());
    const i64 m = (i64)kv.size();
    order.resize((size_t)m);
    keys.clear(); start.clear(); end.clear();
    for (i64 i = 0; i < m; ++i) {
      order[(size_t)i] = kv[(size_t)i].second;
      if (i == 0 || kv[(size_t)i].first != kv[(size_t)i - 1].first) {
        keys.push_back(kv[(size_t)i].first);
        start.push_back(i);
        if (i) end.push_back(i);
      }
    }
    if (m) end.push_back(m);
  }
  static bool finite3(float a, float b, float c) { return std::isfinite(a) && std::isfinite(b) && std::isfinite(c); }
  // returns neighbours sorted by (d2, index)
  void radius(float qx, float qy, float qz, double r, std::vector<int>& idx,
              std::vector<float>& d2) const {
    idx.clear(); d2.clear();
    const float rr = (float)(r * r);
    if (!finite3(qx, qy, qz)) return;
    i64 cx, cy, cz;
    cellOf(qx, qy, qz, cx, cy, cz);
    std::vector<std::pair<float, int> > hits;
    for (i64 ix = cx - 1; ix <= cx + 1; ++ix)
      for (i64 iy = cy - 1; iy <= cy + 1; ++iy)
        for (i64 iz = cz - 1; iz <= cz + 1; ++iz) {
          if (ix < -OFF + 1 || iy < -OFF + 1 || iz < -OFF + 1 || ix >= OFF || iy >= OFF || iz >= OFF) continue;
          uint64_t k = pack(ix, iy, iz);
          std::vector<uint64_t>::const_iterator it = std::lower_bound(keys.begin(), keys.end(), k);
          if (it == keys.end() || *it != k) continue;
          size_t c = (size_t)(it - keys.begin());
          for (i64 s = start[c]; s < end[c]; ++s) {
            i64 p = order[(size_t)s];
            float dx = qx - x[p], dy = qy - y[p], dz = qz - z[p];
            float dd = ((0.0f + dx * dx) + dy * dy) + dz * dz;
            if (dd < rr) hits.push_back(std::make_pair(dd, (int)p));
          }
        }
    std::sort(hits.begin(), hits.end());  // (d2, index) lexicographic == FLANN DistanceIndex<
    idx.resize(hits.size()); d2.resize(hits.size());
    for (size_t i = 0; i < hits.size(); ++i) { d2[i] = hits[i].first; idx[i] = hits[i].second; }
  }
};

}  // namespace orc
