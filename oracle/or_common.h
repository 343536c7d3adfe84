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
//  evaluation orders are restated explicitly (one model everywhere, round 4):
//    * reductions (dot / sum / squaredNorm / norm) of a fixed-size expression without packet
//      access -- Vector3f, Map<Vector3f>, a 3-element block -- go through Redux.h's
//      DefaultTraversal + CompleteUnrolling, i.e. redux_novec_unroller, which splits at
//      HalfLength = Length / 2:  sum of 3 terms = x + (y + z)            (dot3 / sqn3)
//    * aligned 4-vectors (SSE2 packet predux):   dot/squaredNorm = (x + z) + (y + w)
//    * small fixed-size matrix * vector products (Affine3f * Vector3f, Matrix3f * Vector3f) are
//      CoeffBasedProduct coefficients (product_coeff_impl, DefaultTraversal): left to right,
//      ((m0 v0 + m1 v1) + m2 v2)                                         (mv3)
//    * scalar code written out in PCL (squaredEuclideanDistance, flipNormalTowardsViewpoint):
//      left to right as written.
//  Transcendentals: atan2f and acosf are glibc's (sysdeps/ieee754/flt-32/e_atan2f.c,
//  s_atanf.c, e_acosf.c: the fdlibm float routines, unchanged from the ROS-Indigo-era glibc
//  2.19 to 2.35), restated below and PINNED against the host libm bit for bit
//  (tests/test_oracle.py: all floats in [-1, 1] for acosf, 2e7 random pairs for atan2f).
//  cosf/sinf (computeRoots only) are the correctly rounded value: glibc 2.19's x86_64 SSE2
//  s_cosf.S/s_sinf.S evaluate in double and round once; unpinned.
//  Eigen 3.2 scalar division: `v /= s` and `v.normalize()` multiply by the reciprocal
//  (DenseBase::operator/= uses scalar_product_op with Scalar(1)/s, SelfCwiseBinaryOp.h);
//  `v / s` and `v.normalized()` divide (scalar_quotient1_op).
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

// ---- float transcendentals ----------------------------------------------------------
inline int32_t f2w(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }
inline float w2f(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

// glibc __atanf (s_atanf.c, fdlibm): argument reduction to |x| < 7/16 around atan(0.5),
// atan(1), atan(1.5), atan(inf), odd/even split of the degree-11 polynomial
inline float atanf_glibc(float x) {
  static const float atanhi[] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
  static const float atanlo[] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
  static const float aT[] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                             9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                             4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
  const int32_t hx = f2w(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = std::fabs(x);
    if (ix < 0x3f980000) {  // |x| < 1.1875
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
      else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
      else { id = 3; x = -1.0f / x; }
    }
  }
  const float z = x * x, w = z * z;
  const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -r : r;
}

// glibc __ieee754_atan2f (e_atan2f.c, fdlibm)
inline float atan2f_glibc(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
              pi_lo = -8.7422776573e-08f;
  const int32_t hx = f2w(x), ix = hx & 0x7fffffff, hy = f2w(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf_glibc(y);
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    if (m <= 1) return y;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return 0.0f;
      case 1: return -0.0f;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = atanf_glibc(std::fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return w2f(f2w(z) ^ (int32_t)0x80000000);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// glibc __ieee754_acosf (e_acosf.c, fdlibm)
inline float acosf_glibc(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
              pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
              pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
              qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
  const int32_t hx = f2w(x), ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if (hx < 0) {  // x < -0.5
    const float z = (one + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = std::sqrt(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (one - x) * 0.5f;  // x > 0.5
  const float s = std::sqrt(z);
  const float df = w2f(f2w(s) & (int32_t)0xfffff000);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}

inline float cosf_cr(float t) { return (float)std::cos((double)t); }
inline float sinf_cr(float t) { return (float)std::sin((double)t); }
// powf(x, 3) / powf(x, 2) as used by RangeImageBorderExtractor / NarfKeypoint
inline float pow3f_cr(float x) { double d = (double)x; return (float)(d * d * d); }

// ---- small vector algebra with Eigen 3.2 evaluation order ---------------------------
struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
// Vector3f reductions (unvectorised, redux_novec_unroller<0,3>): a0 b0 + (a1 b1 + a2 b2)
inline float dot3(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
inline float sqn3(V3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
// one row of a small fixed-size matrix * Vector3f (CoeffBasedProduct): ((m0 v0 + m1 v1) + m2 v2)
inline float mv3(V3 row, V3 v) { return (row.x * v.x + row.y * v.y) + row.z * v.z; }
// Vector4f with w == 0 (SSE2 predux): ((a0 b0 + a2 b2) + (a1 b1 + 0))
inline float dot4(V3 a, V3 b) { return (a.x * b.x + a.z * b.z) + (a.y * b.y + 0.0f); }
inline float sqn4(V3 a) { return (a.x * a.x + a.z * a.z) + (a.y * a.y + 0.0f); }
inline V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Eigen normalized(): v / sqrt(squaredNorm)
inline V3 normalized3(V3 a) { return divs(a, std::sqrt(sqn3(a))); }
// Eigen 3.2 normalize() in place: v *= 1 / sqrt(squaredNorm)  (operator/= by the reciprocal)
inline V3 normalize3(V3 a) { return mul(a, 1.0f / std::sqrt(sqn3(a))); }

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
  float theta = atan2f_glibc(std::sqrt(-q), half_b) * s_inv3;
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

// ---- Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d>::compute (ComputeEigenvectors) ---------
// (Eigenvalues/SelfAdjointEigenSolver.h, Eigenvalues/Tridiagonalization.h, Jacobi/Jacobi.h,
// MathFunctions.h hypot_impl).  Used by ISSKeypoint3D (values only) and by
// SHOTLocalReferenceFrameEstimation::getLocalRF (values and vectors).
inline double hypot_e(double x, double y) {  // internal::hypot_impl
  const double ax = std::fabs(x), ay = std::fabs(y);
  const double p = std::max(ax, ay);
  if (p == 0.0) return 0.0;
  const double q = std::min(ax, ay);
  const double qp = q / p;
  return p * std::sqrt(1.0 + qp * qp);
}

inline void make_givens(double p, double q, double& c, double& s) {  // JacobiRotation::makeGivens (real)
  if (q == 0.0) {
    c = p < 0.0 ? -1.0 : 1.0;
    s = 0.0;
  } else if (p == 0.0) {
    c = 0.0;
    s = q < 0.0 ? 1.0 : -1.0;
  } else if (std::fabs(p) > std::fabs(q)) {
    const double t = q / p;
    double u = std::sqrt(1.0 + t * t);
    if (p < 0.0) u = -u;
    c = 1.0 / u;
    s = -t * c;
  } else {
    const double t = p / q;
    double u = std::sqrt(1.0 + t * t);
    if (q < 0.0) u = -u;
    s = -1.0 / u;
    c = -t * s;
  }
}

// internal::tridiagonal_qr_step; Q (nullable, column-major 3x3 as Q[col][row]) gets
// Q.applyOnTheRight(k, k+1, rot) = apply_rotation_in_the_plane(col k, col k+1, rot.transpose()):
// x' = c x - s y, y' = s x + c y (returns early for the identity rotation)
inline void tridiagonal_qr_step(double* diag, double* sub, int start, int end, double (*Q)[3]) {
  const double td = (diag[end - 1] - diag[end]) * 0.5;
  const double e = sub[end - 1];
  double mu = diag[end];
  if (td == 0.0) {
    mu -= std::fabs(e);
  } else {
    const double e2 = e * e;
    const double h = hypot_e(td, e);
    if (e2 == 0.0)
      mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
    else
      mu -= e2 / (td + (td > 0.0 ? h : -h));
  }
  double x = diag[start] - mu;
  double z = sub[start];
  for (int k = start; k < end; ++k) {
    double c, s;
    make_givens(x, z, c, s);
    const double sdk = s * diag[k] + c * sub[k];
    const double dkp1 = s * sub[k] + c * diag[k + 1];
    diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
    diag[k + 1] = s * sdk + c * dkp1;
    sub[k] = c * sdk - s * dkp1;
    if (k > start) sub[k - 1] = c * sub[k - 1] - s * z;
    x = sub[k];
    if (k < end - 1) {
      z = -s * sub[k + 1];
      sub[k + 1] = c * sub[k + 1];
    }
    if (Q && !(c == 1.0 && s == 0.0)) {
      for (int i = 0; i < 3; ++i) {
        const double xi = Q[k][i], yi = Q[k + 1][i];
        Q[k][i] = c * xi + (-s) * yi;
        Q[k + 1][i] = -(-s) * xi + c * yi;
      }
    }
  }
}

// a: row-major symmetric 3x3 (the lower triangle is read, as Eigen does); ev ascending.
// V (nullable): V[k] = the eigenvector of ev[k] (column k of Eigen's eigenvectors()).
inline void selfadjoint_eigen3(const double a[9], double ev[3], double (*V)[3]) {
  double m[3][3] = {{a[0], 0.0, 0.0}, {a[3], a[4], 0.0}, {a[6], a[7], a[8]}};
  double scale = 0.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(m[i][j]));
  if (scale == 0.0) scale = 1.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j <= i; ++j) m[i][j] /= scale;  // triangularView<Lower>() /= scale: m / s
  // tridiagonalization_inplace_selector<MatrixType, 3, false>::run (extractQ)
  double diag[3], sub[2], Q[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
  diag[0] = m[0][0];
  const double v1norm2 = m[2][0] * m[2][0];
  if (v1norm2 == 0.0) {
    diag[1] = m[1][1];
    diag[2] = m[2][2];
    sub[0] = m[1][0];
    sub[1] = m[2][1];
  } else {
    const double beta = std::sqrt(m[1][0] * m[1][0] + v1norm2);
    const double inv_beta = 1.0 / beta;
    const double m01 = m[1][0] * inv_beta;
    const double m02 = m[2][0] * inv_beta;
    const double q = 2.0 * m01 * m[2][1] + m02 * (m[2][2] - m[1][1]);
    diag[1] = m[1][1] + m02 * q;
    diag[2] = m[2][2] - m02 * q;
    sub[0] = beta;
    sub[1] = m[2][1] - m01 * q;
    // mat << 1, 0, 0,  0, m01, m02,  0, m02, -m01   (Q[col][row])
    Q[1][1] = m01; Q[1][2] = m02; Q[2][1] = m02; Q[2][2] = -m01;
  }
  // implicit symmetric QR with Wilkinson shift (max 30 * n iterations)
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (std::fabs(sub[i]) <= (std::fabs(diag[i]) + std::fabs(diag[i + 1])) * 1e-12) sub[i] = 0.0;
    while (end > 0 && sub[end - 1] == 0.0) end--;
    if (end <= 0) break;
    iter++;
    if (iter > 30 * 3) break;
    start = end - 1;
    while (start > 0 && sub[start - 1] != 0.0) start--;
    tridiagonal_qr_step(diag, sub, start, end, V ? Q : 0);
  }
  if (iter <= 30 * 3) {  // Success: selection sort, ascending (first minimum wins), columns follow
    for (int i = 0; i < 2; ++i) {
      int k = i;
      for (int j = i + 1; j < 3; ++j)
        if (diag[j] < diag[k]) k = j;
      if (k != i) {
        std::swap(diag[i], diag[k]);
        for (int r = 0; r < 3; ++r) std::swap(Q[i][r], Q[k][r]);
      }
    }
  }
  for (int i = 0; i < 3; ++i) ev[i] = diag[i] * scale;
  if (V)
    for (int k = 0; k < 3; ++k)
      for (int r = 0; r < 3; ++r) V[k][r] = Q[k][r];
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
