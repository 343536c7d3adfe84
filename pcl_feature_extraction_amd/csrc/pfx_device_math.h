// pfx_device_math.h -- gfx950 device arithmetic for the PCL 1.7 path.
//
// Every function reproduces the IEEE operation sequence PCL 1.7 / Eigen 3.2 execute on x86-64
// (SURVEY.md Appendix A), so results are bit-identical to the CPU restatement:
//   * compiled with -ffp-contract=off (no v_fma contraction), default IEEE div/sqrt
//     (v_div_fixup / corrected v_sqrt sequences), f32 denormals on;
//   * Eigen 3.2 fixed-size Vector3f reductions (Redux.h redux_novec_unroller, HalfLength split):
//     x + (y + z); aligned Vector4f (SSE2 predux): (x + z) + (y + w); a row of a small
//     fixed-size matrix * vector product (CoeffBasedProduct): ((m0 v0 + m1 v1) + m2 v2);
//   * atan2f / acosf: glibc's fdlibm float routines (e_atan2f.c, s_atanf.c, e_acosf.c) restated
//     operation for operation (the oracle's are pinned bit for bit against the host libm);
//     cosf / sinf as the correctly rounded result, evaluated in f64 (ocml) and rounded once;
//   * Eigen 3.2 `v /= s` and `v.normalize()` multiply by the reciprocal 1/s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pfx {

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 scale3(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 div3(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
__device__ __forceinline__ float sqn3(f3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
__device__ __forceinline__ float mv3(f3 row, f3 v) { return (row.x * v.x + row.y * v.y) + row.z * v.z; }
__device__ __forceinline__ float dot4(f3 a, f3 b) { return (a.x * b.x + a.z * b.z) + (a.y * b.y + 0.0f); }
__device__ __forceinline__ float sqn4(f3 a) { return (a.x * a.x + a.z * a.z) + (a.y * a.y + 0.0f); }
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 normalized3(f3 a) { return div3(a, sqrtf(sqn3(a))); }

// Eigen 3.2 normalize() in place: v * (1 / sqrt(squaredNorm))
__device__ __forceinline__ f3 normalize3(f3 a) { return scale3(a, 1.0f / sqrtf(sqn3(a))); }

__device__ __forceinline__ float cosf_cr(float t) { return (float)cos((double)t); }
__device__ __forceinline__ float sinf_cr(float t) { return (float)sin((double)t); }

// glibc __atanf (s_atanf.c, fdlibm)
__device__ __forceinline__ float atanf_glibc(float x) {
  const int32_t hx = __float_as_int(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? 1.5707962513e+00f + 7.5497894159e-08f : -1.5707962513e+00f - 7.5497894159e-08f;
  }
  float hi = 0.0f, lo = 0.0f;
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); hi = 4.6364760399e-01f; lo = 5.0121582440e-09f; }
      else { id = 1; x = (x - 1.0f) / (x + 1.0f); hi = 7.8539812565e-01f; lo = 3.7748947079e-08f; }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); hi = 9.8279368877e-01f; lo = 3.4473217170e-08f; }
      else { id = 3; x = -1.0f / x; hi = 1.5707962513e+00f; lo = 7.5497894159e-08f; }
    }
  }
  const float z = x * x, w = z * z;
  const float s1 = z * (3.3333334327e-01f +
                        w * (1.4285714924e-01f + w * (9.0908870101e-02f + w * (6.6610731184e-02f +
                        w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
  const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                        w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
  if (id < 0) return x - x * (s1 + s2);
  const float r = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -r : r;
}

// glibc __ieee754_atan2f (e_atan2f.c, fdlibm)
__device__ __forceinline__ float atan2f_glibc(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
              pi_lo = -8.7422776573e-08f;
  const int32_t hx = __float_as_int(x), ix = hx & 0x7fffffff, hy = __float_as_int(y), iy = hy & 0x7fffffff;
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
      if (m == 0) return pi_o_4 + tiny;
      if (m == 1) return -pi_o_4 - tiny;
      if (m == 2) return 3.0f * pi_o_4 + tiny;
      return -3.0f * pi_o_4 - tiny;
    }
    if (m == 0) return 0.0f;
    if (m == 1) return -0.0f;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = atanf_glibc(fabsf(y / x));
  if (m == 0) return z;
  if (m == 1) return __int_as_float(__float_as_int(z) ^ (int32_t)0x80000000);
  if (m == 2) return pi - (z - pi_lo);
  return (z - pi_lo) - pi;
}

// glibc __ieee754_acosf (e_acosf.c, fdlibm)
__device__ __forceinline__ float acosf_glibc(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
              pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
              pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
              qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
  const int32_t hx = __float_as_int(x), ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if (hx < 0) {
    const float z = (one + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = sqrtf(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (one - x) * 0.5f;
  const float s = sqrtf(z);
  const float df = __int_as_float(__float_as_int(s) & (int32_t)0xfffff000);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}
__device__ __forceinline__ float pow3f_cr(float x) { double d = (double)x; return (float)(d * d * d); }

// squared distance exactly as FLANN L2_Simple: ((0 + dx^2) + dy^2) + dz^2, dx = q - p
__device__ __forceinline__ float flann_d2(float qx, float qy, float qz, float px, float py, float pz) {
  float dx = qx - px, dy = qy - py, dz = qz - pz;
  return ((0.0f + dx * dx) + dy * dy) + dz * dz;
}

// ---- pcl::computeRoots2 / computeRoots (common/impl/eigen.hpp) ---------------------------
__device__ __forceinline__ void computeRoots2(float b, float c, float r[3]) {
  r[0] = 0.0f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.0f) d = 0.0f;
  float sd = sqrtf(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

// m00 m01 m02 m11 m12 m22 (upper triangle, as read by PCL)
__device__ __forceinline__ void computeRoots(float m00, float m01, float m02, float m11, float m12,
                                             float m22, float r[3]) {
  float c0 = m00 * m11 * m22 + 2.0f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 -
             m22 * m01 * m01;
  float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  float c2 = m00 + m11 + m22;
  if (fabsf(c0) < 1.19209290e-07f) {
    computeRoots2(c2, c1, r);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = sqrtf(3.0f);
  float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.0f) a_over_3 = 0.0f;
  float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.0f) q = 0.0f;
  float rho = sqrtf(-a_over_3);
  float theta = atan2f_glibc(sqrtf(-q), half_b) * s_inv3;
  float ct = cosf_cr(theta), st = sinf_cr(theta);
  r[0] = c2_over_3 + 2.0f * rho * ct;
  r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
  r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
  float t;
  if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  if (r[1] >= r[2]) {
    t = r[1]; r[1] = r[2]; r[2] = t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  }
  if (r[0] <= 0.0f) computeRoots2(c2, c1, r);
}

struct Sym3 { float a00, a01, a02, a10, a11, a12, a20, a21, a22; };  // full row-major 3x3

__device__ __forceinline__ float scaleSym(const Sym3& m, Sym3& s) {
  float sc = 0.0f;
  sc = fmaxf(sc, fabsf(m.a00)); sc = fmaxf(sc, fabsf(m.a01)); sc = fmaxf(sc, fabsf(m.a02));
  sc = fmaxf(sc, fabsf(m.a10)); sc = fmaxf(sc, fabsf(m.a11)); sc = fmaxf(sc, fabsf(m.a12));
  sc = fmaxf(sc, fabsf(m.a20)); sc = fmaxf(sc, fabsf(m.a21)); sc = fmaxf(sc, fabsf(m.a22));
  if (sc <= 1.17549435e-38f) sc = 1.0f;
  s.a00 = m.a00 / sc; s.a01 = m.a01 / sc; s.a02 = m.a02 / sc;
  s.a10 = m.a10 / sc; s.a11 = m.a11 / sc; s.a12 = m.a12 / sc;
  s.a20 = m.a20 / sc; s.a21 = m.a21 / sc; s.a22 = m.a22 / sc;
  return sc;
}

__device__ __forceinline__ f3 nullVector(const Sym3& s, float lambda, float* picked) {
  f3 r0 = mk3(s.a00 - lambda, s.a01, s.a02);
  f3 r1 = mk3(s.a10, s.a11 - lambda, s.a12);
  f3 r2 = mk3(s.a20, s.a21, s.a22 - lambda);
  f3 v1 = cross3(r0, r1), v2 = cross3(r0, r2), v3 = cross3(r1, r2);
  float l1 = sqn3(v1), l2 = sqn3(v2), l3 = sqn3(v3);
  if (l1 >= l2 && l1 >= l3) { *picked = l1; return div3(v1, sqrtf(l1)); }
  if (l2 >= l1 && l2 >= l3) { *picked = l2; return div3(v2, sqrtf(l2)); }
  *picked = l3;
  return div3(v3, sqrtf(l3));
}

// pcl::eigen33(mat, eigenvalue, eigenvector): smallest eigenpair
__device__ __forceinline__ void eigen33_min(const Sym3& m, float& lambda, f3& vec) {
  Sym3 s;
  float sc = scaleSym(m, s);
  float ev[3];
  computeRoots(s.a00, s.a01, s.a02, s.a11, s.a12, s.a22, ev);
  lambda = ev[0] * sc;
  float dummy;
  vec = nullVector(s, ev[0], &dummy);
}

__device__ __forceinline__ f3 unitOrthogonal(f3 s) {
  const float prec = 1e-5f;
  bool xs = fabsf(s.x) <= fabsf(s.z) * prec;
  bool ys = fabsf(s.y) <= fabsf(s.z) * prec;
  if (!xs || !ys) {
    float inv = 1.0f / sqrtf(s.x * s.x + s.y * s.y);
    return mk3(-s.y * inv, s.x * inv, 0.0f);
  }
  float inv = 1.0f / sqrtf(s.y * s.y + s.z * s.z);
  return mk3(0.0f, -s.z * inv, s.y * inv);
}

// pcl::eigen33(mat, evecs, evals): evecs[k] = column k, ascending evals
__device__ __forceinline__ void eigen33_full(const Sym3& m, f3 ev[3], float evals[3]) {
  Sym3 s;
  float sc = scaleSym(m, s);
  computeRoots(s.a00, s.a01, s.a02, s.a11, s.a12, s.a22, evals);
  const float eps = 1.19209290e-07f;
  float pk;
  if ((evals[2] - evals[0]) <= eps) {
    ev[0] = mk3(1, 0, 0); ev[1] = mk3(0, 1, 0); ev[2] = mk3(0, 0, 1);
  } else if ((evals[1] - evals[0]) <= eps) {
    ev[2] = nullVector(s, evals[2], &pk);
    ev[1] = unitOrthogonal(ev[2]);
    ev[0] = cross3(ev[1], ev[2]);
  } else if ((evals[2] - evals[1]) <= eps) {
    ev[0] = nullVector(s, evals[0], &pk);
    ev[1] = unitOrthogonal(ev[0]);
    ev[2] = cross3(ev[0], ev[1]);
  } else {
    float mmax[3];
    unsigned min_el = 2, max_el = 2;
    ev[2] = nullVector(s, evals[2], &mmax[2]);
    float l1;
    ev[1] = nullVector(s, evals[1], &l1);
    mmax[1] = l1;
    min_el = l1 <= mmax[min_el] ? 1 : min_el;
    max_el = l1 > mmax[max_el] ? 1 : max_el;
    f3 r0 = mk3(s.a00 - evals[0], s.a01, s.a02);
    f3 r1 = mk3(s.a10, s.a11 - evals[0], s.a12);
    f3 r2 = mk3(s.a20, s.a21, s.a22 - evals[0]);
    f3 v1 = cross3(r0, r1), v2 = cross3(r0, r2), v3 = cross3(r1, r2);
    float len1 = sqn3(v1), len2 = sqn3(v2), len3 = sqn3(v3);
    if (len1 >= len2 && len1 >= len3) { mmax[0] = len1; ev[0] = div3(v1, sqrtf(len1)); }
    else if (len2 >= len1 && len2 >= len3) { mmax[0] = len2; ev[0] = div3(v2, sqrtf(len2)); }
    else { mmax[0] = len3; ev[0] = div3(v3, sqrtf(len3)); }
    min_el = len3 <= mmax[min_el] ? 0 : min_el;
    max_el = len3 > mmax[max_el] ? 0 : max_el;
    unsigned mid_el = 3 - min_el - max_el;
    f3 e0 = ev[0], e1 = ev[1], e2 = ev[2];
    f3 a = (min_el == 0) ? e1 : (min_el == 1 ? e2 : e0);
    f3 b = (min_el == 0) ? e2 : (min_el == 1 ? e0 : e1);
    f3 nmin = normalized3(cross3(a, b));
    if (min_el == 0) e0 = nmin; else if (min_el == 1) e1 = nmin; else e2 = nmin;
    a = (mid_el == 0) ? e1 : (mid_el == 1 ? e2 : e0);
    b = (mid_el == 0) ? e2 : (mid_el == 1 ? e0 : e1);
    f3 nmid = normalized3(cross3(a, b));
    if (mid_el == 0) e0 = nmid; else if (mid_el == 1) e1 = nmid; else e2 = nmid;
    ev[0] = e0; ev[1] = e1; ev[2] = e2;
  }
  evals[0] *= sc; evals[1] *= sc; evals[2] *= sc;
}

}  // namespace pfx
