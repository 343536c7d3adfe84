// pfx_normal_math.h -- PCL's per-point normal from the ordered neighbour sums:
//   accu = sequential float sums {x^2, xy, xz, y^2, yz, z^2, x, y, z} in FLANN order
//   C    = accu * (1/|N|) - mean mean^T  (Eigen 3.2 `accu /= n`);  (lambda, n) = pcl::eigen33(C);  curvature = |lambda / tr C|
//   flip n towards the viewpoint;  |N| < 3 -> NaN
#pragma once
#include "pfx_device_math.h"

namespace pfx {

// term a of the nine covariance chains for neighbour (px, py, pz)
__device__ __forceinline__ float chain_term(int a, float px, float py, float pz) {
  float u = (a == 0 || a == 1 || a == 2 || a == 6) ? px : ((a == 3 || a == 4 || a == 7) ? py : pz);
  float v = (a == 0) ? px : ((a == 1 || a == 3) ? py : pz);
  return (a < 6) ? u * v : u;
}

__device__ __forceinline__ void finish_normal(const float accu_in[9], int k, float px, float py, float pz,
                                              float vpx, float vpy, float vpz, float out[4]) {
  if (k < 3) {
    out[0] = out[1] = out[2] = out[3] = __builtin_nanf("");
    return;
  }
  float a[9];
  const float inv = 1.0f / (float)k;  // `accu /= n`: Eigen 3.2 multiplies by the reciprocal
#pragma unroll
  for (int i = 0; i < 9; ++i) a[i] = accu_in[i] * inv;
  Sym3 C;
  C.a00 = a[0] - a[6] * a[6];
  C.a01 = a[1] - a[6] * a[7];
  C.a02 = a[2] - a[6] * a[8];
  C.a11 = a[3] - a[7] * a[7];
  C.a12 = a[4] - a[7] * a[8];
  C.a22 = a[5] - a[8] * a[8];
  C.a10 = C.a01; C.a20 = C.a02; C.a21 = C.a12;
  float lambda;
  f3 n;
  eigen33_min(C, lambda, n);
  float eig_sum = C.a00 + C.a11 + C.a22;
  float curv = (eig_sum != 0.0f) ? fabsf(lambda / eig_sum) : 0.0f;
  float ax = vpx - px, ay = vpy - py, az = vpz - pz;
  float cos_theta = (ax * n.x + ay * n.y) + az * n.z;
  if (cos_theta < 0.0f) { n.x *= -1.0f; n.y *= -1.0f; n.z *= -1.0f; }
  out[0] = n.x; out[1] = n.y; out[2] = n.z; out[3] = curv;
}

}  // namespace pfx
