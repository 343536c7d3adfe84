// pfx_eigen3.h -- Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d>::compute on the device, the
// operation sequence of oracle/or_common.h selfadjoint_eigen3 (Eigenvalues/SelfAdjointEigenSolver.h,
// Eigenvalues/Tridiagonalization.h 3x3 selector, Jacobi/Jacobi.h makeGivens and
// applyOnTheRight, MathFunctions.h hypot_impl), in double without FMA contraction.
//   ISSKeypoint3D (keypoints.h:177-189): eigenvalues of the scatter matrix;
//   SHOTLocalReferenceFrameEstimation::getLocalRF: eigenvalues and eigenvectors.
#pragma once
#include <hip/hip_runtime.h>

namespace pfx {

__device__ __forceinline__ double hypot_e(double x, double y) {  // internal::hypot_impl
  const double ax = fabs(x), ay = fabs(y);
  const double p = ax > ay ? ax : ay;
  if (p == 0.0) return 0.0;
  const double q = ax > ay ? ay : ax;
  const double qp = q / p;
  return p * sqrt(1.0 + qp * qp);
}

__device__ __forceinline__ void make_givens(double p, double q, double& c, double& s) {
  if (q == 0.0) {
    c = p < 0.0 ? -1.0 : 1.0;
    s = 0.0;
  } else if (p == 0.0) {
    c = 0.0;
    s = q < 0.0 ? 1.0 : -1.0;
  } else if (fabs(p) > fabs(q)) {
    const double t = q / p;
    double u = sqrt(1.0 + t * t);
    if (p < 0.0) u = -u;
    c = 1.0 / u;
    s = -t * c;
  } else {
    const double t = p / q;
    double u = sqrt(1.0 + t * t);
    if (q < 0.0) u = -u;
    s = -1.0 / u;
    c = -t * s;
  }
}

// one implicit QR step on the unreduced block [start, end] of a 3x3 tridiagonal; Q (column k =
// Q[k][.]) gets Q.applyOnTheRight(k, k + 1, rot) = rotation by rot.transpose()
template <bool kVectors>
__device__ __forceinline__ void qr_step(double d[3], double e[2], int start, int end, double Q[3][3]) {
  const double td = (d[end - 1] - d[end]) * 0.5;
  const double ee = e[end - 1];
  double mu = d[end];
  if (td == 0.0) {
    mu -= fabs(ee);
  } else {
    const double e2 = ee * ee;
    const double h = hypot_e(td, ee);
    if (e2 == 0.0)
      mu -= (ee / (td + (td > 0.0 ? 1.0 : -1.0))) * (ee / h);
    else
      mu -= e2 / (td + (td > 0.0 ? h : -h));
  }
  double x = d[start] - mu;
  double z = e[start];
  for (int k = start; k < end; ++k) {
    double c, s;
    make_givens(x, z, c, s);
    const double sdk = s * d[k] + c * e[k];
    const double dkp1 = s * e[k] + c * d[k + 1];
    d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
    d[k + 1] = s * sdk + c * dkp1;
    e[k] = c * sdk - s * dkp1;
    if (k > start) e[k - 1] = c * e[k - 1] - s * z;
    x = e[k];
    if (k < end - 1) {
      z = -s * e[k + 1];
      e[k + 1] = c * e[k + 1];
    }
    if (kVectors && !(c == 1.0 && s == 0.0)) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double xi = Q[k][i], yi = Q[k + 1][i];
        Q[k][i] = c * xi + (-s) * yi;
        Q[k + 1][i] = -(-s) * xi + c * yi;
      }
    }
  }
}

// lower triangle a00, a10, a11, a20, a21, a22 of a symmetric matrix -> ev ascending;
// kVectors: V[k] = eigenvector of ev[k] (Eigen's eigenvectors().col(k))
template <bool kVectors>
__device__ void eigen_selfadjoint3(double a00, double a10, double a11, double a20, double a21, double a22,
                                   double ev[3], double V[3][3]) {
  double scale = fmax(fmax(fmax(fabs(a00), fabs(a10)), fmax(fabs(a11), fabs(a20))), fmax(fabs(a21), fabs(a22)));
  if (scale == 0.0) scale = 1.0;
  a00 /= scale;
  a10 /= scale;
  a11 /= scale;
  a20 /= scale;
  a21 /= scale;
  a22 /= scale;
  double d[3], e[2];
  double Q[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
  d[0] = a00;
  const double v1norm2 = a20 * a20;
  if (v1norm2 == 0.0) {
    d[1] = a11;
    d[2] = a22;
    e[0] = a10;
    e[1] = a21;
  } else {
    const double beta = sqrt(a10 * a10 + v1norm2);
    const double inv_beta = 1.0 / beta;
    const double m01 = a10 * inv_beta;
    const double m02 = a20 * inv_beta;
    const double q = 2.0 * m01 * a21 + m02 * (a22 - a11);
    d[1] = a11 + m02 * q;
    d[2] = a22 - m02 * q;
    e[0] = beta;
    e[1] = a21 - m01 * q;
    if (kVectors) { Q[1][1] = m01; Q[1][2] = m02; Q[2][1] = m02; Q[2][2] = -m01; }
  }
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (fabs(e[i]) <= (fabs(d[i]) + fabs(d[i + 1])) * 1e-12) e[i] = 0.0;
    while (end > 0 && e[end - 1] == 0.0) end--;
    if (end <= 0) break;
    if (++iter > 90) break;
    start = end - 1;
    while (start > 0 && e[start - 1] != 0.0) start--;
    qr_step<kVectors>(d, e, start, end, Q);
  }
  if (iter <= 90) {
    for (int i = 0; i < 2; ++i) {
      int k = i;
      for (int j = i + 1; j < 3; ++j)
        if (d[j] < d[k]) k = j;
      if (k != i) {
        const double t = d[i];
        d[i] = d[k];
        d[k] = t;
        if (kVectors)
          for (int r = 0; r < 3; ++r) { const double u = Q[i][r]; Q[i][r] = Q[k][r]; Q[k][r] = u; }
      }
    }
  }
  ev[0] = d[0] * scale;
  ev[1] = d[1] * scale;
  ev[2] = d[2] * scale;
  if (kVectors)
    for (int k = 0; k < 3; ++k)
      for (int r = 0; r < 3; ++r) V[k][r] = Q[k][r];
}

}  // namespace pfx
