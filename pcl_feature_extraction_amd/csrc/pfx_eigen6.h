// pfx_eigen6.h -- the two small float Eigen 3.2 solvers of HarrisKeypoint6D on the device, lane
// per problem, every index static (fully unrolled loops; runtime bounds become predicates, so
// nothing is spilled to scratch):
//   ColPivHouseholderQR<Matrix3f>::compute(A).solve(b)     (IntensityGradientEstimation)
//   SelfAdjointEigenSolver<Matrix<float,6,6>>::eigenvalues() (HarrisKeypoint6D::responseTomasi)
// The operation sequences (and the SSE2 evaluation orders they assume) are those written out in
// oracle/or_keypoints.cpp (colpiv_solve3, eigen_selfadjoint6f), in float without FMA.
#pragma once
#include <hip/hip_runtime.h>

namespace pfx {

// ---- ColPivHouseholderQR<Matrix3f> (QR/ColPivHouseholderQR.h, Householder/Householder.h) ----
// a: column-major (a[3 c + r])
__device__ __forceinline__ void colpiv_solve3f(const float a[9], const float rhs[3], float xo[3]) {
  float qr[9], hc[3] = {0.f, 0.f, 0.f}, colsq[3];
  int transp[3] = {0, 1, 2};
#pragma unroll
  for (int e = 0; e < 9; ++e) qr[e] = a[e];
#pragma unroll
  for (int c = 0; c < 3; ++c)  // Matrix3f column: fixed size 3, tree-unrolled sum
    colsq[c] = qr[3 * c] * qr[3 * c] + (qr[3 * c + 1] * qr[3 * c + 1] + qr[3 * c + 2] * qr[3 * c + 2]);
  const float eps = 1.1920928955078125e-07f;
  const float maxc = fmaxf(colsq[0], fmaxf(colsq[1], colsq[2]));
  const float thr = maxc * (eps * eps) / 3.0f;
  int nz = 3;
  bool stop = false;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (stop) continue;
    int bi = k;  // maxCoeff(&index): the first maximum
    float best = colsq[k];
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
      if (colsq[j] > best) {
        bi = j;
        best = colsq[j];
      }
    // squared norm of rows k..2 of column bi, left to right
    float bv = 0.f;
#pragma unroll
    for (int j = k; j < 3; ++j) {
      if (j != bi) continue;
      float s = qr[3 * j + k] * qr[3 * j + k];
#pragma unroll
      for (int r = k + 1; r < 3; ++r) s = s + qr[3 * j + r] * qr[3 * j + r];
      bv = s;
      colsq[j] = s;
    }
    if (bv < thr * (float)(3 - k)) {
      nz = k;
#pragma unroll
      for (int j = k; j < 3; ++j) hc[j] = 0.f;
#pragma unroll
      for (int c = k; c < 3; ++c)
#pragma unroll
        for (int r = c + 1; r < 3; ++r) qr[3 * c + r] = 0.f;
      stop = true;
      continue;
    }
    transp[k] = bi;
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
      if (bi == j) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const float t = qr[3 * k + r];
          qr[3 * k + r] = qr[3 * j + r];
          qr[3 * j + r] = t;
        }
        const float t = colsq[k];
        colsq[k] = colsq[j];
        colsq[j] = t;
      }
    const float c0 = qr[3 * k + k];
    float tailsq = 0.f;
    if (k < 2) {
      tailsq = qr[3 * k + k + 1] * qr[3 * k + k + 1];
#pragma unroll
      for (int r = k + 2; r < 3; ++r) tailsq = tailsq + qr[3 * k + r] * qr[3 * k + r];
    }
    float tau, beta;
    if (tailsq == 0.f) {
      tau = 0.f;
      beta = c0;
#pragma unroll
      for (int r = k + 1; r < 3; ++r) qr[3 * k + r] = 0.f;
    } else {
      beta = sqrtf(c0 * c0 + tailsq);
      if (c0 >= 0.f) beta = -beta;
      const float den = c0 - beta;
#pragma unroll
      for (int r = k + 1; r < 3; ++r) qr[3 * k + r] = qr[3 * k + r] / den;
      tau = (beta - c0) / beta;
    }
    qr[3 * k + k] = beta;
    hc[k] = tau;
    if (k < 2) {
#pragma unroll
      for (int c = k + 1; c < 3; ++c) {
        float tmp = qr[3 * k + k + 1] * qr[3 * c + k + 1];
#pragma unroll
        for (int r = k + 2; r < 3; ++r) tmp = tmp + qr[3 * k + r] * qr[3 * c + r];
        tmp = tmp + qr[3 * c + k];
        qr[3 * c + k] = qr[3 * c + k] - tau * tmp;
#pragma unroll
        for (int r = k + 1; r < 3; ++r) qr[3 * c + r] = qr[3 * c + r] - (tau * qr[3 * k + r]) * tmp;
      }
    }
#pragma unroll
    for (int c = k + 1; c < 3; ++c) colsq[c] = colsq[c] - qr[3 * c + k] * qr[3 * c + k];
  }
  if (nz == 0) {
    xo[0] = xo[1] = xo[2] = 0.f;
    return;
  }
  float cv[3] = {rhs[0], rhs[1], rhs[2]};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nz) continue;
    if (k == 2) {
      cv[2] = cv[2] * (1.0f - hc[2]);
      continue;
    }
    float tmp = qr[3 * k + k + 1] * cv[k + 1];
#pragma unroll
    for (int r = k + 2; r < 3; ++r) tmp = tmp + qr[3 * k + r] * cv[r];
    tmp = tmp + cv[k];
    cv[k] = cv[k] - hc[k] * tmp;
#pragma unroll
    for (int r = k + 1; r < 3; ++r) cv[r] = cv[r] - (hc[k] * qr[3 * k + r]) * tmp;
  }
#pragma unroll
  for (int i = 2; i >= 0; --i) {
    if (i >= nz) continue;
    if (cv[i] != 0.f) {
      cv[i] /= qr[3 * i + i];
#pragma unroll
      for (int j = 0; j < i; ++j) cv[j] = cv[j] - cv[i] * qr[3 * i + j];
    }
  }
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nz) continue;
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
      if (transp[k] == j) {
        const int t = perm[k];
        perm[k] = perm[j];
        perm[j] = t;
      }
  }
  xo[0] = xo[1] = xo[2] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= nz) continue;
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (perm[i] == t) xo[t] = cv[i];
  }
}

// ---- SelfAdjointEigenSolver<Matrix<float,6,6>> ---------------------------------------------
__device__ __forceinline__ float sqsum_packet(const float* v, int m) {  // m static after unrolling
  if (m < 4) {
    float s = v[0] * v[0];
#pragma unroll
    for (int i = 1; i < 3; ++i)
      if (i < m) s = s + v[i] * v[i];
    return s;
  }
  const float p0 = v[0] * v[0], p1 = v[1] * v[1], p2 = v[2] * v[2], p3 = v[3] * v[3];
  float s = (p0 + p2) + (p1 + p3);
  if (m > 4) s = s + v[4] * v[4];
  return s;
}

__device__ __forceinline__ float hypot_e32(float x, float y) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float p = fmaxf(ax, ay);
  if (p == 0.f) return 0.f;
  const float q = fminf(ax, ay);
  const float qp = q / p;
  return p * sqrtf(1.0f + qp * qp);
}

__device__ __forceinline__ void make_givens32(float p, float q, float& c, float& s) {
  if (q == 0.f) {
    c = p < 0.f ? -1.f : 1.f;
    s = 0.f;
  } else if (p == 0.f) {
    c = 0.f;
    s = q < 0.f ? 1.f : -1.f;
  } else if (fabsf(p) > fabsf(q)) {
    const float t = q / p;
    float u = sqrtf(1.0f + t * t);
    if (p < 0.f) u = -u;
    c = 1.0f / u;
    s = -t * c;
  } else {
    const float t = p / q;
    float u = sqrtf(1.0f + t * t);
    if (q < 0.f) u = -u;
    s = -1.0f / u;
    c = -t * s;
  }
}

// cv: the 21 upper-triangle sums of responseTomasi (row-major upper = column-major lower);
// returns eigenvalues()[3]
__device__ __forceinline__ float eigen6f_value3(const float cv[21]) {
  float m[36];
  {
    int e = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        if (b < a) {
          m[6 * a + b] = 0.f;
        } else {
          m[6 * a + b] = cv[e];  // column a, row b >= a
          ++e;
        }
      }
  }
  float scale = 0.f;
#pragma unroll
  for (int e = 0; e < 36; ++e) scale = fmaxf(scale, fabsf(m[e]));
  if (scale == 0.f) scale = 1.f;
#pragma unroll
  for (int c = 0; c < 6; ++c)
#pragma unroll
    for (int r = c; r < 6; ++r) m[6 * c + r] = m[6 * c + r] / scale;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int rs = 5 - i;
    float* v = m + 6 * i + i + 1;
    const float c0 = v[0];
    const float tailsq = rs == 1 ? 0.f : sqsum_packet(v + 1, rs - 1);
    float h, beta;
    if (tailsq == 0.f) {
      h = 0.f;
      beta = c0;
#pragma unroll
      for (int r = 1; r < 5; ++r)
        if (r < rs) v[r] = 0.f;
    } else {
      beta = sqrtf(c0 * c0 + tailsq);
      if (c0 >= 0.f) beta = -beta;
      const float den = c0 - beta;
#pragma unroll
      for (int r = 1; r < 5; ++r)
        if (r < rs) v[r] = v[r] / den;
      h = (beta - c0) / beta;
    }
    v[0] = 1.f;
    float res[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float* B = m + 6 * (i + 1) + (i + 1);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j >= rs) continue;
      const float t1 = h * v[j];
      float t2 = 0.f;
      res[j] += B[6 * j + j] * t1;
#pragma unroll
      for (int r = j + 1; r < 5; ++r) {
        if (r >= rs) continue;
        res[r] += B[6 * j + r] * t1;
        t2 += B[6 * j + r] * v[r];
      }
      res[j] += h * t2;
    }
    float dot = res[0] * v[0];
#pragma unroll
    for (int r = 1; r < 5; ++r)
      if (r < rs) dot = dot + res[r] * v[r];
    const float sc = (h * -0.5f) * dot;
#pragma unroll
    for (int r = 0; r < 5; ++r)
      if (r < rs) res[r] = res[r] + sc * v[r];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j >= rs) continue;
      const float a1 = -1.0f * v[j], a2 = -1.0f * res[j];
#pragma unroll
      for (int r = j; r < 5; ++r)
        if (r < rs) B[6 * j + r] = B[6 * j + r] + (a1 * res[r] + a2 * v[r]);
    }
    v[0] = beta;
  }
  float d[6], e[5];
#pragma unroll
  for (int k = 0; k < 6; ++k) d[k] = m[6 * k + k];
#pragma unroll
  for (int k = 0; k < 5; ++k) e[k] = m[6 * k + k + 1];
  auto sel_e = [&](int i) {  // e[i] for a runtime i in [0, 5)
    float v = e[0];
#pragma unroll
    for (int t = 1; t < 5; ++t) v = i == t ? e[t] : v;
    return v;
  };
  auto sel_d = [&](int i) {
    float v = d[0];
#pragma unroll
    for (int t = 1; t < 6; ++t) v = i == t ? d[t] : v;
    return v;
  };
  int end = 5, start = 0, iter = 0;
  const int maxit = 30 * 6;
  while (end > 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i >= start && i < end && fabsf(e[i]) <= (fabsf(d[i]) + fabsf(d[i + 1])) * 1e-5f) e[i] = 0.f;
    while (end > 0 && sel_e(end - 1) == 0.f) end--;
    if (end <= 0) break;
    if (++iter > maxit) break;
    start = end - 1;
    while (start > 0 && sel_e(start - 1) != 0.f) start--;
    const float td = (sel_d(end - 1) - sel_d(end)) * 0.5f;
    const float ee = sel_e(end - 1);
    float mu = sel_d(end);
    if (td == 0.f) {
      mu -= fabsf(ee);
    } else {
      const float e2 = ee * ee;
      const float hh = hypot_e32(td, ee);
      if (e2 == 0.f) mu -= (ee / (td + (td > 0.f ? 1.f : -1.f))) * (ee / hh);
      else mu -= e2 / (td + (td > 0.f ? hh : -hh));
    }
    float x = sel_d(start) - mu, z = sel_e(start);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      if (k < start || k >= end) continue;
      float c, s;
      make_givens32(x, z, c, s);
      const float sdk = s * d[k] + c * e[k];
      const float dkp1 = s * e[k] + c * d[k + 1];
      d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
      d[k + 1] = s * sdk + c * dkp1;
      e[k] = c * sdk - s * dkp1;
      if (k > 0 && k > start) e[k - 1] = c * e[k - 1] - s * z;
      x = e[k];
      if (k < 4 && k < end - 1) {
        z = -s * e[k + 1];
        e[k + 1] = c * e[k + 1];
      }
    }
  }
  if (iter <= maxit) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      int k = i;
      float dk = d[i];
#pragma unroll
      for (int j = i + 1; j < 6; ++j)
        if (d[j] < dk) {
          k = j;
          dk = d[j];
        }
#pragma unroll
      for (int j = i + 1; j < 6; ++j)
        if (k == j) {
          const float t = d[i];
          d[i] = d[j];
          d[j] = t;
        }
    }
  }
  return d[3] * scale;
}

}  // namespace pfx
