// =====================================================================================
//  oracle/or_keypoints.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of the reference's active-list keypoint detectors:
//
//    Keypoints::computeCloudResolution           include/pcl_feature_extraction/keypoints.h:401-428
//    Keypoints::compute, ISS branch               include/pcl_feature_extraction/keypoints.h:177-189
//      -> pcl::ISSKeypoint3D<PointXYZRGB, PointXYZRGB>  (PCL 1.7 keypoints/impl/iss_3d.hpp),
//         salient radius 6 res, non-max radius 4 res, min neighbours 5, gamma21 = gamma32 = 0.975,
//         search::KdTree<PointXYZRGB> (sorted results), no border radius, no normals.
//
//  computeCloudResolution: mean over the points with a finite x of sqrt(d2 of the second
//  nearest neighbour), where the first is the point itself (d2 = 0; a duplicate point gives
//  0 as well).  `sqrt(squaredDistances[1])` takes a float under `using namespace std`
//  (keypoints.h:33), so the term is std::sqrt(float) -- correctly rounded float -- and the sum
//  is a sequential double accumulation in index order, divided by the count.
//
//  ISSKeypoint3D::detectKeypoints (PCL 1.7), per finite point i:
//    getScatterMatrix: N = radiusSearch(i, salient) in FLANN order; if |N| < min_neighbors the
//      matrix stays 0; else cov[a*3+b] += (p_a - c_a) * (p_b - c_b) in double, neighbour order;
//    Eigen::SelfAdjointEigenSolver<Matrix3d>(cov) (Eigen 3.2.0, restated below);
//    e1 >= e2 >= e3; skip (no value) when one is non-finite or e3 < 0;
//    third[i] = e3 when e2/e1 < gamma21 and e3/e2 < gamma32, else 0;
//  then i is a keypoint when third[i] > 0, |radiusSearch(i, non_max)| >= min_neighbors and no
//  neighbour has a larger third value.  Output: the keypoints' cloud indices, ascending.
//
//  Restatement choices (documented in DESIGN.md, unpinned):
//    * skipped points (non-finite or negative eigenvalues) have third = 0.  PCL leaves their
//      prg_mem slot uninitialised (iss_3d.hpp `continue` before the copy) -- undefined;
//    * the reference pushes keypoints from an OpenMP loop under `omp critical` (thread order);
//      the restatement returns them in index order (the single-thread order);
//    * computeCloudResolution skips points with any non-finite coordinate (the reference tests
//      x only and queries the kd-tree with the NaN point otherwise: undefined).
// =====================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "or_common.h"

using orc::i64;
using orc::NeighborGrid;

namespace {

// Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d>: orc::selfadjoint_eigen3 (or_common.h)
using orc::selfadjoint_eigen3;
inline void selfadjoint_eigenvalues3(const double a[9], double ev[3]) { selfadjoint_eigen3(a, ev, 0); }

inline bool finite3(const float* x, const float* y, const float* z, i64 i) {
  return std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i]);
}

// d2 of the second nearest point of the cloud to point i (itself included, FLANN kNN k = 2);
// +inf when the cloud has a single finite point.  Ring search on a grid of cell h.
float second_nn_d2(const NeighborGrid& g, const float* x, const float* y, const float* z, i64 i) {
  const float qx = x[i], qy = y[i], qz = z[i];
  float b1 = INFINITY, b2 = INFINITY;
  auto visit = [&](i64 p) {
    const float dx = qx - x[p], dy = qy - y[p], dz = qz - z[p];
    const float dd = ((0.0f + dx * dx) + dy * dy) + dz * dz;  // flann::L2_Simple
    if (dd < b1) {
      b2 = b1;
      b1 = dd;
    } else if (dd < b2) {
      b2 = dd;
    }
  };
  i64 cx, cy, cz;
  g.cellOf(qx, qy, qz, cx, cy, cz);
  for (i64 R = 1; R <= 4; ++R) {
    b1 = b2 = INFINITY;
    for (i64 ix = cx - R; ix <= cx + R; ++ix)
      for (i64 iy = cy - R; iy <= cy + R; ++iy)
        for (i64 iz = cz - R; iz <= cz + R; ++iz) {
          if (ix < -NeighborGrid::OFF + 1 || iy < -NeighborGrid::OFF + 1 || iz < -NeighborGrid::OFF + 1 ||
              ix >= NeighborGrid::OFF || iy >= NeighborGrid::OFF || iz >= NeighborGrid::OFF)
            continue;
          const uint64_t k = NeighborGrid::pack(ix, iy, iz);
          std::vector<uint64_t>::const_iterator it = std::lower_bound(g.keys.begin(), g.keys.end(), k);
          if (it == g.keys.end() || *it != k) continue;
          const size_t c = (size_t)(it - g.keys.begin());
          for (i64 s = g.start[c]; s < g.end[c]; ++s) visit(g.order[(size_t)s]);
        }
    // everything outside the block is at least R cells (R * cell) away
    const double reach = (double)R * g.cell;
    if ((double)b2 < reach * reach * (1.0 - 1e-6)) return b2;
  }
  b1 = b2 = INFINITY;  // isolated point: every indexed point
  for (size_t s = 0; s < g.order.size(); ++s) visit(g.order[s]);
  return b2;
}

}  // namespace

extern "C" {

// Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d> eigenvalues (ascending) of row-major symmetric
// 3x3 matrices, for the tests of the restatement itself.
int orc_eigen_selfadjoint3(const double* a, i64 n, double* ev) {
  for (i64 i = 0; i < n; ++i) selfadjoint_eigenvalues3(a + 9 * i, ev + 3 * i);
  return 0;
}

// the same with eigenvectors: vec[9 i + 3 k + r] = component r of the eigenvector of ev[3 i + k]
int orc_eigen_selfadjoint3_vectors(const double* a, i64 n, double* ev, double* vec) {
  for (i64 i = 0; i < n; ++i) selfadjoint_eigen3(a + 9 * i, ev + 3 * i, (double(*)[3])(vec + 9 * i));
  return 0;
}

// Keypoints::computeCloudResolution (keypoints.h:401-428).  `terms` (nullable, n floats): the
// per-point sqrt term, NaN where the point does not contribute.
int orc_cloud_resolution(const float* x, const float* y, const float* z, i64 n, double* out, float* terms,
                         int threads) {
  *out = 0.0;
  if (n <= 0) return 0;
  // cell: the mean spacing of the bounding volume (any cell size gives the same answer)
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  i64 nf = 0;
  for (i64 i = 0; i < n; ++i) {
    if (!finite3(x, y, z, i)) continue;
    const float p[3] = {x[i], y[i], z[i]};
    for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], (double)p[d]); hi[d] = std::max(hi[d], (double)p[d]); }
    ++nf;
  }
  std::vector<float> t((size_t)n, NAN);
  if (nf >= 2) {
    double ext = 0.0, vol = 1.0;
    for (int d = 0; d < 3; ++d) ext = std::max(ext, hi[d] - lo[d]);
    for (int d = 0; d < 3; ++d) vol *= std::max(hi[d] - lo[d], ext * 1e-3);
    double h = ext > 0.0 ? 0.5 * std::cbrt(vol / (double)nf) : 1.0;
    NeighborGrid g;
    g.build(x, y, z, n, h);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
#endif
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x, y, z, i)) continue;
      t[(size_t)i] = std::sqrt(second_nn_d2(g, x, y, z, i));  // std::sqrt(float)
    }
  }
  double resolution = 0.0;
  i64 count = 0;
  for (i64 i = 0; i < n; ++i) {
    if (std::isnan(t[(size_t)i])) continue;
    resolution += t[(size_t)i];
    ++count;
  }
  if (count != 0) resolution /= count;
  *out = resolution;
  if (terms)
    for (i64 i = 0; i < n; ++i) terms[i] = t[(size_t)i];
  return 0;
}

// ISSKeypoint3D::compute as configured at keypoints.h:177-189.  idx: keypoint cloud indices
// (ascending), third (nullable, n doubles): the per-point third eigenvalue map.
// Returns 1 for parameters PCL's initCompute rejects (no output), 3 when cap is too small.
int orc_iss_keypoints(const float* x, const float* y, const float* z, i64 n, double salient, double non_max,
                      int min_neighbors, double gamma21, double gamma32, int32_t* idx, i64 cap, i64* n_out,
                      double* third_out, int threads) {
  *n_out = 0;
  if (salient <= 0.0 || non_max <= 0.0 || gamma21 <= 0.0 || gamma32 <= 0.0 || min_neighbors <= 0) return 1;
  if (n <= 0) return 0;
  std::vector<double> third((size_t)n, 0.0);
  std::vector<char> is_max((size_t)n, 0);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  {
    NeighborGrid gs;
    gs.build(x, y, z, n, salient);
#pragma omp parallel
    {
      std::vector<int> nb;
      std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
      for (i64 i = 0; i < n; ++i) {
        if (!finite3(x, y, z, i)) continue;
        gs.radius(x[i], y[i], z[i], salient, nb, dd);
        double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        if ((int)nb.size() >= min_neighbors) {
          const double c[3] = {x[i], y[i], z[i]};
          for (size_t m = 0; m < nb.size(); ++m) {
            const double p[3] = {x[nb[m]], y[nb[m]], z[nb[m]]};
            for (int a = 0; a < 3; ++a)
              for (int b = 0; b < 3; ++b) cov[a * 3 + b] += (p[a] - c[a]) * (p[b] - c[b]);
          }
        }
        double ev[3];
        selfadjoint_eigenvalues3(cov, ev);
        const double e1 = ev[2], e2 = ev[1], e3 = ev[0];
        if (!std::isfinite(e1) || !std::isfinite(e2) || !std::isfinite(e3) || e3 < 0.0) continue;
        if (e2 / e1 < gamma21 && e3 / e2 < gamma32) third[(size_t)i] = e3;
      }
    }
  }
  {
    NeighborGrid gn;
    gn.build(x, y, z, n, non_max);
#pragma omp parallel
    {
      std::vector<int> nb;
      std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
      for (i64 i = 0; i < n; ++i) {
        if (!(third[(size_t)i] > 0.0) || !finite3(x, y, z, i)) continue;
        gn.radius(x[i], y[i], z[i], non_max, nb, dd);
        if ((int)nb.size() < min_neighbors) continue;
        bool m = true;
        for (size_t j = 0; j < nb.size(); ++j)
          if (third[(size_t)i] < third[(size_t)nb[j]]) m = false;
        is_max[(size_t)i] = m;
      }
    }
  }
  i64 k = 0;
  for (i64 i = 0; i < n; ++i)
    if (is_max[(size_t)i]) {
      if (k < cap) idx[k] = (int32_t)i;
      ++k;
    }
  *n_out = k;
  if (third_out)
    for (i64 i = 0; i < n; ++i) third_out[i] = third[(size_t)i];
  return k > cap ? 3 : 0;
}

}  // extern "C"

// =====================================================================================
//  Harris3D: Keypoints::compute HARRIS_3D branch, keypoints.h:150-162
//    HarrisKeypoint3D<PointXYZRGB, PointXYZI> (PCL 1.7 keypoints/impl/harris_3d.hpp), method
//    HARRIS, radius 0.01 (constructor default), setNonMaxSupression(true), setThreshold(1e-6),
//    refine (default true); then Keypoints::getKeypointsCloud (keypoints.h:365-395) snaps each
//    refined corner to its nearest cloud point when that is closer than d2 < 0.0001.
//  Per finite point i (radius r):
//    normals: NormalEstimation at r, viewpoint 0 (the orc_normals restatement);
//    covariance (calculateNormalCovar, SSE branch): over the neighbours with a finite normal,
//      sequential float sums of nx*nx, ny*nx, nz*nx, ny*ny, nz*ny, nz*nz, each divided by
//      float(count) (0 matrix without such neighbours);
//    response: trace = (c00 + c11) + c22; when trace != 0,
//      det = c00*c11*c22 + 2*c01*c02*c12 - c02*c02*c11 - c01*c01*c22 - c12*c12*c00 (left to right)
//      intensity = 0.04f + det - 0.04f * trace * trace, else 0;
//  non-maximum suppression: finite intensity >= threshold and no neighbour within r larger;
//  refineCorners: up to 10 times, over the corner's current r-ball (finite normals),
//    NNT += n n^T, NNTp += (n n^T) p (Matrix3f * Vector3f: ((m0 p0 + m1 p1) + m2 p2)),
//    invert3x3SymMatrix (common/eigen.hpp: adjugate / det, det != 0), corner = NNTInv * NNTp,
//    until |corner - previous|^2 <= 1e-6 (a Vector3f squaredNorm: dx^2 + (dy^2 + dz^2)).
//  Restatement choices (unpinned): neighbour order = FLANN's sorted (d2, index) order -- PCL's
//  NormalEstimation and HarrisKeypoint3D search an unsorted search::KdTree(false), i.e. the
//  kd-tree traversal order, which changes float sums in the last bits; corners in index order
//  (PCL: omp critical order); nearest-point ties -> lowest index (FLANN: first visited).
// =====================================================================================
extern "C" int orc_normals(const float* x, const float* y, const float* z, i64 n, double r, float vpx, float vpy,
                           float vpz, float* nx, float* ny, float* nz, float* curv, int nthreads);

namespace {

struct M3 { float m[9]; };  // column-major, as Eigen's Matrix3f coeff(k)

// pcl::invert3x3SymMatrix (common/impl/eigen.hpp)
float invert3x3Sym(const M3& a, M3& inv) {
  const float* c = a.m;
  const float fd_ee = c[4] * c[8] - c[7] * c[5];
  const float ce_bf = c[2] * c[5] - c[1] * c[8];
  const float be_cd = c[1] * c[5] - c[2] * c[4];
  const float det = c[0] * fd_ee + c[1] * ce_bf + c[2] * be_cd;
  if (det != 0.0f) {
    inv.m[0] = fd_ee;
    inv.m[1] = inv.m[3] = ce_bf;
    inv.m[2] = inv.m[6] = be_cd;
    inv.m[4] = c[0] * c[8] - c[2] * c[2];
    inv.m[5] = inv.m[7] = c[1] * c[2] - c[0] * c[5];
    inv.m[8] = c[0] * c[4] - c[1] * c[1];
    const float rdet = 1.0f / det;  // `inverse /= det`: Eigen 3.2 multiplies by the reciprocal
    for (int k = 0; k < 9; ++k) inv.m[k] *= rdet;
  }
  return det;
}

// Matrix3f (column-major) * Vector3f, Eigen's coefficient-based product order
inline void mat_vec(const M3& a, const float v[3], float out[3]) {
  for (int r = 0; r < 3; ++r) out[r] = (a.m[r] * v[0] + a.m[3 + r] * v[1]) + a.m[6 + r] * v[2];
}

float harris_response(const std::vector<int>& nb, const float* nx, const float* ny, const float* nz) {
  float sxx = 0.f, sxy = 0.f, sxz = 0.f, syy = 0.f, syz = 0.f, szz = 0.f;
  unsigned count = 0;
  for (size_t m = 0; m < nb.size(); ++m) {
    const int j = nb[m];
    if (!std::isfinite(nx[j])) continue;
    sxx += nx[j] * nx[j];
    sxy += ny[j] * nx[j];
    sxz += nz[j] * nx[j];
    syy += ny[j] * ny[j];
    syz += nz[j] * ny[j];
    szz += nz[j] * nz[j];
    ++count;
  }
  float c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (count > 0) {
    const float f = (float)count;
    c[0] = sxx / f; c[1] = sxy / f; c[2] = sxz / f;
    c[5] = syy / f; c[6] = syz / f; c[7] = szz / f;
  }
  const float trace = c[0] + c[5] + c[7];
  if (trace == 0.0f) return 0.0f;
  const float det = c[0] * c[5] * c[7] + 2.0f * c[1] * c[2] * c[6] - c[2] * c[2] * c[5] - c[1] * c[1] * c[7] -
                    c[6] * c[6] * c[0];
  return 0.04f + det - 0.04f * trace * trace;
}

int harris_finish(const float* x, const float* y, const float* z, i64 n, double radius, float threshold, int refine,
                  const NeighborGrid& g, const std::vector<float>& nx, const std::vector<float>& ny,
                  const std::vector<float>& nz, const std::vector<float>& resp, int32_t* idx, i64 cap, i64* n_out,
                  i64* n_corners, float* resp_out, float* corners_out);

}  // namespace

extern "C" {

// resp (nullable, n), corners (nullable, 3 * cap floats: refined xyz in corner order),
// idx[0..cap): snapped cloud indices (getKeypointsCloud), *n_out their number, *n_corners the
// number of corners.  Returns 3 when cap is too small.
int orc_harris3d(const float* x, const float* y, const float* z, i64 n, double radius, float threshold, int refine,
                 int32_t* idx, i64 cap, i64* n_out, i64* n_corners, float* resp_out, float* corners_out,
                 int threads) {
  *n_out = 0;
  *n_corners = 0;
  if (n <= 0) return 0;
  std::vector<float> nx((size_t)n), ny((size_t)n), nz((size_t)n), cv((size_t)n), resp((size_t)n, 0.0f);
  orc_normals(x, y, z, n, radius, 0.f, 0.f, 0.f, nx.data(), ny.data(), nz.data(), cv.data(), threads);
  NeighborGrid g;
  g.build(x, y, z, n, radius);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x, y, z, i)) continue;
      g.radius(x[i], y[i], z[i], radius, nb, dd);
      resp[(size_t)i] = harris_response(nb, nx.data(), ny.data(), nz.data());
    }
  }
  return harris_finish(x, y, z, n, radius, threshold, refine, g, nx, ny, nz, resp, idx, cap, n_out, n_corners,
                       resp_out, corners_out);
}

}  // extern "C"

namespace {

// HarrisKeypoint3D/6D::detectKeypoints after the response: non-maximum suppression, refineCorners
// (harris_3d.hpp / harris_6d.hpp: the same loop), then Keypoints::getKeypointsCloud
int harris_finish(const float* x, const float* y, const float* z, i64 n, double radius, float threshold, int refine,
                  const NeighborGrid& g, const std::vector<float>& nx, const std::vector<float>& ny,
                  const std::vector<float>& nz, const std::vector<float>& resp, int32_t* idx, i64 cap, i64* n_out,
                  i64* n_corners, float* resp_out, float* corners_out) {
  std::vector<char> is_max((size_t)n, 0);
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 i = 0; i < n; ++i) {
      const float v = resp[(size_t)i];
      if (!finite3(x, y, z, i) || !std::isfinite(v) || v < threshold) continue;
      g.radius(x[i], y[i], z[i], radius, nb, dd);
      bool m = true;
      for (size_t k = 0; k < nb.size() && m; ++k)
        if (v < resp[(size_t)nb[k]]) m = false;
      is_max[(size_t)i] = m;
    }
  }
  std::vector<i64> corner_of;
  for (i64 i = 0; i < n; ++i)
    if (is_max[(size_t)i]) corner_of.push_back(i);
  const i64 nc = (i64)corner_of.size();
  std::vector<float> cx((size_t)nc), cy((size_t)nc), cz((size_t)nc);
  for (i64 c = 0; c < nc; ++c) {
    cx[(size_t)c] = x[corner_of[(size_t)c]];
    cy[(size_t)c] = y[corner_of[(size_t)c]];
    cz[(size_t)c] = z[corner_of[(size_t)c]];
  }
  if (refine) {
#pragma omp parallel
    {
      std::vector<int> nb;
      std::vector<float> dd;
#pragma omp for schedule(dynamic, 16)
      for (i64 c = 0; c < nc; ++c) {
        float px = cx[(size_t)c], py = cy[(size_t)c], pz = cz[(size_t)c];
        unsigned iterations = 0;
        float diff;
        do {
          M3 NNT, inv;
          float NNTp[3] = {0.f, 0.f, 0.f};
          for (int k = 0; k < 9; ++k) NNT.m[k] = 0.f;
          const float ox = px, oy = py, oz = pz;
          g.radius(px, py, pz, radius, nb, dd);
          for (size_t k = 0; k < nb.size(); ++k) {
            const int j = nb[k];
            if (!std::isfinite(nx[j])) continue;
            const float nv[3] = {nx[j], ny[j], nz[j]};
            M3 nnT;
            for (int col = 0; col < 3; ++col)
              for (int row = 0; row < 3; ++row) nnT.m[3 * col + row] = nv[row] * nv[col];
            for (int e = 0; e < 9; ++e) NNT.m[e] += nnT.m[e];
            const float p[3] = {x[j], y[j], z[j]};
            float t[3];
            mat_vec(nnT, p, t);
            for (int e = 0; e < 3; ++e) NNTp[e] += t[e];
          }
          if (invert3x3Sym(NNT, inv) != 0.0f) {
            float q[3];
            mat_vec(inv, NNTp, q);
            px = q[0]; py = q[1]; pz = q[2];
          }
          const float dx = px - ox, dy = py - oy, dz = pz - oz;
          diff = dx * dx + (dy * dy + dz * dz);  // (Map - Map).squaredNorm (): Redux.h x + (y + z)
        } while (diff > 1e-6 && ++iterations < 10);
        cx[(size_t)c] = px; cy[(size_t)c] = py; cz[(size_t)c] = pz;
      }
    }
  }
  // getKeypointsCloud: nearest cloud point of each corner, kept when d2 < 0.0001
  std::vector<int32_t> snap((size_t)nc, -1);
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 64)
    for (i64 c = 0; c < nc; ++c) {
      const float px = cx[(size_t)c], py = cy[(size_t)c], pz = cz[(size_t)c];
      if (!std::isfinite(px) || !std::isfinite(py) || !std::isfinite(pz)) continue;
      g.radius(px, py, pz, radius * 1.00001, nb, dd);  // (d2, index) order: nb[0] is the nearest
      if (!nb.empty() && (double)dd[0] < 0.0001) snap[(size_t)c] = nb[0];
    }
  }
  i64 k = 0;
  for (i64 c = 0; c < nc; ++c)
    if (snap[(size_t)c] >= 0) {
      if (k < cap) idx[k] = snap[(size_t)c];
      ++k;
    }
  *n_out = k;
  *n_corners = nc;
  if (resp_out)
    for (i64 i = 0; i < n; ++i) resp_out[i] = resp[(size_t)i];
  if (corners_out)
    for (i64 c = 0; c < nc && c < cap; ++c) {
      corners_out[3 * c] = cx[(size_t)c];
      corners_out[3 * c + 1] = cy[(size_t)c];
      corners_out[3 * c + 2] = cz[(size_t)c];
    }
  return (k > cap || nc > cap) ? 3 : 0;
}

}  // namespace

// =====================================================================================
//  Harris6D: Keypoints::compute HARRIS_6D branch, keypoints.h:164-176
//    HarrisKeypoint6D<PointXYZRGB, PointXYZI> (PCL 1.7 keypoints/impl/harris_6d.hpp): radius
//    0.01 (constructor default), setNonMaxSupression(true), setThreshold(1e-6), refine (default
//    true); then Keypoints::getKeypointsCloud (keypoints.h:365-395) as for Harris3D.
//  detectKeypoints:
//    normals: NormalEstimation<PointXYZRGB, Normal> at r (orc_normals, viewpoint 0);
//    IntensityGradientEstimation<PointXYZRGB, Normal, IntensityGradient> at r
//      (features/impl/intensity_gradient.hpp) with IntensityFieldAccessor<PointXYZRGB>
//      (common/intensity.h): I(p) = float(299 r + 587 g + 114 b) * 0.001f.  Per point, over its
//      neighbours N in FLANN order: centroid = sum of xyz (Vector3f +=) then `/= float(|N|)`
//      (Eigen 3.2: * (1/|N|)); mean = sum of I (float) / float(|N|);
//      computePointIntensityGradient(centroid, mean, normal): |N| < 3 -> NaN; over N:
//        p -= centroid; demean(p, mean) writes I(p) - mean back into the colour
//        (r = u8(I' * 3.34448160535f), g = u8(I' * 1.70357751278f), b = u8(I' * 8.77192982456f),
//        u8 = the low byte of cvttss2si, gcc's x86-64 code for static_cast<uint8_t>(float)),
//        then A += (p p^T) upper, b += p * I(p) with the re-read I;
//        x = A.colPivHouseholderQr().solve(b) (restated below); gradient = (I3 - n n^T) x;
//    normalisation: len = |g|^2 (float); len > 200 -> g *= float(1.0 / sqrt(double(len)));
//    responseTomasi: per finite point, over N with a finite normal_x and finite gradient[0], the
//      21 float sums of v v^T with v = (nx, ny, nz, gx, gy, gz) (no normalisation); intensity =
//      eigenvalues()[3] of SelfAdjointEigenSolver<Matrix<float,6,6>> (restated below); 0 for a
//      non-finite point;
//    non-maximum suppression, refineCorners and the snap: harris_finish (as Harris3D).
//  Eigen 3.2 evaluation orders (SSE2 build): a fixed-size non-vectorisable sum (Matrix3f column)
//  is tree-unrolled (Redux.h redux_novec_unroller: x0 + (x1 + x2)); a dynamic-size sum is left
//  to right unless its operand has packet access (Matrix<float,6,6> blocks), where the first 4*j
//  terms go through the 4-wide SSE predux ((t0 + t2) + (t1 + t3)) and the rest follow in order;
//  SelfadjointMatrixVector.h takes its scalar path below 8 rows; `v / s` divides, `v /= s`
//  multiplies by 1/s except TriangularView::operator/= (= m_matrix / s, divides).
//  Restatement choices (unpinned): FLANN's sorted order (PCL: unsorted kd-trees, as Harris3D);
//  corners in index order (PCL: omp critical); sqrt(float) as glibc's double sqrt (GCC 4.8's
//  <cmath> has no global float overload); NaN responses are not corners.
// =====================================================================================
namespace {

inline float h6_intensity(uint32_t rgb) {
  const int r = (int)((rgb >> 16) & 255u), g = (int)((rgb >> 8) & 255u), b = (int)(rgb & 255u);
  return (float)(299 * r + 587 * g + 114 * b) * 0.001f;
}
// static_cast<uint8_t>(float) as x86-64 gcc emits it: cvttss2si (truncation, INT_MIN when out
// of range or NaN), low byte
inline int h6_u8(float v) {
  const int32_t i = (v > -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : INT32_MIN;
  return i & 255;
}
// IntensityFieldAccessor<PointXYZRGB>::demean followed by operator()
inline float h6_demeaned(uint32_t rgb, float mean) {
  const float iv = h6_intensity(rgb) - mean;
  const int r = h6_u8(iv * 3.34448160535f), g = h6_u8(iv * 1.70357751278f), b = h6_u8(iv * 8.77192982456f);
  return (float)(299 * r + 587 * g + 114 * b) * 0.001f;
}

// Eigen 3.2 ColPivHouseholderQR<Matrix3f>::compute(A).solve(rhs) (QR/ColPivHouseholderQR.h,
// Householder/Householder.h).  a: column-major (a[3 c + r]).
void colpiv_solve3(const float a[9], const float rhs[3], float x[3]) {
  float qr[9], hc[3] = {0.f, 0.f, 0.f}, colsq[3];
  int transp[3] = {0, 1, 2};
  for (int e = 0; e < 9; ++e) qr[e] = a[e];
  for (int c = 0; c < 3; ++c)  // Matrix3f column: fixed size 3, tree-unrolled
    colsq[c] = qr[3 * c] * qr[3 * c] + (qr[3 * c + 1] * qr[3 * c + 1] + qr[3 * c + 2] * qr[3 * c + 2]);
  const float eps = std::numeric_limits<float>::epsilon();
  const float maxc = std::max(colsq[0], std::max(colsq[1], colsq[2]));
  const float thr = maxc * (eps * eps) / 3.0f;
  int nz = 3;
  for (int k = 0; k < 3; ++k) {
    int bi = k;
    for (int j = k + 1; j < 3; ++j)
      if (colsq[j] > colsq[bi]) bi = j;  // maxCoeff(&index): first maximum
    float bv = qr[3 * bi + k] * qr[3 * bi + k];  // tail(rows - k) of a column: left to right
    for (int r = k + 1; r < 3; ++r) bv = bv + qr[3 * bi + r] * qr[3 * bi + r];
    colsq[bi] = bv;
    if (bv < thr * (float)(3 - k)) {
      nz = k;
      for (int j = k; j < 3; ++j) hc[j] = 0.f;
      for (int c = k; c < 3; ++c)
        for (int r = c + 1; r < 3; ++r) qr[3 * c + r] = 0.f;
      break;
    }
    transp[k] = bi;
    if (k != bi) {
      for (int r = 0; r < 3; ++r) std::swap(qr[3 * k + r], qr[3 * bi + r]);
      std::swap(colsq[k], colsq[bi]);
    }
    // makeHouseholderInPlace on qr(k..2, k)
    const float c0 = qr[3 * k + k];
    float tailsq = 0.f;
    if (k < 2) {
      tailsq = qr[3 * k + k + 1] * qr[3 * k + k + 1];
      for (int r = k + 2; r < 3; ++r) tailsq = tailsq + qr[3 * k + r] * qr[3 * k + r];
    }
    float tau, beta;
    if (tailsq == 0.f) {
      tau = 0.f;
      beta = c0;
      for (int r = k + 1; r < 3; ++r) qr[3 * k + r] = 0.f;
    } else {
      beta = std::sqrt(c0 * c0 + tailsq);
      if (c0 >= 0.f) beta = -beta;
      const float den = c0 - beta;
      for (int r = k + 1; r < 3; ++r) qr[3 * k + r] = qr[3 * k + r] / den;
      tau = (beta - c0) / beta;
    }
    qr[3 * k + k] = beta;
    hc[k] = tau;
    // applyHouseholderOnTheLeft(essential = qr(k+1..2, k), tau) on qr(k..2, k+1..2)
    for (int c = k + 1; c < 3; ++c) {
      if (k == 2) break;
      float tmp = qr[3 * k + k + 1] * qr[3 * c + k + 1];
      for (int r = k + 2; r < 3; ++r) tmp = tmp + qr[3 * k + r] * qr[3 * c + r];
      tmp = tmp + qr[3 * c + k];
      qr[3 * c + k] = qr[3 * c + k] - tau * tmp;
      for (int r = k + 1; r < 3; ++r) qr[3 * c + r] = qr[3 * c + r] - (tau * qr[3 * k + r]) * tmp;
    }
    for (int c = k + 1; c < 3; ++c) colsq[c] = colsq[c] - qr[3 * c + k] * qr[3 * c + k];
  }
  if (nz == 0) {
    x[0] = x[1] = x[2] = 0.f;
    return;
  }
  // c = Q^T rhs: H_0 first, rows k..2 (a one-row block is scaled by 1 - tau)
  float cv[3] = {rhs[0], rhs[1], rhs[2]};
  for (int k = 0; k < nz; ++k) {
    if (k == 2) {
      cv[2] = cv[2] * (1.0f - hc[2]);
      continue;
    }
    float tmp = qr[3 * k + k + 1] * cv[k + 1];
    for (int r = k + 2; r < 3; ++r) tmp = tmp + qr[3 * k + r] * cv[r];
    tmp = tmp + cv[k];
    cv[k] = cv[k] - hc[k] * tmp;
    for (int r = k + 1; r < 3; ++r) cv[r] = cv[r] - (hc[k] * qr[3 * k + r]) * tmp;
  }
  // R(0..nz) upper-triangular solve in place (triangular_solve_vector, column-major Upper)
  for (int i = nz - 1; i >= 0; --i) {
    if (cv[i] != 0.f) {
      cv[i] /= qr[3 * i + i];
      for (int j = 0; j < i; ++j) cv[j] = cv[j] - cv[i] * qr[3 * i + j];
    }
  }
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < nz; ++k) std::swap(perm[k], perm[transp[k]]);
  x[0] = x[1] = x[2] = 0.f;
  for (int i = 0; i < nz; ++i) x[perm[i]] = cv[i];
}

// sum of the squares of v[0..m) as Eigen 3.2 reduces a dynamic-size block of a packet-capable
// matrix: the first 4 j terms through the SSE predux, the rest in order (m < 4: in order)
inline float h6_sqsum(const float* v, int m) {
  if (m < 4) {
    float s = v[0] * v[0];
    for (int i = 1; i < m; ++i) s = s + v[i] * v[i];
    return s;
  }
  float p0 = v[0] * v[0], p1 = v[1] * v[1], p2 = v[2] * v[2], p3 = v[3] * v[3];
  int i = 4;
  if (m >= 8) {
    float q0 = v[4] * v[4], q1 = v[5] * v[5], q2 = v[6] * v[6], q3 = v[7] * v[7];
    p0 = p0 + q0; p1 = p1 + q1; p2 = p2 + q2; p3 = p3 + q3;
    i = 8;
  }
  float s = (p0 + p2) + (p1 + p3);
  for (; i < m; ++i) s = s + v[i] * v[i];
  return s;
}

inline float h6_hypot(float x, float y) {  // internal::hypot_impl<float>
  const float ax = std::fabs(x), ay = std::fabs(y);
  const float p = std::max(ax, ay);
  if (p == 0.f) return 0.f;
  const float q = std::min(ax, ay);
  const float qp = q / p;
  return p * std::sqrt(1.0f + qp * qp);
}

inline void h6_givens(float p, float q, float& c, float& s) {  // JacobiRotation::makeGivens (real)
  if (q == 0.f) {
    c = p < 0.f ? -1.f : 1.f;
    s = 0.f;
  } else if (p == 0.f) {
    c = 0.f;
    s = q < 0.f ? 1.f : -1.f;
  } else if (std::fabs(p) > std::fabs(q)) {
    const float t = q / p;
    float u = std::sqrt(1.0f + t * t);
    if (p < 0.f) u = -u;
    c = 1.0f / u;
    s = -t * c;
  } else {
    const float t = p / q;
    float u = std::sqrt(1.0f + t * t);
    if (q < 0.f) u = -u;
    s = -1.0f / u;
    c = -t * s;
  }
}

// Eigen 3.2 SelfAdjointEigenSolver<Matrix<float,6,6>>::compute(A).eigenvalues() (A: lower
// triangle read, column-major m[6 c + r]); returns false when the QR iteration does not converge
// (then the values are unsorted, as Eigen leaves them)
bool eigen_selfadjoint6f(const float A[36], float ev[6]) {
  const int n = 6;
  float m[36];
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < n; ++r) m[6 * c + r] = r >= c ? A[6 * c + r] : 0.f;
  float scale = 0.f;
  for (int e = 0; e < 36; ++e) scale = std::max(scale, std::fabs(m[e]));  // cwiseAbs().maxCoeff()
  if (scale == 0.f) scale = 1.f;
  for (int c = 0; c < n; ++c)
    for (int r = c; r < n; ++r) m[6 * c + r] = m[6 * c + r] / scale;  // TriangularView /= : divides
  // Tridiagonalization.h tridiagonalization_inplace (generic selector), lower triangle
  float hco[5];
  for (int i = 0; i < n - 1; ++i) {
    const int rs = n - i - 1;  // remaining size
    float* v = m + 6 * i + i + 1;  // column i, rows i+1..n-1
    // makeHouseholderInPlace(h, beta): c0 = v[0], tail = v[1..rs)
    const float c0 = v[0];
    const float tailsq = rs == 1 ? 0.f : h6_sqsum(v + 1, rs - 1);
    float h, beta;
    if (tailsq == 0.f) {
      h = 0.f;
      beta = c0;
      for (int r = 1; r < rs; ++r) v[r] = 0.f;
    } else {
      beta = std::sqrt(c0 * c0 + tailsq);
      if (c0 >= 0.f) beta = -beta;
      const float den = c0 - beta;
      for (int r = 1; r < rs; ++r) v[r] = v[r] / den;
      h = (beta - c0) / beta;
    }
    v[0] = 1.f;
    // hco(i..) = h * (B v), B = bottom-right rs x rs lower view (selfadjoint_matrix_vector_product,
    // scalar path, alpha = h extracted from the rhs expression, rhs = v)
    float res[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    const float* B = m + 6 * (i + 1) + (i + 1);  // B(r, c) = B[6 c + r]
    for (int j = 0; j < rs; ++j) {
      const float t1 = h * v[j];
      float t2 = 0.f;
      res[j] += B[6 * j + j] * t1;
      for (int r = j + 1; r < rs; ++r) {
        res[r] += B[6 * j + r] * t1;
        t2 += B[6 * j + r] * v[r];
      }
      res[j] += h * t2;
    }
    // += (h * -0.5 * (hco . v)) v   (dot: CwiseBinaryOp of a 5-vector block, no packets: in order)
    float dot = res[0] * v[0];
    for (int r = 1; r < rs; ++r) dot = dot + res[r] * v[r];
    const float sc = (h * -0.5f) * dot;
    for (int r = 0; r < rs; ++r) res[r] = res[r] + sc * v[r];
    // rankUpdate(v, res, -1): column j of the lower view: B(j.., j) += (-v_j) res(j..) + (-res_j) v(j..)
    float* Bw = m + 6 * (i + 1) + (i + 1);
    for (int j = 0; j < rs; ++j) {
      const float a1 = -1.0f * v[j], a2 = -1.0f * res[j];
      for (int r = j; r < rs; ++r) Bw[6 * j + r] = Bw[6 * j + r] + (a1 * res[r] + a2 * v[r]);
    }
    v[0] = beta;
    hco[i] = h;
  }
  float d[6], e[5];
  for (int k = 0; k < n; ++k) d[k] = m[6 * k + k];
  for (int k = 0; k < n - 1; ++k) e[k] = m[6 * k + k + 1];
  (void)hco;
  int end = n - 1, start = 0, iter = 0;
  const int maxit = 30 * n;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (std::fabs(e[i]) <= (std::fabs(d[i]) + std::fabs(d[i + 1])) * 1e-5f) e[i] = 0.f;  // isMuchSmallerThan
    while (end > 0 && e[end - 1] == 0.f) end--;
    if (end <= 0) break;
    if (++iter > maxit) break;
    start = end - 1;
    while (start > 0 && e[start - 1] != 0.f) start--;
    // tridiagonal_qr_step
    const float td = (d[end - 1] - d[end]) * 0.5f;
    const float ee = e[end - 1];
    float mu = d[end];
    if (td == 0.f) {
      mu -= std::fabs(ee);
    } else {
      const float e2 = ee * ee;
      const float hh = h6_hypot(td, ee);
      if (e2 == 0.f) mu -= (ee / (td + (td > 0.f ? 1.f : -1.f))) * (ee / hh);
      else mu -= e2 / (td + (td > 0.f ? hh : -hh));
    }
    float x = d[start] - mu, z = e[start];
    for (int k = start; k < end; ++k) {
      float c, s;
      h6_givens(x, z, c, s);
      const float sdk = s * d[k] + c * e[k];
      const float dkp1 = s * e[k] + c * d[k + 1];
      d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
      d[k + 1] = s * sdk + c * dkp1;
      e[k] = c * sdk - s * dkp1;
      if (k > start) e[k - 1] = c * e[k - 1] - s * z;
      x = e[k];
      if (k < end - 1) {
        z = -s * e[k + 1];
        e[k + 1] = c * e[k + 1];
      }
    }
  }
  const bool ok = iter <= maxit;
  if (ok)
    for (int i = 0; i < n - 1; ++i) {
      int k = i;
      for (int j = i + 1; j < n; ++j)
        if (d[j] < d[k]) k = j;
      if (k != i) std::swap(d[i], d[k]);
    }
  for (int k = 0; k < n; ++k) ev[k] = d[k] * scale;
  return ok;
}

// IntensityGradientEstimation::computeFeature + computePointIntensityGradient for point i over
// its FLANN-ordered neighbours nb
void h6_gradient(const float* x, const float* y, const float* z, const uint32_t* rgb, const std::vector<int>& nb,
                 float nxi, float nyi, float nzi, float g[3]) {
  const size_t k = nb.size();
  float cx = 0.f, cy = 0.f, cz = 0.f, mi = 0.f;
  for (size_t m = 0; m < k; ++m) {
    const int j = nb[m];
    cx += x[j];
    cy += y[j];
    cz += z[j];
    mi += h6_intensity(rgb[j]);
  }
  const float rk = 1.0f / (float)k;  // centroid /= float(k): Eigen 3.2 reciprocal
  cx *= rk;
  cy *= rk;
  cz *= rk;
  mi /= (float)k;
  if (k < 3) {
    g[0] = g[1] = g[2] = orc::kNaN;
    return;
  }
  float A00 = 0.f, A01 = 0.f, A02 = 0.f, A11 = 0.f, A12 = 0.f, A22 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
  for (size_t m = 0; m < k; ++m) {
    const int j = nb[m];
    const float px = x[j] - cx, py = y[j] - cy, pz = z[j] - cz;
    const float iv = h6_demeaned(rgb[j], mi);
    A00 += px * px;
    A01 += px * py;
    A02 += px * pz;
    A11 += py * py;
    A12 += py * pz;
    A22 += pz * pz;
    b0 += px * iv;
    b1 += py * iv;
    b2 += pz * iv;
  }
  const float A[9] = {A00, A01, A02, A01, A11, A12, A02, A12, A22};
  const float bv[3] = {b0, b1, b2};
  float xs[3];
  colpiv_solve3(A, bv, xs);
  // (Identity - n n^T) * x: Matrix3f * Vector3f, ((m0 x0 + m1 x1) + m2 x2)
  const float nv[3] = {nxi, nyi, nzi};
  float P[9];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) P[3 * c + r] = (r == c ? 1.0f : 0.0f) - nv[r] * nv[c];
  for (int r = 0; r < 3; ++r) g[r] = (P[r] * xs[0] + P[3 + r] * xs[1]) + P[6 + r] * xs[2];
}

void h6_normalise(float g[3]) {  // HarrisKeypoint6D::detectKeypoints, "remove this magic number"
  float len = (g[0] * g[0] + g[1] * g[1]) + g[2] * g[2];
  if (len > 200.0) {
    len = (float)(1.0 / std::sqrt((double)len));
    g[0] = g[0] * len;
    g[1] = g[1] * len;
    g[2] = g[2] * len;
  } else {  // harris_6d.hpp: gradient_x = gradient_y = gradient_z = 0 (a NaN len lands here too)
    g[0] = g[1] = g[2] = 0.0f;
  }
}

float h6_response(const std::vector<int>& nb, const float* nx, const float* ny, const float* nz, const float* gx,
                  const float* gy, const float* gz) {
  float cv[21];
  for (int e = 0; e < 21; ++e) cv[e] = 0.f;
  for (size_t m = 0; m < nb.size(); ++m) {
    const int j = nb[m];
    if (!std::isfinite(nx[j]) || !std::isfinite(gx[j])) continue;
    const float v[6] = {nx[j], ny[j], nz[j], gx[j], gy[j], gz[j]};
    int e = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b) cv[e++] += v[a] * v[b];
  }
  float A[36];
  int e = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b, ++e) {
      A[6 * a + b] = cv[e];  // (row b, column a): lower triangle
      A[6 * b + a] = cv[e];
    }
  float ev[6];
  eigen_selfadjoint6f(A, ev);
  return ev[3];
}

}  // namespace

extern "C" {

// Eigen restatements exposed for the tests
int orc_eigen_selfadjoint6f(const float* a, i64 n, float* ev) {
  int bad = 0;
  for (i64 i = 0; i < n; ++i) bad += eigen_selfadjoint6f(a + 36 * i, ev + 6 * i) ? 0 : 1;
  return bad;
}
int orc_colpiv_solve3f(const float* a, const float* b, i64 n, float* x) {
  for (i64 i = 0; i < n; ++i) colpiv_solve3(a + 9 * i, b + 3 * i, x + 3 * i);
  return 0;
}

// rgb: packed 0x00RRGGBB (PointXYZRGB's float rgb field as bits).  grad_out (nullable, 3 n
// floats): the normalised intensity gradients; the rest as orc_harris3d.
int orc_harris6d(const float* x, const float* y, const float* z, const uint32_t* rgb, i64 n, double radius,
                 float threshold, int refine, int32_t* idx, i64 cap, i64* n_out, i64* n_corners, float* resp_out,
                 float* corners_out, float* grad_out, int threads) {
  *n_out = 0;
  *n_corners = 0;
  if (n <= 0) return 0;
  std::vector<float> nx((size_t)n), ny((size_t)n), nz((size_t)n), cv((size_t)n), resp((size_t)n, 0.0f);
  std::vector<float> gx((size_t)n, orc::kNaN), gy((size_t)n, orc::kNaN), gz((size_t)n, orc::kNaN);
  orc_normals(x, y, z, n, radius, 0.f, 0.f, 0.f, nx.data(), ny.data(), nz.data(), cv.data(), threads);
  NeighborGrid g;
  g.build(x, y, z, n, radius);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x, y, z, i)) continue;  // the dense branch never sees these; not a neighbour either
      g.radius(x[i], y[i], z[i], radius, nb, dd);
      float gr[3];
      h6_gradient(x, y, z, rgb, nb, nx[(size_t)i], ny[(size_t)i], nz[(size_t)i], gr);
      h6_normalise(gr);
      gx[(size_t)i] = gr[0];
      gy[(size_t)i] = gr[1];
      gz[(size_t)i] = gr[2];
    }
  }
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 256)
    for (i64 i = 0; i < n; ++i) {
      if (!finite3(x, y, z, i)) continue;
      g.radius(x[i], y[i], z[i], radius, nb, dd);
      resp[(size_t)i] = h6_response(nb, nx.data(), ny.data(), nz.data(), gx.data(), gy.data(), gz.data());
    }
  }
  if (grad_out)
    for (i64 i = 0; i < n; ++i) {
      grad_out[3 * i] = gx[(size_t)i];
      grad_out[3 * i + 1] = gy[(size_t)i];
      grad_out[3 * i + 2] = gz[(size_t)i];
    }
  return harris_finish(x, y, z, n, radius, threshold, refine, g, nx, ny, nz, resp, idx, cap, n_out, n_corners,
                       resp_out, corners_out);
}

}  // extern "C"

extern "C" {
// the u8 model above vs the host compiler's own code for static_cast<uint8_t>(float) (the cast
// is undefined for negative values in C++; x86-64 gcc emits cvttss2si and keeps the low byte):
// test-only pin of the model
int orc_u8_cast_model(const float* v, i64 n, int32_t* out) {
  for (i64 i = 0; i < n; ++i) out[i] = h6_u8(v[i]);
  return 0;
}
__attribute__((noinline)) static uint8_t native_u8(volatile float v) { return static_cast<uint8_t>(v); }
int orc_u8_cast_native(const float* v, i64 n, int32_t* out) {
  for (i64 i = 0; i < n; ++i) out[i] = native_u8(v[i]);
  return 0;
}
}  // extern "C"
