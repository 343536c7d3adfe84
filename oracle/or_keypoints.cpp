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
//    until |corner - previous|^2 <= 1e-6.
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
    for (int k = 0; k < 9; ++k) inv.m[k] /= det;
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
          diff = (dx * dx + dy * dy) + dz * dz;
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

}  // extern "C"
