// =====================================================================================
//  oracle/or_shot.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of SHOTEstimationOMP<PointXYZRGB,Normal,SHOT352> as called from
//  evaluation.cpp:766-785 via Features<T>::compute (features.h:175-196), SURVEY A.7:
//    SHOTLocalReferenceFrameEstimation::getLocalRF   (features/impl/shot_lrf.hpp)
//    SHOTEstimation::computePointSHOT / createBinDistanceShape / interpolateSingleChannel /
//    normalizeHistogram                               (features/impl/shot.hpp)
//  Restatement choices (DESIGN.md "SHOT"):
//    * Eigen 3.2.0's SelfAdjointEigenSolver<Matrix3d> (values AND vectors: the closed-form 3x3
//      Householder Q times the Givens rotations of the implicit QR steps) is restated operation
//      for operation (or_common.h selfadjoint_eigen3), `cov_m /= sum` as Eigen 3.2's
//      multiplication by the reciprocal;
//    * unqualified sqrt/acos/atan2 on float/double arguments resolve to the C double functions.
// =====================================================================================
#include "or_common.h"
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace orc;

namespace {

const double PST_PI = 3.1415926535897932384626433832795;
inline V3 v3f(const double* v) { return v3((float)v[0], (float)v[1], (float)v[2]); }
const double PST_RAD_45 = 0.78539816339744830961566084581988;
const double PST_RAD_90 = 1.5707963267948966192313216916398;
const double PST_RAD_135 = 2.3561944901923449288469825374596;
const double PST_RAD_PI_7_8 = 2.7488935718910690836548129603691;

// SHOTLocalReferenceFrameEstimation::getLocalRF; returns false (rf = NaN) on failure
bool localRF(const float* sx, const float* sy, const float* sz, float cx, float cy, float cz,
             const std::vector<int>& nb, const std::vector<float>& d2, double radius, float rf[9]) {
  std::vector<double> vx, vy, vz;
  vx.reserve(nb.size()); vy.reserve(nb.size()); vz.reserve(nb.size());
  double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  double sum = 0.0;
  for (size_t i = 0; i < nb.size(); ++i) {
    const int p = nb[i];
    if (sx[p] == cx && sy[p] == cy && sz[p] == cz) continue;
    const double v[3] = {(double)(sx[p] - cx), (double)(sy[p] - cy), (double)(sz[p] - cz)};
    const double distance = radius - std::sqrt((double)d2[i]);
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) cov[a][b] += distance * (v[a] * v[b]);
    sum += distance;
    vx.push_back(v[0]); vy.push_back(v[1]); vz.push_back(v[2]);
  }
  const int valid = (int)vx.size();
  if (valid < 5) {
    for (int k = 0; k < 9; ++k) rf[k] = kNaN;
    return false;
  }
  // `cov_m /= sum` (Eigen 3.2: times the reciprocal), then SelfAdjointEigenSolver<Matrix3d>
  const double inv_sum = 1.0 / sum;
  double covr[9];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) covr[3 * a + b] = cov[a][b] * inv_sum;
  double ev[3], V[3][3];  // V[k]: eigenvector of ev[k]
  selfadjoint_eigen3(covr, ev, V);
  if (!std::isfinite(ev[0]) || !std::isfinite(ev[1]) || !std::isfinite(ev[2])) {
    for (int k = 0; k < 9; ++k) rf[k] = kNaN;
    return false;
  }
  double v1[3] = {V[2][0], V[2][1], V[2][2]}, v3[3] = {V[0][0], V[0][1], V[0][2]};
  // vij.row(ne).dot(v) on a column-major Dynamic x 4 matrix row: ((x + y) + z) + 0
  auto dotv = [&](int ne, const double* v) { return ((vx[ne] * v[0] + vy[ne] * v[1]) + vz[ne] * v[2]) + 0.0; };
  int plusT = 0, plusN = 0;
  for (int ne = 0; ne < valid; ++ne) {
    if (dotv(ne, v1) >= 0) ++plusT;
    if (dotv(ne, v3) >= 0) ++plusN;
  }
  plusT = 2 * plusT - valid;
  if (plusT == 0) {
    const int points = 5, median = valid / 2;
    for (int i = -points / 2; i <= points / 2; ++i)
      if (dotv(median - i, v1) > 0) ++plusT;
    if (plusT < points / 2 + 1) for (int k = 0; k < 3; ++k) v1[k] *= -1;
  } else if (plusT < 0) {
    for (int k = 0; k < 3; ++k) v1[k] *= -1;
  }
  plusN = 2 * plusN - valid;
  if (plusN == 0) {
    const int points = 5, median = valid / 2;
    for (int i = -points / 2; i <= points / 2; ++i)
      if (dotv(median - i, v3) > 0) ++plusN;
    if (plusN < points / 2 + 1) for (int k = 0; k < 3; ++k) v3[k] *= -1;
  } else if (plusN < 0) {
    for (int k = 0; k < 3; ++k) v3[k] *= -1;
  }
  V3 x = v3f(v1), z = v3f(v3);
  V3 y = cross(z, x);
  rf[0] = x.x; rf[1] = x.y; rf[2] = x.z;
  rf[3] = y.x; rf[4] = y.y; rf[5] = y.z;
  rf[6] = z.x; rf[7] = z.y; rf[8] = z.z;
  return true;
}

void computeSHOT(const float* sx, const float* sy, const float* sz, const float* nx, const float* ny,
                 const float* nz, float cx, float cy, float cz, const float rf[9], const std::vector<int>& nb,
                 const std::vector<float>& d2, double radius, float shot[352]) {
  const int nr_bins = 10, desc_len = 352, maxAngularSectors = 32;
  if (nb.size() < 5) {
    for (int k = 0; k < desc_len; ++k) shot[k] = kNaN;
    return;
  }
  const double radius3_4 = (radius * 3) / 4, radius1_4 = radius / 4, radius1_2 = radius / 2;
  const V3 fx = v3(rf[0], rf[1], rf[2]), fy = v3(rf[3], rf[4], rf[5]), fz = v3(rf[6], rf[7], rf[8]);
  // createBinDistanceShape
  std::vector<double> binDistance(nb.size());
  for (size_t i = 0; i < nb.size(); ++i) {
    const int p = nb[i];
    if (!std::isfinite(nx[p]) || !std::isfinite(ny[p]) || !std::isfinite(nz[p])) {
      binDistance[i] = std::numeric_limits<double>::quiet_NaN();
      continue;
    }
    double cosineDesc = dot4(v3(nx[p], ny[p], nz[p]), fz);
    if (cosineDesc > 1.0) cosineDesc = 1.0;
    if (cosineDesc < -1.0) cosineDesc = -1.0;
    binDistance[i] = ((1.0 + cosineDesc) * nr_bins) / 2;
  }
  for (int k = 0; k < desc_len; ++k) shot[k] = 0.0f;
  // interpolateSingleChannel
  for (size_t i = 0; i < nb.size(); ++i) {
    if (!std::isfinite(binDistance[i])) continue;
    const int p = nb[i];
    const V3 delta = v3(sx[p] - cx, sy[p] - cy, sz[p] - cz);
    const double distance = std::sqrt((double)d2[i]);
    if (std::fabs(distance - 0.0) < 1E-15) continue;
    double xInFeatRef = dot4(delta, fx);
    double yInFeatRef = dot4(delta, fy);
    double zInFeatRef = dot4(delta, fz);
    if (std::fabs(yInFeatRef) < 1E-30) yInFeatRef = 0;
    if (std::fabs(xInFeatRef) < 1E-30) xInFeatRef = 0;
    if (std::fabs(zInFeatRef) < 1E-30) zInFeatRef = 0;
    unsigned char bit4 = ((yInFeatRef > 0) || ((yInFeatRef == 0.0) && (xInFeatRef < 0))) ? 1 : 0;
    unsigned char bit3 = (unsigned char)(((xInFeatRef > 0) || ((xInFeatRef == 0.0) && (yInFeatRef > 0))) ? !bit4 : bit4);
    int desc_index = (bit4 << 3) + (bit3 << 2);
    desc_index = desc_index << 1;
    if ((xInFeatRef * yInFeatRef > 0) || (xInFeatRef == 0.0))
      desc_index += (std::fabs(xInFeatRef) >= std::fabs(yInFeatRef)) ? 0 : 4;
    else
      desc_index += (std::fabs(xInFeatRef) > std::fabs(yInFeatRef)) ? 4 : 0;
    desc_index += zInFeatRef > 0 ? 1 : 0;
    desc_index += (distance > radius1_2) ? 2 : 0;
    const int step_index = (int)std::floor(binDistance[i] + 0.5);
    const int volume_index = desc_index * (nr_bins + 1);
    binDistance[i] -= step_index;
    double intWeight = (1 - std::fabs(binDistance[i]));
    if (binDistance[i] > 0)
      shot[volume_index + ((step_index + 1) % nr_bins)] += (float)binDistance[i];
    else
      shot[volume_index + ((step_index - 1 + nr_bins) % nr_bins)] += -(float)binDistance[i];
    if (distance > radius1_2) {
      const double radiusDistance = (distance - radius3_4) / radius1_2;
      if (distance > radius3_4) {
        intWeight += 1 - radiusDistance;
      } else {
        intWeight += 1 + radiusDistance;
        shot[(desc_index - 2) * (nr_bins + 1) + step_index] -= (float)radiusDistance;
      }
    } else {
      const double radiusDistance = (distance - radius1_4) / radius1_2;
      if (distance < radius1_4) {
        intWeight += 1 + radiusDistance;
      } else {
        intWeight += 1 - radiusDistance;
        shot[(desc_index + 2) * (nr_bins + 1) + step_index] += (float)radiusDistance;
      }
    }
    double inclinationCos = zInFeatRef / distance;
    if (inclinationCos < -1.0) inclinationCos = -1.0;
    if (inclinationCos > 1.0) inclinationCos = 1.0;
    const double inclination = std::acos(inclinationCos);
    if (inclination > PST_RAD_90 || (std::fabs(inclination - PST_RAD_90) < 1e-30 && zInFeatRef <= 0)) {
      const double inclinationDistance = (inclination - PST_RAD_135) / PST_RAD_90;
      if (inclination > PST_RAD_135) {
        intWeight += 1 - inclinationDistance;
      } else {
        intWeight += 1 + inclinationDistance;
        shot[(desc_index + 1) * (nr_bins + 1) + step_index] -= (float)inclinationDistance;
      }
    } else {
      const double inclinationDistance = (inclination - PST_RAD_45) / PST_RAD_90;
      if (inclination < PST_RAD_45) {
        intWeight += 1 + inclinationDistance;
      } else {
        intWeight += 1 - inclinationDistance;
        shot[(desc_index - 1) * (nr_bins + 1) + step_index] += (float)inclinationDistance;
      }
    }
    if (yInFeatRef != 0.0 || xInFeatRef != 0.0) {
      const double azimuth = std::atan2(yInFeatRef, xInFeatRef);
      const int sel = desc_index >> 2;
      const double angularSectorSpan = PST_RAD_45;
      const double angularSectorStart = -PST_RAD_PI_7_8;
      double azimuthDistance = (azimuth - (angularSectorStart + angularSectorSpan * sel)) / angularSectorSpan;
      azimuthDistance = std::max(-0.5, std::min(azimuthDistance, 0.5));
      if (azimuthDistance > 0) {
        intWeight += 1 - azimuthDistance;
        const int interp_index = (desc_index + 4) % maxAngularSectors;
        shot[interp_index * (nr_bins + 1) + step_index] += (float)azimuthDistance;
      } else {
        const int interp_index = (desc_index - 4 + maxAngularSectors) % maxAngularSectors;
        intWeight += 1 + azimuthDistance;
        shot[interp_index * (nr_bins + 1) + step_index] -= (float)azimuthDistance;
      }
    }
    shot[volume_index + step_index] += (float)intWeight;
  }
  // normalizeHistogram
  double acc_norm = 0;
  for (int j = 0; j < desc_len; ++j) acc_norm += shot[j] * shot[j];
  acc_norm = std::sqrt(acc_norm);
  for (int j = 0; j < desc_len; ++j) shot[j] /= (float)acc_norm;
  (void)PST_PI;
}

}  // namespace

extern "C" int orc_shot(const float* sx, const float* sy, const float* sz, const float* snx, const float* sny,
                        const float* snz, i64 n_surf, const float* qx, const float* qy, const float* qz, i64 nq,
                        double radius, float* desc, float* rf_out, int nthreads) {
  NeighborGrid g;
  g.build(sx, sy, sz, n_surf, radius);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    std::vector<int> nb;
    std::vector<float> dd;
#pragma omp for schedule(dynamic, 8)
    for (i64 q = 0; q < nq; ++q) {
      float* d = desc + q * 352;
      float* rf = rf_out + q * 9;
      const float cx = qx[q], cy = qy[q], cz = qz[q];
      if (!(std::isfinite(cx) && std::isfinite(cy) && std::isfinite(cz))) {
        for (int k = 0; k < 352; ++k) d[k] = kNaN;
        for (int k = 0; k < 9; ++k) rf[k] = kNaN;
        continue;
      }
      g.radius(cx, cy, cz, radius, nb, dd);
      float lrf[9];
      bool ok = localRF(sx, sy, sz, cx, cy, cz, nb, dd, radius, lrf);
      if (!ok || nb.empty()) {
        for (int k = 0; k < 352; ++k) d[k] = kNaN;
        for (int k = 0; k < 9; ++k) rf[k] = kNaN;
        continue;
      }
      computeSHOT(sx, sy, sz, snx, sny, snz, cx, cy, cz, lrf, nb, dd, radius, d);
      for (int k = 0; k < 9; ++k) rf[k] = lrf[k];
    }
  }
  return 0;
}
