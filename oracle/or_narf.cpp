// =====================================================================================
//  oracle/or_narf.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of the NARF keypoint branch of Keypoints::compute
//  (include/pcl_feature_extraction/keypoints.h:199-231), i.e. of PCL 1.7's
//    RangeImagePlanar::createFromPointCloudWithFixedSize     (confidence H)
//    RangeImageBorderExtractor                                (confidence M)
//    NarfKeypoint::compute                                    (confidence M/L)
//  PCL 1.7 source files restated (not in this container): range_image/impl/range_image.hpp,
//  range_image_planar.hpp, features/src/range_image_border_extractor.cpp + impl/*.hpp,
//  common/impl/vector_average.hpp, keypoints/src/narf_keypoint.cpp.
//  Documented restatement choices (see DESIGN.md "NARF"):
//    * interest image: the dense ("complete") formula at full resolution
//      (calculateCompleteInterestImage); PCL's default sparse traversal only as a reconstruction
//      (interestImageSparse, confidence L, params[7] = 2); the scale-space variant is not restated
//      (planar images have no angular resolution).
//    * VectorAverage covariance is used as a full symmetric matrix.
//    * histogram cell of a NaN / negative angle -> 0 (UB in PCL).
//  Round 4 (one Eigen 3.2 model, or_common.h): Vector3f dot / squaredNorm / norm / normalized()
//  reduce as x + (y + z) (range = transformedPoint.norm () in getImagePoint, the viewing
//  direction and normal flip of getSurfaceInformation, eigen33's cross-product lengths, the
//  border-direction cosines and normalize (), getTransFromUnitVectorsZY, the greedy selection's
//  squaredNorm); the viewer-frame rotation of nkdGetDirectionAngle is an Affine3f * Vector3f
//  product (left to right); get3dDirection intersects the neighbour pixel's viewing ray with
//  the local plane (normal_no_jumps, neighborhood_mean_no_jumps) as PCL 1.7 does (rounds 1-3
//  projected along the normal through the point).
//  Single-threaded except the per-pixel interest loop (OpenMP, order-free).
// =====================================================================================
#include "or_common.h"
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace orc;

namespace {

// PCL BorderTrait bit order (common/point_types.h)
enum {
  OBSTACLE_BORDER = 0, SHADOW_BORDER, VEIL_POINT, SHADOW_BORDER_TOP, SHADOW_BORDER_RIGHT,
  SHADOW_BORDER_BOTTOM, SHADOW_BORDER_LEFT, OBSTACLE_BORDER_TOP, OBSTACLE_BORDER_RIGHT,
  OBSTACLE_BORDER_BOTTOM, OBSTACLE_BORDER_LEFT, VEIL_POINT_TOP, VEIL_POINT_RIGHT,
  VEIL_POINT_BOTTOM, VEIL_POINT_LEFT
};
inline uint32_t bit(int t) { return 1u << t; }

// Alternative readings of the medium / low confidence statements of SURVEY A.5 / A.6, for the
// sensitivity table of scripts/narf_alt_report.py (VERDICT r04 #2c: which statements the keypoint
// set hinges on).  0 (always, outside that report) = the restatement as documented; each bit
// swaps ONE statement for its most plausible other reading (orc_narf_set_alt).
enum : int {
  kAltPlaneFullWindow = 1 << 0,  // A.5.1 local plane: every pixel of the 5x5 window, 9 closest (not step 2, 4 closest)
  kAltUpdateWithCentre = 1 << 1, // A.5.3 updatedScoreAccordingToNeighborValues: 3x3 mean incl. the centre
  kAltUpdateNoEarlyOut = 1 << 2, // A.5.3 ... without the early return below minimum_border_probability
  kAltShadowUnupdated = 1 << 3,  // A.5.4 shadow pass: every direction reads the un-updated scores
  kAltCurvatureNoSqrt = 1 << 4,  // A.5.7 principal curvature magnitude = lambda_max (not its sqrt)
  kAltBeamsNotCut = 1 << 5,      // A.5.7 curvature beams skip veil/shadow pixels instead of ending
  kAltGrowOr = 1 << 6,           // A.6 region grow: accept only within 2 px AND within R (not OR)
  kAltPosLessEq2 = 1 << 7,       // A.6 positive score: scs when pixel distance <= 2 (not < 2)
  kAltNegNotSquared = 1 << 8,    // A.6 negative score not squared
  kAltAngleAtan2 = 1 << 9,       // A.6 direction angle: 0.5 normAngle(2 atan2(v_y, v_x)) (not acos(v_x))
  kAltCellRound = 1 << 10,       // A.6 histogram cell: lrint without floorf
  kAltAcvNoSqrt = 1 << 11,       // A.6 interest = negative x max(h_i h_j nd) (no sqrt)
};
int g_alt = 0;
inline bool alt(int b) { return (g_alt & b) != 0; }

const float kInf = std::numeric_limits<float>::infinity();

struct P4 { float x, y, z, range; };

struct Affine {  // 3x4 row-major [R | t]
  float m[3][4];
  V3 apply(V3 p) const {  // Eigen: res = t; res += linear * p  ->  t + ((r0 x + r1 y) + r2 z)
    V3 r;
    r.x = m[0][3] + (m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z);
    r.y = m[1][3] + (m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z);
    r.z = m[2][3] + (m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z);
    return r;
  }
};

struct Camera {
  int w, h;
  float cx, cy, fx, fy;
  float pose[16];
  int frame;
  float noise, min_range;
};

struct RangeImage {
  int w = 0, h = 0;
  float cx, cy, fx, fy, fxr, fyr;
  Affine to_world, to_ri;
  std::vector<P4> pts;

  bool inImage(int x, int y) const { return x >= 0 && x < w && y >= 0 && y < h; }
  bool isValid(int x, int y) const { return inImage(x, y) && std::isfinite(pts[(size_t)y * w + x].range); }
  bool isValidIdx(int i) const { return std::isfinite(pts[(size_t)i].range); }
  bool isMaxRange(int x, int y) const {
    if (!inImage(x, y)) return false;
    float r = pts[(size_t)y * w + x].range;
    return std::isinf(r) && r > 0;
  }
  P4 getPoint(int x, int y) const {
    if (!inImage(x, y)) { P4 u = {kNaN, kNaN, kNaN, -kInf}; return u; }
    return pts[(size_t)y * w + x];
  }
  V3 sensorPos() const { return v3(to_world.m[0][3], to_world.m[1][3], to_world.m[2][3]); }
  // RangeImagePlanar::calculate3DPoint
  V3 calc3D(float ix, float iy, float range) const {
    float dx = (ix + 0.0f - cx) * fxr, dy = (iy + 0.0f - cy) * fyr;
    V3 p;
    p.z = range / (std::sqrt(dx * dx + dy * dy + 1));
    p.x = dx * p.z;
    p.y = dy * p.z;
    return to_world.apply(p);
  }
  // RangeImagePlanar::getImagePoint
  void imagePoint(V3 point, float& ix, float& iy, float& range) const {
    V3 t = to_ri.apply(point);
    if (t.z <= 0) { ix = iy = range = -1.0f; return; }
    range = std::sqrt(sqn3(t));
    ix = cx + fx * t.x / t.z - 0.0f;
    iy = cy + fy * t.y / t.z - 0.0f;
  }
};

inline int lrintf_i(float v) { return (int)std::lrint(v); }

// ---- RangeImagePlanar::createFromPointCloudWithFixedSize ---------------------------------
void createRangeImage(const float* X, const float* Y, const float* Z, i64 n, const Camera& c, RangeImage& ri) {
  ri.w = c.w; ri.h = c.h;
  ri.cx = c.cx; ri.cy = c.cy; ri.fx = c.fx; ri.fy = c.fy;
  ri.fxr = 1 / c.fx; ri.fyr = 1 / c.fy;
  // to_world = sensor_pose * coordinate-frame transformation (CAMERA_FRAME = identity)
  float F[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  if (c.frame == 1) {  // LASER_FRAME
    float L[4][4] = {{0, 0, 1, 0}, {-1, 0, 0, 0}, {0, -1, 0, 0}, {0, 0, 0, 1}};
    std::memcpy(F, L, sizeof(F));
  }
  float W[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      W[i][j] = ((c.pose[i * 4 + 0] * F[0][j] + c.pose[i * 4 + 1] * F[1][j]) + c.pose[i * 4 + 2] * F[2][j]) +
                c.pose[i * 4 + 3] * F[3][j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) ri.to_world.m[i][j] = W[i][j];
  // inverse(Isometry): R^T, -(R^T t)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) ri.to_ri.m[i][j] = W[j][i];
  for (int i = 0; i < 3; ++i)
    ri.to_ri.m[i][3] = -(ri.to_ri.m[i][0] * W[0][3] + ri.to_ri.m[i][1] * W[1][3] + ri.to_ri.m[i][2] * W[2][3]);

  const size_t size = (size_t)ri.w * ri.h;
  P4 unobs = {kNaN, kNaN, kNaN, -kInf};
  ri.pts.assign(size, unobs);
  std::vector<int> counters(size, 0);
  for (i64 i = 0; i < n; ++i) {
    if (!(std::isfinite(X[i]) && std::isfinite(Y[i]) && std::isfinite(Z[i]))) continue;
    float xr, yr, rng;
    ri.imagePoint(v3(X[i], Y[i], Z[i]), xr, yr, rng);
    int x = lrintf_i(xr), y = lrintf_i(yr);
    if (rng < c.min_range || !ri.inImage(x, y)) continue;
    int fx0 = (int)std::lrint(std::floor((double)xr)), fy0 = (int)std::lrint(std::floor((double)yr));
    int cx0 = (int)std::lrint(std::ceil((double)xr)), cy0 = (int)std::lrint(std::ceil((double)yr));
    int nxs[4] = {fx0, fx0, cx0, cx0}, nys[4] = {fy0, cy0, fy0, cy0};
    for (int k = 0; k < 4; ++k) {
      int nx_ = nxs[k], ny_ = nys[k];
      if (nx_ == x && ny_ == y) continue;
      if (!ri.inImage(nx_, ny_)) continue;
      size_t np = (size_t)ny_ * ri.w + nx_;
      if (counters[np] == 0) {
        float& nr = ri.pts[np].range;
        nr = std::isinf(nr) ? rng : std::min(nr, rng);
      }
    }
    size_t ap = (size_t)y * ri.w + x;
    float& r_at = ri.pts[ap].range;
    int& counter = counters[ap];
    bool add = false, replace = false;
    if (counter == 0) replace = true;
    else if (rng < r_at - c.noise) replace = true;
    else if (std::fabs(rng - r_at) <= c.noise) add = true;
    if (replace) { counter = 1; r_at = rng; }
    else if (add) { ++counter; r_at += (rng - r_at) / counter; }
  }
  // recalculate3DPointPositions
  for (int y = 0; y < ri.h; ++y)
    for (int x = 0; x < ri.w; ++x) {
      P4& p = ri.pts[(size_t)y * ri.w + x];
      if (!std::isinf(p.range)) {
        V3 q = ri.calc3D((float)x, (float)y, p.range);
        p.x = q.x; p.y = q.y; p.z = q.z;
      }
    }
}

// ---- VectorAverage3f (common/impl/vector_average.hpp) -------------------------------------
// add(): `covariance_(i, j) = (1.0f-alpha)*(covariance_(i, j) + alpha*diff[i]*diff[j])` -- the
// product parses left to right, (alpha * diff[i]) * diff[j] (round 4; was alpha * (d_i d_j))
struct VecAvg {
  int n = 0;
  float acc_w = 0.0f;
  V3 mean = {0, 0, 0};
  float cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  void add(V3 s) {
    ++n;
    acc_w += 1.0f;
    float alpha = 1.0f / acc_w;
    V3 diff = sub(s, mean);
    mean = orc::add(mean, v3(alpha * diff.x, alpha * diff.y, alpha * diff.z));
    float d[3] = {diff.x, diff.y, diff.z};
    for (int i = 0; i < 3; ++i)
      for (int j = i; j < 3; ++j) cov[i][j] = (1.0f - alpha) * (cov[i][j] + alpha * d[i] * d[j]);
  }
  void pca(float evals[3], V3 evecs[3]) const {
    float m[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) m[i][j] = (j >= i) ? cov[i][j] : cov[j][i];
    eigen33_full(m, evecs, evals);
  }
};

struct Surface {
  bool valid = false;
  V3 normal_no_jumps;
  V3 mean_no_jumps;  // LocalSurface::neighborhood_mean_no_jumps (get3dDirection's plane)
  float max_nb_d2 = 0.0f;
};

float sqDist(const P4& a, const P4& b) {  // pcl::squaredEuclideanDistance(p1, p2): diff = p2 - p1
  float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
  return dx * dx + dy * dy + dz * dz;
}

// RangeImage::getSurfaceInformation (no-jumps part; the all-neighbour PCA feeds nothing on this path)
bool surfaceInformation(const RangeImage& ri, int x, int y, int radius, const P4& point, int no_of_closest,
                        int step, Surface& s) {
  struct ND { float d; P4 p; };
  ND nb[64];
  int cnt = 0;
  for (int y2 = y - radius; y2 <= y + radius; y2 += step)
    for (int x2 = x - radius; x2 <= x + radius; x2 += step) {
      if (!ri.isValid(x2, y2)) continue;
      P4 p = ri.getPoint(x2, y2);
      nb[cnt].p = p;
      nb[cnt].d = sqDist(point, p);
      ++cnt;
    }
  // std::sort on <= 16 elements is libstdc++'s insertion sort (stable), by distance
  for (int i = 1; i < cnt; ++i) {
    ND v = nb[i];
    int j = i;
    while (j > 0 && v.d < nb[j - 1].d) { nb[j] = nb[j - 1]; --j; }
    nb[j] = v;
  }
  int k = std::min(cnt, no_of_closest);
  s.max_nb_d2 = nb[k - 1].d;
  float max_d2 = s.max_nb_d2 * 4.0f;
  VecAvg va;
  for (int i = 0; i < cnt; ++i) {
    if (nb[i].d > max_d2) break;
    va.add(v3(nb[i].p.x, nb[i].p.y, nb[i].p.z));
  }
  if (va.n < 3) return false;
  float ev[3];
  V3 evec[3];
  va.pca(ev, evec);
  V3 normal = evec[0];
  V3 view = normalized3(sub(ri.sensorPos(), v3(point.x, point.y, point.z)));
  if (dot3(normal, view) < 0.0f) normal = mul(normal, -1.0f);
  s.normal_no_jumps = normal;
  s.mean_no_jumps = va.mean;  // `mean = vector_average.getMean ()`
  s.valid = true;
  return true;
}

struct Params {
  float support_size;
  int max_no_of_interest_points;
  float min_distance_between_interest_points, optimal_distance_to_high_surface_change, min_interest_value,
      min_surface_change_score;
  int do_nms;
  int pixel_radius_borders, pixel_radius_plane_extraction, pixel_radius_border_direction;
  float minimum_border_probability;
  int pixel_radius_principal_curvature;
};

struct Border {
  const RangeImage& ri;
  const Params& P;
  int w, h;
  std::vector<Surface> surf;
  std::vector<float> sL, sR, sT, sB;
  std::vector<int> shL, shR, shT, shB;  // shadow border indices (-1 none)
  std::vector<char> has_shadow;
  std::vector<uint32_t> traits;
  std::vector<char> dir_valid;
  std::vector<V3> dir;
  std::vector<float> scs;
  std::vector<V3> scd;
  Border(const RangeImage& r, const Params& p) : ri(r), P(p), w(r.w), h(r.h) {}

  void get1dPointAverage(int x, int y, int dx, int dy, int no_of_points, P4& avg) const {
    float weight_sum = 1.0f;
    avg = ri.getPoint(x, y);
    if (std::isinf(avg.range)) {
      if (avg.range > 0.0f) return;
      weight_sum = 0.0f;
      avg.x = avg.y = avg.z = avg.range = 0.0f;
    }
    int x2 = x, y2 = y;
    for (int step = 1; step < no_of_points; ++step) {
      x2 += dx; y2 += dy;
      if (!ri.isValid(x2, y2)) continue;
      const P4& p = ri.pts[(size_t)y2 * w + x2];
      avg.x += p.x; avg.y += p.y; avg.z += p.z; avg.range += p.range;
      weight_sum += 1.0f;
    }
    if (weight_sum <= 0.0f) { P4 u = {kNaN, kNaN, kNaN, -kInf}; avg = u; return; }
    float nf = 1.0f / weight_sum;
    avg.x *= nf; avg.y *= nf; avg.z *= nf; avg.range *= nf;
  }

  float neighborDistanceChangeScore(const Surface& s, int x, int y, int ox, int oy, int pixel_radius) const {
    P4 point = ri.getPoint(x, y);
    P4 nb;
    get1dPointAverage(x + ox, y + oy, ox, oy, pixel_radius, nb);
    if (std::isinf(nb.range)) return nb.range < 0.0f ? 0.0f : 1.0f;
    float nd2 = sqDist(nb, point);
    if (nd2 <= s.max_nb_d2) return 0.0f;
    float ret = 1.0f - std::sqrt(s.max_nb_d2 / nd2);
    if (nb.range < point.range) ret = -ret;
    return ret;
  }

  void localSurfaces() {
    surf.assign((size_t)w * h, Surface());
    int step = (P.pixel_radius_plane_extraction / 2) + 1;
    int nn = (int)std::pow((double)(P.pixel_radius_plane_extraction / step + 1), 2.0);
    if (alt(kAltPlaneFullWindow)) {
      step = 1;
      nn = (P.pixel_radius_plane_extraction + 1) * (P.pixel_radius_plane_extraction + 1);
    }
#pragma omp parallel for schedule(dynamic, 8)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        if (!ri.isValid(x, y)) continue;
        Surface s;
        if (surfaceInformation(ri, x, y, P.pixel_radius_plane_extraction, ri.getPoint(x, y), nn, step, s))
          surf[(size_t)y * w + x] = s;
      }
  }

  void borderScores() {
    size_t n = (size_t)w * h;
    sL.assign(n, 0.f); sR.assign(n, 0.f); sT.assign(n, 0.f); sB.assign(n, 0.f);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        size_t i = (size_t)y * w + x;
        if (!surf[i].valid) continue;
        sL[i] = neighborDistanceChangeScore(surf[i], x, y, -1, 0, P.pixel_radius_borders);
        sR[i] = neighborDistanceChangeScore(surf[i], x, y, 1, 0, P.pixel_radius_borders);
        sT[i] = neighborDistanceChangeScore(surf[i], x, y, 0, -1, P.pixel_radius_borders);
        sB[i] = neighborDistanceChangeScore(surf[i], x, y, 0, 1, P.pixel_radius_borders);
      }
  }

  float updatedScore(int x, int y, const std::vector<float>& s) const {
    const float bonus = 0.5f;
    float b = s[(size_t)y * w + x];
    if (!alt(kAltUpdateNoEarlyOut) && b + bonus * (1.0f - b) < P.minimum_border_probability) return b;
    float avg = 0.0f, ws = 0.0f;
    for (int y2 = y - 1; y2 <= y + 1; ++y2)
      for (int x2 = x - 1; x2 <= x + 1; ++x2) {
        if (!ri.inImage(x2, y2) || (x2 == x && y2 == y && !alt(kAltUpdateWithCentre))) continue;
        avg += s[(size_t)y2 * w + x2];
        ws += 1.0f;
      }
    avg /= ws;
    if (avg * b < 0.0f) return b;
    return b + bonus * avg * (1.0f - std::fabs(b));
  }
  void updateScores(std::vector<float>& s) {
    std::vector<float> ns(s.size());
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) ns[(size_t)y * w + x] = updatedScore(x, y, s);
    s.swap(ns);
  }

  bool changeScoreShadow(int x, int y, int ox, int oy, std::vector<float>& scores,
                         const std::vector<float>& other, int& sidx) {
    float& b = scores[(size_t)y * w + x];
    sidx = -1;
    if (b < P.minimum_border_probability) return false;
    if (b == 1.0f) {
      if (ri.isMaxRange(x + ox, y + oy)) { sidx = (y + oy) * w + x + ox; return true; }
    }
    float best = 0.0f;
    for (int d = 1; d <= P.pixel_radius_borders; ++d) {
      int nx_ = x + d * ox, ny_ = y + d * oy;
      if (!ri.inImage(nx_, ny_)) continue;
      float s = other[(size_t)ny_ * w + nx_];
      if (s < best) { sidx = ny_ * w + nx_; best = s; }
    }
    if (sidx >= 0) {
      b *= std::max(0.9f, 1 - pow3f_cr(1 + best));
      if (b >= P.minimum_border_probability) return true;
    }
    sidx = -1;
    b = 0.0f;
    return false;
  }

  void shadowBorders() {
    size_t n = (size_t)w * h;
    shL.assign(n, -1); shR.assign(n, -1); shT.assign(n, -1); shB.assign(n, -1);
    has_shadow.assign(n, 0);
    // (alternative reading: the opposite-direction scores read before any update)
    const std::vector<float> oL = sL, oR = sR, oT = sT, oB = sB;
    const bool un = alt(kAltShadowUnupdated);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        size_t i = (size_t)y * w + x;
        int s;
        if (changeScoreShadow(x, y, -1, 0, sL, un ? oR : sR, s)) { has_shadow[i] = 1; shL[i] = s; }
        if (changeScoreShadow(x, y, 1, 0, sR, un ? oL : sL, s)) { has_shadow[i] = 1; shR[i] = s; }
        if (changeScoreShadow(x, y, 0, -1, sT, un ? oB : sB, s)) { has_shadow[i] = 1; shT[i] = s; }
        if (changeScoreShadow(x, y, 0, 1, sB, un ? oT : sT, s)) { has_shadow[i] = 1; shB[i] = s; }
      }
  }

  bool checkIfMaximum(int x, int y, int ox, int oy, const std::vector<float>& s, int sidx) const {
    float b = s[(size_t)y * w + x];
    int nx_ = x - ox, ny_ = y - oy;
    if (ri.inImage(nx_, ny_) && s[(size_t)ny_ * w + nx_] > b) return false;
    for (int d = 1; d <= P.pixel_radius_borders; ++d) {
      nx_ = x + d * ox; ny_ = y + d * oy;
      if (!ri.inImage(nx_, ny_)) continue;
      int ni = ny_ * w + nx_;
      if (ni == sidx) return true;
      if (s[(size_t)ni] > b) return false;
    }
    return true;
  }

  void classify() {
    traits.assign((size_t)w * h, 0u);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int i = y * w + x;
        if (!has_shadow[(size_t)i]) continue;
        uint32_t& bt = traits[(size_t)i];
        int s = shL[(size_t)i];
        if (s >= 0 && checkIfMaximum(x, y, -1, 0, sL, s)) {
          bt |= bit(OBSTACLE_BORDER) | bit(OBSTACLE_BORDER_LEFT);
          traits[(size_t)s] |= bit(SHADOW_BORDER) | bit(SHADOW_BORDER_RIGHT);
          int sx = s % w;
          for (int i3 = y * w + sx + 1; i3 < i; ++i3) traits[(size_t)i3] |= bit(VEIL_POINT) | bit(VEIL_POINT_RIGHT);
        }
        s = shR[(size_t)i];
        if (s >= 0 && checkIfMaximum(x, y, 1, 0, sR, s)) {
          bt |= bit(OBSTACLE_BORDER) | bit(OBSTACLE_BORDER_RIGHT);
          traits[(size_t)s] |= bit(SHADOW_BORDER) | bit(SHADOW_BORDER_LEFT);
          int sx = s % w, sy = s / w;
          for (int i3 = i + 1; i3 < sy * w + sx; ++i3) traits[(size_t)i3] |= bit(VEIL_POINT) | bit(VEIL_POINT_LEFT);
        }
        s = shT[(size_t)i];
        if (s >= 0 && checkIfMaximum(x, y, 0, -1, sT, s)) {
          bt |= bit(OBSTACLE_BORDER) | bit(OBSTACLE_BORDER_TOP);
          traits[(size_t)s] |= bit(SHADOW_BORDER) | bit(SHADOW_BORDER_BOTTOM);
          int sy = s / w;
          for (int i3 = (sy + 1) * w + x; i3 < i; i3 += w) traits[(size_t)i3] |= bit(VEIL_POINT) | bit(VEIL_POINT_BOTTOM);
        }
        s = shB[(size_t)i];
        if (s >= 0 && checkIfMaximum(x, y, 0, 1, sB, s)) {
          bt |= bit(OBSTACLE_BORDER) | bit(OBSTACLE_BORDER_BOTTOM);
          traits[(size_t)s] |= bit(SHADOW_BORDER) | bit(SHADOW_BORDER_TOP);
          int sy = s / w;
          for (int i3 = i + w; i3 < sy * w + x; i3 += w) traits[(size_t)i3] |= bit(VEIL_POINT) | bit(VEIL_POINT_TOP);
        }
      }
  }

  bool get3dDirection(int x, int y, V3& direction) const {
    uint32_t bt = traits[(size_t)y * w + x];
    int dx = 0, dy = 0;
    if (bt & bit(OBSTACLE_BORDER_LEFT)) --dx;
    if (bt & bit(OBSTACLE_BORDER_RIGHT)) ++dx;
    if (bt & bit(OBSTACLE_BORDER_TOP)) --dy;
    if (bt & bit(OBSTACLE_BORDER_BOTTOM)) ++dy;
    if (dx == 0 && dy == 0) return false;
    P4 point = ri.getPoint(x, y);
    V3 pt = v3(point.x, point.y, point.z);
    V3 nbp = ri.calc3D((float)(x + dx), (float)(y + dy), point.range);
    const Surface& s = surf[(size_t)y * w + x];
    if (s.valid) {
      // "Get the point that lies on the local plane approximation": the viewing ray through the
      // neighbour pixel meets the plane (normal_no_jumps, neighborhood_mean_no_jumps)
      //   lambda = n.dot(mean - sensor) / n.dot(viewing_direction)
      //   neighbor_point = lambda * viewing_direction + sensor_pos
      const V3 sensor = ri.sensorPos();
      const V3 vd = sub(nbp, sensor);
      const V3 nrm = s.normal_no_jumps;
      const float lambda = dot3(nrm, sub(s.mean_no_jumps, sensor)) / dot3(nrm, vd);
      nbp = add(mul(vd, lambda), sensor);
    }
    direction = sub(nbp, pt);
    direction = normalize3(direction);  // `direction.normalize ()`
    return true;
  }

  void borderDirections() {
    size_t n = (size_t)w * h;
    std::vector<char> raw_valid(n, 0);
    std::vector<V3> raw(n, v3(0, 0, 0));
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        size_t i = (size_t)y * w + x;
        if (!(traits[i] & bit(OBSTACLE_BORDER))) continue;
        V3 d;
        if (get3dDirection(x, y, d)) { raw[i] = d; raw_valid[i] = 1; }
      }
    dir_valid.assign(n, 0);
    dir.assign(n, v3(0, 0, 0));
    const int radius = P.pixel_radius_border_direction;
    const int min_weight = radius + 1;
    const float min_cos = cosf_cr(120.0f * 0.017453292519943295769236907684886127134428718885417f);
    const float thr = 0.95f * P.minimum_border_probability;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        size_t i = (size_t)y * w + x;
        if (!raw_valid[i]) continue;
        V3 avg = raw[i];
        float ws = 1.0f;
        for (int y2 = std::max(0, y - radius); y2 <= std::min(y + radius, h - 1); ++y2)
          for (int x2 = std::max(0, x - radius); x2 <= std::min(x + radius, w - 1); ++x2) {
            size_t i2 = (size_t)y2 * w + x2;
            if (!raw_valid[i2] || i2 == i) continue;
            float ca = dot3(raw[i2], raw[i]);
            if (ca < min_cos) continue;
            float between = neighborDistanceChangeScore(surf[i], x, y, x2 - x, y2 - y, 1);
            if (std::fabs(between) >= thr) continue;
            avg = add(avg, raw[i2]);
            ws += 1.0f;
          }
        if (std::lrint(ws) < min_weight) continue;
        dir[i] = normalize3(avg);  // `average_border_direction->normalize ()`
        dir_valid[i] = 1;
      }
  }

  bool mainPrincipalCurvature(int x, int y, int radius, float& mag, V3& main_dir) const {
    mag = 0.0f;
    size_t i = (size_t)y * w + x;
    if (!surf[i].valid) return false;
    VecAvg va;
    bool beam[9];
    for (int step = 1; step <= radius; ++step) {
      int bi = 0;
      for (int y2 = y - step; y2 <= y + step; y2 += step)
        for (int x2 = x - step; x2 <= x + step; x2 += step) {
          bool& bv = beam[bi++];
          if (step == 1) {
            bv = !(x2 == x && y2 == y);
          } else if (!bv) {
            continue;
          }
          if (!ri.isValid(x2, y2)) continue;
          size_t i2 = (size_t)y2 * w + x2;
          if (traits[i2] & (bit(VEIL_POINT) | bit(SHADOW_BORDER))) {
            if (!alt(kAltBeamsNotCut)) bv = false;
            continue;
          }
          if (!surf[i2].valid) continue;
          va.add(surf[i2].normal_no_jumps);
        }
    }
    if (va.n < 3) return false;
    float ev[3];
    V3 evec[3];
    va.pca(ev, evec);
    main_dir = evec[2];
    mag = alt(kAltCurvatureNoSqrt) ? ev[2] : std::sqrt(ev[2]);
    if (!std::isfinite(mag)) return false;
    return true;
  }

  void surfaceChanges() {
    size_t n = (size_t)w * h;
    scs.assign(n, 0.0f);
    scd.assign(n, v3(0, 0, 0));
#pragma omp parallel for schedule(dynamic, 8)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        size_t i = (size_t)y * w + x;
        if (traits[i] & (bit(VEIL_POINT) | bit(SHADOW_BORDER))) continue;
        if (dir_valid[i]) {
          scs[i] = 1.0f;
          scd[i] = dir[i];
        } else {
          float m;
          V3 d = v3(0, 0, 0);
          if (!mainPrincipalCurvature(x, y, P.pixel_radius_principal_curvature, m, d)) {
            scs[i] = 0.0f;
            scd[i] = d;
            continue;
          }
          scs[i] = m;
          scd[i] = d;
        }
      }
  }

  void run() {
    localSurfaces();
    borderScores();
    updateScores(sL); updateScores(sR); updateScores(sT); updateScores(sB);
    shadowBorders();
    classify();
    borderDirections();
    surfaceChanges();
  }
};

// normAngle (common/angles.hpp)
inline float normAngle(float a) {
  const float pi = (float)M_PI;
  return a >= 0 ? std::fmod(a + pi, 2.0f * pi) - pi : -(std::fmod(pi - a, 2.0f * pi) - pi);
}

struct InterestPoint { float x, y, z, strength; };
bool isBetter(const InterestPoint& a, const InterestPoint& b) { return a.strength > b.strength; }

void interestImage(const RangeImage& ri, const Border& B, const Params& P, std::vector<float>& interest) {
  const int w = ri.w, h = ri.h;
  const size_t n = (size_t)w * h;
  interest.assign(n, 0.0f);
  const float search_radius = 0.5f * P.support_size;
  const float radius_squared = search_radius * search_radius;
  const float radius_reciprocal = 1.0f / search_radius;
  const int hist_size = 18;
  const float deg = 0.017453292519943295769236907684886127134428718885417f;
  const float d90 = 90.0f * deg, d180 = 180.0f * deg;
  const V3 sensor = ri.sensorPos();
#pragma omp parallel
  {
    std::vector<char> touched(n, 0);
    std::vector<int> queue;
#pragma omp for schedule(dynamic, 16)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const int index = y * w + x;
        if (!ri.isValidIdx(index)) continue;
        if (B.traits[(size_t)index] & (bit(SHADOW_BORDER) | bit(VEIL_POINT))) continue;
        const P4 point = ri.pts[(size_t)index];
        // getRotationToViewerCoordinateFrame -> getTransFromUnitVectorsZY(z = view, y = (0,-1,0))
        V3 view = normalized3(sub(v3(point.x, point.y, point.z), sensor));
        V3 tmp0 = normalized3(cross(v3(0.0f, -1.0f, 0.0f), view));
        V3 tmp1 = normalized3(cross(view, tmp0));
        V3 tmp2 = normalized3(view);
        float hist[18];
        for (int k = 0; k < hist_size; ++k) hist[k] = 0.0f;
        float negative_score = 1.0f;
        queue.clear();
        queue.push_back(index);
        touched[(size_t)index] = 1;
        for (size_t qi = 0; qi < queue.size(); ++qi) {
          const int index2 = queue[qi];
          if (!ri.isValidIdx(index2)) continue;
          if (B.traits[(size_t)index2] & (bit(SHADOW_BORDER) | bit(VEIL_POINT))) continue;
          const int y2 = index2 / w, x2 = index2 - y2 * w;
          const P4 point2 = ri.pts[(size_t)index2];
          const float pixelDistance = (float)std::max(std::abs(x2 - x), std::abs(y2 - y));
          const float distance_squared = sqDist(point, point2);
          if (alt(kAltGrowOr) ? (pixelDistance > 2.0f || distance_squared > radius_squared)
                              : (pixelDistance > 2.0f && distance_squared > radius_squared))
            continue;
          for (int y3 = std::max(0, y2 - 1); y3 <= std::min(h - 1, y2 + 1); ++y3)
            for (int x3 = std::max(0, x2 - 1); x3 <= std::min(w - 1, x2 + 1); ++x3) {
              int index3 = y3 * w + x3;
              if (!touched[(size_t)index3]) { queue.push_back(index3); touched[(size_t)index3] = 1; }
            }
          const float scs = B.scs[(size_t)index2];
          if (scs < P.min_surface_change_score) continue;
          const V3 dir = B.scd[(size_t)index2];
          const float distance = std::sqrt(distance_squared);
          const float distance_factor = radius_reciprocal * distance;
          // nkdGetScores
          float neg = 1.0f - 0.5f * scs * std::max(1.0f - distance_factor / P.optimal_distance_to_high_surface_change, 0.0f);
          if (!alt(kAltNegNotSquared)) neg = neg * neg;
          const bool near = alt(kAltPosLessEq2) ? pixelDistance <= 2.0 : pixelDistance < 2.0;
          const float pos = near ? scs : scs * (1.0f - distance_factor);
          // nkdGetDirectionAngle: (rotation * direction).head<2> (), Affine3f * Vector3f (mv3 rows)
          V3 rot = v3(0.0f + mv3(tmp0, dir), 0.0f + mv3(tmp1, dir), 0.0f + mv3(tmp2, dir));
          float inv = std::sqrt(rot.x * rot.x + rot.y * rot.y);
          float dvx = rot.x * (1.0f / inv);  // Vector2f::normalize (): times the reciprocal
          float angle = 0.5f * normAngle(2.0f * acosf_glibc(dvx));
          if (alt(kAltAngleAtan2)) angle = 0.5f * normAngle(2.0f * std::atan2(rot.y * (1.0f / inv), dvx));
          float cellf = alt(kAltCellRound) ? (angle + d90) / d180 * hist_size
                                           : std::floor((angle + d90) / d180 * hist_size);
          int cell;
          if (!(cellf == cellf)) cell = 0;  // NaN -> lrint -> INT_MIN -> (int) 0
          else cell = std::min(hist_size - 1, (int)std::lrint(cellf));
          if (cell < 0) cell = 0;
          hist[cell] = std::max(hist[cell], pos);
          negative_score = std::min(negative_score, neg);
        }
        for (size_t qi = 0; qi < queue.size(); ++qi) touched[(size_t)queue[qi]] = 0;
        float acv = 0.0f;
        for (int c1 = 0; c1 < hist_size - 1; ++c1) {
          if (hist[c1] == 0.0f) continue;
          for (int c2 = c1 + 1; c2 < hist_size; ++c2) {
            if (hist[c2] == 0.0f) continue;
            float nd = 2.0f * (float)(c2 - c1) / (float)hist_size;
            nd = (nd <= 1.0f ? nd : 2.0f - nd);
            acv = std::max(hist[c1] * hist[c2] * nd, acv);
          }
        }
        if (!alt(kAltAcvNoSqrt)) acv = std::sqrt(acv);
        interest[(size_t)index] = negative_score * acv;
      }
  }
}

// Reconstruction (confidence L) of PCL 1.7's NarfKeypoint::calculateSparseInterestImage, the
// mode PCL's default Parameters (calculate_sparse_interest_image = true) select.  Its source
// (keypoints/src/narf_keypoint.cpp) is not in this container and the NARF paper does not describe
// it; the header documents it as "some heuristics to decide which areas of the interest image can
// be left out".  What is restated here is the increased-radius scheme its locals name
// (increased_radius = 1.5 R, radius_overhead = increased_radius - R, neighbours within the
// overhead): pixels are visited in raster order; a visited pixel p grows its region with the
// acceptance widened to the increased radius, computes its own interest exactly as the complete
// formula does (contributions only from pixels within pixel distance 2 or within R of p, but
// reached through the widened region), and bounds the interest of every pixel within the overhead
// of p -- whose R-balls lie inside p's increased ball -- by the angle-change value of a histogram of
// the raw surface-change scores over the increased region (pos <= scs, neg <= 1).  When that bound
// is below min_interest_value those pixels are left out (interest 0, never visited).  The bound is
// heuristic (the overhead pixels' own viewer rotations and region paths differ from p's), which is
// exactly where this mode can depart from the complete one; tests/test_oracle_narf_sparse.py
// measures whether it does on the reference's clouds and the bench scans.
void interestImageSparse(const RangeImage& ri, const Border& B, const Params& P, std::vector<float>& interest) {
  const int w = ri.w, h = ri.h;
  const size_t n = (size_t)w * h;
  interest.assign(n, 0.0f);
  const float search_radius = 0.5f * P.support_size, radius_squared = search_radius * search_radius,
              radius_reciprocal = 1.0f / search_radius, increased_radius = 1.5f * search_radius,
              increased_radius_squared = increased_radius * increased_radius,
              radius_overhead = increased_radius - search_radius,
              radius_overhead_squared = radius_overhead * radius_overhead;
  const int hist_size = 18;
  const float deg = 0.017453292519943295769236907684886127134428718885417f;
  const float d90 = 90.0f * deg, d180 = 180.0f * deg;
  const V3 sensor = ri.sensorPos();
  std::vector<char> touched(n, 0), done(n, 0);
  std::vector<int> queue, overhead;
  auto acv_of = [&](const float* hist) {
    float acv = 0.0f;
    for (int c1 = 0; c1 < hist_size - 1; ++c1) {
      if (hist[c1] == 0.0f) continue;
      for (int c2 = c1 + 1; c2 < hist_size; ++c2) {
        if (hist[c2] == 0.0f) continue;
        float nd = 2.0f * (float)(c2 - c1) / (float)hist_size;
        nd = (nd <= 1.0f ? nd : 2.0f - nd);
        acv = std::max(hist[c1] * hist[c2] * nd, acv);
      }
    }
    return std::sqrt(acv);
  };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int index = y * w + x;
      if (done[(size_t)index]) continue;
      if (!ri.isValidIdx(index)) continue;
      if (B.traits[(size_t)index] & (bit(SHADOW_BORDER) | bit(VEIL_POINT))) continue;
      done[(size_t)index] = 1;
      const P4 point = ri.pts[(size_t)index];
      V3 view = normalized3(sub(v3(point.x, point.y, point.z), sensor));
      V3 tmp0 = normalized3(cross(v3(0.0f, -1.0f, 0.0f), view));
      V3 tmp1 = normalized3(cross(view, tmp0));
      V3 tmp2 = normalized3(view);
      float hist[18], bound_hist[18];
      for (int k = 0; k < hist_size; ++k) hist[k] = bound_hist[k] = 0.0f;
      float negative_score = 1.0f;
      queue.clear();
      overhead.clear();
      queue.push_back(index);
      touched[(size_t)index] = 1;
      for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int index2 = queue[qi];
        if (!ri.isValidIdx(index2)) continue;
        if (B.traits[(size_t)index2] & (bit(SHADOW_BORDER) | bit(VEIL_POINT))) continue;
        const int y2 = index2 / w, x2 = index2 - y2 * w;
        const P4 point2 = ri.pts[(size_t)index2];
        const float pixelDistance = (float)std::max(std::abs(x2 - x), std::abs(y2 - y));
        const float distance_squared = sqDist(point, point2);
        if (pixelDistance > 2.0f && distance_squared > increased_radius_squared) continue;
        for (int y3 = std::max(0, y2 - 1); y3 <= std::min(h - 1, y2 + 1); ++y3)
          for (int x3 = std::max(0, x2 - 1); x3 <= std::min(w - 1, x2 + 1); ++x3) {
            int index3 = y3 * w + x3;
            if (!touched[(size_t)index3]) { queue.push_back(index3); touched[(size_t)index3] = 1; }
          }
        if (distance_squared <= radius_overhead_squared) overhead.push_back(index2);
        const float scs = B.scs[(size_t)index2];
        if (scs < P.min_surface_change_score) continue;
        const V3 dir = B.scd[(size_t)index2];
        V3 rot = v3(0.0f + mv3(tmp0, dir), 0.0f + mv3(tmp1, dir), 0.0f + mv3(tmp2, dir));
        float inv = std::sqrt(rot.x * rot.x + rot.y * rot.y);
        float dvx = rot.x * (1.0f / inv);
        float angle = 0.5f * normAngle(2.0f * acosf_glibc(dvx));
        float cellf = std::floor((angle + d90) / d180 * hist_size);
        int cell;
        if (!(cellf == cellf)) cell = 0;
        else cell = std::min(hist_size - 1, (int)std::lrint(cellf));
        if (cell < 0) cell = 0;
        bound_hist[cell] = std::max(bound_hist[cell], scs);
        if (pixelDistance > 2.0f && distance_squared > radius_squared) continue;  // not in p's own region
        const float distance_factor = radius_reciprocal * std::sqrt(distance_squared);
        float neg = 1.0f - 0.5f * scs * std::max(1.0f - distance_factor / P.optimal_distance_to_high_surface_change, 0.0f);
        neg = neg * neg;
        const float pos = (pixelDistance < 2.0) ? scs : scs * (1.0f - distance_factor);
        hist[cell] = std::max(hist[cell], pos);
        negative_score = std::min(negative_score, neg);
      }
      for (size_t qi = 0; qi < queue.size(); ++qi) touched[(size_t)queue[qi]] = 0;
      interest[(size_t)index] = negative_score * acv_of(hist);
      if (acv_of(bound_hist) < P.min_interest_value)
        for (size_t k = 0; k < overhead.size(); ++k) done[(size_t)overhead[k]] = 1;
    }
}

// Second reading of the same locals (confidence L): one region grow to the increased radius
// around a seed p serves every not yet computed pixel q within the overhead of p (q's R-ball lies
// inside the grown ball), whose interest is then formed from the seed's contributor list (the
// complete formula's acceptance -- pixel distance <= 2 or distance <= R -- measured from q, but
// the connectivity of the seed's region); seeds in raster order.  params[7] = 3.
void interestImageSeeded(const RangeImage& ri, const Border& B, const Params& P, std::vector<float>& interest) {
  const int w = ri.w, h = ri.h;
  const size_t n = (size_t)w * h;
  interest.assign(n, 0.0f);
  const float search_radius = 0.5f * P.support_size, radius_squared = search_radius * search_radius,
              radius_reciprocal = 1.0f / search_radius, increased_radius = 1.5f * search_radius,
              increased_radius_squared = increased_radius * increased_radius,
              radius_overhead = increased_radius - search_radius,
              radius_overhead_squared = radius_overhead * radius_overhead;
  const int hist_size = 18;
  const float deg = 0.017453292519943295769236907684886127134428718885417f;
  const float d90 = 90.0f * deg, d180 = 180.0f * deg;
  const V3 sensor = ri.sensorPos();
  std::vector<char> touched(n, 0), done(n, 0);
  std::vector<int> queue, overhead, contrib;
  auto usable = [&](int i) {
    return ri.isValidIdx(i) && !(B.traits[(size_t)i] & (bit(SHADOW_BORDER) | bit(VEIL_POINT)));
  };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int index = y * w + x;
      if (done[(size_t)index] || !usable(index)) continue;
      const P4 point = ri.pts[(size_t)index];
      queue.clear();
      overhead.clear();
      contrib.clear();
      queue.push_back(index);
      touched[(size_t)index] = 1;
      for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int index2 = queue[qi];
        if (!usable(index2)) continue;
        const int y2 = index2 / w, x2 = index2 - y2 * w;
        const float pixelDistance = (float)std::max(std::abs(x2 - x), std::abs(y2 - y));
        const float distance_squared = sqDist(point, ri.pts[(size_t)index2]);
        if (pixelDistance > 2.0f && distance_squared > increased_radius_squared) continue;
        for (int y3 = std::max(0, y2 - 1); y3 <= std::min(h - 1, y2 + 1); ++y3)
          for (int x3 = std::max(0, x2 - 1); x3 <= std::min(w - 1, x2 + 1); ++x3) {
            int index3 = y3 * w + x3;
            if (!touched[(size_t)index3]) { queue.push_back(index3); touched[(size_t)index3] = 1; }
          }
        if (distance_squared <= radius_overhead_squared && !done[(size_t)index2]) overhead.push_back(index2);
        if (B.scs[(size_t)index2] >= P.min_surface_change_score) contrib.push_back(index2);
      }
      for (size_t qi = 0; qi < queue.size(); ++qi) touched[(size_t)queue[qi]] = 0;
      for (size_t oi = 0; oi < overhead.size(); ++oi) {
        const int iq = overhead[oi];
        const int yq = iq / w, xq = iq - yq * w;
        const P4 pq = ri.pts[(size_t)iq];
        V3 view = normalized3(sub(v3(pq.x, pq.y, pq.z), sensor));
        V3 tmp0 = normalized3(cross(v3(0.0f, -1.0f, 0.0f), view));
        V3 tmp1 = normalized3(cross(view, tmp0));
        V3 tmp2 = normalized3(view);
        float hist[18];
        for (int k = 0; k < hist_size; ++k) hist[k] = 0.0f;
        float negative_score = 1.0f;
        for (size_t ci = 0; ci < contrib.size(); ++ci) {
          const int is = contrib[ci];
          const int ys = is / w, xs = is - ys * w;
          const float pixelDistance = (float)std::max(std::abs(xs - xq), std::abs(ys - yq));
          const float distance_squared = sqDist(pq, ri.pts[(size_t)is]);
          if (pixelDistance > 2.0f && distance_squared > radius_squared) continue;
          const float scs = B.scs[(size_t)is];
          const V3 dir = B.scd[(size_t)is];
          const float distance_factor = radius_reciprocal * std::sqrt(distance_squared);
          float neg = 1.0f - 0.5f * scs * std::max(1.0f - distance_factor / P.optimal_distance_to_high_surface_change, 0.0f);
          neg = neg * neg;
          const float pos = (pixelDistance < 2.0) ? scs : scs * (1.0f - distance_factor);
          V3 rot = v3(0.0f + mv3(tmp0, dir), 0.0f + mv3(tmp1, dir), 0.0f + mv3(tmp2, dir));
          float inv = std::sqrt(rot.x * rot.x + rot.y * rot.y);
          float dvx = rot.x * (1.0f / inv);
          float angle = 0.5f * normAngle(2.0f * acosf_glibc(dvx));
          float cellf = std::floor((angle + d90) / d180 * hist_size);
          int cell;
          if (!(cellf == cellf)) cell = 0;
          else cell = std::min(hist_size - 1, (int)std::lrint(cellf));
          if (cell < 0) cell = 0;
          hist[cell] = std::max(hist[cell], pos);
          negative_score = std::min(negative_score, neg);
        }
        float acv = 0.0f;
        for (int c1 = 0; c1 < hist_size - 1; ++c1) {
          if (hist[c1] == 0.0f) continue;
          for (int c2 = c1 + 1; c2 < hist_size; ++c2) {
            if (hist[c2] == 0.0f) continue;
            float nd = 2.0f * (float)(c2 - c1) / (float)hist_size;
            nd = (nd <= 1.0f ? nd : 2.0f - nd);
            acv = std::max(hist[c1] * hist[c2] * nd, acv);
          }
        }
        interest[(size_t)iq] = negative_score * std::sqrt(acv);
        done[(size_t)iq] = 1;
      }
    }
}

void keypoints(const RangeImage& ri, const std::vector<float>& interest, const Params& P, std::vector<int>& out) {
  const int w = ri.w, h = ri.h;
  std::vector<InterestPoint> tmp;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int index = y * w + x;
      float iv = interest[(size_t)index];
      if (iv < P.min_interest_value) continue;
      bool is_max = true;
      for (int y2 = y - 1; y2 <= y + 1 && is_max && P.do_nms; ++y2)
        for (int x2 = x - 1; x2 <= x + 1; ++x2) {
          if (!ri.inImage(x2, y2)) continue;
          if (interest[(size_t)y2 * w + x2] <= iv) continue;
          is_max = false;
          break;
        }
      if (!is_max) continue;
      const P4& p = ri.pts[(size_t)index];
      InterestPoint ip = {p.x, p.y, p.z, iv};
      tmp.push_back(ip);
    }
  std::sort(tmp.begin(), tmp.end(), isBetter);
  const float md = P.min_distance_between_interest_points * P.support_size;
  const float min_d2 = md * md;
  std::vector<InterestPoint> accepted;
  std::vector<char> mark((size_t)w * h, 0);
  for (size_t k = 0; k < tmp.size(); ++k) {
    if (P.max_no_of_interest_points > 0 && (int)accepted.size() >= P.max_no_of_interest_points) break;
    const InterestPoint& ip = tmp[k];
    bool too_close = false;
    for (size_t k2 = 0; k2 < accepted.size(); ++k2) {
      const InterestPoint& q = accepted[k2];
      V3 d = v3(ip.x - q.x, ip.y - q.y, ip.z - q.z);
      if (sqn3(d) < min_d2) { too_close = true; break; }
    }
    if (too_close) continue;
    accepted.push_back(ip);
    float xr, yr, rr;
    ri.imagePoint(v3(ip.x, ip.y, ip.z), xr, yr, rr);
    int ix = lrintf_i(xr), iy = lrintf_i(yr);
    if (ri.isValid(ix, iy)) mark[(size_t)iy * w + ix] = 1;
  }
  out.clear();
  for (int i = 0; i < w * h; ++i)
    if (mark[(size_t)i]) out.push_back(i);
}

Camera makeCamera(int w, int h, float cx, float cy, float fx, float fy, const float* pose, int frame, float noise,
                  float min_range) {
  Camera c;
  c.w = w; c.h = h; c.cx = cx; c.cy = cy; c.fx = fx; c.fy = fy;
  for (int i = 0; i < 16; ++i) c.pose[i] = pose ? pose[i] : ((i % 5 == 0) ? 1.0f : 0.0f);
  c.frame = frame; c.noise = noise; c.min_range = min_range;
  return c;
}

}  // namespace

extern "C" {

// the alternative-reading selector (test infrastructure: scripts/narf_alt_report.py only)
void orc_narf_set_alt(int mask) { g_alt = mask; }

// out: w*h*4 floats (x, y, z, range)
int orc_range_image_planar(const float* x, const float* y, const float* z, i64 n, int w, int h, float cx, float cy,
                           float fx, float fy, const float* pose, int frame, float noise, float min_range, float* out) {
  RangeImage ri;
  createRangeImage(x, y, z, n, makeCamera(w, h, cx, cy, fx, fy, pose, frame, noise, min_range), ri);
  std::memcpy(out, ri.pts.data(), sizeof(P4) * ri.pts.size());
  return 0;
}

// params: float[16] packed as in pfx_narf_params order:
//  support, max_no, min_dist, opt_dist, min_interest, min_scs, nms, sparse (2: reconstruction), poly(0), straight(0),
//  prb, prpe, prbd, min_border_prob, prpc
// debug_* optional (w*h): interest, surface change score, traits
int orc_narf_keypoints(const float* x, const float* y, const float* z, i64 n, int w, int h, float cx, float cy,
                       float fx, float fy, const float* pose, int frame, float noise, float min_range,
                       const float* params, int* out, i64 cap, i64* n_out, float* dbg_interest, float* dbg_scs,
                       uint32_t* dbg_traits, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  Params P;
  P.support_size = params[0];
  P.max_no_of_interest_points = (int)params[1];
  P.min_distance_between_interest_points = params[2];
  P.optimal_distance_to_high_surface_change = params[3];
  P.min_interest_value = params[4];
  P.min_surface_change_score = params[5];
  P.do_nms = (int)params[6];
  P.pixel_radius_borders = (int)params[10];
  P.pixel_radius_plane_extraction = (int)params[11];
  P.pixel_radius_border_direction = (int)params[12];
  P.minimum_border_probability = params[13];
  P.pixel_radius_principal_curvature = (int)params[14];
  RangeImage ri;
  createRangeImage(x, y, z, n, makeCamera(w, h, cx, cy, fx, fy, pose, frame, noise, min_range), ri);
  Border B(ri, P);
  B.run();
  std::vector<float> interest;
  // params[7]: 2 = the reconstruction of PCL's sparse traversal (interestImageSparse); 0 / 1 =
  // the complete formula (the GPU's output in either of its modes)
  if ((int)params[7] == 2) interestImageSparse(ri, B, P, interest);
  else if ((int)params[7] == 3) interestImageSeeded(ri, B, P, interest);
  else interestImage(ri, B, P, interest);
  std::vector<int> kp;
  keypoints(ri, interest, P, kp);
  *n_out = (i64)kp.size();
  for (size_t i = 0; i < kp.size() && (i64)i < cap; ++i) out[i] = kp[i];
  size_t npx = (size_t)w * h;
  if (dbg_interest) std::memcpy(dbg_interest, interest.data(), sizeof(float) * npx);
  if (dbg_scs) std::memcpy(dbg_scs, B.scs.data(), sizeof(float) * npx);
  if (dbg_traits) std::memcpy(dbg_traits, B.traits.data(), sizeof(uint32_t) * npx);
  return (i64)kp.size() > cap ? 3 : 0;
}

}  // extern "C"
