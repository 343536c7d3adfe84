// pfx_pcl.hpp -- PCL 1.7-compatible C++ facade over the libpfx C-ABI (include/pfx.h).
//
// The reference's wrapper headers call PCL's class API on the hot path and nothing else:
//   include/pcl_feature_extraction/keypoints.h:199-231  RangeImagePlanar, RangeImageBorderExtractor,
//                                                       NarfKeypoint, PointCloud<int>
//   include/pcl_feature_extraction/features.h:175-196   Feature / FeatureFromNormals (polymorphic,
//                                                       probed with dynamic_pointer_cast),
//                                                       search::KdTree, setRadiusSearch, compute
//   include/pcl_feature_extraction/tools.h:22-32        NormalEstimationOMP
//   src/evaluation.cpp:593-612, :766-785                FPFHEstimation, SHOTEstimationOMP
//   include/pcl_feature_extraction/features.h:224-273   KdTreeFLANN<FeatureT>::nearestKSearch,
//                                                       Correspondence(s), boost::thread / ref
// This header provides those names in namespace pcl (plus the minimal Eigen subset the calls
// touch), implemented on the GPU through libpfx, so the wrapper headers compile unchanged when
// this header stands in for the PCL includes.  Point types keep PCL's 16-byte-aligned layouts.
//
// Behaviour mirrors PCL 1.7: compute() never throws on algorithmic failure -- a failed
// initCompute / device error prints PCL_ERROR and leaves an empty output cloud; per-point failure
// is NaN in the row, is_dense = false.  Objects are not re-entrant; one libpfx context per
// process (device from $PFX_DEVICE, default 0), calls are synchronous on the caller's thread.
//
// Define PFX_PCL_BOOST_SHIM before including to get boost::shared_ptr / dynamic_pointer_cast
// aliases for code written against PCL 1.7's boost pointers (features.h:181-182).
#ifndef PFX_PCL_HPP_
#define PFX_PCL_HPP_

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pfx.h"

#ifndef PCL_ERROR
#define PCL_ERROR(...) std::fprintf(stderr, __VA_ARGS__)
#endif

#ifdef PFX_PCL_BOOST_SHIM
namespace boost {
using std::dynamic_pointer_cast;
using std::ref;
using std::shared_ptr;
using std::thread;  // features.h:234-239 runs the two getCorrespondences on boost::thread
}  // namespace boost
#endif

// ---- the Eigen subset used by keypoints.h:207-210 ------------------------------------------
namespace Eigen {

struct Vector3f {
  float v[3] = {0, 0, 0};
  Vector3f() = default;
  Vector3f(float x, float y, float z) : v{x, y, z} {}
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};

struct Vector4f {
  float v[4] = {0, 0, 0, 0};
  Vector4f() = default;
  Vector4f(float x, float y, float z, float w) : v{x, y, z, w} {}
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
  static Vector4f Zero() { return Vector4f(); }
};

struct Quaternionf {
  float qw = 1, qx = 0, qy = 0, qz = 0;
  Quaternionf() = default;
  Quaternionf(float w, float x, float y, float z) : qw(w), qx(x), qy(y), qz(z) {}
  static Quaternionf Identity() { return Quaternionf(); }
  float w() const { return qw; }
  float x() const { return qx; }
  float y() const { return qy; }
  float z() const { return qz; }
};

struct Translation3f {
  float t[3];
  Translation3f(float x, float y, float z) : t{x, y, z} {}
};

// 4x4 affine transform, row-major storage
struct Affine3f {
  float m[16];
  Affine3f() { setIdentity(); }
  explicit Affine3f(const Translation3f& tr) {
    setIdentity();
    m[3] = tr.t[0]; m[7] = tr.t[1]; m[11] = tr.t[2];
  }
  // Eigen's Quaternion::toRotationMatrix (unit quaternion)
  explicit Affine3f(const Quaternionf& q) {
    setIdentity();
    const float tx = 2.f * q.qx, ty = 2.f * q.qy, tz = 2.f * q.qz;
    const float twx = tx * q.qw, twy = ty * q.qw, twz = tz * q.qw;
    const float txx = tx * q.qx, txy = ty * q.qx, txz = tz * q.qx;
    const float tyy = ty * q.qy, tyz = tz * q.qy, tzz = tz * q.qz;
    m[0] = 1.f - (tyy + tzz); m[1] = txy - twz;         m[2] = txz + twy;
    m[4] = txy + twz;         m[5] = 1.f - (txx + tzz); m[6] = tyz - twx;
    m[8] = txz - twy;         m[9] = tyz + twx;         m[10] = 1.f - (txx + tyy);
  }
  static Affine3f Identity() { return Affine3f(); }
  void setIdentity() {
    for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f;
  }
  float& operator()(int r, int c) { return m[4 * r + c]; }
  float operator()(int r, int c) const { return m[4 * r + c]; }
  Affine3f operator*(const Affine3f& o) const {
    Affine3f r;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        float s = 0.f;
        for (int k = 0; k < 4; ++k) s += m[4 * i + k] * o.m[4 * k + j];
        r.m[4 * i + j] = s;
      }
    return r;
  }
};

// 4x4 float matrix (registration's getBestTransformation), row-major storage
struct Matrix4f {
  float m[16];
  Matrix4f() { setIdentity(); }
  static Matrix4f Identity() { return Matrix4f(); }
  void setIdentity() {
    for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f;
  }
  float& operator()(int r, int c) { return m[4 * r + c]; }
  float operator()(int r, int c) const { return m[4 * r + c]; }
};

}  // namespace Eigen

namespace pcl {

namespace detail {
// one libpfx context per process (thread-affine use, as PCL objects are not re-entrant)
inline pfx_ctx* context() {
  static pfx_ctx* ctx = [] {
    pfx_ctx* c = nullptr;
    const char* dev = std::getenv("PFX_DEVICE");
    if (pfx_ctx_create(dev ? std::atoi(dev) : 0, &c) != PFX_OK) {
      PCL_ERROR("[pfx_pcl] no HIP device: %s\n", c ? pfx_last_error(c) : "pfx_ctx_create failed");
      return static_cast<pfx_ctx*>(nullptr);
    }
    return c;
  }();
  return ctx;
}
inline float nanf() { return std::numeric_limits<float>::quiet_NaN(); }
// serialises calls that may come from several threads at once (features.h:234-239 queries two
// descriptor trees on two threads; a libpfx context is not re-entrant)
inline std::mutex& context_mutex() {
  static std::mutex m;
  return m;
}
}  // namespace detail

// ---- point types (PCL 1.7 layouts, 16-byte aligned) ----------------------------------------
struct alignas(16) PointXYZRGB {
  float x = 0, y = 0, z = 0, data_pad = 1.f;
  union { float rgb; uint32_t rgba = 0; };
  float pad_[3] = {0, 0, 0};
};
struct alignas(16) Normal {
  float normal_x = 0, normal_y = 0, normal_z = 0, data_pad = 0.f;
  float curvature = 0;
  float pad_[3] = {0, 0, 0};
};
struct alignas(16) PointWithRange {
  float x = 0, y = 0, z = 0, data_pad = 1.f;
  float range = 0;
  float pad_[3] = {0, 0, 0};
};
struct alignas(16) PointXYZI {
  float x = 0, y = 0, z = 0, data_pad = 1.f;
  float intensity = 0;
  float pad_[3] = {0, 0, 0};
};
struct FPFHSignature33 { float histogram[33]; };
struct SHOT352 { float descriptor[352]; float rf[9]; };
struct ReferenceFrame { float x_axis[3], y_axis[3], z_axis[3]; };

template <typename T>
class PointCloud {
 public:
  typedef std::shared_ptr<PointCloud<T> > Ptr;
  typedef std::shared_ptr<const PointCloud<T> > ConstPtr;
  std::vector<T> points;
  uint32_t width = 0, height = 1;
  bool is_dense = true;
  Eigen::Vector4f sensor_origin_ = Eigen::Vector4f(0, 0, 0, 0);
  Eigen::Quaternionf sensor_orientation_ = Eigen::Quaternionf::Identity();
  size_t size() const { return points.size(); }
  bool empty() const { return points.empty(); }
  void push_back(const T& p) { points.push_back(p); width = (uint32_t)points.size(); height = 1; }
  void resize(size_t n) { points.resize(n); width = (uint32_t)n; height = 1; }
  void clear() { points.clear(); width = 0; height = 1; }
  T& operator[](size_t i) { return points[i]; }
  const T& operator[](size_t i) const { return points[i]; }
};

namespace detail {
struct SoA {
  std::vector<float> x, y, z;
};
template <typename P>
inline SoA soa_xyz(const PointCloud<P>& c) {
  SoA s;
  const size_t n = c.size();
  s.x.resize(n); s.y.resize(n); s.z.resize(n);
  for (size_t i = 0; i < n; ++i) { s.x[i] = c.points[i].x; s.y[i] = c.points[i].y; s.z[i] = c.points[i].z; }
  return s;
}
inline SoA soa_normals(const PointCloud<Normal>& c) {
  SoA s;
  const size_t n = c.size();
  s.x.resize(n); s.y.resize(n); s.z.resize(n);
  for (size_t i = 0; i < n; ++i) {
    s.x[i] = c.points[i].normal_x; s.y[i] = c.points[i].normal_y; s.z[i] = c.points[i].normal_z;
  }
  return s;
}
inline bool ok(pfx_status st, const char* who) {
  if (st == PFX_OK) return true;
  PCL_ERROR("[pcl::%s::compute] %s\n", who, context() ? pfx_last_error(context()) : "no device");
  return false;
}
}  // namespace detail

namespace search {
// The GPU path builds its own uniform-grid index; the tree object only carries the type.
template <typename PointT>
class KdTree {
 public:
  typedef std::shared_ptr<KdTree<PointT> > Ptr;
  explicit KdTree(bool sorted = true) : sorted_(sorted) {}
  virtual ~KdTree() = default;
 private:
  bool sorted_;
};
}  // namespace search

// ---- Feature hierarchy (features.h:175-196 probes FeatureFromNormals by dynamic cast) -------
template <typename PointInT, typename PointOutT>
class Feature {
 public:
  typedef PointCloud<PointInT> PointCloudIn;
  typedef typename PointCloudIn::ConstPtr PointCloudInConstPtr;
  typedef PointCloud<PointOutT> PointCloudOut;
  typedef std::shared_ptr<Feature<PointInT, PointOutT> > Ptr;
  typedef typename search::KdTree<PointInT>::Ptr KdTreePtr;
  virtual ~Feature() = default;
  void setInputCloud(const PointCloudInConstPtr& cloud) { input_ = cloud; }
  void setSearchSurface(const PointCloudInConstPtr& cloud) { surface_ = cloud; }
  void setSearchMethod(const KdTreePtr& tree) { tree_ = tree; }
  void setRadiusSearch(double r) { search_radius_ = r; }
  void setKSearch(int k) { k_ = k; }
  double getRadiusSearch() const { return search_radius_; }
  // Feature::compute: initCompute -> computeFeature -> deinitCompute
  void compute(PointCloudOut& output) {
    output.clear();
    if (!input_ || input_->empty() || k_ != 0 || !(search_radius_ > 0.0)) {
      PCL_ERROR("[pcl::%s::compute] initCompute failed (needs an input cloud and a radius; "
                "k-NN search is not on the accelerated path)\n", name_.c_str());
      return;
    }
    if (!detail::context()) return;
    computeFeature(output);
  }

 protected:
  virtual void computeFeature(PointCloudOut& output) = 0;
  const PointCloudIn& surface() const { return surface_ ? *surface_ : *input_; }
  bool input_is_surface() const { return !surface_ || surface_.get() == input_.get(); }
  std::string name_ = "Feature";
  PointCloudInConstPtr input_, surface_;
  KdTreePtr tree_;
  double search_radius_ = 0.0;
  int k_ = 0;
};

template <typename PointInT, typename PointNT, typename PointOutT>
class FeatureFromNormals : public Feature<PointInT, PointOutT> {
 public:
  typedef typename PointCloud<PointNT>::ConstPtr PointCloudNConstPtr;
  typedef std::shared_ptr<FeatureFromNormals<PointInT, PointNT, PointOutT> > Ptr;
  void setInputNormals(const PointCloudNConstPtr& normals) { normals_ = normals; }

 protected:
  PointCloudNConstPtr normals_;
};

// NormalEstimationOMP<In, Normal> (tools.h:22-32): viewpoint (0,0,0) unless set
template <typename PointInT, typename PointOutT>
class NormalEstimationOMP : public Feature<PointInT, PointOutT> {
 public:
  explicit NormalEstimationOMP(unsigned int /*nr_threads*/ = 0) { this->name_ = "NormalEstimationOMP"; }
  void setViewPoint(float vx, float vy, float vz) { vp_[0] = vx; vp_[1] = vy; vp_[2] = vz; }
  void setNumberOfThreads(unsigned int) {}

 protected:
  void computeFeature(PointCloud<PointOutT>& out) override {
    const PointCloud<PointInT>& in = *this->input_;
    if (!this->input_is_surface()) {
      PCL_ERROR("[pcl::NormalEstimationOMP::compute] a search surface other than the input is not on "
                "the accelerated path\n");
      return;
    }
    const detail::SoA s = detail::soa_xyz(in);
    const size_t n = in.size();
    std::vector<float> nx(n), ny(n), nz(n), cv(n);
    if (!detail::ok(pfx_normals(detail::context(), s.x.data(), s.y.data(), s.z.data(), (int64_t)n,
                                this->search_radius_, vp_, nx.data(), ny.data(), nz.data(), cv.data()),
                    "NormalEstimationOMP"))
      return;
    out.resize(n);
    out.is_dense = true;
    for (size_t i = 0; i < n; ++i) {
      out.points[i].normal_x = nx[i]; out.points[i].normal_y = ny[i];
      out.points[i].normal_z = nz[i]; out.points[i].curvature = cv[i];
      if (std::isnan(nx[i])) out.is_dense = false;
    }
  }
  float vp_[3] = {0.f, 0.f, 0.f};
};

// FPFHEstimation<In, Normal, FPFHSignature33> (evaluation.cpp:597)
template <typename PointInT, typename PointNT, typename PointOutT = FPFHSignature33>
class FPFHEstimation : public FeatureFromNormals<PointInT, PointNT, PointOutT> {
 public:
  typedef std::shared_ptr<FPFHEstimation<PointInT, PointNT, PointOutT> > Ptr;
  FPFHEstimation() { this->name_ = "FPFHEstimation"; }

 protected:
  void computeFeature(PointCloud<PointOutT>& out) override {
    const PointCloud<PointInT>& surf = this->surface();
    if (!this->normals_ || this->normals_->size() != surf.size()) {
      PCL_ERROR("[pcl::FPFHEstimation::compute] normals missing or not matching the surface\n");
      return;
    }
    const detail::SoA s = detail::soa_xyz(surf), nrm = detail::soa_normals(*this->normals_);
    const detail::SoA q = detail::soa_xyz(*this->input_);
    const size_t nq = this->input_->size();
    std::vector<float> h(nq * 33);
    if (!detail::ok(pfx_fpfh(detail::context(), s.x.data(), s.y.data(), s.z.data(), nrm.x.data(), nrm.y.data(),
                             nrm.z.data(), (int64_t)surf.size(), q.x.data(), q.y.data(), q.z.data(), (int64_t)nq,
                             this->input_is_surface() ? 1 : 0, this->search_radius_, h.data()),
                    "FPFHEstimation"))
      return;
    out.resize(nq);
    out.is_dense = true;
    for (size_t i = 0; i < nq; ++i) {
      for (int b = 0; b < 33; ++b) out.points[i].histogram[b] = h[i * 33 + b];
      if (std::isnan(h[i * 33])) out.is_dense = false;
    }
  }
};

// SHOTEstimationOMP<In, Normal, SHOT352> + SHOTLocalReferenceFrameEstimation (evaluation.cpp:770)
template <typename PointInT, typename PointNT, typename PointOutT = SHOT352,
          typename PointRFT = ReferenceFrame>
class SHOTEstimationOMP : public FeatureFromNormals<PointInT, PointNT, PointOutT> {
 public:
  typedef std::shared_ptr<SHOTEstimationOMP<PointInT, PointNT, PointOutT, PointRFT> > Ptr;
  explicit SHOTEstimationOMP(unsigned int /*nr_threads*/ = 0) { this->name_ = "SHOTEstimationOMP"; }
  void setNumberOfThreads(unsigned int) {}

 protected:
  void computeFeature(PointCloud<PointOutT>& out) override {
    const PointCloud<PointInT>& surf = this->surface();
    if (!this->normals_ || this->normals_->size() != surf.size()) {
      PCL_ERROR("[pcl::SHOTEstimationOMP::compute] normals missing or not matching the surface\n");
      return;
    }
    const detail::SoA s = detail::soa_xyz(surf), nrm = detail::soa_normals(*this->normals_);
    const detail::SoA q = detail::soa_xyz(*this->input_);
    const size_t nq = this->input_->size();
    std::vector<float> d(nq * 352), rf(nq * 9);
    if (!detail::ok(pfx_shot(detail::context(), s.x.data(), s.y.data(), s.z.data(), nrm.x.data(), nrm.y.data(),
                             nrm.z.data(), (int64_t)surf.size(), q.x.data(), q.y.data(), q.z.data(), (int64_t)nq,
                             this->search_radius_, d.data(), rf.data()),
                    "SHOTEstimationOMP"))
      return;
    out.resize(nq);
    out.is_dense = true;
    for (size_t i = 0; i < nq; ++i) {
      for (int b = 0; b < 352; ++b) out.points[i].descriptor[b] = d[i * 352 + b];
      for (int b = 0; b < 9; ++b) out.points[i].rf[b] = rf[i * 9 + b];
      if (std::isnan(d[i * 352])) out.is_dense = false;
    }
  }
};

// ---- range image + NARF (keypoints.h:203-224) ---------------------------------------------
class RangeImage : public PointCloud<PointWithRange> {
 public:
  enum CoordinateFrame { CAMERA_FRAME = 0, LASER_FRAME = 1 };
  virtual ~RangeImage() = default;
};

class RangeImagePlanar : public RangeImage {
 public:
  // Keeps the SoA cloud and the camera for the accelerated NARF pass and materialises the
  // range image itself (PointWithRange per pixel, like PCL) through pfx_range_image_planar.
  template <typename PointCloudType>
  void createFromPointCloudWithFixedSize(const PointCloudType& cloud, int di_width, int di_height,
                                         float di_center_x, float di_center_y, float di_focal_length_x,
                                         float di_focal_length_y, const Eigen::Affine3f& sensor_pose,
                                         CoordinateFrame coordinate_frame = CAMERA_FRAME,
                                         float noise_level = 0.0f, float min_range = 0.0f) {
    cloud_ = detail::soa_xyz(cloud);
    pfx_camera_default(&cam_);
    cam_.width = di_width; cam_.height = di_height;
    cam_.center_x = di_center_x; cam_.center_y = di_center_y;
    cam_.focal_length_x = di_focal_length_x; cam_.focal_length_y = di_focal_length_y;
    for (int i = 0; i < 16; ++i) cam_.sensor_pose[i] = sensor_pose.m[i];
    cam_.coordinate_frame = (int32_t)coordinate_frame;
    cam_.noise_level = noise_level;
    cam_.min_range = min_range;
    width = (uint32_t)di_width;
    height = (uint32_t)di_height;
    points.clear();
    if (!detail::context()) return;
    std::vector<float> pr((size_t)di_width * di_height * 4);
    if (!detail::ok(pfx_range_image_planar(detail::context(), cloud_.x.data(), cloud_.y.data(), cloud_.z.data(),
                                           (int64_t)cloud_.x.size(), &cam_, pr.data()),
                    "RangeImagePlanar"))
      return;
    points.resize((size_t)di_width * di_height);
    for (size_t i = 0; i < points.size(); ++i) {
      points[i].x = pr[4 * i]; points[i].y = pr[4 * i + 1]; points[i].z = pr[4 * i + 2];
      points[i].range = pr[4 * i + 3];
    }
    is_dense = false;
  }
  const detail::SoA& source_cloud() const { return cloud_; }
  const pfx_camera& camera() const { return cam_; }

 private:
  detail::SoA cloud_;
  pfx_camera cam_;
};

class RangeImageBorderExtractor {
 public:
  struct Parameters {
    int pixel_radius_borders = 3;
    int pixel_radius_plane_extraction = 2;
    int pixel_radius_border_direction = 2;
    float minimum_border_probability = 0.8f;
    int pixel_radius_principal_curvature = 2;
  };
  explicit RangeImageBorderExtractor(const RangeImage* = nullptr) {}
  Parameters& getParameters() { return parameters_; }

 private:
  Parameters parameters_;
};

class NarfKeypoint {
 public:
  struct Parameters {
    float support_size = -1.0f;
    int max_no_of_interest_points = -1;
    float min_distance_between_interest_points = 0.25f;
    float optimal_distance_to_high_surface_change = 0.25f;
    float min_interest_value = 0.45f;
    float min_surface_change_score = 0.2f;
    int optimal_range_image_patch_size = 10;
    float distance_for_additional_points = 0.0f;
    bool add_points_on_straight_edges = false;
    bool do_non_maximum_suppression = true;
    int no_of_polynomial_approximations_per_point = 0;
    int max_no_of_threads = 1;
    bool use_recursive_scale_reduction = false;
    // PCL's default (true).  Both values compute the COMPLETE interest formula here (true only
    // prunes pixels that cannot reach min_interest_value: same keypoints); PCL 1.7's sparse
    // heuristics are not reproduced -- unpinned, measured sensitivity 1-2 keypoints per reference
    // cloud (pfx.h)
    bool calculate_sparse_interest_image = true;
  };
  explicit NarfKeypoint(RangeImageBorderExtractor* border_extractor = nullptr, float support_size = -1.0f)
      : border_extractor_(border_extractor) {
    parameters_.support_size = support_size;
  }
  void setRangeImage(const RangeImage* range_image) {
    range_image_ = dynamic_cast<const RangeImagePlanar*>(range_image);
  }
  Parameters& getParameters() { return parameters_; }
  // NarfKeypoint::compute: ascending pixel indices of the keypoints
  void compute(PointCloud<int>& out) {
    out.clear();
    if (!range_image_ || !(parameters_.support_size > 0.0f)) {
      PCL_ERROR("[pcl::NarfKeypoint::compute] needs a RangeImagePlanar and support_size > 0\n");
      return;
    }
    if (!detail::context()) return;
    pfx_narf_params p;
    pfx_narf_params_default(&p);
    p.support_size = parameters_.support_size;
    p.max_no_of_interest_points = parameters_.max_no_of_interest_points;
    p.min_distance_between_interest_points = parameters_.min_distance_between_interest_points;
    p.optimal_distance_to_high_surface_change = parameters_.optimal_distance_to_high_surface_change;
    p.min_interest_value = parameters_.min_interest_value;
    p.min_surface_change_score = parameters_.min_surface_change_score;
    p.do_non_maximum_suppression = parameters_.do_non_maximum_suppression ? 1 : 0;
    p.calculate_sparse_interest_image = parameters_.calculate_sparse_interest_image ? 1 : 0;
    p.no_of_polynomial_approximations_per_point = parameters_.no_of_polynomial_approximations_per_point ? 1 : 0;
    p.add_points_on_straight_edges = parameters_.add_points_on_straight_edges ? 1 : 0;
    if (border_extractor_) {
      const RangeImageBorderExtractor::Parameters& b = border_extractor_->getParameters();
      p.pixel_radius_borders = b.pixel_radius_borders;
      p.pixel_radius_plane_extraction = b.pixel_radius_plane_extraction;
      p.pixel_radius_border_direction = b.pixel_radius_border_direction;
      p.minimum_border_probability = b.minimum_border_probability;
      p.pixel_radius_principal_curvature = b.pixel_radius_principal_curvature;
    }
    const detail::SoA& c = range_image_->source_cloud();
    const pfx_camera cam = range_image_->camera();
    std::vector<int32_t> idx((size_t)cam.width * cam.height);
    int64_t k = 0;
    if (!detail::ok(pfx_narf_keypoints(detail::context(), c.x.data(), c.y.data(), c.z.data(), (int64_t)c.x.size(),
                                       &cam, &p, idx.data(), (int64_t)idx.size(), &k),
                    "NarfKeypoint"))
      return;
    out.points.assign(idx.begin(), idx.begin() + k);
    out.width = (uint32_t)k;
    out.height = 1;
  }

 private:
  RangeImageBorderExtractor* border_extractor_;
  const RangeImagePlanar* range_image_ = nullptr;
  Parameters parameters_;
};

// ---- ISS keypoints (keypoints.h:177-189) ------------------------------------------------------
// ISSKeypoint3D<In, Out, NormalT>: the reference's setters, compute() -> the keypoints' xyz in
// index order (pfx_iss_keypoints; PCL pushes them from an OpenMP loop).  A
// parameter initCompute rejects (radius, threshold or min neighbours <= 0) -> PCL_ERROR and an
// empty output.  Border radius / normals are not on the accelerated path (the reference sets
// neither).
template <typename PointInT, typename PointOutT, typename NormalT = Normal>
class ISSKeypoint3D {
 public:
  typedef typename PointCloud<PointInT>::ConstPtr PointCloudInConstPtr;
  typedef typename search::KdTree<PointInT>::Ptr KdTreePtr;
  explicit ISSKeypoint3D(double salient_radius = 0.0001) : salient_radius_(salient_radius) {}
  void setInputCloud(const PointCloudInConstPtr& cloud) { input_ = cloud; }
  void setSearchMethod(const KdTreePtr& tree) { tree_ = tree; }
  void setSalientRadius(double r) { salient_radius_ = r; }
  void setNonMaxRadius(double r) { non_max_radius_ = r; }
  void setMinNeighbors(int k) { min_neighbors_ = k; }
  void setThreshold21(double t) { gamma_21_ = t; }
  void setThreshold32(double t) { gamma_32_ = t; }
  const std::vector<int>& getKeypointsIndices() const { return indices_; }
  void compute(PointCloud<PointOutT>& output) {
    output.clear();
    indices_.clear();
    if (!input_) {
      PCL_ERROR("[pcl::ISSKeypoint3D::compute] no input cloud\n");
      return;
    }
    if (!detail::context()) return;
    const detail::SoA c = detail::soa_xyz(*input_);
    std::vector<int32_t> idx(c.x.size() + 1);
    int64_t k = 0;
    if (!detail::ok(pfx_iss_keypoints(detail::context(), c.x.data(), c.y.data(), c.z.data(), (int64_t)c.x.size(),
                                      salient_radius_, non_max_radius_, min_neighbors_, gamma_21_, gamma_32_,
                                      idx.data(), (int64_t)idx.size(), &k, nullptr),
                    "ISSKeypoint3D"))
      return;
    for (int64_t j = 0; j < k; ++j) {
      PointOutT p;
      p.x = input_->points[idx[j]].x;
      p.y = input_->points[idx[j]].y;
      p.z = input_->points[idx[j]].z;
      output.push_back(p);
      indices_.push_back(idx[j]);
    }
  }

 private:
  PointCloudInConstPtr input_;
  KdTreePtr tree_;
  double salient_radius_, non_max_radius_ = 0.0, gamma_21_ = 0.975, gamma_32_ = 0.975;
  int min_neighbors_ = 5;
  std::vector<int> indices_;
};

// Keypoints::computeCloudResolution (keypoints.h:401-428) is the reference's own helper; its
// body becomes this call (same value: see DESIGN.md, F3)
template <typename PointT>
inline double cloudResolution(const typename PointCloud<PointT>::ConstPtr& cloud) {
  if (!cloud || !detail::context()) return 0.0;
  const detail::SoA c = detail::soa_xyz(*cloud);
  double res = 0.0;
  if (!detail::ok(pfx_cloud_resolution(detail::context(), c.x.data(), c.y.data(), c.z.data(), (int64_t)c.x.size(),
                                       &res),
                  "computeCloudResolution"))
    return 0.0;
  return res;
}

// ---- HarrisKeypoint3D / HarrisKeypoint6D (keypoints.h:150-176) --------------------------------
// compute(): the corners as PCL outputs them -- refined position, intensity = the response of
// the corner's own point -- in corner (index) order (PCL: omp critical order).
// Only the reference's configuration is accelerated: method HARRIS (3D) with non-maximum
// suppression; anything else -> PCL_ERROR + empty output.  The radius defaults to PCL's 0.01.
namespace detail {
template <typename PointOutT, typename PointInT>
inline void harris_output(const PointCloud<PointInT>& in, const std::vector<float>& resp,
                          const std::vector<float>& corners, const std::vector<int32_t>& cidx, int64_t nc,
                          PointCloud<PointOutT>& out) {
  for (int64_t c = 0; c < nc; ++c) {
    PointOutT p;
    p.x = corners[3 * c];
    p.y = corners[3 * c + 1];
    p.z = corners[3 * c + 2];
    p.intensity = resp[(size_t)cidx[c]];
    out.push_back(p);
  }
  (void)in;
  out.is_dense = true;
}
}  // namespace detail

template <typename PointInT, typename PointOutT, typename NormalT = Normal>
class HarrisKeypoint3D {
 public:
  typedef typename PointCloud<PointInT>::ConstPtr PointCloudInConstPtr;
  enum ResponseMethod { HARRIS = 1, NOBLE, LOWE, TOMASI, CURVATURE };
  explicit HarrisKeypoint3D(ResponseMethod method = HARRIS, float radius = 0.01f, float threshold = 0.0f)
      : method_(method), radius_(radius), threshold_(threshold) {}
  void setInputCloud(const PointCloudInConstPtr& cloud) { input_ = cloud; }
  void setMethod(ResponseMethod m) { method_ = m; }
  void setRadius(float r) { radius_ = r; }
  void setRadiusSearch(double r) { radius_ = (float)r; }
  void setThreshold(float t) { threshold_ = t; }
  void setNonMaxSupression(bool b) { nonmax_ = b; }
  void setRefine(bool b) { refine_ = b; }
  void compute(PointCloud<PointOutT>& output) {
    output.clear();
    if (!input_) {
      PCL_ERROR("[pcl::HarrisKeypoint3D::compute] no input cloud\n");
      return;
    }
    if (method_ != HARRIS || !nonmax_) {
      PCL_ERROR("[pcl::HarrisKeypoint3D::compute] only method HARRIS with non-maximum suppression is accelerated\n");
      return;
    }
    if (!detail::context()) return;
    const detail::SoA c = detail::soa_xyz(*input_);
    const size_t n = c.x.size();
    std::vector<int32_t> idx(n + 1), cidx(n + 1);
    std::vector<float> resp(n + 1), corners(3 * (n + 1));
    int64_t k = 0, nc = 0;
    if (!detail::ok(pfx_harris3d_keypoints(detail::context(), c.x.data(), c.y.data(), c.z.data(), (int64_t)n, radius_,
                                           threshold_, 1, refine_ ? 1 : 0, idx.data(), (int64_t)n + 1, &k, resp.data(),
                                           corners.data(), &nc, cidx.data()),
                    "HarrisKeypoint3D"))
      return;
    detail::harris_output(*input_, resp, corners, cidx, nc, output);
  }

 private:
  PointCloudInConstPtr input_;
  ResponseMethod method_;
  float radius_, threshold_;
  bool nonmax_ = false, refine_ = true;
};

// HarrisKeypoint6D<PointXYZRGB, ...>: the colour intensity comes from the points' rgb field
template <typename PointInT, typename PointOutT, typename NormalT = Normal>
class HarrisKeypoint6D {
 public:
  typedef typename PointCloud<PointInT>::ConstPtr PointCloudInConstPtr;
  explicit HarrisKeypoint6D(float radius = 0.01f, float threshold = 0.0f) : radius_(radius), threshold_(threshold) {}
  void setInputCloud(const PointCloudInConstPtr& cloud) { input_ = cloud; }
  void setRadius(float r) { radius_ = r; }
  void setRadiusSearch(double r) { radius_ = (float)r; }
  void setThreshold(float t) { threshold_ = t; }
  void setNonMaxSupression(bool b) { nonmax_ = b; }
  void setRefine(bool b) { refine_ = b; }
  void compute(PointCloud<PointOutT>& output) {
    output.clear();
    if (!input_) {
      PCL_ERROR("[pcl::HarrisKeypoint6D::compute] no input cloud\n");
      return;
    }
    if (!nonmax_) {
      PCL_ERROR("[pcl::HarrisKeypoint6D::compute] only non-maximum suppression is accelerated\n");
      return;
    }
    if (!detail::context()) return;
    const detail::SoA c = detail::soa_xyz(*input_);
    const size_t n = c.x.size();
    std::vector<uint32_t> rgb(n + 1);
    for (size_t i = 0; i < n; ++i) rgb[i] = input_->points[i].rgba & 0x00ffffffu;
    std::vector<int32_t> idx(n + 1), cidx(n + 1);
    std::vector<float> resp(n + 1), corners(3 * (n + 1));
    int64_t k = 0, nc = 0;
    if (!detail::ok(pfx_harris6d_keypoints(detail::context(), c.x.data(), c.y.data(), c.z.data(), rgb.data(),
                                           (int64_t)n, radius_, threshold_, 1, refine_ ? 1 : 0, idx.data(),
                                           (int64_t)n + 1, &k, resp.data(), corners.data(), &nc, nullptr, cidx.data()),
                    "HarrisKeypoint6D"))
      return;
    detail::harris_output(*input_, resp, corners, cidx, nc, output);
  }

 private:
  PointCloudInConstPtr input_;
  float radius_, threshold_;
  bool nonmax_ = false, refine_ = true;
};

// ---- descriptor matching (features.h:224-273) ------------------------------------------------
struct Correspondence {
  int index_query = 0;
  int index_match = -1;
  float distance = std::numeric_limits<float>::max();
  Correspondence() = default;
  Correspondence(int q, int m, float d) : index_query(q), index_match(m), distance(d) {}
};
typedef std::vector<Correspondence> Correspondences;
typedef std::shared_ptr<Correspondences> CorrespondencesPtr;
typedef std::shared_ptr<const Correspondences> CorrespondencesConstPtr;

namespace detail {
// DefaultFeatureRepresentation: the compared floats of a descriptor and the point stride
template <typename T> struct DescriptorLayout;
template <> struct DescriptorLayout<FPFHSignature33> { static constexpr int dim = 33, stride = 33; };
template <> struct DescriptorLayout<SHOT352> { static constexpr int dim = 352, stride = 361; };
}  // namespace detail

// KdTreeFLANN<FeatureT> with nearestKSearch(k = 1), as the reference uses it (features.h:258-272):
// exact 1-NN under FLANN's L2_Simple on the GPU (pfx_nearest_descriptors).  The reference asks
// one source row at a time; the first query of a source cloud answers all its rows in one GPU
// pass and the following calls read that batch (the cloud must not change in between, as with
// the reference's loop).  A row without a match (non-finite values: undefined in FLANN) returns
// 0 neighbours with k_indices = {0}, which the mutual check of findCorrespondences rejects
// (target rows never match a non-finite source row).
template <typename PointT>
class KdTreeFLANN {
 public:
  typedef typename PointCloud<PointT>::ConstPtr PointCloudConstPtr;
  typedef std::shared_ptr<KdTreeFLANN<PointT> > Ptr;
  explicit KdTreeFLANN(bool sorted = true) : sorted_(sorted) {}
  void setInputCloud(const PointCloudConstPtr& cloud) {
    target_ = cloud;
    batch_src_ = nullptr;
  }
  int nearestKSearch(const PointCloud<PointT>& cloud, int index, int k, std::vector<int>& k_indices,
                     std::vector<float>& k_sqr_distances) const {
    if (k != 1 || !target_ || index < 0 || (size_t)index >= cloud.size()) {
      PCL_ERROR("[pcl::KdTreeFLANN::nearestKSearch] only k = 1 over a set input cloud is accelerated\n");
      return 0;
    }
    if (batch_src_ != &cloud || batch_n_ != cloud.size()) {
      idx_.assign(cloud.size(), -1);
      dist_.assign(cloud.size(), detail::nanf());
      std::lock_guard<std::mutex> lock(detail::context_mutex());
      typedef detail::DescriptorLayout<PointT> L;
      if (!detail::context() ||
          !detail::ok(pfx_nearest_descriptors(detail::context(), reinterpret_cast<const float*>(cloud.points.data()),
                                              (int64_t)cloud.size(), L::stride,
                                              reinterpret_cast<const float*>(target_->points.data()),
                                              (int64_t)target_->size(), L::stride, L::dim, idx_.data(), dist_.data()),
                      "KdTreeFLANN"))
        idx_.assign(cloud.size(), -1);
      batch_src_ = &cloud;
      batch_n_ = cloud.size();
    }
    k_indices.assign(1, idx_[index] < 0 ? 0 : idx_[index]);
    k_sqr_distances.assign(1, dist_[index]);
    return idx_[index] < 0 ? 0 : 1;
  }
  int nearestKSearch(const PointT& point, int k, std::vector<int>& k_indices, std::vector<float>& k_sqr_distances) const {
    PointCloud<PointT> one;
    one.push_back(point);
    KdTreeFLANN<PointT> tmp;
    tmp.setInputCloud(target_);
    return tmp.nearestKSearch(one, 0, k, k_indices, k_sqr_distances);
  }

 private:
  bool sorted_;
  PointCloudConstPtr target_;
  mutable const PointCloud<PointT>* batch_src_ = nullptr;
  mutable size_t batch_n_ = 0;
  mutable std::vector<int32_t> idx_;
  mutable std::vector<float> dist_;
};

// KdTreeFLANN over a point cloud (Keypoints::getKeypointsCloud, keypoints.h:374-392): exact
// nearestKSearch(k = 1) as radius searches on the GPU (pfx_radius_search) over a growing ball --
// the first non-empty ball holds the nearest point, the first entry of FLANN's (d2, index) order
template <>
class KdTreeFLANN<PointXYZRGB> {
 public:
  typedef PointCloud<PointXYZRGB>::ConstPtr PointCloudConstPtr;
  explicit KdTreeFLANN(bool sorted = true) : sorted_(sorted) {}
  void setInputCloud(const PointCloudConstPtr& cloud) {
    target_ = cloud;
    soa_ = cloud ? detail::soa_xyz(*cloud) : detail::SoA();
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = 0; i < soa_.x.size(); ++i) {
      const float p[3] = {soa_.x[i], soa_.y[i], soa_.z[i]};
      if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))) continue;
      for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], p[d]); hi[d] = std::max(hi[d], p[d]); }
    }
    extent_ = 0.0;
    for (int d = 0; d < 3; ++d) extent_ = std::max(extent_, (double)hi[d] - (double)lo[d]);
  }
  int nearestKSearch(const PointXYZRGB& point, int k, std::vector<int>& k_indices,
                     std::vector<float>& k_sqr_distances) const {
    k_indices.clear();
    k_sqr_distances.clear();
    if (k != 1 || !target_ || soa_.x.empty()) {
      if (k != 1) PCL_ERROR("[pcl::KdTreeFLANN::nearestKSearch] only k = 1 is accelerated\n");
      return 0;
    }
    if (!(std::isfinite(point.x) && std::isfinite(point.y) && std::isfinite(point.z)) || !detail::context())
      return 0;
    std::lock_guard<std::mutex> lock(detail::context_mutex());
    const float qx = point.x, qy = point.y, qz = point.z;
    // the ball must reach the farthest point of the cloud's box: its diagonal from any point in it
    const double limit = 4.0 * (extent_ + std::fabs((double)qx) + std::fabs((double)qy) + std::fabs((double)qz)) + 1.0;
    for (double r = 0.01; r <= limit; r *= 4.0) {
      int64_t cnt = 0;
      int32_t idx = -1;
      float d2 = 0.f;
      if (!detail::ok(pfx_radius_search(detail::context(), soa_.x.data(), soa_.y.data(), soa_.z.data(),
                                        (int64_t)soa_.x.size(), &qx, &qy, &qz, 1, r, &cnt, &idx, &d2, 1),
                      "KdTreeFLANN"))
        return 0;
      if (cnt > 0) {
        k_indices.assign(1, idx);
        k_sqr_distances.assign(1, d2);
        return 1;
      }
    }
    return 0;
  }

 private:
  bool sorted_;
  PointCloudConstPtr target_;
  detail::SoA soa_;
  double extent_ = 0.0;
};

// ---- RANSAC correspondence rejection (features.h:282-297) -------------------------------------
namespace registration {
// CorrespondenceRejectorSampleConsensus<PointT>: PCL's fixed-seed sample sequence and adaptive
// stop, every hypothesis scored on the GPU (pfx_ransac_rejector)
template <typename PointT>
class CorrespondenceRejectorSampleConsensus {
 public:
  typedef typename PointCloud<PointT>::ConstPtr PointCloudConstPtr;
  void setInputSource(const PointCloudConstPtr& c) { source_ = c; }
  void setInputTarget(const PointCloudConstPtr& c) { target_ = c; }
  void setInputCorrespondences(const CorrespondencesConstPtr& c) { input_ = c; }
  void setInlierThreshold(double t) { threshold_ = t; }
  void setMaximumIterations(int n) { max_iterations_ = n; }
  double getInlierThreshold() const { return threshold_; }
  int getMaximumIterations() const { return max_iterations_; }
  Eigen::Matrix4f getBestTransformation() const { return best_; }
  // CorrespondenceRejector::getCorrespondences -> applyRejection(correspondences)
  void getCorrespondences(Correspondences& out) {
    out.clear();
    best_.setIdentity();
    if (!input_ || !source_ || !target_) {
      PCL_ERROR("[pcl::registration::CorrespondenceRejectorSampleConsensus::getCorrespondences] no input\n");
      return;
    }
    getRemainingCorrespondences(*input_, out);
  }
  void getRemainingCorrespondences(const Correspondences& original, Correspondences& remaining) {
    remaining.clear();
    best_.setIdentity();
    if (!source_ || !target_ || !detail::context()) return;
    const detail::SoA s = detail::soa_xyz(*source_), t = detail::soa_xyz(*target_);
    const size_t n = original.size();
    std::vector<int32_t> q(n + 1), m(n + 1), keep(n + 1);
    for (size_t i = 0; i < n; ++i) {
      q[i] = original[i].index_query;
      m[i] = original[i].index_match;
    }
    int64_t nk = 0;
    float T[16];
    std::lock_guard<std::mutex> lock(detail::context_mutex());
    if (!detail::ok(pfx_ransac_rejector(detail::context(), s.x.data(), s.y.data(), s.z.data(), (int64_t)s.x.size(),
                                        t.x.data(), t.y.data(), t.z.data(), (int64_t)t.x.size(), q.data(), m.data(),
                                        (int64_t)n, threshold_, max_iterations_, keep.data(), &nk, T),
                    "CorrespondenceRejectorSampleConsensus"))
      return;
    for (int64_t j = 0; j < nk; ++j) remaining.push_back(original[(size_t)keep[j]]);
    for (int i = 0; i < 16; ++i) best_.m[i] = T[i];
  }

 private:
  PointCloudConstPtr source_, target_;
  CorrespondencesConstPtr input_;
  double threshold_ = 0.05;
  int max_iterations_ = 1000;
  Eigen::Matrix4f best_;
};
}  // namespace registration

}  // namespace pcl

#endif  // PFX_PCL_HPP_
