// facade_driver.cpp -- the reference's NARF / ISS / Harris + Features flow written against
// include/pfx_pcl.hpp.
//
// Mirrors, call for call, include/pcl_feature_extraction/keypoints.h:199-231 (NARF branch),
// features.h:175-196 (Features<T>::compute with the FeatureFromNormals probe) and tools.h:22-32
// (estimateNormals), as src/evaluation.cpp:593-612 / :766-785 drive them.  Reads a PCL 1.7 binary
// PCD (x y z rgb, 16 B per point), writes raw float/int arrays for tests/test_facade.py:
//   facade_driver <cloud.pcd> <out_dir> [<target.pcd>]
//   -> keypoints.i32, normals.f32 (n x 4), fpfh.f32 (K x 33), shot.f32 (K x 352), shot_rf.f32 (K x 9)
//   with a target cloud also: fpfh_target.f32 and corr.i32 (index_query, index_match pairs) of
//   features.h:224-273 (findCorrespondences / getCorrespondences, verbatim below), then
//   features.h:282-297 (filterCorrespondences) -> filtered.i32, transformation.f32; and the
//   Harris3D / Harris6D branches (keypoints.h:150-176 + getKeypointsCloud keypoints.h:365-395)
//   -> harris{3,6}d_xyz.f32 (snapped cloud points), harris{3,6}d_corners.f32 (x, y, z, intensity).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#define PFX_PCL_BOOST_SHIM
#include "pfx_pcl.hpp"

using namespace pcl;
typedef PointXYZRGB PointRGB;
typedef PointCloud<PointRGB> PointCloudRGB;

static bool read_pcd(const char* path, PointCloudRGB& c) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string line;
  size_t n = 0;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string key;
    ss >> key;
    if (key == "POINTS") ss >> n;
    if (key == "DATA") {
      std::string kind;
      ss >> kind;
      if (kind != "binary") return false;
      break;
    }
  }
  std::vector<float> raw(n * 4);
  f.read(reinterpret_cast<char*>(raw.data()), (std::streamsize)(raw.size() * sizeof(float)));
  if (!f) return false;
  c.points.resize(n);
  for (size_t i = 0; i < n; ++i) {
    c.points[i].x = raw[4 * i]; c.points[i].y = raw[4 * i + 1]; c.points[i].z = raw[4 * i + 2];
    c.points[i].rgb = raw[4 * i + 3];
  }
  c.width = (uint32_t)n;
  c.height = 1;
  return true;
}

template <typename T>
static void dump(const std::string& path, const T* p, size_t count) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (f) { std::fwrite(p, sizeof(T), count, f); std::fclose(f); }
}

// features.h:224-273, Features<FeatureType>::findCorrespondences / getCorrespondences, verbatim
// apart from the class scaffolding (boost::thread / boost::ref through PFX_PCL_BOOST_SHIM)
template <typename FeatureType>
struct Features {
  void findCorrespondences(typename PointCloud<FeatureType>::Ptr source,
                           typename PointCloud<FeatureType>::Ptr target,
                           CorrespondencesPtr& correspondences)
  {
    std::vector<int> source2target;
    std::vector<int> target2source;

    boost::thread thread1(&Features::getCorrespondences, this, boost::ref(source), boost::ref(target), boost::ref(source2target));
    boost::thread thread2(&Features::getCorrespondences, this, boost::ref(target), boost::ref(source), boost::ref(target2source));

    // Wait until both threads have finished
    thread1.join();
    thread2.join();

    // now populate the correspondences vector
    std::vector<std::pair<unsigned, unsigned> > c;
    for (unsigned c_idx = 0; c_idx < source2target.size (); ++c_idx)
      if (target2source[source2target[c_idx]] == (int)c_idx)
        c.push_back(std::make_pair(c_idx, source2target[c_idx]));

    correspondences->resize(c.size());
    for (unsigned c_idx = 0; c_idx < c.size(); ++c_idx)
    {
      (*correspondences)[c_idx].index_query = c[c_idx].first;
      (*correspondences)[c_idx].index_match = c[c_idx].second;
    }
  }

  void getCorrespondences(typename PointCloud<FeatureType>::Ptr source,
                          typename PointCloud<FeatureType>::Ptr target,
                          std::vector<int>& source2target)
  {
    const int k = 1;
    std::vector<int> k_indices(k);
    std::vector<float> k_dist(k);
    source2target.clear();
    KdTreeFLANN<FeatureType> descriptor_kdtree;

    // Find the index of the best match for each keypoint
    // From source to target
    descriptor_kdtree.setInputCloud(target);
    source2target.resize(source->size());
    for (size_t i = 0; i < source->size(); ++i)
    {
      descriptor_kdtree.nearestKSearch(*source, i, k, k_indices, k_dist);
      source2target[i] = k_indices[0];
    }
  }
};

// tools.h:22-32
static void estimateNormals(const PointCloudRGB::Ptr& cloud, PointCloud<Normal>::Ptr& normals, double radius) {
  NormalEstimationOMP<PointRGB, Normal> normal_estimation_omp;
  normal_estimation_omp.setInputCloud(cloud);
  normal_estimation_omp.setRadiusSearch(radius);
  search::KdTree<PointRGB>::Ptr kdtree_omp(new search::KdTree<PointRGB>);
  normal_estimation_omp.setSearchMethod(kdtree_omp);
  normal_estimation_omp.compute(*normals);
}

// features.h:175-196
template <typename FeatureType>
static void features_compute(typename Feature<PointRGB, FeatureType>::Ptr feature_extractor, double feat_radius,
                             double normal_radius, const PointCloudRGB::Ptr cloud,
                             const PointCloudRGB::Ptr keypoints, typename PointCloud<FeatureType>::Ptr& descriptors,
                             PointCloud<Normal>::Ptr* normals_out = nullptr) {
  typename FeatureFromNormals<PointRGB, Normal, FeatureType>::Ptr feature_from_normals =
      boost::dynamic_pointer_cast<FeatureFromNormals<PointRGB, Normal, FeatureType> >(feature_extractor);
  if (feature_from_normals) {
    PointCloud<Normal>::Ptr normals(new PointCloud<Normal>);
    estimateNormals(cloud, normals, normal_radius);
    feature_from_normals->setInputNormals(normals);
    if (normals_out) *normals_out = normals;
  }
  feature_extractor->setSearchSurface(cloud);
  feature_extractor->setInputCloud(keypoints);
  search::KdTree<PointRGB>::Ptr kdtree(new search::KdTree<PointRGB>);
  feature_extractor->setSearchMethod(kdtree);
  feature_extractor->setRadiusSearch(feat_radius);
  feature_extractor->compute(*descriptors);
}

// keypoints.h:199-231 (NARF branch) -> the keypoint cloud (and the raw pixel indices)
static PointCloudRGB::Ptr narf_keypoints(const PointCloudRGB::Ptr& cloud, PointCloud<int>::Ptr& keypoints) {
  int image_size_x = 640, image_size_y = 480;
  float center_x = (640.0f / 2.0f), center_y = (480.0f / 2.0f);
  float focal_length_x = 525.0f;
  Eigen::Affine3f sensor_pose = Eigen::Affine3f(Eigen::Translation3f(cloud->sensor_origin_[0],
                                                                     cloud->sensor_origin_[1],
                                                                     cloud->sensor_origin_[2])) *
                                Eigen::Affine3f(cloud->sensor_orientation_);
  float noise_level = 0.0f, minimum_range = 0.0f;
  RangeImagePlanar range_image;
  range_image.createFromPointCloudWithFixedSize(*cloud, image_size_x, image_size_y, center_x, center_y,
                                                focal_length_x, focal_length_x, sensor_pose,
                                                RangeImage::CAMERA_FRAME, noise_level, minimum_range);
  keypoints.reset(new PointCloud<int>);
  RangeImageBorderExtractor border_extractor;
  NarfKeypoint detector(&border_extractor);
  detector.setRangeImage(&range_image);
  detector.getParameters().support_size = 0.2f;
  detector.compute(*keypoints);
  PointCloudRGB::Ptr cloud_keypoints(new PointCloudRGB);
  for (size_t i = 0; i < keypoints->points.size(); ++i)
    if ((size_t)keypoints->points[i] < cloud->size())  // keypoints.h:229 indexes the cloud by pixel index
      cloud_keypoints->points.push_back(cloud->points[keypoints->points[i]]);
  return cloud_keypoints;
}

// keypoints.h:401-428, Keypoints::computeCloudResolution: the reference's own helper, its body
// replaced by the libpfx call
static double computeCloudResolution(const PointCloudRGB::Ptr& cloud) { return cloudResolution<PointRGB>(cloud); }

// keypoints.h:177-189 (ISS branch), verbatim
static void iss_keypoints(const PointCloudRGB::Ptr& cloud, PointCloudRGB::Ptr& cloud_keypoints) {
  cloud_keypoints.reset(new PointCloudRGB);
    ISSKeypoint3D<PointRGB, PointRGB> detector;
    detector.setInputCloud(cloud);
    search::KdTree<PointRGB>::Ptr kdtree(new search::KdTree<PointRGB>);
    detector.setSearchMethod(kdtree);
    double resolution = computeCloudResolution(cloud);
    detector.setSalientRadius(6 * resolution);
    detector.setNonMaxRadius(4 * resolution);
    detector.setMinNeighbors(5);
    detector.setThreshold21(0.975);
    detector.setThreshold32(0.975);
    detector.compute(*cloud_keypoints);
}

// keypoints.h:365-395, Keypoints::getKeypointsCloud (the reference's own helper), against the
// facade's KdTreeFLANN<PointRGB>
static void getKeypointsCloud(const PointCloudRGB::Ptr& cloud, const PointCloud<PointXYZI>::Ptr& keypoints,
                              PointCloudRGB::Ptr& cloud_keypoints) {
  cloud_keypoints.reset(new PointCloudRGB);
  if (!cloud || !keypoints || cloud->points.empty() || keypoints->points.empty()) return;
  KdTreeFLANN<PointRGB> kdtree;
  kdtree.setInputCloud(cloud);
  for (size_t i = 0; i < keypoints->size(); ++i) {
    PointXYZI pt_tmp = keypoints->points[i];
    PointRGB pt;
    pt.x = pt_tmp.x;
    pt.y = pt_tmp.y;
    pt.z = pt_tmp.z;
    if (!std::isfinite(pt.x) || !std::isfinite(pt.y) || !std::isfinite(pt.z)) continue;
    std::vector<int> idx_vec;
    std::vector<float> dist;
    if (kdtree.nearestKSearch(pt, 1, idx_vec, dist) > 0) {
      if (dist[0] < 0.0001) cloud_keypoints->points.push_back(cloud->points[idx_vec[0]]);
    }
  }
}

// keypoints.h:150-176, the HARRIS_3D and HARRIS_6D branches of Keypoints::compute
static void harris_keypoints(const PointCloudRGB::Ptr& cloud, bool six, PointCloud<PointXYZI>::Ptr& keypoints,
                             PointCloudRGB::Ptr& cloud_keypoints) {
  keypoints.reset(new PointCloud<PointXYZI>);
  if (!six) {
    HarrisKeypoint3D<PointRGB, PointXYZI> harris3d;
    harris3d.setNonMaxSupression(true);
    harris3d.setInputCloud(cloud);
    harris3d.setThreshold(1e-6);
    harris3d.compute(*keypoints);
  } else {
    HarrisKeypoint6D<PointRGB, PointXYZI> harris6d;
    harris6d.setNonMaxSupression(true);
    harris6d.setInputCloud(cloud);
    harris6d.setThreshold(1e-6);
    harris6d.compute(*keypoints);
  }
  getKeypointsCloud(cloud, keypoints, cloud_keypoints);
}

// features.h:282-297, Features<T>::filterCorrespondences
static void filterCorrespondences(const PointCloudRGB::Ptr source, const PointCloudRGB::Ptr target,
                                  CorrespondencesPtr correspondences, CorrespondencesPtr& filtered_correspondences,
                                  Eigen::Matrix4f& transformation) {
  registration::CorrespondenceRejectorSampleConsensus<PointRGB> rejector;
  rejector.setInputSource(source);
  rejector.setInputTarget(target);
  rejector.setInputCorrespondences(correspondences);
  rejector.setInlierThreshold(0.015);
  rejector.setMaximumIterations(1000);
  rejector.getCorrespondences(*filtered_correspondences);
  transformation = rejector.getBestTransformation();
}

static void dump_xyz(const std::string& path, const PointCloudRGB& c) {
  std::vector<float> v;
  for (const PointRGB& p : c.points) {
    v.push_back(p.x);
    v.push_back(p.y);
    v.push_back(p.z);
  }
  dump(path, v.data(), v.size());
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s cloud.pcd out_dir\n", argv[0]);
    return 2;
  }
  PointCloudRGB::Ptr cloud(new PointCloudRGB);
  if (!read_pcd(argv[1], *cloud)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const std::string out = argv[2];

  // ---- keypoints.h:199-231 (NARF) ----
  PointCloud<int>::Ptr keypoints;
  PointCloudRGB::Ptr cloud_keypoints = narf_keypoints(cloud, keypoints);
  dump(out + "/keypoints.i32", keypoints->points.data(), keypoints->points.size());

  // ---- evaluation.cpp:593-612 (FPFH, r 0.08, normals r 0.05) ----
  Feature<PointRGB, FPFHSignature33>::Ptr fpfh(new FPFHEstimation<PointRGB, Normal, FPFHSignature33>);
  PointCloud<FPFHSignature33>::Ptr fdesc(new PointCloud<FPFHSignature33>);
  PointCloud<Normal>::Ptr normals;
  features_compute<FPFHSignature33>(fpfh, 0.08, 0.05, cloud, cloud_keypoints, fdesc, &normals);
  dump(out + "/normals.f32", reinterpret_cast<const float*>(normals->points.data()), normals->size() * 8);
  dump(out + "/fpfh.f32", reinterpret_cast<const float*>(fdesc->points.data()), fdesc->size() * 33);

  // ---- evaluation.cpp:766-785 (SHOT, r 0.08) ----
  Feature<PointRGB, SHOT352>::Ptr shot(new SHOTEstimationOMP<PointRGB, Normal, SHOT352>);
  PointCloud<SHOT352>::Ptr sdesc(new PointCloud<SHOT352>);
  features_compute<SHOT352>(shot, 0.08, 0.05, cloud, cloud_keypoints, sdesc);
  std::vector<float> d, rf;
  for (const SHOT352& s : sdesc->points) {
    d.insert(d.end(), s.descriptor, s.descriptor + 352);
    rf.insert(rf.end(), s.rf, s.rf + 9);
  }
  dump(out + "/shot.f32", d.data(), d.size());
  dump(out + "/shot_rf.f32", rf.data(), rf.size());
  std::printf("points %zu keypoints %zu fpfh %zu shot %zu\n", cloud->size(), keypoints->size(), fdesc->size(),
              sdesc->size());

  // ---- keypoints.h:177-189 (ISS, the reference's active list) ----
  PointCloudRGB::Ptr iss_kp;
  iss_keypoints(cloud, iss_kp);
  std::vector<float> iss_xyz;
  for (const PointRGB& p : iss_kp->points) {
    iss_xyz.push_back(p.x);
    iss_xyz.push_back(p.y);
    iss_xyz.push_back(p.z);
  }
  dump(out + "/iss_xyz.f32", iss_xyz.data(), iss_xyz.size());
  const double res = computeCloudResolution(cloud);
  dump(out + "/resolution.f64", &res, 1);
  std::printf("iss keypoints %zu\n", iss_kp->size());

  // ---- keypoints.h:150-176 (Harris3D / Harris6D) + getKeypointsCloud ----
  for (int six = 0; six < 2; ++six) {
    PointCloud<PointXYZI>::Ptr hk;
    PointCloudRGB::Ptr hkp;
    harris_keypoints(cloud, six != 0, hk, hkp);
    dump_xyz(out + (six ? "/harris6d_xyz.f32" : "/harris3d_xyz.f32"), *hkp);
    std::vector<float> corners;
    for (const PointXYZI& p : hk->points) {
      corners.push_back(p.x);
      corners.push_back(p.y);
      corners.push_back(p.z);
      corners.push_back(p.intensity);
    }
    dump(out + (six ? "/harris6d_corners.f32" : "/harris3d_corners.f32"), corners.data(), corners.size());
    std::printf("harris%dd corners %zu keypoints %zu\n", six ? 6 : 3, hk->size(), hkp->size());
  }

  // ---- evaluation.cpp:342 (feat.findCorrespondences) between this cloud and a target ----
  if (argc > 3) {
    PointCloudRGB::Ptr target(new PointCloudRGB);
    if (!read_pcd(argv[3], *target)) {
      std::fprintf(stderr, "cannot read %s\n", argv[3]);
      return 2;
    }
    PointCloud<int>::Ptr tkp;
    PointCloudRGB::Ptr target_keypoints = narf_keypoints(target, tkp);
    PointCloud<FPFHSignature33>::Ptr tdesc(new PointCloud<FPFHSignature33>);
    Feature<PointRGB, FPFHSignature33>::Ptr tfpfh(new FPFHEstimation<PointRGB, Normal, FPFHSignature33>);
    features_compute<FPFHSignature33>(tfpfh, 0.08, 0.05, target, target_keypoints, tdesc);
    dump(out + "/fpfh_target.f32", reinterpret_cast<const float*>(tdesc->points.data()), tdesc->size() * 33);
    CorrespondencesPtr corr(new Correspondences);
    Features<FPFHSignature33> feat;
    feat.findCorrespondences(fdesc, tdesc, corr);
    std::vector<int32_t> pairs;
    for (const Correspondence& c : *corr) {
      pairs.push_back(c.index_query);
      pairs.push_back(c.index_match);
    }
    dump(out + "/corr.i32", pairs.data(), pairs.size());
    std::printf("target keypoints %zu correspondences %zu\n", tdesc->size(), corr->size());
    // ---- features.h:282-297 (filterCorrespondences) on the keypoint clouds ----
    CorrespondencesPtr filtered(new Correspondences);
    Eigen::Matrix4f T;
    filterCorrespondences(cloud_keypoints, target_keypoints, corr, filtered, T);
    std::vector<int32_t> kept;
    for (const Correspondence& c : *filtered) {
      kept.push_back(c.index_query);
      kept.push_back(c.index_match);
    }
    dump(out + "/filtered.i32", kept.data(), kept.size());
    dump(out + "/transformation.f32", T.m, 16);
    dump_xyz(out + "/src_kp_xyz.f32", *cloud_keypoints);
    dump_xyz(out + "/tgt_kp_xyz.f32", *target_keypoints);
    std::printf("filtered correspondences %zu\n", filtered->size());
  }
  return 0;
}
