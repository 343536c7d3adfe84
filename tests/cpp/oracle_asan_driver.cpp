// AddressSanitizer / UBSan run of the CPU restatement (SURVEY §5 "sanitizers"): every oracle entry
// point on a subsample of one of the reference's clouds plus a handful of degenerate inputs
// (empty, single point, duplicates, NaN rows).  Built and run by tests/test_sanitizers.py with
//   g++ -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all ... oracle/*.cpp
// Test infrastructure only: the oracle is the checker, never the product.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

typedef int64_t i64;
extern "C" {
int orc_radius_search(const float*, const float*, const float*, i64, const float*, const float*, const float*, i64,
                      double, i64*, int*, float*, i64);
int orc_normals(const float*, const float*, const float*, i64, double, float, float, float, float*, float*, float*,
                float*, int);
int orc_fpfh(const float*, const float*, const float*, const float*, const float*, const float*, i64, const float*,
             const float*, const float*, i64, int, double, float*, int);
int orc_shot(const float*, const float*, const float*, const float*, const float*, const float*, i64, const float*,
             const float*, const float*, i64, double, float*, float*, int);
int orc_narf_keypoints(const float*, const float*, const float*, i64, int, int, float, float, float, float,
                       const float*, int, float, float, const float*, int*, i64, i64*, float*, float*, uint32_t*, int);
int orc_cloud_resolution(const float*, const float*, const float*, i64, double*, float*, int);
int orc_iss_keypoints(const float*, const float*, const float*, i64, double, double, int, double, double, int32_t*,
                      i64, i64*, double*, int);
int orc_harris3d(const float*, const float*, const float*, i64, double, float, int, int32_t*, i64, i64*, i64*, float*,
                 float*, int);
int orc_correspondences(const float*, i64, const float*, i64, int, int32_t*, int32_t*, i64, i64*, int);
int orc_ransac_rejector(const float*, const float*, const float*, i64, const float*, const float*, const float*, i64,
                        const int32_t*, const int32_t*, i64, double, int, int32_t*, i64*, float*, i64*);
}

namespace {

// binary PCD with FIELDS x y z rgb, SIZE 4 x4 (the reference's clouds)
bool read_pcd(const char* path, std::vector<float>& x, std::vector<float>& y, std::vector<float>& z) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string line;
  long n = 0;
  while (std::getline(f, line)) {
    if (line.rfind("POINTS", 0) == 0) n = std::atol(line.c_str() + 6);
    if (line.rfind("DATA", 0) == 0) break;
  }
  std::vector<float> rec((size_t)n * 4);
  f.read(reinterpret_cast<char*>(rec.data()), (std::streamsize)(rec.size() * sizeof(float)));
  if (!f) return false;
  for (long i = 0; i < n; ++i) {
    x.push_back(rec[4 * i]);
    y.push_back(rec[4 * i + 1]);
    z.push_back(rec[4 * i + 2]);
  }
  return true;
}

int failures = 0;
void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL %s\n", what);
    ++failures;
  }
}

void run_all(const std::vector<float>& x, const std::vector<float>& y, const std::vector<float>& z, const char* tag) {
  const i64 n = (i64)x.size();
  const float* X = x.data();
  const float* Y = y.data();
  const float* Z = z.data();
  std::vector<float> nx(n + 1), ny(n + 1), nz(n + 1), cv(n + 1);
  check(orc_normals(X, Y, Z, n, 0.05, 0, 0, 0, nx.data(), ny.data(), nz.data(), cv.data(), 2) == 0, "normals");
  std::vector<i64> cnt(n + 1);
  const i64 cap = 64;
  std::vector<int> idx((size_t)(n + 1) * cap);
  std::vector<float> d2((size_t)(n + 1) * cap);
  check(orc_radius_search(X, Y, Z, n, X, Y, Z, n, 0.02, cnt.data(), idx.data(), d2.data(), cap) == 0, "radius");
  const i64 nq = n < 7 ? n : 7;
  std::vector<float> qx(X, X + nq), qy(Y, Y + nq), qz(Z, Z + nq);
  std::vector<float> f((size_t)(nq + 1) * 33), f2((size_t)(n + 1) * 33);
  check(orc_fpfh(X, Y, Z, nx.data(), ny.data(), nz.data(), n, qx.data(), qy.data(), qz.data(), nq, 0, 0.08, f.data(),
                 1) >= 0, "fpfh");  // returns |S|
  check(orc_fpfh(X, Y, Z, nx.data(), ny.data(), nz.data(), n, X, Y, Z, n, 1, 0.05, f2.data(), 2) >= 0, "fpfh all");
  std::vector<float> sd((size_t)(nq + 1) * 352), rf((size_t)(nq + 1) * 9);
  check(orc_shot(X, Y, Z, nx.data(), ny.data(), nz.data(), n, qx.data(), qy.data(), qz.data(), nq, 0.08, sd.data(),
                 rf.data(), 2) == 0, "shot");
  const float pose[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  const float params[15] = {0.2f, -1, 0.25f, 0.25f, 0.45f, 0.2f, 1, 1, 0, 0, 3, 2, 2, 0.8f, 2};
  std::vector<int> kp(640 * 480);
  i64 nk = 0;
  check(orc_narf_keypoints(X, Y, Z, n, 640, 480, 320, 240, 525, 525, pose, 0, 0, 0, params, kp.data(), 640 * 480,
                           &nk, nullptr, nullptr, nullptr, 1) == 0, "narf");
  double res = 0;
  std::vector<float> terms(n + 1);
  check(orc_cloud_resolution(X, Y, Z, n, &res, terms.data(), 2) == 0, "resolution");
  std::vector<int32_t> ik(n + 1);
  std::vector<double> third(n + 1);
  i64 ni = 0;
  if (res > 0)
    check(orc_iss_keypoints(X, Y, Z, n, 6 * res, 4 * res, 5, 0.975, 0.975, ik.data(), n + 1, &ni, third.data(), 2) ==
              0, "iss");
  std::vector<int32_t> hk(n + 1);
  std::vector<float> resp(n + 1), cor((size_t)3 * (n + 1));
  i64 nh = 0, nc = 0;
  check(orc_harris3d(X, Y, Z, n, 0.01, 1e-6f, 1, hk.data(), n + 1, &nh, &nc, resp.data(), cor.data(), 2) == 0,
        "harris3d");
  // matching + RANSAC on the first half of the FPFH rows against the second half
  const i64 h = n / 2;
  std::vector<int32_t> q(h + 1), m(h + 1), keep(h + 1);
  i64 nm = 0, nkeep = 0, it = 0;
  check(orc_correspondences(f2.data(), h, f2.data() + h * 33, n - h, 33, q.data(), m.data(), h + 1, &nm, 2) == 0,
        "correspondences");
  float T[16];
  check(orc_ransac_rejector(X, Y, Z, h, X + h, Y + h, Z + h, n - h, q.data(), m.data(), nm, 0.015, 1000, keep.data(),
                            &nkeep, T, &it) == 0, "ransac");
  std::printf("%s: n=%lld narf=%lld iss=%lld harris=%lld corr=%lld kept=%lld\n", tag, (long long)n, (long long)nk,
              (long long)ni, (long long)nh, (long long)nm, (long long)nkeep);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s cloud.pcd [stride]\n", argv[0]);
    return 2;
  }
  std::vector<float> x, y, z;
  if (!read_pcd(argv[1], x, y, z)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const int stride = argc > 2 ? std::atoi(argv[2]) : 8;
  std::vector<float> sx, sy, sz;
  for (size_t i = 0; i < x.size(); i += (size_t)stride) {
    sx.push_back(x[i]);
    sy.push_back(y[i]);
    sz.push_back(z[i]);
  }
  run_all(sx, sy, sz, "subsample");
  // degenerate inputs: empty, one point, duplicates, NaN rows
  std::vector<float> e;
  run_all(e, e, e, "empty");
  std::vector<float> one{0.1f}, onez{1.0f};
  run_all(one, one, onez, "single");
  std::vector<float> dx(50, 0.2f), dy(50, -0.1f), dz(50, 1.5f);
  run_all(dx, dy, dz, "duplicates");
  std::vector<float> nx2(sx.begin(), sx.begin() + (sx.size() < 2000 ? sx.size() : 2000));
  std::vector<float> ny2(sy.begin(), sy.begin() + nx2.size()), nz2(sz.begin(), sz.begin() + nx2.size());
  for (size_t i = 0; i < nx2.size(); i += 17) nx2[i] = std::nanf("");
  run_all(nx2, ny2, nz2, "nan rows");
  if (failures) return 1;
  std::printf("oracle sanitizer run clean\n");
  return 0;
}
