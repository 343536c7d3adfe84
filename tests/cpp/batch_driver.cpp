// The multi-GPU scan batch from a C++ host (include/pfx.h pfx_batch_*): what the reference's
// per-scan loop (evaluation.cpp:272-852) becomes for the (Narf, FPFH) pair when the host stays
// C++.  usage: batch_driver <out_dir> <devices, e.g. 0 or 0,1> <scan.f32>...
// Each scan file holds n x, then n y, then n z floats.  Writes desc.f32 (sum K x 33), idx.i32
// (sum K) and rows.i64 (K per scan) in scan order.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "pfx.h"

static std::vector<float> read_f32(const char* path) {
  std::vector<float> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize((size_t)bytes / sizeof(float));
  if (std::fread(v.data(), sizeof(float), v.size(), f) != v.size()) v.clear();
  std::fclose(f);
  return v;
}

template <class T>
static bool write(const std::string& path, const T* p, size_t n) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(p, sizeof(T), n, f) == n;
  std::fclose(f);
  return ok;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s out_dir devices scan.f32...\n", argv[0]);
    return 2;
  }
  const std::string out = argv[1];
  std::vector<int> devices;
  for (const char* p = argv[2]; *p;) {
    devices.push_back(std::atoi(p));
    while (*p && *p != ',') ++p;
    if (*p == ',') ++p;
  }
  std::vector<std::vector<float>> clouds;
  std::vector<const float*> x, y, z;
  std::vector<int64_t> n;
  for (int i = 3; i < argc; ++i) {
    clouds.push_back(read_f32(argv[i]));
    if (clouds.back().empty() || clouds.back().size() % 3) {
      std::fprintf(stderr, "bad scan file %s\n", argv[i]);
      return 2;
    }
  }
  for (auto& c : clouds) {
    const int64_t m = (int64_t)c.size() / 3;
    x.push_back(c.data());
    y.push_back(c.data() + m);
    z.push_back(c.data() + 2 * m);
    n.push_back(m);
  }
  pfx_batch* b = nullptr;
  if (pfx_batch_create(devices.data(), (int)devices.size(), &b) != PFX_OK) {
    std::fprintf(stderr, "pfx_batch_create failed\n");
    return 1;
  }
  pfx_camera cam;
  pfx_camera_default(&cam);  // keypoints.h:203-216
  pfx_narf_params params;
  pfx_narf_params_default(&params);
  params.support_size = 0.2f;  // keypoints.h:223
  const int64_t cap = 1 << 20;
  std::vector<float> desc((size_t)cap * 33);
  std::vector<int32_t> idx((size_t)cap);
  std::vector<int64_t> rows(clouds.size());
  // Features<FPFHSignature33>(est, feat_radius 0.08, normal_radius 0.05): evaluation.cpp:167-168
  pfx_status st = pfx_batch_narf_fpfh(b, (int)clouds.size(), x.data(), y.data(), z.data(), n.data(), &cam, &params,
                                      0.05, 0.08, desc.data(), idx.data(), cap, rows.data());
  if (st != PFX_OK) {
    std::fprintf(stderr, "pfx_batch_narf_fpfh: %s\n", pfx_batch_last_error(b));
    pfx_batch_destroy(b);
    return 1;
  }
  int64_t total = 0;
  for (int64_t k : rows) total += k;
  bool ok = write(out + "/desc.f32", desc.data(), (size_t)total * 33) &&
            write(out + "/idx.i32", idx.data(), (size_t)total) && write(out + "/rows.i64", rows.data(), rows.size());
  pfx_batch_destroy(b);
  std::printf("%zu scans on %zu device(s): %lld descriptor rows\n", clouds.size(), devices.size(), (long long)total);
  return ok ? 0 : 1;
}
