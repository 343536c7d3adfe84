// pfx_pcd.hip -- PCD v0.7 loading straight into the device SoA layout.
//
// Replaces pcl::io::loadPCDFile<PointXYZRGB> (evaluation.cpp:226-235) on the path's input side:
// the reference parses the file into an AoS PointCloud<PointXYZRGB> and every libpfx entry point
// would then unpack it to SoA; here the file's data block goes to the device once and one
// kernel unpacks x, y, z (any field order / point size) into the float SoA the kernels read.
//   DATA binary             -> raw block H2D (pinned staging), k_pcd_unpack
//   DATA ascii              -> host parse (strtof: correctly rounded, "nan" accepted), H2D
//   DATA binary_compressed  -> PFX_ERR_UNSUPPORTED (the reference's data files are binary;
//                              pcl::io::savePCDFile writes ascii)
// The header is parsed as PCL 1.7's PCDReader::readHeader does for these keys: VERSION, FIELDS,
// SIZE, TYPE, COUNT (default 1), WIDTH, HEIGHT (default 1), VIEWPOINT (default 0 0 0 1 0 0 0),
// POINTS (default WIDTH * HEIGHT), DATA; '#' comment lines are skipped.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pfx_internal.h"

namespace pfx {
namespace {

__global__ void k_pcd_unpack(const uint8_t* __restrict__ raw, int64_t n, int point_size, int ox, int oy, int oz,
                             float* __restrict__ x, float* __restrict__ y, float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = raw + i * point_size;
  if (((point_size | ox | oy | oz) & 3) == 0) {  // the usual case: 4-byte aligned float fields
    x[i] = *reinterpret_cast<const float*>(p + ox);
    y[i] = *reinterpret_cast<const float*>(p + oy);
    z[i] = *reinterpret_cast<const float*>(p + oz);
    return;
  }
  auto rd = [&](int o) {  // fields after 1- or 2-byte fields: byte-wise (little-endian)
    const uint32_t b = (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) |
                       ((uint32_t)p[o + 3] << 24);
    return __uint_as_float(b);
  };
  x[i] = rd(ox);
  y[i] = rd(oy);
  z[i] = rd(oz);
}

struct File {
  FILE* f = nullptr;
  explicit File(const char* path) : f(std::fopen(path, "rb")) {}
  ~File() { if (f) std::fclose(f); }
};

std::vector<std::string> split(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r')) ++i;
    size_t j = i;
    while (j < s.size() && s[j] != ' ' && s[j] != '\t' && s[j] != '\r') ++j;
    if (j > i) out.push_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

// parses the header; on return the stream is positioned at the data block
pfx_status parse_header(FILE* f, pfx_pcd_header& h, std::string& err) {
  std::memset(&h, 0, sizeof(h));
  h.height = 1;
  h.x_offset = h.y_offset = h.z_offset = -1;
  const float vp0[7] = {0, 0, 0, 1, 0, 0, 0};
  std::memcpy(h.viewpoint, vp0, sizeof(vp0));
  std::vector<std::string> fields, types;
  std::vector<int> sizes, counts;
  bool have_points = false, have_data = false;
  char line[65536];
  long pos = 0;
  while (std::fgets(line, sizeof(line), f)) {
    pos = std::ftell(f);
    std::string s(line);
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    std::vector<std::string> t = split(s);
    if (t.empty() || t[0][0] == '#') continue;
    const std::string& key = t[0];
    if (key == "FIELDS" || key == "COLUMNS") fields.assign(t.begin() + 1, t.end());
    else if (key == "SIZE") { sizes.clear(); for (size_t i = 1; i < t.size(); ++i) sizes.push_back(std::atoi(t[i].c_str())); }
    else if (key == "TYPE") types.assign(t.begin() + 1, t.end());
    else if (key == "COUNT") { counts.clear(); for (size_t i = 1; i < t.size(); ++i) counts.push_back(std::atoi(t[i].c_str())); }
    else if (key == "WIDTH" && t.size() > 1) h.width = std::atoi(t[1].c_str());
    else if (key == "HEIGHT" && t.size() > 1) h.height = std::atoi(t[1].c_str());
    else if (key == "VIEWPOINT") { for (size_t i = 1; i < t.size() && i <= 7; ++i) h.viewpoint[i - 1] = std::strtof(t[i].c_str(), nullptr); }
    else if (key == "POINTS" && t.size() > 1) { h.points = std::atoll(t[1].c_str()); have_points = true; }
    else if (key == "DATA" && t.size() > 1) {
      const std::string& d = t[1];
      h.data = d == "ascii" ? 0 : d == "binary" ? 1 : d == "binary_compressed" ? 2 : -1;
      have_data = true;
      break;
    }
  }
  if (!have_data || h.data < 0) { err = "pcd: no DATA ascii|binary|binary_compressed line"; return PFX_ERR_INVALID; }
  if (fields.empty() || sizes.size() != fields.size() || types.size() != fields.size()) {
    err = "pcd: FIELDS / SIZE / TYPE disagree";
    return PFX_ERR_INVALID;
  }
  if (counts.empty()) counts.assign(fields.size(), 1);
  if (counts.size() != fields.size()) { err = "pcd: COUNT disagrees with FIELDS"; return PFX_ERR_INVALID; }
  if (!have_points) h.points = (int64_t)h.width * h.height;
  h.nfields = (int32_t)fields.size();
  int off = 0, col = 0;
  for (size_t i = 0; i < fields.size(); ++i) {
    const bool f32 = types[i] == "F" && sizes[i] == 4 && counts[i] == 1;
    int32_t* dst = fields[i] == "x" ? &h.x_offset : fields[i] == "y" ? &h.y_offset : fields[i] == "z" ? &h.z_offset : nullptr;
    if (dst) {
      if (!f32) { err = "pcd: field " + fields[i] + " is not a single float32"; return PFX_ERR_UNSUPPORTED; }
      *dst = h.data == 0 ? col : off;  // ascii: column index, binary: byte offset
    }
    off += sizes[i] * counts[i];
    col += counts[i];
  }
  h.point_size = h.data == 0 ? col : off;
  h.data_offset = pos;
  if (h.x_offset < 0 || h.y_offset < 0 || h.z_offset < 0) { err = "pcd: no x y z fields"; return PFX_ERR_UNSUPPORTED; }
  if (h.points < 0) { err = "pcd: negative POINTS"; return PFX_ERR_INVALID; }
  return PFX_OK;
}

}  // namespace

pfx_status pcd_read_header(const char* path, pfx_pcd_header* out, std::string& err) {
  File file(path);
  if (!file.f) { err = std::string("pcd: cannot open ") + path; return PFX_ERR_INVALID; }
  return parse_header(file.f, *out, err);
}

int64_t pcd_load_xyz_dev(pfx_ctx* ctx, const char* path, float* d_x, float* d_y, float* d_z, int64_t cap,
                         pfx_pcd_header* hdr_out) {
  File file(path);
  if (!file.f) throw Error(PFX_ERR_INVALID, std::string("pcd: cannot open ") + path);
  pfx_pcd_header h;
  std::string err;
  const pfx_status st0 = parse_header(file.f, h, err);
  if (st0 != PFX_OK) throw Error(st0, err + " (" + path + ")");
  if (hdr_out) *hdr_out = h;
  if (h.data == 2) throw Error(PFX_ERR_UNSUPPORTED, std::string("pcd: DATA binary_compressed not supported (") + path + ")");
  const int64_t n = h.points;
  if (n > cap) return n;  // caller buffer too small: the count tells
  if (n == 0) return 0;
  hipStream_t st = ctx->stream;
  TimeScope ts(ctx, "pcd_load");
  if (h.data == 1) {
    const size_t bytes = (size_t)n * (size_t)h.point_size;
    void* pinned = nullptr;
    PFX_HIP(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    const size_t got = std::fread(pinned, 1, bytes, file.f);
    if (got != bytes) {
      (void)hipHostFree(pinned);
      throw Error(PFX_ERR_INVALID, std::string("pcd: truncated binary data in ") + path);
    }
    uint8_t* raw = ctx->buf("pcd_raw").as<uint8_t>(bytes);
    hipError_t e = hipMemcpyAsync(raw, pinned, bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      k_pcd_unpack<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(raw, n, h.point_size, h.x_offset, h.y_offset,
                                                                h.z_offset, d_x, d_y, d_z);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);  // the pinned block is released below
    (void)hipHostFree(pinned);
    if (e != hipSuccess) throw Error(PFX_ERR_DEVICE, std::string("pcd load: ") + hipGetErrorString(e));
    return n;
  }
  // ascii: one point per line, `point_size` columns
  std::vector<float> xs((size_t)n), ys((size_t)n), zs((size_t)n);
  std::vector<char> rest;
  {
    const long start = std::ftell(file.f);
    std::fseek(file.f, 0, SEEK_END);
    const long end = std::ftell(file.f);
    std::fseek(file.f, start, SEEK_SET);
    rest.resize((size_t)(end - start) + 1);
    const size_t got = std::fread(rest.data(), 1, (size_t)(end - start), file.f);
    rest[got] = '\0';
  }
  char* c = rest.data();
  for (int64_t i = 0; i < n; ++i) {
    for (int col = 0; col < h.point_size; ++col) {
      char* e = nullptr;
      const float v = std::strtof(c, &e);
      if (e == c) throw Error(PFX_ERR_INVALID, std::string("pcd: truncated ascii data in ") + path);
      if (col == h.x_offset) xs[(size_t)i] = v;
      if (col == h.y_offset) ys[(size_t)i] = v;
      if (col == h.z_offset) zs[(size_t)i] = v;
      c = e;
    }
  }
  PFX_HIP(hipMemcpyAsync(d_x, xs.data(), sizeof(float) * n, hipMemcpyHostToDevice, st));
  PFX_HIP(hipMemcpyAsync(d_y, ys.data(), sizeof(float) * n, hipMemcpyHostToDevice, st));
  PFX_HIP(hipMemcpyAsync(d_z, zs.data(), sizeof(float) * n, hipMemcpyHostToDevice, st));
  PFX_HIP(hipStreamSynchronize(st));  // the host vectors go out of scope
  return n;
}

}  // namespace pfx
