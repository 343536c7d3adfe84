// pfx_narf.hip -- NARF keypoints on the planar range image (keypoints.h:199-231) on gfx950:
//   RangeImagePlanar::createFromPointCloudWithFixedSize      k_ri_*
//   RangeImageBorderExtractor                                k_surface .. k_scs
//   NarfKeypoint::compute                                    k_interest, k_nms
// One thread per pixel for the image passes (640x480 = 307,200 px, 16-B/px SoA float4
// images in HBM), one wave per pixel for the interest region-grow (bitmap + queue in LDS).
// The only sequential steps -- std::sort of the few hundred NMS survivors and the greedy
// minimum-distance selection -- run on the host exactly as PCL does.
//
// Order-dependent PCL steps and how they are made parallel without changing results:
//   * z-buffer: with noise_level 0 the result is min(direct hits) else min(fills):
//     two atomicMin images on the float bits (ranges > 0 order like uints).
//   * shadow borders are updated in place in raster order: the R/B passes only read the
//     not-yet-updated L/T scores, the L/T passes read the final R/B scores -> two phases.
//   * border traits are set-only -> atomicOr.
//   * interest region-grow: the accepted set is the 8-connected component of p, histogram
//     max / negative min are order-free -> level-parallel BFS.
#include <algorithm>
#include <cstring>

#include "pfx_device_math.h"
#include <cstdio>

#include "pfx_internal.h"

namespace pfx {

enum {
  T_OBSTACLE_BORDER = 0, T_SHADOW_BORDER, T_VEIL_POINT, T_SHADOW_BORDER_TOP, T_SHADOW_BORDER_RIGHT,
  T_SHADOW_BORDER_BOTTOM, T_SHADOW_BORDER_LEFT, T_OBSTACLE_BORDER_TOP, T_OBSTACLE_BORDER_RIGHT,
  T_OBSTACLE_BORDER_BOTTOM, T_OBSTACLE_BORDER_LEFT, T_VEIL_POINT_TOP, T_VEIL_POINT_RIGHT,
  T_VEIL_POINT_BOTTOM, T_VEIL_POINT_LEFT
};
#define TB(t) (1u << (t))

struct NarfState {
  int w = 0, h = 0;
  DevBuf direct, fill, pts, surf, smean, svalid, sL, sR, sT, sB, uL, uR, uT, uB, shadow, traits, rawdir, dir, scs, scd,
      interest, cand, counters, rowp, sat, work, fb1, pk;
  std::vector<float> h_interest, h_scs, h_range;
  std::vector<uint32_t> h_traits;
  bool have_debug = false;
  // pinned host block of the readbacks (counters, NMS survivors, validity bits): async DMA copies,
  // not pageable staging through a blit kernel (which waited ~1 ms for CU slots beside the
  // normal estimation's list kernels and held the runtime lock the other host thread launches through)
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  void* host(size_t need) {
    if (need > pinned_bytes) {
      if (pinned) PFX_HIP(hipHostFree(pinned));
      pinned_bytes = need + need / 2 + 4096;
      PFX_HIP(hipHostMalloc(&pinned, pinned_bytes, hipHostMallocDefault));
    }
    return pinned;
  }
  void release() {
    if (pinned) (void)hipHostFree(pinned);
    pinned = nullptr;
    pinned_bytes = 0;
    DevBuf* all[] = {&direct, &fill, &pts, &surf, &smean, &svalid, &sL, &sR, &sT, &sB, &uL, &uR, &uT, &uB, &shadow,
                     &traits, &rawdir, &dir, &scs, &scd, &interest, &cand, &counters, &rowp, &sat, &work, &fb1, &pk};
    for (auto* b : all) b->release();
  }
};

namespace {

struct Aff { float m[12]; };  // row-major 3x4 [R | t]

struct Img {
  int w, h;
  float cx, cy, fx, fy, fxr, fyr;
  Aff to_world, to_ri;
};

__device__ __forceinline__ f3 aff_apply(const Aff& a, f3 p) {
  return mk3(a.m[3] + (a.m[0] * p.x + a.m[1] * p.y + a.m[2] * p.z),
             a.m[7] + (a.m[4] * p.x + a.m[5] * p.y + a.m[6] * p.z),
             a.m[11] + (a.m[8] * p.x + a.m[9] * p.y + a.m[10] * p.z));
}

__device__ __forceinline__ bool in_image(const Img& I, int x, int y) { return x >= 0 && x < I.w && y >= 0 && y < I.h; }

__device__ __forceinline__ f3 calc3d(const Img& I, float ix, float iy, float range) {
  float dx = (ix + 0.0f - I.cx) * I.fxr, dy = (iy + 0.0f - I.cy) * I.fyr;
  f3 p;
  p.z = range / (sqrtf(dx * dx + dy * dy + 1));
  p.x = dx * p.z;
  p.y = dy * p.z;
  return aff_apply(I.to_world, p);
}

__device__ __forceinline__ void image_point(const Img& I, f3 pt, float& ix, float& iy, float& range) {
  f3 t = aff_apply(I.to_ri, pt);
  if (t.z <= 0) { ix = iy = range = -1.0f; return; }
  range = sqrtf(sqn3(t));
  ix = I.cx + I.fx * t.x / t.z - 0.0f;
  iy = I.cy + I.fy * t.y / t.z - 0.0f;
}

__device__ __forceinline__ float sq_dist(float4 a, float4 b) {  // diff = b - a
  float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
  return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ float4 get_point(const Img& I, const float4* __restrict__ P, int x, int y) {
  if (!in_image(I, x, y)) return make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), -INFINITY);
  return P[y * I.w + x];
}
__device__ __forceinline__ bool is_valid(const Img& I, const float4* __restrict__ P, int x, int y) {
  return in_image(I, x, y) && isfinite(P[y * I.w + x].w);
}

// ---- range image ---------------------------------------------------------------------------
__global__ void k_ri_init(uint32_t* __restrict__ direct, uint32_t* __restrict__ fill, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { direct[i] = 0xffffffffu; fill[i] = 0xffffffffu; }
}

__global__ void k_ri_project(Img I, const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                             int64_t n, float min_range, uint32_t* __restrict__ direct, uint32_t* __restrict__ fill) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float px = X[i], py = Y[i], pz = Z[i];
  if (!(isfinite(px) && isfinite(py) && isfinite(pz))) return;
  float xr, yr, rng;
  image_point(I, mk3(px, py, pz), xr, yr, rng);
  int x = (int)rintf(xr), y = (int)rintf(yr);
  if (rng < min_range || !in_image(I, x, y)) return;
  int fx0 = (int)floorf(xr), fy0 = (int)floorf(yr), cx0 = (int)ceilf(xr), cy0 = (int)ceilf(yr);
  int nxs[4] = {fx0, fx0, cx0, cx0}, nys[4] = {fy0, cy0, fy0, cy0};
  uint32_t rb = __float_as_uint(rng);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (nxs[k] == x && nys[k] == y) continue;
    if (!in_image(I, nxs[k], nys[k])) continue;
    atomicMin(&fill[nys[k] * I.w + nxs[k]], rb);
  }
  atomicMin(&direct[y * I.w + x], rb);
}

__global__ void k_ri_finalize(Img I, const uint32_t* __restrict__ direct, const uint32_t* __restrict__ fill,
                              float4* __restrict__ P) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  uint32_t d = direct[i], f = fill[i];
  float r = d != 0xffffffffu ? __uint_as_float(d) : (f != 0xffffffffu ? __uint_as_float(f) : -INFINITY);
  float4 o = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), r);
  if (!isinf(r)) {
    int y = i / I.w, x = i - y * I.w;
    f3 q = calc3d(I, (float)x, (float)y, r);
    o.x = q.x; o.y = q.y; o.z = q.z;
  }
  P[i] = o;
}

// ---- VectorAverage3f -------------------------------------------------------------------------
struct VecAvg {
  int n;
  float acc_w;
  f3 mean;
  float c00, c01, c02, c11, c12, c22;
  __device__ void init() { n = 0; acc_w = 0.f; mean = mk3(0, 0, 0); c00 = c01 = c02 = c11 = c12 = c22 = 0.f; }
  __device__ void add(f3 s) {
    ++n;
    acc_w += 1.0f;
    float alpha = 1.0f / acc_w;
    f3 d = sub3(s, mean);
    mean = add3(mean, mk3(alpha * d.x, alpha * d.y, alpha * d.z));
    float om = 1.0f - alpha;
    // `(1.0f-alpha)*(covariance_(i, j) + alpha*diff[i]*diff[j])`: (alpha * d_i) * d_j
    c00 = om * (c00 + alpha * d.x * d.x);
    c01 = om * (c01 + alpha * d.x * d.y);
    c02 = om * (c02 + alpha * d.x * d.z);
    c11 = om * (c11 + alpha * d.y * d.y);
    c12 = om * (c12 + alpha * d.y * d.z);
    c22 = om * (c22 + alpha * d.z * d.z);
  }
  __device__ void pca(float ev[3], f3 evec[3]) const {
    Sym3 m;
    m.a00 = c00; m.a01 = c01; m.a02 = c02;
    m.a10 = c01; m.a11 = c11; m.a12 = c12;
    m.a20 = c02; m.a21 = c12; m.a22 = c22;
    eigen33_full(m, evec, ev);
  }
};

// RangeImage::getSurfaceInformation (no-jumps part), radius/step from the border parameters
// surf = (normal_no_jumps, max_neighbor_distance_squared), smean = neighborhood_mean_no_jumps
__global__ void k_surface(Img I, const float4* __restrict__ P, int radius, int step, int no_of_closest,
                          float4* __restrict__ surf, float4* __restrict__ smean, uint8_t* __restrict__ svalid) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  svalid[i] = 0;
  int y = i / I.w, x = i - y * I.w;
  float4 point = P[i];
  if (!isfinite(point.w)) return;
  float nd[25];
  float4 np[25];
  int cnt = 0;
  for (int y2 = y - radius; y2 <= y + radius; y2 += step)
    for (int x2 = x - radius; x2 <= x + radius; x2 += step) {
      if (!is_valid(I, P, x2, y2) || cnt >= 25) continue;
      float4 q = P[y2 * I.w + x2];
      float d = sq_dist(point, q);
      int j = cnt++;
      while (j > 0 && d < nd[j - 1]) { nd[j] = nd[j - 1]; np[j] = np[j - 1]; --j; }
      nd[j] = d;
      np[j] = q;
    }
  int k = cnt < no_of_closest ? cnt : no_of_closest;
  float maxd2 = nd[k - 1];
  float lim = maxd2 * 4.0f;
  VecAvg va;
  va.init();
  for (int j = 0; j < cnt; ++j) {
    if (nd[j] > lim) break;
    va.add(mk3(np[j].x, np[j].y, np[j].z));
  }
  if (va.n < 3) return;
  float ev[3];
  f3 evec[3];
  va.pca(ev, evec);
  f3 normal = evec[0];
  f3 sensor = mk3(I.to_world.m[3], I.to_world.m[7], I.to_world.m[11]);
  f3 view = normalized3(sub3(sensor, mk3(point.x, point.y, point.z)));
  if (dot3(normal, view) < 0.0f) normal = scale3(normal, -1.0f);
  surf[i] = make_float4(normal.x, normal.y, normal.z, maxd2);
  smean[i] = make_float4(va.mean.x, va.mean.y, va.mean.z, 0.0f);
  svalid[i] = 1;
}

__device__ __forceinline__ float4 point_avg(const Img& I, const float4* __restrict__ P, int x, int y, int dx, int dy,
                                            int no_of_points) {
  float ws = 1.0f;
  float4 a = get_point(I, P, x, y);
  if (isinf(a.w)) {
    if (a.w > 0.0f) return a;
    ws = 0.0f;
    a = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int x2 = x, y2 = y;
  for (int s = 1; s < no_of_points; ++s) {
    x2 += dx; y2 += dy;
    if (!is_valid(I, P, x2, y2)) continue;
    float4 p = P[y2 * I.w + x2];
    a.x += p.x; a.y += p.y; a.z += p.z; a.w += p.w;
    ws += 1.0f;
  }
  if (ws <= 0.0f) return make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), -INFINITY);
  float nf = 1.0f / ws;
  a.x *= nf; a.y *= nf; a.z *= nf; a.w *= nf;
  return a;
}

__device__ __forceinline__ float dist_change_score(const Img& I, const float4* __restrict__ P, float maxd2, int x,
                                                   int y, int ox, int oy, int pixel_radius) {
  float4 point = get_point(I, P, x, y);
  float4 nb = point_avg(I, P, x + ox, y + oy, ox, oy, pixel_radius);
  if (isinf(nb.w)) return nb.w < 0.0f ? 0.0f : 1.0f;
  float nd2 = sq_dist(nb, point);
  if (nd2 <= maxd2) return 0.0f;
  float ret = 1.0f - sqrtf(maxd2 / nd2);
  if (nb.w < point.w) ret = -ret;
  return ret;
}

__global__ void k_border_scores(Img I, const float4* __restrict__ P, const float4* __restrict__ surf,
                                const uint8_t* __restrict__ svalid, int prb, float* __restrict__ sL,
                                float* __restrict__ sR, float* __restrict__ sT, float* __restrict__ sB) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  float l = 0.f, r = 0.f, t = 0.f, b = 0.f;
  if (svalid[i]) {
    int y = i / I.w, x = i - y * I.w;
    float maxd2 = surf[i].w;
    l = dist_change_score(I, P, maxd2, x, y, -1, 0, prb);
    r = dist_change_score(I, P, maxd2, x, y, 1, 0, prb);
    t = dist_change_score(I, P, maxd2, x, y, 0, -1, prb);
    b = dist_change_score(I, P, maxd2, x, y, 0, 1, prb);
  }
  sL[i] = l; sR[i] = r; sT[i] = t; sB[i] = b;
}

__device__ __forceinline__ float updated_score(const Img& I, const float* __restrict__ s, int x, int y, float minp) {
  const float bonus = 0.5f;
  float b = s[y * I.w + x];
  if (b + bonus * (1.0f - b) < minp) return b;
  float avg = 0.0f, ws = 0.0f;
  for (int y2 = y - 1; y2 <= y + 1; ++y2)
    for (int x2 = x - 1; x2 <= x + 1; ++x2) {
      if (!in_image(I, x2, y2) || (x2 == x && y2 == y)) continue;
      avg += s[y2 * I.w + x2];
      ws += 1.0f;
    }
  avg /= ws;
  if (avg * b < 0.0f) return b;
  return b + bonus * avg * (1.0f - fabsf(b));
}

__global__ void k_update_scores(Img I, float minp, const float* __restrict__ iL, const float* __restrict__ iR,
                                const float* __restrict__ iT, const float* __restrict__ iB, float* __restrict__ oL,
                                float* __restrict__ oR, float* __restrict__ oT, float* __restrict__ oB) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  int y = i / I.w, x = i - y * I.w;
  oL[i] = updated_score(I, iL, x, y, minp);
  oR[i] = updated_score(I, iR, x, y, minp);
  oT[i] = updated_score(I, iT, x, y, minp);
  oB[i] = updated_score(I, iB, x, y, minp);
}

__device__ __forceinline__ bool is_max_range(const Img& I, const float4* __restrict__ P, int x, int y) {
  if (!in_image(I, x, y)) return false;
  float r = P[y * I.w + x].w;
  return isinf(r) && r > 0;
}

// changeScoreAccordingToShadowBorderValue; returns new score, sets sidx (-1 if none)
__device__ __forceinline__ float shadow_pass(const Img& I, const float4* __restrict__ P, int x, int y, int ox, int oy,
                                             float b, const float* __restrict__ other, int prb, float minp, int& sidx) {
  sidx = -1;
  if (b < minp) return b;
  if (b == 1.0f && is_max_range(I, P, x + ox, y + oy)) { sidx = (y + oy) * I.w + x + ox; return b; }
  float best = 0.0f;
  for (int d = 1; d <= prb; ++d) {
    int nx = x + d * ox, ny = y + d * oy;
    if (!in_image(I, nx, ny)) continue;
    float s = other[ny * I.w + nx];
    if (s < best) { sidx = ny * I.w + nx; best = s; }
  }
  if (sidx >= 0) {
    b *= fmaxf(0.9f, 1 - pow3f_cr(1 + best));
    if (b >= minp) return b;
  }
  sidx = -1;
  return 0.0f;
}

// phase 1: R and B passes (read the not-yet-updated L / T scores)
__global__ void k_shadow_rb(Img I, const float4* __restrict__ P, int prb, float minp, const float* __restrict__ sL,
                            float* __restrict__ sR, const float* __restrict__ sT, float* __restrict__ sB,
                            int4* __restrict__ sh) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  int y = i / I.w, x = i - y * I.w;
  int a, c;
  sR[i] = shadow_pass(I, P, x, y, 1, 0, sR[i], sL, prb, minp, a);
  sB[i] = shadow_pass(I, P, x, y, 0, 1, sB[i], sT, prb, minp, c);
  int4 s = sh[i];
  s.y = a;  // right
  s.w = c;  // bottom
  sh[i] = s;
}

// phase 2: L and T passes (read the final R / B scores)
__global__ void k_shadow_lt(Img I, const float4* __restrict__ P, int prb, float minp, float* __restrict__ sL,
                            const float* __restrict__ sR, float* __restrict__ sT, const float* __restrict__ sB,
                            int4* __restrict__ sh) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  int y = i / I.w, x = i - y * I.w;
  int a, c;
  sL[i] = shadow_pass(I, P, x, y, -1, 0, sL[i], sR, prb, minp, a);
  sT[i] = shadow_pass(I, P, x, y, 0, -1, sT[i], sB, prb, minp, c);
  int4 s = sh[i];
  s.x = a;  // left
  s.z = c;  // top
  sh[i] = s;
}

__device__ __forceinline__ bool check_max(const Img& I, const float* __restrict__ s, int x, int y, int ox, int oy,
                                          int sidx, int prb) {
  float b = s[y * I.w + x];
  int nx = x - ox, ny = y - oy;
  if (in_image(I, nx, ny) && s[ny * I.w + nx] > b) return false;
  for (int d = 1; d <= prb; ++d) {
    nx = x + d * ox; ny = y + d * oy;
    if (!in_image(I, nx, ny)) continue;
    int ni = ny * I.w + nx;
    if (ni == sidx) return true;
    if (s[ni] > b) return false;
  }
  return true;
}

__global__ void k_classify(Img I, int prb, const float* __restrict__ sL, const float* __restrict__ sR,
                           const float* __restrict__ sT, const float* __restrict__ sB, const int4* __restrict__ sh,
                           uint32_t* __restrict__ traits) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  int4 s = sh[i];
  if (s.x < 0 && s.y < 0 && s.z < 0 && s.w < 0) return;
  int y = i / I.w, x = i - y * I.w;
  const int w = I.w;
  uint32_t own = 0;
  if (s.x >= 0 && check_max(I, sL, x, y, -1, 0, s.x, prb)) {
    own |= TB(T_OBSTACLE_BORDER) | TB(T_OBSTACLE_BORDER_LEFT);
    atomicOr(&traits[s.x], TB(T_SHADOW_BORDER) | TB(T_SHADOW_BORDER_RIGHT));
    int sx = s.x % w;
    for (int i3 = y * w + sx + 1; i3 < i; ++i3) atomicOr(&traits[i3], TB(T_VEIL_POINT) | TB(T_VEIL_POINT_RIGHT));
  }
  if (s.y >= 0 && check_max(I, sR, x, y, 1, 0, s.y, prb)) {
    own |= TB(T_OBSTACLE_BORDER) | TB(T_OBSTACLE_BORDER_RIGHT);
    atomicOr(&traits[s.y], TB(T_SHADOW_BORDER) | TB(T_SHADOW_BORDER_LEFT));
    int sx = s.y % w, sy = s.y / w;
    for (int i3 = i + 1; i3 < sy * w + sx; ++i3) atomicOr(&traits[i3], TB(T_VEIL_POINT) | TB(T_VEIL_POINT_LEFT));
  }
  if (s.z >= 0 && check_max(I, sT, x, y, 0, -1, s.z, prb)) {
    own |= TB(T_OBSTACLE_BORDER) | TB(T_OBSTACLE_BORDER_TOP);
    atomicOr(&traits[s.z], TB(T_SHADOW_BORDER) | TB(T_SHADOW_BORDER_BOTTOM));
    int sy = s.z / w;
    for (int i3 = (sy + 1) * w + x; i3 < i; i3 += w) atomicOr(&traits[i3], TB(T_VEIL_POINT) | TB(T_VEIL_POINT_BOTTOM));
  }
  if (s.w >= 0 && check_max(I, sB, x, y, 0, 1, s.w, prb)) {
    own |= TB(T_OBSTACLE_BORDER) | TB(T_OBSTACLE_BORDER_BOTTOM);
    atomicOr(&traits[s.w], TB(T_SHADOW_BORDER) | TB(T_SHADOW_BORDER_TOP));
    int sy = s.w / w;
    for (int i3 = i + w; i3 < sy * w + x; i3 += w) atomicOr(&traits[i3], TB(T_VEIL_POINT) | TB(T_VEIL_POINT_TOP));
  }
  if (own) atomicOr(&traits[i], own);
}

// RangeImageBorderExtractor::get3dDirection for obstacle borders; rawdir.w = 1 if valid
__global__ void k_border_dir_raw(Img I, const float4* __restrict__ P, const float4* __restrict__ surf,
                                 const float4* __restrict__ smean, const uint8_t* __restrict__ svalid, const uint32_t* __restrict__ traits,
                                 float4* __restrict__ rawdir) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  uint32_t bt = traits[i];
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bt & TB(T_OBSTACLE_BORDER)) {
    int dx = 0, dy = 0;
    if (bt & TB(T_OBSTACLE_BORDER_LEFT)) --dx;
    if (bt & TB(T_OBSTACLE_BORDER_RIGHT)) ++dx;
    if (bt & TB(T_OBSTACLE_BORDER_TOP)) --dy;
    if (bt & TB(T_OBSTACLE_BORDER_BOTTOM)) ++dy;
    if (dx != 0 || dy != 0) {
      int y = i / I.w, x = i - y * I.w;
      float4 point = P[i];
      f3 pt = mk3(point.x, point.y, point.z);
      f3 nbp = calc3d(I, (float)(x + dx), (float)(y + dy), point.w);
      if (svalid[i]) {
        // the neighbour pixel's viewing ray meets the local plane (normal_no_jumps,
        // neighborhood_mean_no_jumps): lambda = n.(mean - sensor) / n.(nbp - sensor)
        const float4 s = surf[i], m = smean[i];
        const f3 nrm = mk3(s.x, s.y, s.z);
        const f3 sensor = mk3(I.to_world.m[3], I.to_world.m[7], I.to_world.m[11]);
        const f3 vd = sub3(nbp, sensor);
        const float lambda = dot3(nrm, sub3(mk3(m.x, m.y, m.z), sensor)) / dot3(nrm, vd);
        nbp = add3(scale3(vd, lambda), sensor);
      }
      f3 d = normalize3(sub3(nbp, pt));  // get3dDirection: `direction.normalize ()`
      out = make_float4(d.x, d.y, d.z, 1.0f);
    }
  }
  rawdir[i] = out;
}

__global__ void k_border_dir_avg(Img I, const float4* __restrict__ P, const float4* __restrict__ surf,
                                 const float4* __restrict__ rawdir, int radius, float min_cos, float thr,
                                 float4* __restrict__ dir) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  float4 r0 = rawdir[i];
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r0.w != 0.0f) {
    int y = i / I.w, x = i - y * I.w;
    f3 base = mk3(r0.x, r0.y, r0.z);
    f3 avg = base;
    float ws = 1.0f;
    float maxd2 = surf[i].w;
    int y0 = max(0, y - radius), y1 = min(y + radius, I.h - 1);
    int x0 = max(0, x - radius), x1 = min(x + radius, I.w - 1);
    for (int y2 = y0; y2 <= y1; ++y2)
      for (int x2 = x0; x2 <= x1; ++x2) {
        int i2 = y2 * I.w + x2;
        float4 r2 = rawdir[i2];
        if (r2.w == 0.0f || i2 == i) continue;
        f3 nb = mk3(r2.x, r2.y, r2.z);
        if (dot3(nb, base) < min_cos) continue;
        float between = dist_change_score(I, P, maxd2, x, y, x2 - x, y2 - y, 1);
        if (fabsf(between) >= thr) continue;
        avg = add3(avg, nb);
        ws += 1.0f;
      }
    if ((int)rintf(ws) >= radius + 1) {
      f3 d = normalize3(avg);  // `average_border_direction->normalize ()`
      out = make_float4(d.x, d.y, d.z, 1.0f);
    }
  }
  dir[i] = out;
}

__global__ void k_surface_change(Img I, const float4* __restrict__ P, const float4* __restrict__ surf,
                                 const uint8_t* __restrict__ svalid, const uint32_t* __restrict__ traits,
                                 const float4* __restrict__ dir, int radius, float* __restrict__ scs,
                                 float4* __restrict__ scd) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  float score = 0.0f;
  f3 d = mk3(0.f, 0.f, 0.f);
  const uint32_t skip = TB(T_VEIL_POINT) | TB(T_SHADOW_BORDER);
  if (!(traits[i] & skip)) {
    float4 bd = dir[i];
    if (bd.w != 0.0f) {
      score = 1.0f;
      d = mk3(bd.x, bd.y, bd.z);
    } else if (svalid[i]) {
      int y = i / I.w, x = i - y * I.w;
      VecAvg va;
      va.init();
      bool beam[9];
      for (int step = 1; step <= radius; ++step) {
        int bi = 0;
        for (int y2 = y - step; y2 <= y + step; y2 += step)
          for (int x2 = x - step; x2 <= x + step; x2 += step) {
            int b = bi++;
            if (step == 1) {
              beam[b] = !(x2 == x && y2 == y);
            } else if (!beam[b]) {
              continue;
            }
            if (!is_valid(I, P, x2, y2)) continue;
            int i2 = y2 * I.w + x2;
            if (traits[i2] & skip) { beam[b] = false; continue; }
            if (!svalid[i2]) continue;
            float4 s2 = surf[i2];
            va.add(mk3(s2.x, s2.y, s2.z));
          }
      }
      if (va.n >= 3) {
        float ev[3];
        f3 evec[3];
        va.pca(ev, evec);
        float mag = sqrtf(ev[2]);
        if (isfinite(mag)) {
          score = mag;
          d = evec[2];
        }
      }
    }
  }
  scs[i] = score;
  scd[i] = make_float4(d.x, d.y, d.z, 0.0f);
}

// ---- NARF interest image: one wave (64-thread block) per pixel ------------------------------
// The region grow of pixel p can only accept pixels whose 3D point lies within R of p (or within
// 2 px), so it stays inside a window whose half-size follows from the pinhole projection:
//   |du| <= fx R (tz + |tx|) / ((tz - R) tz)   (t = p in the range-image frame, tz > R).
// The touched bitmap covers that window (+3 px margin) in LDS; pixels whose window exceeds the
// LDS budget (very close to the sensor) go to the full-image variant.  A pixel touched outside
// its window raises the error flag (the bound is a checked invariant, not an assumption).
constexpr int kWinWords = 2048;     // 65,536-pixel window (e.g. 256 x 256)
constexpr int kFullWords = 9600;    // 640 x 480 bits
constexpr int kQueue = 2048;        // ring buffer of pending pixels
constexpr int kContribCap = 2048;   // k_interest_ff: contributing pixels compacted per batch (4 KB LDS)

__device__ __forceinline__ float norm_angle(float a) {
  const float pi = 3.14159265358979323846f;
  return a >= 0 ? fmodf(a + pi, 2.0f * pi) - pi : -(fmodf(pi - a, 2.0f * pi) - pi);
}

// Row prefix counts of "contributing" pixels (valid, not shadow/veil, scs >= thr): with
// thr = min_scs a pixel whose region-grow window holds none of them has interest exactly 0 (no
// histogram entry, no negative score: 1 * sqrt(0)), so it skips the region grow; the sparse mode
// raises thr (see narf_dev).  rowp is h x (w+1).
__global__ void k_contrib_rows(Img I, const float4* __restrict__ P, const uint32_t* __restrict__ traits,
                               const float* __restrict__ scs, float min_scs, int* __restrict__ rowp) {
  __shared__ int part[1024];
  const int y = blockIdx.x, tid = threadIdx.x;  // one row per workgroup, w <= 1024
  const uint32_t skip = TB(T_SHADOW_BORDER) | TB(T_VEIL_POINT);
  int v = 0;
  if (tid < I.w) {
    const int i = y * I.w + tid;
    v = (isfinite(P[i].w) && !(traits[i] & skip) && scs[i] >= min_scs) ? 1 : 0;
  }
  part[tid] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int add = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += add;
    __syncthreads();
  }
  if (tid < I.w) rowp[y * (I.w + 1) + tid + 1] = part[tid];
  if (tid == 0) rowp[y * (I.w + 1)] = 0;
}

// Packed pixel for the flood-fill masks: (x, y, z, flags) with flags in the bits of w --
// bit 0: valid and not shadow / veil (the grow may accept it), bit 1: scs >= min_scs.
__global__ void k_pack_px(Img I, const float4* __restrict__ P, const uint32_t* __restrict__ traits,
                          const float* __restrict__ scs, float min_scs, float4* __restrict__ pk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  const uint32_t skip = TB(T_SHADOW_BORDER) | TB(T_VEIL_POINT);
  const float4 p = P[i];
  const uint32_t f = ((isfinite(p.w) && !(traits[i] & skip)) ? 1u : 0u) | (scs[i] >= min_scs ? 2u : 0u);
  pk[i] = make_float4(p.x, p.y, p.z, __uint_as_float(f));
}

// Summed-area table of the contributing pixels: sat[y][x] = count in rows [0, y) x columns
// [0, x), (h + 1) x (w + 1) ints, from the row prefixes (one thread per column).
__global__ void k_contrib_sat(Img I, const int* __restrict__ rowp, int* __restrict__ sat) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x > I.w) return;
  int acc = 0;
  sat[x] = 0;
  for (int y = 0; y < I.h; ++y) {
    acc += rowp[y * (I.w + 1) + x];
    sat[(y + 1) * (I.w + 1) + x] = acc;
  }
}

// does the window hold a contributing pixel?  (four table reads, the same in every lane)
__device__ __forceinline__ bool window_contributes(const Img& I, const int* __restrict__ sat, int x0, int y0,
                                                   int ww, int wh, int lane) {
  (void)lane;
  const int W = I.w + 1;
  const int c = sat[(y0 + wh) * W + x0 + ww] - sat[y0 * W + x0 + ww] - sat[(y0 + wh) * W + x0] + sat[y0 * W + x0];
  return c != 0;
}

// histogram cell of the direction angle: 0.5 * normAngle(2 acosf(dvx)) (NarfKeypoint,
// nkdGetDirectionAngle) with glibc's acosf.  The hardware acosf is within 1e-5 of it; the map is
// monotone on each side of acos = pi/2 (where normAngle wraps), so equal cells at both ends of the
// interval (same side) are exact, otherwise glibc's value (pfx_device_math.h) is used.
__device__ __forceinline__ int angle_cell_of(float ac, float d90, float d180) {
  const float angle = 0.5f * norm_angle(2.0f * ac);
  const float cellf = floorf((angle + d90) / d180 * 18);
  if (!(cellf == cellf)) return 0;
  int cell = min(17, (int)rintf(cellf));
  return cell < 0 ? 0 : cell;
}

__device__ __attribute__((noinline)) int angle_cell_exact(float dvx, float d90, float d180) {
  return angle_cell_of(acosf_glibc(dvx), d90, d180);
}

__device__ __forceinline__ int angle_cell(float dvx, float d90, float d180) {
  const float a = acosf(dvx);
  if (!(a == a)) return angle_cell_exact(dvx, d90, d180);
  const float lo = a - 1e-5f, hi = a + 1e-5f;
  const float half_pi = 1.57079632679489661923f;
  if ((lo < half_pi) == (hi < half_pi)) {
    const int cl = angle_cell_of(lo, d90, d180), ch = angle_cell_of(hi, d90, d180);
    if (cl == ch) return cl;
  }
  return angle_cell_exact(dvx, d90, d180);
}

struct InterestParams {
  float radius_squared, radius_reciprocal, min_scs, opt_dist, d90, d180;
  float prune_below;  // sparse mode: min_interest_value (pixels that cannot reach it may stay 0); else -1
  double R;  // search radius for the window bound
  double R_prune;  // sparse mode: radius within which a pixel can reach pos >= min_interest_value
};

// region-grow window of pixel (x, y): |du| <= fx R (tz + |tx|) / ((tz - R) tz) (+3 px margin
// for touched neighbours), the whole image when the point is within ~R of the sensor plane
__device__ __forceinline__ void interest_window(const Img& I, float4 point, int x, int y, double R, int& x0,
                                                int& y0, int& ww, int& wh) {
  x0 = 0; y0 = 0; ww = I.w; wh = I.h;
  const f3 t = aff_apply(I.to_ri, mk3(point.x, point.y, point.z));
  const double tz = t.z;
  if (!(tz > 1.02 * R)) return;
  const double den = (tz - R) * tz;
  const double wx = (double)I.fx * R * (tz + fabs((double)t.x)) / den * 1.01 + 3.0;
  const double wy = (double)I.fy * R * (tz + fabs((double)t.y)) / den * 1.01 + 3.0;
  const int hx = wx > 1e6 ? 1000000 : (int)ceil(wx), hy = wy > 1e6 ? 1000000 : (int)ceil(wy);
  x0 = max(0, x - hx); y0 = max(0, y - hy);
  ww = min(I.w - 1, x + hx) - x0 + 1;
  wh = min(I.h - 1, y + hy) - y0 + 1;
}

// NarfKeypoint's per-pixel contribution of an accepted pixel with scs >= min_scs: histogram
// maximum of the positive score per direction cell, minimum of the negative score (both
// order-free, LDS atomics on float bit patterns of non-negative values)
__device__ __forceinline__ float negative_score(const InterestParams& ip, float sc, float df) {
  const float neg = 1.0f - 0.5f * sc * fmaxf(1.0f - df / ip.opt_dist, 0.0f);
  return neg * neg;
}

__device__ __forceinline__ void contribute(const InterestParams& ip, float sc, float4 dv, float d2, float pd, f3 tmp0,
                                           f3 tmp1, f3 tmp2, unsigned* hist, unsigned* neg_bits) {
  const f3 dir = mk3(dv.x, dv.y, dv.z);
  const float distance = sqrtf(d2);
  const float df = ip.radius_reciprocal * distance;
  const float neg = negative_score(ip, sc, df);
  const float pos = (pd < 2.0f) ? sc : sc * (1.0f - df);
  // (rotation * direction).head<2> (): Affine3f * Vector3f, rows left to right
  const f3 rot = mk3(0.0f + mv3(tmp0, dir), 0.0f + mv3(tmp1, dir), 0.0f + mv3(tmp2, dir));
  const float nrm = sqrtf(rot.x * rot.x + rot.y * rot.y);
  const float dvx = rot.x * (1.0f / nrm);  // Vector2f::normalize (): times the reciprocal
  const int cell = angle_cell(dvx, ip.d90, ip.d180);
  if (pos > 0.0f) atomicMax(&hist[cell], __float_as_uint(pos));
  if (neg < 1.0f) atomicMin(neg_bits, __float_as_uint(neg));
}

// interest = negative score * sqrt(max over cell pairs of h1 h2 normalised angle distance)
__device__ __forceinline__ float interest_value(const unsigned* hist, unsigned neg_bits) {
  float h[18];
  for (int c = 0; c < 18; ++c) h[c] = __uint_as_float(hist[c]);
  float acv = 0.0f;
  for (int c1 = 0; c1 < 17; ++c1) {
    if (h[c1] == 0.0f) continue;
    for (int c2 = c1 + 1; c2 < 18; ++c2) {
      if (h[c2] == 0.0f) continue;
      float nd = 2.0f * (float)(c2 - c1) / (float)18;
      nd = (nd <= 1.0f ? nd : 2.0f - nd);
      float v = h[c1] * h[c2] * nd;
      acv = (v < acv) ? acv : v;
    }
  }
  acv = sqrtf(acv);
  return __uint_as_float(neg_bits) * acv;
}

// rotation to the viewer frame: getTransFromUnitVectorsZY(view, (0,-1,0))
__device__ __forceinline__ void viewer_frame(const Img& I, float4 point, f3& tmp0, f3& tmp1, f3& tmp2) {
  const f3 sensor = mk3(I.to_world.m[3], I.to_world.m[7], I.to_world.m[11]);
  const f3 view = normalized3(sub3(mk3(point.x, point.y, point.z), sensor));
  tmp0 = normalized3(cross3(mk3(0.0f, -1.0f, 0.0f), view));
  tmp1 = normalized3(cross3(view, tmp0));
  tmp2 = normalized3(view);
}

template <int WORDS, bool FULL>
__global__ void __launch_bounds__(64) k_interest(Img I, const float4* __restrict__ P, const uint32_t* __restrict__ traits,
                                                 const float* __restrict__ scs, const float4* __restrict__ scd,
                                                 const int* __restrict__ sat, InterestParams ip,
                                                 const int* __restrict__ list, const int* __restrict__ n_list,
                                                 float* __restrict__ interest, int* __restrict__ fallback,
                                                 int* __restrict__ n_fallback, int* __restrict__ err,
                                                 unsigned long long* __restrict__ work) {
  __shared__ uint32_t bitmap[WORDS];
  __shared__ int queue[kQueue];
  __shared__ unsigned hist[18];
  __shared__ unsigned neg_bits;
  const int lane = threadIdx.x;
  const int npx = list ? *n_list : I.w * I.h;
  const uint32_t skip = TB(T_SHADOW_BORDER) | TB(T_VEIL_POINT);
  unsigned long long n_grown = 0, n_window = 0, n_visits = 0;  // lane 0: region-grow statistics
  for (int it = blockIdx.x; it < npx; it += gridDim.x) {
    const int index = list ? list[it] : it;
    const float4 point = P[index];
    if (!isfinite(point.w) || (traits[index] & skip)) {
      if (lane == 0) interest[index] = 0.0f;
      continue;
    }
    const int y = index / I.w, x = index - y * I.w;
    int x0 = 0, y0 = 0, ww = I.w, wh = I.h;
    if (!FULL) interest_window(I, point, x, y, ip.R, x0, y0, ww, wh);
    if (!FULL && (int64_t)ww * wh > (int64_t)WORDS * 32) {
      if (lane == 0) fallback[atomicAdd(n_fallback, 1)] = index;
      continue;
    }
    if (lane == 0) { n_grown += 1; n_window += (unsigned long long)ww * wh; }
    const int nwords = (ww * wh + 31) >> 5;
    for (int k = lane; k < nwords; k += 64) bitmap[k] = 0u;
    f3 tmp0, tmp1, tmp2;
    viewer_frame(I, point, tmp0, tmp1, tmp2);
    if (lane < 18) hist[lane] = 0u;
    __syncthreads();
    if (lane == 0) {
      neg_bits = __float_as_uint(1.0f);
      queue[0] = index;
      const int lb = (y - y0) * ww + (x - x0);
      bitmap[lb >> 5] |= 1u << (lb & 31);
    }
    __syncthreads();
    // breadth-first region grow; the queue tail is wave-uniform (one wave per workgroup)
    int head = 0, tail = 1;
    while (head < tail) {
      const int take = min(tail - head, 64);
      const bool act = lane < take;
      int index2 = index, x2 = x, y2 = y;
      bool ok = false;
      float pd = 0.0f, d2 = 0.0f;
      if (act) {
        index2 = queue[(head + lane) & (kQueue - 1)];
        y2 = index2 / I.w;
        x2 = index2 - y2 * I.w;
        const float4 point2 = P[index2];
        ok = isfinite(point2.w) && !(traits[index2] & skip);
        pd = (float)max(abs(x2 - x), abs(y2 - y));
        d2 = sq_dist(point, point2);
        if (ok && pd > 2.0f && d2 > ip.radius_squared) ok = false;
      }
      // the 8-neighbourhood of accepted pixels: newly touched pixels are appended with one
      // ballot per neighbour offset
#pragma unroll
      for (int nb = 0; nb < 9; ++nb) {
        const int x3 = x2 + nb % 3 - 1, y3 = y2 + nb / 3 - 1;
        bool fresh = false;
        if (ok && x3 >= 0 && x3 < I.w && y3 >= 0 && y3 < I.h) {
          const int lx = x3 - x0, ly = y3 - y0;
          if (lx < 0 || lx >= ww || ly < 0 || ly >= wh) {
            atomicOr(err, 2);
          } else {
            const int lb = ly * ww + lx;
            const uint32_t bitm = 1u << (lb & 31);
            if (!(bitmap[lb >> 5] & bitm)) fresh = !(atomicOr(&bitmap[lb >> 5], bitm) & bitm);
          }
        }
        const uint64_t m = __ballot(fresh);
        if (fresh) queue[(tail + __popcll(m & __lanemask_lt())) & (kQueue - 1)] = y3 * I.w + x3;
        tail += __popcll(m);
      }
      if (ok) {
        const float sc = scs[index2];
        if (sc >= ip.min_scs) contribute(ip, sc, scd[index2], d2, pd, tmp0, tmp1, tmp2, hist, &neg_bits);
      }
      head += take;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (tail - head > kQueue) {
        if (lane == 0) atomicOr(err, 1);
        break;
      }
    }
    __syncthreads();
    if (lane == 0) {
      interest[index] = interest_value(hist, neg_bits);
      n_visits += (unsigned long long)tail;
    }
    __syncthreads();
  }
  if (lane == 0 && work && n_grown) {
    atomicAdd(&work[0], n_grown);
    atomicAdd(&work[1], n_window);
    atomicAdd(&work[2], n_visits);
  }
}

// Sparse mode, reverse bound: interest(p) <= max pos over p's region (see k_interest_classify),
// so p can reach min_interest_value only through a contributing pixel q (accepted, scs >= min_scs)
// with pos(q) = sc_q (pd <= 1) or sc_q (1 - d / R) >= min_interest_value, i.e. sc_q >= it and
// d = |p - q| <= R (1 - min_interest_value / sc_q).  One wave per such q (few: the high surface-
// change pixels) marks every pixel within that distance (or within 1 px) -- the only candidates.
__global__ void __launch_bounds__(256) k_interest_reach(Img I, const float4* __restrict__ PK,
                                                        const float* __restrict__ scs, InterestParams ip,
                                                        uint8_t* __restrict__ reach) {
  const int lane = threadIdx.x & 63;
  const int npx = I.w * I.h;
  for (int q = blockIdx.x * 4 + (threadIdx.x >> 6); q < npx; q += gridDim.x * 4) {
    const float4 pq = PK[q];
    const float sc = scs[q];
    if ((__float_as_uint(pq.w) & 3u) != 3u || !(sc >= ip.prune_below)) continue;  // wave-uniform
    const int yq = q / I.w, xq = q - yq * I.w;
    const double Rq = ip.R * std::max(0.0, 1.0 - 0.999 * (double)ip.prune_below / (double)sc);
    const float rq2 = (float)(Rq * Rq * 1.0001);
    int x0, y0, ww, wh;
    interest_window(I, pq, xq, yq, Rq, x0, y0, ww, wh);
    for (int r = 0; r < wh; ++r) {
      const int py = y0 + r;
      for (int c = lane; c < ww; c += 64) {
        const int px = x0 + c, p = py * I.w + px;
        const int pd = max(abs(px - xq), abs(py - yq));
        if (pd <= 1 || sq_dist(pq, PK[p]) <= rq2) reach[p] = 1;
      }
    }
  }
}

// Which pixels need the region grow: valid, not shadow / veil, and a contributing pixel in the
// window (summed-area table).  Sparse mode (prune_below = min_interest_value) adds two bounds
// under which the pixel cannot reach min_interest_value (its interest then stays 0):
//  * p and its accepted contributing 8-neighbours are always in the region (pd <= 1 needs no
//    distance test), so interest = neg * sqrt(acv) <= their smallest negative score (acv <= 1);
//  * interest <= max pos (acv <= pos_max^2, neg <= 1) and pos = sc (1 - d / R) for pd >= 2 with
//    sc <= 1, so only a contributing pixel with scs >= min_interest_value within
//    R_prune = R (1 - 0.99 min_interest_value) of p (or within 2 px) can lift p to it.
// Pixels that pass are listed for k_interest_ff; every other pixel's interest is written as 0.
__global__ void __launch_bounds__(256) k_interest_classify(Img I, const float4* __restrict__ P,
                                                           const float4* __restrict__ PK,
                                                           const uint32_t* __restrict__ traits,
                                                           const float* __restrict__ scs,
                                                           const int* __restrict__ rowp, InterestParams ip,
                                                           const uint8_t* __restrict__ reach,
                                                           float* __restrict__ interest, int* __restrict__ list,
                                                           int* __restrict__ n_list,
                                                           unsigned long long* __restrict__ work) {
  const int index = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t skip = TB(T_SHADOW_BORDER) | TB(T_VEIL_POINT);
  bool grow = false, pruned = false;
  if (index < I.w * I.h) {
    const float4 point = P[index];
    if (isfinite(point.w) && !(traits[index] & skip)) {
      const int y = index / I.w, x = index - y * I.w;
      if (ip.prune_below > 0.0f) {
        // sparse mode: k_interest_reach's mark (it implies a contributing pixel in the window,
        // so no summed-area test), then the neighbours' negative-score bound
        grow = reach[index] != 0;
        if (grow) {
          float nb = 1.0f;
          for (int k = 0; k < 9; ++k) {
            const int xq = x + k % 3 - 1, yq = y + k / 3 - 1;
            if (xq < 0 || xq >= I.w || yq < 0 || yq >= I.h) continue;
            const int iq = yq * I.w + xq;
            const float4 q = PK[iq];
            if ((__float_as_uint(q.w) & 3u) != 3u) continue;
            const float df = ip.radius_reciprocal * sqrtf(sq_dist(point, q));
            nb = fminf(nb, negative_score(ip, scs[iq], df));
          }
          grow = !(nb < ip.prune_below);
        }
        pruned = !grow;
      } else {
        int x0, y0, ww, wh;
        interest_window(I, point, x, y, ip.R, x0, y0, ww, wh);
        grow = window_contributes(I, rowp, x0, y0, ww, wh, lane);
      }
    }
    if (!grow) interest[index] = 0.0f;
  }
  const uint64_t m = __ballot(grow);
  if (m) {
    const int leader = __builtin_ctzll(m);
    int base = 0;
    if (lane == leader) base = atomicAdd(n_list, __popcll(m));
    base = __shfl(base, leader);
    if (grow) list[base + __popcll(m & ((1ull << lane) - 1ull))] = index;
  }
  const uint64_t mp = __ballot(pruned);
  if (mp && lane == 0 && work) atomicAdd(&work[3], (unsigned long long)__popcll(mp));
}

// ---- flood-fill region grow (windows of <= 128 rows x <= 128 columns) ---------------------
// Lane l holds rows l and l + 64 of the window, each as two 64-bit masks: A = pixels the region
// grow accepts (valid, not shadow/veil, within 2 px or R of p) and C = accepted pixels that
// contribute (scs >= min_scs).  PCL's breadth-first grow accepts exactly the 8-connected
// component of p in A, obtained here by R <- dilate3x3(R) & A until stable (bit shifts within a
// row, lane shuffles across rows).  Larger windows go to the queue-based k_interest.
struct Rows2 {  // [half h: rows l + 64 h][word w: columns 64 w .. 64 w + 63]
  uint64_t m00 = 0, m01 = 0, m10 = 0, m11 = 0;
};

// m of lane l <- v (v and l wave-uniform): one compare and two v_cndmask
__device__ __forceinline__ void put_row(uint64_t& m, uint64_t v, int l) {
  m = ((int)threadIdx.x == l) ? v : m;
}

// whole-wave lane shifts by one (DPP wave_shr:1 / wave_shl:1, no LDS round trip): lane i gets
// lane i - 1 (up) or lane i + 1 (down); the lane shifted in from outside the wave gets 0
__device__ __forceinline__ uint64_t lane_up1(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xf, 0xf, true);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t lane_dn1(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x130, 0xf, 0xf, true);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t lane_get(uint64_t v, int l) {  // l wave-uniform
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// horizontal 3-dilation of one row held as (lo, hi) words
__device__ __forceinline__ void hdil(uint64_t lo, uint64_t hi, uint64_t& dlo, uint64_t& dhi) {
  dlo = lo | (lo << 1) | (lo >> 1) | (hi << 63);
  dhi = hi | (hi << 1) | (hi >> 1) | (lo >> 63);
}

#ifdef PFX_SHOT_PROFILE
__device__ unsigned long long g_ff_prof[8];  // cycles: window test, masks, flood fill, contributions
#define FF_T(v) const long long v = clock64()
#define FF_ADD(i, a, b) if (lane == 0) atomicAdd(&g_ff_prof[i], (unsigned long long)((b) - (a)))
#else
#define FF_T(v)
#define FF_ADD(i, a, b)
#endif

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5, 8))) k_interest_ff(Img I, const float4* __restrict__ P,
                                                    const float4* __restrict__ PK,
                                                    const uint32_t* __restrict__ traits,
                                                    const float* __restrict__ scs, const float4* __restrict__ scd,
                                                    const int* __restrict__ rowp, InterestParams ip,
                                                    const int* __restrict__ list, const int* __restrict__ n_list,
                                                    float* __restrict__ interest, int* __restrict__ fallback,
                                                    int* __restrict__ n_fallback, int* __restrict__ err,
                                                    unsigned long long* __restrict__ work) {
  __shared__ unsigned hist[18];
  __shared__ unsigned neg_bits;
  __shared__ uint16_t s_px[kContribCap];
  const int lane = threadIdx.x;
  unsigned long long n_grown = 0, n_window = 0, n_visits = 0;
  const int n = *n_list;
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const int index = list[it];
    const float4 point = P[index];
    const int y = index / I.w, x = index - y * I.w;
    int x0, y0, ww, wh;
    interest_window(I, point, x, y, ip.R, x0, y0, ww, wh);
    if (wh > 128 || ww > 128) {
      if (lane == 0) fallback[atomicAdd(n_fallback, 1)] = index;
      continue;
    }
    // acceptance / contribution masks (lanes = columns); four rows per iteration so that their
    // loads are in flight together (the window rows are independent)
    FF_T(q1);
    // Acceptance / contribution masks, computed lazily in groups of four rows (lanes = columns;
    // branch-free per row: the two ballots are the row's masks, written into lane (r & 63)): the
    // band of computed rows starts around p and grows while the component reaches its first or
    // last row -- rows the component cannot reach are never loaded (outside the band A = 0, so
    // the fill cannot enter them before they exist).
    Rows2 A, C;
    const int nwd = ww > 64 ? 2 : 1;
    auto rows4 = [&](int r0) {
      for (int wd = 0; wd < nwd; ++wd) {
        const int c = wd * 64 + lane;
        const bool col = c < ww;
        const int cc = col ? c : 0;
        float4 p2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int rr = r0 + u < wh ? r0 + u : wh - 1;  // clamped: rows past the window are ignored
          p2[u] = PK[(y0 + rr) * I.w + x0 + cc];
        }
        const int adx = abs(x0 + cc - x);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r0 + u;
          if (r >= wh) break;  // wave-uniform
          const uint32_t f = __float_as_uint(p2[u].w);
          const int pd = max(adx, abs(y0 + r - y));
          const float d2 = sq_dist(point, p2[u]);
          // PCL: accepted unless (pd > 2 && d2 > R^2)
          const bool acc = col & ((f & 1u) != 0u) & ((pd <= 2) | !(d2 > ip.radius_squared));
          const bool con = acc & ((f & 2u) != 0u);
          const uint64_t ma = __ballot(acc), mc = __ballot(con);
          const int l = r & 63;
          if (r < 64) {
            if (wd == 0) { put_row(A.m00, ma, l); put_row(C.m00, mc, l); }
            else { put_row(A.m01, ma, l); put_row(C.m01, mc, l); }
          } else {
            if (wd == 0) { put_row(A.m10, ma, l); put_row(C.m10, mc, l); }
            else { put_row(A.m11, ma, l); put_row(C.m11, mc, l); }
          }
        }
      }
    };
    // does the component hold a pixel in window row r?  (wave-uniform)
    Rows2 R;
    auto row_hit = [&](int r) {
      const uint64_t v = r < 64 ? (R.m00 | R.m01) : (R.m10 | R.m11);
      const int l = r & 63;
      return (__builtin_amdgcn_readlane((int)(uint32_t)v, l) | __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l)) != 0;
    };
    const int ry = y - y0, rx = x - x0;
    // computed rows [blo, bhi), four-row groups, at first the groups of rows ry - 1 .. ry + 1
    int blo = max(ry - 1, 0) & ~3, bhi = min(((ry + 1) | 3) + 1, wh);
    for (int r0 = blo; r0 < bhi; r0 += 4) rows4(r0);
    int rows_done = bhi - blo;
    FF_T(q2);
    // 8-connected component of p in A
    if (lane == (ry & 63)) {
      const uint64_t bit = 1ull << (rx & 63);
      if (ry < 64) { if (rx < 64) R.m00 = bit; else R.m01 = bit; }
      else { if (rx < 64) R.m10 = bit; else R.m11 = bit; }
    }
    while (true) {
      uint64_t h00, h01, h10, h11;
      hdil(R.m00, R.m01, h00, h01);
      hdil(R.m10, R.m11, h10, h11);
      // row above: lane-1 of the same half; lane 0 of the upper half takes lane 63 of the lower
      uint64_t u00 = lane_up1(h00), u01 = lane_up1(h01), u10 = lane_up1(h10), u11 = lane_up1(h11);
      uint64_t d00 = lane_dn1(h00), d01 = lane_dn1(h01), d10 = lane_dn1(h10), d11 = lane_dn1(h11);
      if (wh > 64) {  // the two halves meet: row 63 (lane 63, lower) and row 64 (lane 0, upper)
        const uint64_t l63_0 = lane_get(h00, 63), l63_1 = lane_get(h01, 63);
        const uint64_t f0_0 = lane_get(h10, 0), f0_1 = lane_get(h11, 0);
        if (lane == 0) { u10 = l63_0; u11 = l63_1; }
        if (lane == 63) { d00 = f0_0; d01 = f0_1; }
      }
      Rows2 N;
      N.m00 = (h00 | u00 | d00) & A.m00;
      N.m01 = (h01 | u01 | d01) & A.m01;
      N.m10 = (h10 | u10 | d10) & A.m10;
      N.m11 = (h11 | u11 | d11) & A.m11;
      const bool changed = N.m00 != R.m00 || N.m01 != R.m01 || N.m10 != R.m10 || N.m11 != R.m11;
      R = N;
      // the band grows as soon as the component reaches its edge row
      bool grew = false;
      if (blo > 0 && row_hit(blo)) {
        blo -= 4;
        rows4(blo);
        rows_done += 4;
        grew = true;
      }
      if (bhi < wh && row_hit(bhi - 1)) {
        rows4(bhi);
        rows_done += min(4, wh - bhi);
        bhi = min(bhi + 4, wh);
        grew = true;
      }
      if (!grew && !__ballot(changed)) break;
    }
    // checked invariant: the component stays strictly inside the window (unless at the image edge)
    {
      const uint64_t last0 = (ww <= 64) ? (1ull << (ww - 1)) : 0ull;
      const uint64_t last1 = (ww > 64) ? (1ull << (ww - 65)) : 0ull;
      const uint64_t row_lo = R.m00 | R.m01, row_hi = R.m10 | R.m11;
      bool edge = false;
      if (y0 > 0 && lane == 0) edge |= row_lo != 0;
      if (y0 + wh < I.h && lane == ((wh - 1) & 63)) edge |= (wh - 1 < 64 ? row_lo : row_hi) != 0;
      if (x0 > 0) edge |= ((R.m00 | R.m10) & 1ull) != 0;
      if (x0 + ww < I.w) edge |= (((R.m00 | R.m10) & last0) | ((R.m01 | R.m11) & last1)) != 0;
      if (__ballot(edge) && lane == 0) atomicOr(err, 2);
    }
    FF_T(q3);
    FF_ADD(1, q1, q2);
    FF_ADD(2, q2, q3);
    // contributions of the accepted contributing pixels
    f3 tmp0, tmp1, tmp2;
    viewer_frame(I, point, tmp0, tmp1, tmp2);
    if (lane < 18) hist[lane] = 0u;
    if (lane == 0) neg_bits = __float_as_uint(1.0f);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    {
      // the accepted contributing pixels compacted into LDS as window-relative (row << 8 | col)
      // (lane l lists rows l and 64 + l), then contributed 64 at a time by full waves
      const uint64_t M00 = R.m00 & C.m00, M01 = R.m01 & C.m01, M10 = R.m10 & C.m10, M11 = R.m11 & C.m11;
      const int c0 = __popcll(M00) + __popcll(M01), c1 = __popcll(M10) + __popcll(M11);
      int i0 = c0, i1 = c1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int a = __shfl_up(i0, o), b = __shfl_up(i1, o);
        if (lane >= o) { i0 += a; i1 += b; }
      }
      const int tot0 = __shfl(i0, 63);
      const int T = tot0 + __shfl(i1, 63);
      for (int base = 0; base < T; base += kContribCap) {
        int p = i0 - c0 - base;
        auto emit = [&](uint64_t m, int row, int col0) {
          while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            if (p >= 0 && p < kContribCap) s_px[p] = (uint16_t)((row << 8) | (col0 + b));
            ++p;
          }
        };
        emit(M00, lane, 0);
        emit(M01, lane, 64);
        p = tot0 + i1 - c1 - base;
        emit(M10, 64 + lane, 0);
        emit(M11, 64 + lane, 64);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int nb = min(T - base, kContribCap);
        for (int e = lane; e < nb; e += 64) {
          const int v = s_px[e];
          const int xx = x0 + (v & 255), yy = y0 + (v >> 8);
          const int idx2 = yy * I.w + xx;
          const float4 p2 = PK[idx2];
          const float sv = scs[idx2];
          const float4 dv = scd[idx2];
          const float pd = (float)max(abs(xx - x), abs(yy - y));
          contribute(ip, sv, dv, sq_dist(point, p2), pd, tmp0, tmp1, tmp2, hist, &neg_bits);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    FF_T(q4);
    FF_ADD(3, q3, q4);
    const int accepted = __popcll(R.m00) + __popcll(R.m01) + __popcll(R.m10) + __popcll(R.m11);
    int tot = accepted;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if (lane == 0) {
      interest[index] = interest_value(hist, neg_bits);
      n_grown += 1;
      n_window += (unsigned long long)ww * rows_done;
      n_visits += (unsigned long long)tot;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && work && n_grown) {
    atomicAdd(&work[0], n_grown);
    atomicAdd(&work[1], n_window);
    atomicAdd(&work[2], n_visits);
  }
}

__global__ void k_nms(Img I, const float* __restrict__ interest, float min_interest, int nms,
                      int* __restrict__ cand, int* __restrict__ ncand) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= I.w * I.h) return;
  float iv = interest[i];
  if (iv < min_interest) return;
  int y = i / I.w, x = i - y * I.w;
  bool is_max = true;
  for (int y2 = y - 1; y2 <= y + 1 && is_max && nms; ++y2)
    for (int x2 = x - 1; x2 <= x + 1; ++x2) {
      if (!in_image(I, x2, y2)) continue;
      if (interest[y2 * I.w + x2] <= iv) continue;
      is_max = false;
      break;
    }
  if (!is_max) return;
  cand[atomicAdd(ncand, 1)] = i;
}

__global__ void k_gather_cand(const int* __restrict__ cand, int nc, const float4* __restrict__ P,
                              const float* __restrict__ interest, float4* __restrict__ out) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nc) return;
  int i = cand[k];
  float4 p = P[i];
  out[k] = make_float4(p.x, p.y, p.z, interest[i]);
}

__global__ void k_valid_bits(const float4* __restrict__ P, int npx, uint32_t* __restrict__ bits) {
  int wd = blockIdx.x * blockDim.x + threadIdx.x;
  if (wd * 32 >= npx) return;
  uint32_t v = 0;
  for (int b = 0; b < 32; ++b) {
    int i = wd * 32 + b;
    if (i < npx && isfinite(P[i].w)) v |= 1u << b;
  }
  bits[wd] = v;
}

struct HostInterestPoint { float x, y, z, strength; };
bool host_better(const HostInterestPoint& a, const HostInterestPoint& b) { return a.strength > b.strength; }

Img make_img(const pfx_camera& c) {
  Img I;
  I.w = c.width; I.h = c.height;
  I.cx = c.center_x; I.cy = c.center_y; I.fx = c.focal_length_x; I.fy = c.focal_length_y;
  I.fxr = 1 / c.focal_length_x; I.fyr = 1 / c.focal_length_y;
  float F[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  if (c.coordinate_frame == 1) {
    float L[4][4] = {{0, 0, 1, 0}, {-1, 0, 0, 0}, {0, -1, 0, 0}, {0, 0, 0, 1}};
    std::memcpy(F, L, sizeof(F));
  }
  float W[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      W[i][j] = ((c.sensor_pose[i * 4 + 0] * F[0][j] + c.sensor_pose[i * 4 + 1] * F[1][j]) +
                 c.sensor_pose[i * 4 + 2] * F[2][j]) + c.sensor_pose[i * 4 + 3] * F[3][j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) I.to_world.m[i * 4 + j] = W[i][j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I.to_ri.m[i * 4 + j] = W[j][i];
  for (int i = 0; i < 3; ++i)
    I.to_ri.m[i * 4 + 3] = -(I.to_ri.m[i * 4 + 0] * W[0][3] + I.to_ri.m[i * 4 + 1] * W[1][3] +
                             I.to_ri.m[i * 4 + 2] * W[2][3]);
  return I;
}

// host mirror of image_point (same float operation order)
void host_image_point(const Img& I, float px, float py, float pz, float& ix, float& iy) {
  const float* a = I.to_ri.m;
  float tx = a[3] + (a[0] * px + a[1] * py + a[2] * pz);
  float ty = a[7] + (a[4] * px + a[5] * py + a[6] * pz);
  float tz = a[11] + (a[8] * px + a[9] * py + a[10] * pz);
  if (tz <= 0) { ix = iy = -1.0f; return; }
  ix = I.cx + I.fx * tx / tz - 0.0f;
  iy = I.cy + I.fy * ty / tz - 0.0f;
}

NarfState& state(pfx_ctx* ctx) {
  if (!ctx->narf) ctx->narf = new NarfState();
  return *ctx->narf;
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

void range_image_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, const pfx_camera& cam,
                     float4* d_points) {
  PFX_CHECK(cam.width > 0 && cam.height > 0 && (int64_t)cam.width * cam.height < (int64_t(1) << 30),
            "range image: bad image size");
  if (cam.noise_level != 0.0f)
    throw Error(PFX_ERR_UNSUPPORTED, "range image: noise_level != 0 (running-average z-buffer) not supported");
  NarfState& S = state(ctx);
  hipStream_t st = ctx->stream;
  Img I = make_img(cam);
  const int npx = I.w * I.h;
  uint32_t* direct = S.direct.as<uint32_t>(npx);
  uint32_t* fill = S.fill.as<uint32_t>(npx);
  TimeScope ts(ctx, "range_image");
  k_ri_init<<<nblk(npx), 256, 0, st>>>(direct, fill, npx);
  if (n > 0) k_ri_project<<<nblk(n), 256, 0, st>>>(I, x, y, z, n, cam.min_range, direct, fill);
  k_ri_finalize<<<nblk(npx), 256, 0, st>>>(I, direct, fill, d_points);
  check_launch("range image");
}

int64_t narf_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, const pfx_camera& cam,
                 const pfx_narf_params& p, std::vector<int32_t>& out) {
  PFX_CHECK(p.support_size > 0.0f, "narf: support_size must be > 0");
  if (p.no_of_polynomial_approximations_per_point != 0 || p.add_points_on_straight_edges != 0)
    throw Error(PFX_ERR_UNSUPPORTED, "narf: polynomial refinement / straight-edge points not supported");
  PFX_CHECK(p.pixel_radius_plane_extraction >= 0 && p.pixel_radius_plane_extraction <= 4,
            "narf: pixel_radius_plane_extraction must be in [0, 4]");
  NarfState& S = state(ctx);
  hipStream_t st = ctx->stream;
  // the whole keypoint call on its stream (host round trips included): a stage timer
  TimeScope total(ctx, "narf", true);
  Img I = make_img(cam);
  S.w = I.w;
  S.h = I.h;
  const int npx = I.w * I.h;
  PFX_CHECK(npx <= kFullWords * 32 && I.w <= 1024, "narf: image larger than 640x480 pixels is not supported");
  float4* P = S.pts.as<float4>(npx);
  range_image_dev(ctx, x, y, z, n, cam, P);
  float4* surf = S.surf.as<float4>(npx);
  float4* smean = S.smean.as<float4>(npx);
  uint8_t* svalid = S.svalid.as<uint8_t>(npx);
  float *sL = S.sL.as<float>(npx), *sR = S.sR.as<float>(npx), *sT = S.sT.as<float>(npx), *sB = S.sB.as<float>(npx);
  float *uL = S.uL.as<float>(npx), *uR = S.uR.as<float>(npx), *uT = S.uT.as<float>(npx), *uB = S.uB.as<float>(npx);
  int4* sh = S.shadow.as<int4>(npx);
  uint32_t* traits = S.traits.as<uint32_t>(npx);
  float4* rawdir = S.rawdir.as<float4>(npx);
  float4* dir = S.dir.as<float4>(npx);
  float* scs = S.scs.as<float>(npx);
  float4* scd = S.scd.as<float4>(npx);
  float* interest = S.interest.as<float>(npx);
  int* cand = S.cand.as<int>(npx);
  int* counters = S.counters.as<int>(5);
  {
    TimeScope ts(ctx, "narf_border");
    const int step = (p.pixel_radius_plane_extraction / 2) + 1;
    const int nn = (int)std::pow((double)(p.pixel_radius_plane_extraction / step + 1), 2.0);
    k_surface<<<nblk(npx), 256, 0, st>>>(I, P, p.pixel_radius_plane_extraction, step, nn, surf, smean, svalid);
    k_border_scores<<<nblk(npx), 256, 0, st>>>(I, P, surf, svalid, p.pixel_radius_borders, sL, sR, sT, sB);
    k_update_scores<<<nblk(npx), 256, 0, st>>>(I, p.minimum_border_probability, sL, sR, sT, sB, uL, uR, uT, uB);
    PFX_HIP(hipMemsetAsync(sh, 0xff, sizeof(int4) * npx, st));
    PFX_HIP(hipMemsetAsync(traits, 0, sizeof(uint32_t) * npx, st));
    k_shadow_rb<<<nblk(npx), 256, 0, st>>>(I, P, p.pixel_radius_borders, p.minimum_border_probability, uL, uR, uT,
                                           uB, sh);
    k_shadow_lt<<<nblk(npx), 256, 0, st>>>(I, P, p.pixel_radius_borders, p.minimum_border_probability, uL, uR, uT,
                                           uB, sh);
    k_classify<<<nblk(npx), 256, 0, st>>>(I, p.pixel_radius_borders, uL, uR, uT, uB, sh, traits);
    k_border_dir_raw<<<nblk(npx), 256, 0, st>>>(I, P, surf, smean, svalid, traits, rawdir);
    const float deg = 0.017453292519943295769236907684886127134428718885417f;
    const float min_cos = (float)std::cos((double)(120.0f * deg));
    const float thr = 0.95f * p.minimum_border_probability;
    k_border_dir_avg<<<nblk(npx), 256, 0, st>>>(I, P, surf, rawdir, p.pixel_radius_border_direction, min_cos, thr,
                                                dir);
    k_surface_change<<<nblk(npx), 256, 0, st>>>(I, P, surf, svalid, traits, dir, p.pixel_radius_principal_curvature,
                                                scs, scd);
    check_launch("narf border extraction");
  }
  InterestParams ip;
  const float search_radius = 0.5f * p.support_size;
  ip.radius_squared = search_radius * search_radius;
  ip.radius_reciprocal = 1.0f / search_radius;
  ip.min_scs = p.min_surface_change_score;
  ip.opt_dist = p.optimal_distance_to_high_surface_change;
  const float deg = 0.017453292519943295769236907684886127134428718885417f;
  ip.d90 = 90.0f * deg;
  ip.d180 = 180.0f * deg;
  ip.R = search_radius;
  ip.prune_below = p.calculate_sparse_interest_image ? p.min_interest_value : -1.0f;
  ip.R_prune = ip.R * std::max(0.0, 1.0 - 0.99 * (double)p.min_interest_value);
  PFX_HIP(hipMemsetAsync(counters, 0, 5 * sizeof(int), st));
  int* rowp = S.rowp.as<int>((I.w + 1) * I.h);
  int* sat = S.sat.as<int>((I.w + 1) * (I.h + 1));
  unsigned long long* work = S.work.as<unsigned long long>(4);
  PFX_HIP(hipMemsetAsync(work, 0, 4 * sizeof(unsigned long long), st));
  {
    TimeScope ts(ctx, "narf_interest");
    // calculate_sparse_interest_image (PCL default): a pixel can only reach min_interest_value
    // if a contributing pixel with scs >= min_interest_value lies in its region (interest =
    // neg * sqrt(max h1 h2 nd) <= max scs, neg <= 1); pixels without one keep interest 0, which
    // changes no keypoint (NMS and selection only look at pixels >= min_interest_value).
    // (sparse mode: k_interest_reach's marks replace the summed-area window test)
    if (!p.calculate_sparse_interest_image) {
      k_contrib_rows<<<I.h, 1024, 0, st>>>(I, P, traits, scs, ip.min_scs, rowp);
      k_contrib_sat<<<(unsigned)((I.w + 1 + 255) / 256), 256, 0, st>>>(I, rowp, sat);
    }
    int* fb1 = S.fb1.as<int>(npx);
    float4* pk = S.pk.as<float4>(npx);
    k_pack_px<<<nblk(npx), 256, 0, st>>>(I, P, traits, scs, ip.min_scs, pk);
    int* grow_list = reinterpret_cast<int*>(uL);  // uL is dead after k_classify
    uint8_t* reach = S.svalid.as<uint8_t>(npx);    // svalid is dead after k_surface_change
    if (ip.prune_below > 0.0f) {
      PFX_HIP(hipMemsetAsync(reach, 0, npx, st));
      k_interest_reach<<<512, 256, 0, st>>>(I, pk, scs, ip, reach);
      check_launch("k_interest_reach");
    }
    k_interest_classify<<<nblk(npx), 256, 0, st>>>(I, P, pk, traits, scs, sat, ip, reach, interest, grow_list,
                                                   counters + 4, work);
    check_launch("k_interest_classify");
    // waves per CU: 20 alone (interest 0.47 ms); 4 beside the normal estimation of the
    // overlapped step (sweep 20/12/8/4/3/2/1: 161.4/161.4/162.1/162.6/162.7/162.2/159.2 Mpoints/s),
    // where the latency-bound grid build and list set-up on the other stream need wave slots
    const int ff_w = ctx->shared_device ? 4 : 20;
    k_interest_ff<<<256 * ff_w, 64, 0, st>>>(I, P, pk, traits, scs, scd, sat, ip, grow_list, counters + 4, interest,
                                            fb1, counters + 3, counters + 1, work);
    check_launch("k_interest_ff");
    // windows beyond the flood-fill masks: queue-based grow in a windowed LDS bitmap (one
    // workgroup per CU: such windows are few, and an empty launch must not queue a thousand
    // workgroups behind the concurrent list kernels)
    k_interest<kWinWords, false><<<256, 64, 0, st>>>(I, P, traits, scs, scd, sat, ip, fb1, counters + 3,
                                                          interest, cand, counters + 2, counters + 1, work);
    check_launch("k_interest");
    // beyond the windowed bitmap: the whole image (the count stays on the device; no host round
    // trip -- the workgroups exit at once when there is nothing to grow)
    // (a few workgroups: such pixels lie within ~R of the sensor plane and are rare; an empty
    // launch must not hold LDS the concurrent normal estimation needs)
    k_interest<kFullWords, true><<<32, 64, 0, st>>>(I, P, traits, scs, scd, sat, ip, cand, counters + 2, interest,
                                                     nullptr, nullptr, counters + 1, work);
    check_launch("k_interest_full");
  }
  {
    TimeScope ts(ctx, "narf_nms");
    k_nms<<<nblk(npx), 256, 0, st>>>(I, interest, p.min_interest_value, p.do_non_maximum_suppression, cand, counters);
    check_launch("k_nms");
  }
#ifdef PFX_SHOT_PROFILE
  {
    unsigned long long pr[8];
    PFX_HIP(hipStreamSynchronize(st));
    PFX_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_ff_prof), sizeof(pr)));
    fprintf(stderr, "narf ff cycles (summed over pixels): - %llu first rows %llu flood + lazy rows %llu contrib %llu\n", pr[0],
            pr[1], pr[2], pr[3]);
    const unsigned long long z[8] = {};
    PFX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ff_prof), z, sizeof(z)));
  }
#endif
  const int nwords = (npx + 31) / 32;
  // pinned readback block: [4 counters | 4 work words | npx NMS survivors (float4) | npx indices | bits]
  char* hb = static_cast<char*>(S.host(64 + (size_t)npx * (sizeof(float4) + sizeof(int)) + sizeof(uint32_t) * nwords));
  int* h_cnt = reinterpret_cast<int*>(hb);
  unsigned long long* h_work = reinterpret_cast<unsigned long long*>(hb + 16);
  float4* h_pts = reinterpret_cast<float4*>(hb + 64);
  int* h_cand = reinterpret_cast<int*>(hb + 64 + (size_t)npx * sizeof(float4));
  uint32_t* h_valid = reinterpret_cast<uint32_t*>(hb + 64 + (size_t)npx * (sizeof(float4) + sizeof(int)));
  PFX_HIP(hipMemcpyAsync(h_cnt, counters, 4 * sizeof(int), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(h_work, work, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  ctx->stats["narf_interest_grown"] = (int64_t)h_work[0];
  ctx->stats["narf_interest_fullimage"] = h_cnt[2];
  ctx->stats["narf_interest_queue_grown"] = h_cnt[3];
  ctx->stats["narf_interest_window_px"] = (int64_t)h_work[1];
  ctx->stats["narf_interest_visits"] = (int64_t)h_work[2];
  ctx->stats["narf_interest_pruned"] = (int64_t)h_work[3];
  if (h_cnt[1] & 1) throw Error(PFX_ERR_CAPACITY, "narf: interest region-grow queue overflow");
  if (h_cnt[1] & 2) throw Error(PFX_ERR_DEVICE, "narf: interest region left its window bound (internal error)");
  const int nc = h_cnt[0];
  // NMS survivors (point + strength) and the image's validity bits go to the host in one copy
  float4* cpts = S.rawdir.as<float4>(npx);  // rawdir is dead after k_border_dir_avg: reuse
  uint32_t* vbits = reinterpret_cast<uint32_t*>(S.sL.as<float>(npx));  // sL is dead after the update
  {
    TimeScope ts(ctx, "narf_gather");
    if (nc > 0) k_gather_cand<<<nblk(nc), 256, 0, st>>>(cand, nc, P, interest, cpts);
    k_valid_bits<<<nblk(nwords), 256, 0, st>>>(P, npx, vbits);
    check_launch("k_gather_cand");
  }
  if (nc > 0) {
    PFX_HIP(hipMemcpyAsync(h_pts, cpts, sizeof(float4) * nc, hipMemcpyDeviceToHost, st));
    PFX_HIP(hipMemcpyAsync(h_cand, cand, sizeof(int) * nc, hipMemcpyDeviceToHost, st));
  }
  PFX_HIP(hipMemcpyAsync(h_valid, vbits, sizeof(uint32_t) * nwords, hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  // k_gather_cand wrote (x, y, z, strength) plus the pixel index in the sort key: restore raster order
  std::vector<std::pair<int, float4>> ordered(nc);
  for (int k = 0; k < nc; ++k) ordered[k] = std::make_pair(h_cand[k], h_pts[k]);
  std::sort(ordered.begin(), ordered.end(),
            [](const std::pair<int, float4>& a, const std::pair<int, float4>& b) { return a.first < b.first; });
  std::vector<HostInterestPoint> tmp(nc);
  for (int k = 0; k < nc; ++k) {
    const float4& q = ordered[k].second;
    tmp[k] = HostInterestPoint{q.x, q.y, q.z, q.w};
  }
  std::sort(tmp.begin(), tmp.end(), host_better);
  const float md = p.min_distance_between_interest_points * p.support_size;
  const float min_d2 = md * md;
  std::vector<HostInterestPoint> accepted;
  std::vector<int> marked;
  for (size_t k = 0; k < tmp.size(); ++k) {
    if (p.max_no_of_interest_points > 0 && (int)accepted.size() >= p.max_no_of_interest_points) break;
    const HostInterestPoint& a = tmp[k];
    bool too_close = false;
    for (const HostInterestPoint& b : accepted) {
      float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
      // (a - b).squaredNorm () on Vector3f maps: dx^2 + (dy^2 + dz^2)
      if (dx * dx + (dy * dy + dz * dz) < min_d2) { too_close = true; break; }
    }
    if (too_close) continue;
    accepted.push_back(a);
    float ixr, iyr;
    host_image_point(I, a.x, a.y, a.z, ixr, iyr);
    int ix = (int)std::lrint(ixr), iy = (int)std::lrint(iyr);
    if (ix >= 0 && ix < I.w && iy >= 0 && iy < I.h) {
      const int pix = iy * I.w + ix;
      if (h_valid[pix >> 5] & (1u << (pix & 31))) marked.push_back(pix);
    }
  }
  std::sort(marked.begin(), marked.end());
  marked.erase(std::unique(marked.begin(), marked.end()), marked.end());
  out.assign(marked.begin(), marked.end());
  S.have_debug = true;
  ctx->stats["narf_candidates"] = nc;
  ctx->stats["narf_keypoints"] = (int64_t)out.size();
  // which interest formula ran: 0 = NarfKeypoint::calculateCompleteInterestImage (both values of
  // calculate_sparse_interest_image; PCL's sparse heuristics are not reproduced -- pfx.h)
  ctx->stats["narf_interest_formula"] = 0;
  return (int64_t)out.size();
}

void narf_debug(pfx_ctx* ctx, const std::string& which, void* out, int64_t count) {
  if (!ctx->narf || !ctx->narf->have_debug) throw Error(PFX_ERR_INVALID, "narf_debug: no NARF run yet");
  NarfState& S = *ctx->narf;
  const int64_t npx = (int64_t)S.w * S.h;
  if (count < npx) throw Error(PFX_ERR_CAPACITY, "narf_debug: buffer smaller than width*height");
  PFX_HIP(hipStreamSynchronize(ctx->stream));
  if (which == "interest") {
    PFX_HIP(hipMemcpy(out, S.interest.ptr, sizeof(float) * npx, hipMemcpyDeviceToHost));
  } else if (which == "surface_change") {
    PFX_HIP(hipMemcpy(out, S.scs.ptr, sizeof(float) * npx, hipMemcpyDeviceToHost));
  } else if (which == "border_traits") {
    PFX_HIP(hipMemcpy(out, S.traits.ptr, sizeof(uint32_t) * npx, hipMemcpyDeviceToHost));
  } else if (which == "range") {
    std::vector<float4> pts(npx);
    PFX_HIP(hipMemcpy(pts.data(), S.pts.ptr, sizeof(float4) * npx, hipMemcpyDeviceToHost));
    float* o = static_cast<float*>(out);
    for (int64_t i = 0; i < npx; ++i) o[i] = pts[i].w;
  } else {
    throw Error(PFX_ERR_INVALID, "narf_debug: unknown image " + which);
  }
}

void narf_release(pfx_ctx* ctx) {
  if (ctx->narf) {
    ctx->narf->release();
    delete ctx->narf;
    ctx->narf = nullptr;
  }
}

}  // namespace pfx
