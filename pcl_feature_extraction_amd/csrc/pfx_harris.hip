// pfx_harris.hip -- the reference's active-list Harris3D keypoints:
//
//   Keypoints::compute, HARRIS_3D branch          keypoints.h:150-162
//     pcl::HarrisKeypoint3D<PointXYZRGB, PointXYZI> (PCL 1.7 harris_3d.hpp): method HARRIS,
//     radius 0.01 (constructor default), non-maximum suppression, threshold 1e-6, corner
//     refinement (default on)
//   Keypoints::getKeypointsCloud (PointXYZI)       keypoints.h:365-395
//     each refined corner -> its nearest cloud point, kept when d2 < 0.0001
//
// Arithmetic restated in oracle/or_keypoints.cpp (orc_harris3d); neighbour order = FLANN's
// sorted (d2, index) order (PCL searches an unsorted kd-tree here: unpinned).
// Design (MI355X): the normal estimation's FLANN-ordered lists (radius 0.01, pfx_nblist) are
// built once and serve the normals, the response chains and the suppression; lane per point
// for those, wave per corner for the refinement (its neighbourhood moves with the corner: the
// wave gathers the ball of the current position as (d2, index) keys, sorts them in LDS and one
// lane runs PCL's float loop), the snap to the nearest cloud point in the same wave.
#include <cstring>
#include <algorithm>
#include <rocprim/rocprim.hpp>

#include "pfx_internal.h"
#include "pfx_nblist.h"
#include "pfx_neighbors.h"
#include "pfx_eigen6.h"
#include "pfx_wave_sort.h"

namespace pfx {

namespace {

// HarrisKeypoint3D::responseHarris (calculateNormalCovar's SSE branch): lane per list, six
// float chains over the neighbours with a finite normal in list order, / float(count), then
// intensity = 0.04f + det - 0.04f * trace * trace (0 when trace == 0)
__global__ void __launch_bounds__(256) k_harris_response(GridView g, NbLists L, const float* __restrict__ nx,
                                                         const float* __restrict__ ny, const float* __restrict__ nz,
                                                         float* __restrict__ resp) {
  __shared__ int32_t s_rt[9 * 256];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  if (j >= L.nq) return;  // no barriers below
  const int32_t p = L.qpos[j];
  const int k = L.cnt[j];
  const uint32_t key = L.skeys[p];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    block_run(g, key, r, s, len);
    s_rt[r * 256 + tid] = s;
  }
  const uint32_t* lst = L.list + L.off[j];
  const int lg = L.lg[j];
  float sxx = 0.f, sxy = 0.f, sxz = 0.f, syy = 0.f, syz = 0.f, szz = 0.f;
  unsigned count = 0;
  constexpr int kB = 8;
  const int last = k - 1;  // branch-free batches: clamped loads, exact-zero padded terms
  for (int m0 = 0; m0 < k; m0 += kB) {
    float a[kB], b[kB], c[kB];
#pragma unroll
    for (int t = 0; t < kB; ++t) {
      const int m = m0 + t < last ? m0 + t : last;
      const uint32_t e = lst[(int64_t)m << lg];
      const int32_t q = g.perm[s_rt[entry_run(e) * 256 + tid] + (int32_t)entry_off(e)];
      a[t] = nx[q];
      b[t] = ny[q];
      c[t] = nz[q];
    }
#pragma unroll
    for (int t = 0; t < kB; ++t) {
      const bool in = m0 + t < k && isfinite(a[t]);
      sxx = sxx + (in ? a[t] * a[t] : 0.f);
      sxy = sxy + (in ? b[t] * a[t] : 0.f);
      sxz = sxz + (in ? c[t] * a[t] : 0.f);
      syy = syy + (in ? b[t] * b[t] : 0.f);
      syz = syz + (in ? c[t] * b[t] : 0.f);
      szz = szz + (in ? c[t] * c[t] : 0.f);
      count += in ? 1u : 0u;
    }
  }
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c5 = 0.f, c6 = 0.f, c7 = 0.f;
  if (count > 0) {
    const float f = (float)count;
    c0 = sxx / f;
    c1 = sxy / f;
    c2 = sxz / f;
    c5 = syy / f;
    c6 = syz / f;
    c7 = szz / f;
  }
  const float trace = c0 + c5 + c7;
  float v = 0.f;
  if (trace != 0.f) {
    const float det = c0 * c5 * c7 + 2.0f * c1 * c2 * c6 - c2 * c2 * c5 - c1 * c1 * c7 - c6 * c6 * c0;
    v = 0.04f + det - 0.04f * trace * trace;
  }
  resp[g.perm[p]] = v;
}

// non-maximum suppression over the same lists (order-free): finite response >= threshold and
// no neighbour with a larger one
__global__ void __launch_bounds__(256) k_harris_nms(GridView g, NbLists L, const float* __restrict__ resp,
                                                    float thr, uint8_t* __restrict__ flag) {
  __shared__ int32_t s_rt[9 * 256];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  if (j >= L.nq) return;
  const int32_t p = L.qpos[j];
  const int32_t i = g.perm[p];
  const float v = resp[i];
  if (!isfinite(v) || v < thr) return;
  const uint32_t key = L.skeys[p];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    block_run(g, key, r, s, len);
    s_rt[r * 256 + tid] = s;
  }
  const uint32_t* lst = L.list + L.off[j];
  const int lg = L.lg[j], k = L.cnt[j];
  bool is_max = true;
  for (int m = 0; m < k && is_max; ++m) {
    const uint32_t e = lst[(int64_t)m << lg];
    if (v < resp[g.perm[s_rt[entry_run(e) * 256 + tid] + (int32_t)entry_off(e)]]) is_max = false;
  }
  if (is_max) flag[i] = 1;
}

// ---- Harris6D (keypoints.h:164-176): IntensityGradientEstimation + responseTomasi ----------
// IntensityFieldAccessor<PointXYZRGB>: I = float(299 r + 587 g + 114 b) * 0.001f
__device__ __forceinline__ float rgb_intensity(uint32_t c) {
  const int r = (int)((c >> 16) & 255u), g = (int)((c >> 8) & 255u), b = (int)(c & 255u);
  return (float)(299 * r + 587 * g + 114 * b) * 0.001f;
}
// static_cast<uint8_t>(float) as x86-64 gcc compiles it (cvttss2si, low byte): the demeaned
// intensities are far inside int32, where v_cvt_i32_f32 truncates the same way
__device__ __forceinline__ int u8_trunc(float v) { return ((int32_t)v) & 255; }
// IntensityFieldAccessor::demean (write I - mean back into r, g, b) followed by operator()
__device__ __forceinline__ float rgb_demeaned(uint32_t c, float mean) {
  const float iv = rgb_intensity(c) - mean;
  const int r = u8_trunc(iv * 3.34448160535f), g = u8_trunc(iv * 1.70357751278f), b = u8_trunc(iv * 8.77192982456f);
  return (float)(299 * r + 587 * g + 114 * b) * 0.001f;
}

// IntensityGradientEstimation::computeFeature + computePointIntensityGradient, then
// HarrisKeypoint6D's normalisation (|g|^2 > 200 -> unit length, else 0): lane per list, two passes over
// the FLANN-ordered r-neighbours (centroid and mean intensity, then the demeaned 3x3 system)
__global__ void __launch_bounds__(256) k_intensity_gradient(GridView g, NbLists L, const uint32_t* __restrict__ rgb,
                                                            const float* __restrict__ nx, const float* __restrict__ ny,
                                                            const float* __restrict__ nz, float* __restrict__ gx,
                                                            float* __restrict__ gy, float* __restrict__ gz,
                                                            float* __restrict__ grad_out) {
  __shared__ int32_t s_rt[9 * 256];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  if (j >= L.nq) return;  // no barriers below
  const int32_t p = L.qpos[j];
  const int k = L.cnt[j];
  const uint32_t key = L.skeys[p];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    block_run(g, key, r, s, len);
    s_rt[r * 256 + tid] = s;
  }
  const uint32_t* lst = L.list + L.off[j];
  const int lg = L.lg[j];
  auto nbr = [&](int m) { const uint32_t e = lst[(int64_t)m << lg];
                          return g.perm[s_rt[entry_run(e) * 256 + tid] + (int32_t)entry_off(e)]; };
  float cx = 0.f, cy = 0.f, cz = 0.f, mi = 0.f;
  for (int m = 0; m < k; ++m) {
    const int32_t q = nbr(m);
    cx += g.ux[q];
    cy += g.uy[q];
    cz += g.uz[q];
    mi += rgb_intensity(rgb[q]);
  }
  const float rk = 1.0f / (float)k;  // centroid /= float(k): Eigen 3.2 reciprocal
  cx *= rk;
  cy *= rk;
  cz *= rk;
  mi /= (float)k;
  const int32_t i = g.perm[p];
  float o[3];
  if (k < 3) {
    // IntensityGradientEstimation writes NaN; the normalisation's len > 200 test fails on NaN
    // and its else branch zeroes the gradient
    o[0] = o[1] = o[2] = 0.0f;
  } else {
    float A00 = 0.f, A01 = 0.f, A02 = 0.f, A11 = 0.f, A12 = 0.f, A22 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
    for (int m = 0; m < k; ++m) {
      const int32_t q = nbr(m);
      const float px = g.ux[q] - cx, py = g.uy[q] - cy, pz = g.uz[q] - cz;
      const float iv = rgb_demeaned(rgb[q], mi);
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
    colpiv_solve3f(A, bv, xs);
    const float nv[3] = {nx[i], ny[i], nz[i]};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      // Identity - n n^T.  The empty asm pins each coefficient in a register: otherwise the
      // compiler folds (0 - p) * x into x * (-p), which is -0 where the reference's x86 code
      // (IEEE: 0 - (+0) = +0) gets +0 -- the sign of zero gradient components
      float m0 = (r == 0 ? 1.0f : 0.0f) - nv[r] * nv[0];
      float m1 = (r == 1 ? 1.0f : 0.0f) - nv[r] * nv[1];
      float m2 = (r == 2 ? 1.0f : 0.0f) - nv[r] * nv[2];
      asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
      o[r] = (m0 * xs[0] + m1 * xs[1]) + m2 * xs[2];
    }
    float len = (o[0] * o[0] + o[1] * o[1]) + o[2] * o[2];
    if (len > 200.0f) {
      len = (float)(1.0 / sqrt((double)len));
      o[0] = o[0] * len;
      o[1] = o[1] * len;
      o[2] = o[2] * len;
    } else {  // harris_6d.hpp: gradient_x = gradient_y = gradient_z = 0 (NaN gradients included)
      o[0] = o[1] = o[2] = 0.0f;
    }
  }
  gx[i] = o[0];
  gy[i] = o[1];
  gz[i] = o[2];
  if (grad_out) {
    grad_out[3 * (int64_t)i] = o[0];
    grad_out[3 * (int64_t)i + 1] = o[1];
    grad_out[3 * (int64_t)i + 2] = o[2];
  }
}

// HarrisKeypoint6D::responseTomasi: lane per list, the 21 float sums of v v^T over the
// neighbours with a finite normal_x and gradient[0] (v = normal, gradient), then the fourth
// eigenvalue of the 6x6 (pfx_eigen6.h)
__global__ void __launch_bounds__(256) k_harris6d_response(GridView g, NbLists L, const float* __restrict__ nx,
                                                           const float* __restrict__ ny, const float* __restrict__ nz,
                                                           const float* __restrict__ gx, const float* __restrict__ gy,
                                                           const float* __restrict__ gz, float* __restrict__ resp) {
  __shared__ int32_t s_rt[9 * 256];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + tid;
  if (j >= L.nq) return;
  const int32_t p = L.qpos[j];
  const int k = L.cnt[j];
  const uint32_t key = L.skeys[p];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    int32_t s, len;
    block_run(g, key, r, s, len);
    s_rt[r * 256 + tid] = s;
  }
  const uint32_t* lst = L.list + L.off[j];
  const int lg = L.lg[j];
  float cv[21];
#pragma unroll
  for (int e = 0; e < 21; ++e) cv[e] = 0.f;
  for (int m = 0; m < k; ++m) {
    const uint32_t en = lst[(int64_t)m << lg];
    const int32_t q = g.perm[s_rt[entry_run(en) * 256 + tid] + (int32_t)entry_off(en)];
    const float a = nx[q], ga = gx[q];
    if (!isfinite(a) || !isfinite(ga)) continue;
    const float v[6] = {a, ny[q], nz[q], ga, gy[q], gz[q]};
    int e = 0;
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int w = u; w < 6; ++w) {
        cv[e] = cv[e] + v[u] * v[w];
        ++e;
      }
  }
  resp[g.perm[p]] = eigen6f_value3(cv);
}

// matrices column-major as Eigen's Matrix3f::coeff(k)
__device__ __forceinline__ void mat_vec3(const float a[9], const float v[3], float o[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = (a[r] * v[0] + a[3 + r] * v[1]) + a[6 + r] * v[2];
}

// pcl::invert3x3SymMatrix (common/impl/eigen.hpp)
__device__ __forceinline__ float invert3x3_sym(const float c[9], float inv[9]) {
  const float fd_ee = c[4] * c[8] - c[7] * c[5];
  const float ce_bf = c[2] * c[5] - c[1] * c[8];
  const float be_cd = c[1] * c[5] - c[2] * c[4];
  const float det = c[0] * fd_ee + c[1] * ce_bf + c[2] * be_cd;
  if (det != 0.0f) {
    inv[0] = fd_ee;
    inv[1] = inv[3] = ce_bf;
    inv[2] = inv[6] = be_cd;
    inv[4] = c[0] * c[8] - c[2] * c[2];
    inv[5] = inv[7] = c[1] * c[2] - c[0] * c[5];
    inv[8] = c[0] * c[4] - c[1] * c[1];
    const float rdet = 1.0f / det;  // `inverse /= det`: Eigen 3.2 multiplies by the reciprocal
#pragma unroll
    for (int k = 0; k < 9; ++k) inv[k] *= rdet;
  }
  return det;
}

// the (d2, caller index) keys of every cloud point with d2 < rr around (px, py, pz), written to
// key[0..min(k, kWaveSortCap)); returns k (wave-uniform)
__device__ int wave_ball_keys(const GridView& g, float px, float py, float pz, float rr, uint64_t* key, int lane) {
  Runs R;
  query_runs(g, px, py, pz, R);
  const int32_t T = R.pref[9];
  int k = 0;
  for (int32_t t0 = 0; t0 < T; t0 += 64) {
    const int32_t t = t0 + lane;
    bool hit = false;
    uint64_t kv = 0;
    if (t < T) {
      const int32_t pos = run_pos(R, t);
      const float4 v = g.sp[pos];
      const float d2 = flann_d2(px, py, pz, v.x, v.y, v.z);
      hit = d2 < rr;
      kv = nb_key(d2, g.perm[pos]);
    }
    const uint64_t m = __ballot(hit);
    const int slot = k + __popcll(m & lanemask_lt());
    if (hit && slot < kWaveSortCap) key[slot] = kv;
    k += __popcll(m);
  }
  return k;
}

// smallest key among the ball's candidates (no cap): the nearest point, lowest index on ties
__device__ uint64_t wave_ball_min(const GridView& g, float px, float py, float pz, float rr, int lane) {
  Runs R;
  query_runs(g, px, py, pz, R);
  const int32_t T = R.pref[9];
  uint64_t best = ~0ull;
  for (int32_t t = lane; t < T; t += 64) {
    const int32_t pos = run_pos(R, t);
    const float4 v = g.sp[pos];
    const float d2 = flann_d2(px, py, pz, v.x, v.y, v.z);
    if (d2 < rr) best = min(best, nb_key(d2, g.perm[pos]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) best = min(best, (uint64_t)__shfl_xor((long long)best, o));
  return best;
}

// HarrisKeypoint3D::refineCorners + getKeypointsCloud, wave per corner (dynamic queue).  A ball
// with more than kWaveSortCap points is walked in order by repeated wave minima instead.
__global__ void __launch_bounds__(256) k_harris_refine(GridView g, const int32_t* __restrict__ corner, int nc,
                                                       const float* __restrict__ nx, const float* __restrict__ ny,
                                                       const float* __restrict__ nz, float rr, float rr_snap,
                                                       int refine, int* __restrict__ head,
                                                       float* __restrict__ corners_xyz, int32_t* __restrict__ snap) {
  __shared__ uint64_t s_key[4][kWaveSortCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* key = s_key[wv];
  for (;;) {
    int c = 0;
    if (lane == 0) c = atomicAdd(head, 1);
    c = __shfl(c, 0);
    if (c >= nc) break;
    const int32_t i0 = corner[c];
    float px = g.ux[i0], py = g.uy[i0], pz = g.uz[i0];
    for (int it = 0; refine && it < 10; ++it) {
      const float ox = px, oy = py, oz = pz;
      const int k = wave_ball_keys(g, px, py, pz, rr, key, lane);
      float NNT[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, NNTp[3] = {0, 0, 0};
      auto add = [&](int32_t j) {  // one neighbour, PCL's float order
        const float a = nx[j];
        if (!isfinite(a)) return;
        const float nv[3] = {a, ny[j], nz[j]};
        float nnT[9];
#pragma unroll
        for (int col = 0; col < 3; ++col)
#pragma unroll
          for (int row = 0; row < 3; ++row) nnT[3 * col + row] = nv[row] * nv[col];
#pragma unroll
        for (int e = 0; e < 9; ++e) NNT[e] += nnT[e];
        const float pp[3] = {g.ux[j], g.uy[j], g.uz[j]};
        float t[3];
        mat_vec3(nnT, pp, t);
        NNTp[0] += t[0];
        NNTp[1] += t[1];
        NNTp[2] += t[2];
      };
      if (k <= kWaveSortCap) {
        wave_sort_keys(key, k, lane);
        if (lane == 0)
          for (int m = 0; m < k; ++m) add(key_idx(key[m]));
      } else {  // dense ball: walk the keys in order, one wave minimum per step
        uint64_t last = 0;
        for (int m = 0; m < k; ++m) {
          Runs R;
          query_runs(g, px, py, pz, R);
          uint64_t best = ~0ull;
          for (int32_t t = lane; t < R.pref[9]; t += 64) {
            const int32_t pos = run_pos(R, t);
            const float4 v = g.sp[pos];
            const float d2 = flann_d2(px, py, pz, v.x, v.y, v.z);
            const uint64_t kv = nb_key(d2, g.perm[pos]);
            if (d2 < rr && (m == 0 || kv > last)) best = min(best, kv);
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) best = min(best, (uint64_t)__shfl_xor((long long)best, o));
          last = best;
          if (lane == 0) add(key_idx(best));
        }
      }
      float inv[9];
      if (lane == 0 && invert3x3_sym(NNT, inv) != 0.0f) {
        float q[3];
        mat_vec3(inv, NNTp, q);
        px = q[0];
        py = q[1];
        pz = q[2];
      }
      px = __shfl(px, 0);
      py = __shfl(py, 0);
      pz = __shfl(pz, 0);
      const float dx = px - ox, dy = py - oy, dz = pz - oz;
      const float diff = dx * dx + (dy * dy + dz * dz);  // Vector3f squaredNorm (Redux.h x + (y + z))
      wave_lds_sync();  // the key region is rewritten by the next ball
      if (!(diff > 1e-6)) break;
    }
    int32_t s = -1;
    if (isfinite(px) && isfinite(py) && isfinite(pz)) {
      const uint64_t best = wave_ball_min(g, px, py, pz, rr_snap, lane);
      if (best != ~0ull && (double)key_d2(best) < 0.0001) s = key_idx(best);
    }
    if (lane == 0) {
      snap[c] = s;
      corners_xyz[3 * (int64_t)c] = px;
      corners_xyz[3 * (int64_t)c + 1] = py;
      corners_xyz[3 * (int64_t)c + 2] = pz;
    }
  }
}

struct NonNeg {
  __device__ bool operator()(int32_t v) const { return v >= 0; }
};

}  // namespace

namespace {

__global__ void k_fill_f32(float* __restrict__ p, int64_t n, float v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}
void fill_f32(pfx_ctx* ctx, float* p, int64_t n, float v) {
  if (n <= 0) return;
  k_fill_f32<<<(unsigned)ceil_div(n, 256), 256, 0, ctx->stream>>>(p, n, v);
  check_launch("k_fill_f32");
}

// HarrisKeypoint3D/6D::detectKeypoints after the response (resp, caller order): non-maximum
// suppression over the normals' lists, refineCorners (the same loop in harris_3d.hpp and
// harris_6d.hpp) and Keypoints::getKeypointsCloud
int64_t harris_finish_dev(pfx_ctx* ctx, int64_t n, double radius, float threshold, int refine, const float* nx,
                          const float* ny, const float* nz, float* resp, int32_t* out, int64_t cap,
                          float* corners_out, int64_t* n_corners, const char* tag, int32_t* corner_idx_out) {
  hipStream_t st = ctx->stream;
  const NbLists& L = ctx->normals->L;
  const Grid& G = ctx->grid_a;
  uint8_t* flag = ctx->buf("h3_flag").as<uint8_t>(n);
  PFX_HIP(hipMemsetAsync(flag, 0, n, st));
  if (L.nq > 0) {
    const unsigned nb = (unsigned)ceil_div(L.nq, 256);
    k_harris_nms<<<nb, 256, 0, st>>>(view(G), L, resp, threshold, flag);
    check_launch("k_harris_nms");
  }
  // corners in index order
  int32_t* corner = ctx->buf("h3_corner").as<int32_t>(n);
  int64_t* d_cnt = ctx->buf("h3_cnt").as<int64_t>(2);
  size_t tb = 0;
  PFX_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<int32_t>(0), flag, corner, d_cnt, (size_t)n, st));
  void* tmp = ctx->buf("h3_tmp").get(tb + 16);
  PFX_HIP(rocprim::select(tmp, tb, rocprim::counting_iterator<int32_t>(0), flag, corner, d_cnt, (size_t)n, st));
  int64_t nc = 0;
  PFX_HIP(hipMemcpyAsync(&nc, d_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (n_corners) *n_corners = nc;
  ctx->stats[std::string(tag) + "_corners"] = nc;
  if (nc == 0) return 0;
  int32_t* snap = ctx->buf("h3_snap").as<int32_t>(nc);
  float* cxyz = ctx->buf("h3_cxyz").as<float>(3 * nc);
  int* head = ctx->buf("h3_head").as<int>(1);
  PFX_HIP(hipMemsetAsync(head, 0, sizeof(int), st));
  {
    TimeScope ts(ctx, std::string(tag) + "_refine");
    const float rr = (float)(radius * radius);
    // the snap's d2 < 0.0001 test needs every point up to that distance: a ball a little larger
    // than the radius (the grid's cells are >= radius, so the 3x3x3 block still holds it)
    const float rr_snap = (float)((radius * 1.00001) * (radius * 1.00001));
    const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(nc, 4), 2048);
    k_harris_refine<<<blocks, 256, 0, st>>>(view(G), corner, (int)nc, nx, ny, nz, rr, rr_snap, refine, head, cxyz,
                                            snap);
    check_launch("k_harris_refine");
  }
  int32_t* sel = ctx->buf("h3_sel").as<int32_t>(nc);
  size_t tb2 = 0;
  PFX_HIP(rocprim::select(nullptr, tb2, snap, sel, d_cnt + 1, (size_t)nc, NonNeg(), st));
  void* tmp2 = ctx->buf("h3_tmp2").get(tb2 + 16);
  PFX_HIP(rocprim::select(tmp2, tb2, snap, sel, d_cnt + 1, (size_t)nc, NonNeg(), st));
  int64_t k = 0;
  PFX_HIP(hipMemcpyAsync(&k, d_cnt + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipStreamSynchronize(st));
  if (k <= cap && k > 0) PFX_HIP(hipMemcpyAsync(out, sel, sizeof(int32_t) * k, hipMemcpyDeviceToDevice, st));
  if (corners_out && nc <= cap)
    PFX_HIP(hipMemcpyAsync(corners_out, cxyz, sizeof(float) * 3 * nc, hipMemcpyDeviceToDevice, st));
  if (corner_idx_out && nc <= cap)  // the corners' own cloud indices (PCL's output intensity is theirs)
    PFX_HIP(hipMemcpyAsync(corner_idx_out, corner, sizeof(int32_t) * nc, hipMemcpyDeviceToDevice, st));
  return k;
}


}  // namespace

int64_t harris3d_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double radius,
                     float threshold, int refine, int32_t* out, int64_t cap, float* resp_out, float* corners_out,
                     int64_t* n_corners, int32_t* corner_idx_out) {
  PFX_CHECK(n >= 0, "harris3d: negative point count");
  PFX_CHECK(radius > 0.0, "harris3d: radius must be > 0");
  if (n_corners) *n_corners = 0;
  if (n == 0) return 0;
  hipStream_t st = ctx->stream;
  TimeScope total(ctx, "harris3d", true);
  // HarrisKeypoint3D::initCompute: NormalEstimation at the keypoint radius, viewpoint 0
  float* nx = ctx->buf("h3_nx").as<float>(n);
  float* ny = ctx->buf("h3_ny").as<float>(n);
  float* nz = ctx->buf("h3_nz").as<float>(n);
  float* cv = ctx->buf("h3_cv").as<float>(n);
  normals_lists_dev(ctx, x, y, z, n, radius, nx, ny, nz, cv);
  const float vp[3] = {0.f, 0.f, 0.f};
  normals_chains_dev(ctx, ctx, nullptr, 1, vp, nx, ny, nz, cv);
  const NbLists& L = ctx->normals->L;
  const Grid& G = ctx->grid_a;
  float* resp = resp_out ? resp_out : ctx->buf("h3_resp").as<float>(n);
  PFX_HIP(hipMemsetAsync(resp, 0, sizeof(float) * n, st));
  if (L.nq > 0) {
    TimeScope ts(ctx, "harris3d_response");
    const unsigned nb = (unsigned)ceil_div(L.nq, 256);
    k_harris_response<<<nb, 256, 0, st>>>(view(G), L, nx, ny, nz, resp);
    check_launch("k_harris_response");
  }
  return harris_finish_dev(ctx, n, radius, threshold, refine, nx, ny, nz, resp, out, cap, corners_out, n_corners,
                           "harris3d", corner_idx_out);
}

int64_t harris6d_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, const uint32_t* rgb, int64_t n,
                     double radius, float threshold, int refine, int32_t* out, int64_t cap, float* resp_out,
                     float* corners_out, int64_t* n_corners, float* grad_out, int32_t* corner_idx_out) {
  PFX_CHECK(n >= 0, "harris6d: negative point count");
  PFX_CHECK(radius > 0.0, "harris6d: radius must be > 0");
  if (n_corners) *n_corners = 0;
  if (n == 0) return 0;
  hipStream_t st = ctx->stream;
  TimeScope total(ctx, "harris6d", true);
  // HarrisKeypoint6D::detectKeypoints: NormalEstimation at the keypoint radius, viewpoint 0
  float* nx = ctx->buf("h3_nx").as<float>(n);
  float* ny = ctx->buf("h3_ny").as<float>(n);
  float* nz = ctx->buf("h3_nz").as<float>(n);
  float* cv = ctx->buf("h3_cv").as<float>(n);
  normals_lists_dev(ctx, x, y, z, n, radius, nx, ny, nz, cv);
  const float vp[3] = {0.f, 0.f, 0.f};
  normals_chains_dev(ctx, ctx, nullptr, 1, vp, nx, ny, nz, cv);
  const NbLists& L = ctx->normals->L;
  const Grid& G = ctx->grid_a;
  float* gx = ctx->buf("h6_gx").as<float>(n);
  float* gy = ctx->buf("h6_gy").as<float>(n);
  float* gz = ctx->buf("h6_gz").as<float>(n);
  float* resp = resp_out ? resp_out : ctx->buf("h3_resp").as<float>(n);
  // points off the lists (non-finite) keep a NaN gradient and a zero response
  fill_f32(ctx, gx, n, __builtin_nanf(""));
  fill_f32(ctx, gy, n, __builtin_nanf(""));
  fill_f32(ctx, gz, n, __builtin_nanf(""));
  if (grad_out) fill_f32(ctx, grad_out, 3 * n, __builtin_nanf(""));
  PFX_HIP(hipMemsetAsync(resp, 0, sizeof(float) * n, st));
  if (L.nq > 0) {
    const unsigned nb = (unsigned)ceil_div(L.nq, 256);
    {
      TimeScope ts(ctx, "harris6d_gradient");
      k_intensity_gradient<<<nb, 256, 0, st>>>(view(G), L, rgb, nx, ny, nz, gx, gy, gz, grad_out);
      check_launch("k_intensity_gradient");
    }
    {
      TimeScope ts(ctx, "harris6d_response");
      k_harris6d_response<<<nb, 256, 0, st>>>(view(G), L, nx, ny, nz, gx, gy, gz, resp);
      check_launch("k_harris6d_response");
    }
  }
  return harris_finish_dev(ctx, n, radius, threshold, refine, nx, ny, nz, resp, out, cap, corners_out, n_corners,
                           "harris6d", corner_idx_out);
}

}  // namespace pfx
