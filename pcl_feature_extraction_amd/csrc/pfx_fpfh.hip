// pfx_fpfh.hip -- FPFHEstimation<PointXYZRGB,Normal,FPFHSignature33> (evaluation.cpp:593-612,
// features.h:175-196) on gfx950.  SURVEY A.3.
//
//   S        = union of the radius-r neighbourhoods of the queries (or every surface point
//              when input == surface, PCL's special case)            k_fpfh_mark + select
//   SPFH(p)  = 3 x 11 bins of the pair features (p, q), q in N(p)\{p}: each hit adds the same
//              float hist_incr = 100/(|N(p)|-1); the float value of a bin therefore depends
//              only on its hit count c (c sequential adds), so bins are counted with LDS
//              atomics (order-free) and materialised by c ordered adds      k_fpfh_spfh
//   FPFH(q)  = sum over N(q) in FLANN order, skipping d2 == 0, of SPFH(nbr) / d2 (float per bin,
//              double per 11-bin block), then each block scaled to 100      k_fpfh_weight
// SPFH rows are stored by caller index (n_surface x 33 floats, row-major) -- only rows in S
// are written/read.  Neighbour normals are read from a cell-ordered float4 copy (runs of the
// grid are contiguous), positions/coordinates from the grid's packed copy.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_nblist.h"
#include "pfx_neighbors.h"

namespace pfx {
namespace {

constexpr int kBins = 11;
constexpr int kDesc = 33;
constexpr int kCapW = 8192;   // sorted-neighbour capacity of the weighting kernel (LDS: keys + sort scratch)
constexpr int64_t kCapWGlobal = 1 << 22;  // ... of its global-scratch pass (overflow queries)
constexpr int kWOvfBlocks = 16;           // workgroups of that pass
constexpr int kChunkW = 128;  // SPFH rows staged per chunk in the weighting kernel
constexpr int kWT = 1024;     // weighting workgroup: few queries, each as wide as possible
constexpr int kHistCopies = 16;  // SPFH per-wave counter copies

// PCL 1.7 `acos (fabs (a1)) > acos (fabs (a2))` (double acos, correctly rounded by glibc):
// acos is strictly decreasing and distinct floats >= 2^-26 map to distinct rounded values, so
// the test is |a1| < |a2|; below 2^-26 acos(x) rounds as H + (L - x), pi/2 = H + L.
__device__ __forceinline__ bool acos_greater(float a1, float a2) {
  float x1 = fabsf(a1), x2 = fabsf(a2);
  if (x1 >= 1.4901161e-08f || x2 >= 1.4901161e-08f) return x1 < x2;
  const double H = 1.5707963267948966, L = 6.123233995736766e-17;
  return (H + (L - (double)x1)) > (H + (L - (double)x2));
}

__device__ __forceinline__ int bin_of(double v) {
  if (!(v == v)) return 0;  // static_cast<int>(NaN) == INT_MIN on x86 -> clamped to 0
  double f = floor(v);
  int h = (f >= 2147483647.0 || f < -2147483648.0) ? (int)0x80000000 : (int)f;
  return h < 0 ? 0 : (h >= kBins ? kBins - 1 : h);
}

__device__ __forceinline__ double f1_scaled(double f1) {
  const float d_pi = 1.0f / (2.0f * 3.14159265358979323846f);
  return (double)kBins * ((f1 + 3.14159265358979323846) * (double)d_pi);
}

// bin of f1 = glibc's atan2f (PCL: `atan2f (w.dot (n2), n1.dot (n2))`, the fdlibm float routine,
// pfx_device_math.h).  The hardware float atan2 and glibc's are both within a few ulp (< 1e-5 rad)
// of the true value and the bin map is monotone, so when both ends of that interval fall in one
// bin the bin is exact; otherwise (a bin edge within 1e-5 rad) glibc's value is computed.
__device__ __attribute__((noinline)) int bin_f1_exact(float y, float x) {
  return bin_of(f1_scaled((double)atan2f_glibc(y, x)));
}

__device__ __forceinline__ int bin_f1(float y, float x) {
  const float f = atan2f(y, x);
  if (!(f == f)) return 0;  // NaN argument: the exact value is NaN too
  const int lo = bin_of(f1_scaled((double)f - 1e-5)), hi = bin_of(f1_scaled((double)f + 1e-5));
  return lo == hi ? lo : bin_f1_exact(y, x);
}

// pcl::computePairFeatures (features/src/pfh.cpp) + the three bin indices of
// computePointSPFHSignature; Vector4f maps with w = 0.  Degenerate pairs give f = 0.
__device__ __forceinline__ void pair_bins(f3 p1, f3 n1, f3 p2, f3 n2, int& h1, int& h2, int& h3) {
  f3 dp = sub3(p2, p1);
  const float f4 = sqrtf(sqn4(dp));
  const int b_zero_f1 = bin_of(f1_scaled(0.0)), b_zero = bin_of((double)kBins * ((0.0 + 1.0) * 0.5));
  if (f4 == 0.0f) { h1 = b_zero_f1; h2 = h3 = b_zero; return; }
  f3 n1c = n1, n2c = n2;
  const float angle1 = dot4(n1c, dp) / f4;
  const float angle2 = dot4(n2c, dp) / f4;
  float f3o;
  if (acos_greater(angle1, angle2)) {
    n1c = n2; n2c = n1;
    dp = scale3(dp, -1.0f);
    f3o = -angle2;
  } else {
    f3o = angle1;
  }
  f3 v = cross3(dp, n1c);
  const float v_norm = sqrtf(sqn4(v));
  if (v_norm == 0.0f) { h1 = b_zero_f1; h2 = h3 = b_zero; return; }
  v = scale3(v, 1.0f / v_norm);  // `v /= v_norm`: Eigen 3.2 multiplies by the reciprocal
  const f3 w = cross3(n1c, v);
  const float f2 = dot4(v, n2c);
  h1 = bin_f1(dot4(w, n2c), dot4(n1c, n2c));
  h2 = bin_of((double)kBins * (((double)f2 + 1.0) * 0.5));
  h3 = bin_of((double)kBins * (((double)f3o + 1.0) * 0.5));
}

// c sequential float additions of incr starting from 0 (PCL's hist_incr loop), in O(binades):
// inside a binade of s every step adds the same multiple of ulp(s) (incr's position between two
// grid points does not depend on s; an exact half-way case needs one step first, see below);
// steps that would reach the next binade are taken one by one.
__device__ __forceinline__ float repeated_add(float incr, int c) {
  float s = 0.0f;
  int rem = c;
  while (rem > 0) {
    s = s + incr;
    --rem;
    if (rem == 0 || !(s > 0.0f) || !isfinite(s)) break;
    const int e = ilogbf(s);
    const double ulp = ldexp(1.0, e - 23), top = ldexp(1.0, e + 1);
    const double t = (double)incr / ulp;
    if (t - floor(t) == 0.5) {
      // tie: s + incr rounds to even, so one more step leaves s an even multiple of ulp, and from
      // there every step inside this binade adds the same amount (checked against the plain loop
      // for 100 / (k - 1), k < 6000, and random increments)
      s = s + incr;
      --rem;
      if (rem == 0 || ilogbf(s) != e) continue;
    }
    const double delta = (double)(s + incr) - (double)s;
    if (delta <= 0.0) {  // s no longer changes
      rem = 0;
      break;
    }
    int64_t n = (int64_t)ceil((top - (double)s) / delta) - 1;  // s + n delta < top
    if (n > rem) n = rem;
    if (n > 0) {
      s = (float)((double)s + (double)n * delta);
      rem -= (int)n;
    }
  }
  for (; rem > 0; --rem) s = s + incr;  // (after a break on a non-finite or zero sum)
  return s;
}

// ---- fast path of pair_bins ----
// The same float operations as pair_bins up to the first division; then approximate quotients
// (v_rcp / v_rsq), a polynomial atan2 and the bin maps, each feature checked against its bin
// edges with a bound on |approximate - exact-path value| (fractions of a bin: tol).  Any check
// too close to call (an edge within the bound, |angle1| ~ |angle2|, non-finite normals, tiny
// angles) returns false and the caller runs the exact pair_bins.  Bounds (normals |n| <= 1.01):
//   f3 = dot/f4:            |approx - exact| <= 4e-7         used 1e-6
//   f2 = v . n2:            v components within 4e-7, dot    used 4e-6
//   f1 = atan2(w . n2, x):  y within 8e-6 -> 8e-6 / r, atan poly + ops 6e-7, CR rounding 1.2e-7
//                                                            used 1e-6 + 8e-6 / r
// (polynomial: max |atan_poly(a) - atan(a)| = 1.5e-7 on [0, 1] in float Horner, measured).
__device__ __forceinline__ float atan_poly(float a) {
  const float z = a * a;
  float p = -0.00405456405133009f;
  p = p * z + 0.021862948313355446f;
  p = p * z + -0.0559123195707798f;
  p = p * z + 0.0964219719171524f;
  p = p * z + -0.1390862911939621f;
  p = p * z + 0.19946566224098206f;
  p = p * z + -0.33329859375953674f;
  p = p * z + 0.9999993443489075f;
  return p * a;
}

// float evaluation of the bin maps for the fast path: the exact maps are evaluated in double;
// the float forms below differ from them by at most 2.1e-6 bin units (f1: pi rounding + the sum
// and product roundings, x 11/(2 pi); f2/f3: two roundings, x 5.5), so kBinMapSlack is added
// to each feature's tolerance -- no double-precision work per pair.
constexpr float kBinMapSlack = 3e-6f;

__device__ __forceinline__ bool bin_fast_f(float v, float tol, int& h) {
  const float m = floorf(v);
  const float fr = v - m;  // exact (|v| < 2^23)
  if (!(fr > tol && fr < 1.0f - tol)) return false;  // also rejects NaN
  const int b = (int)m;
  h = b < 0 ? 0 : (b >= kBins ? kBins - 1 : b);
  return true;
}

// bin_fast_f without a branch: h is always written (clamped in float, so a NaN or huge value
// converts safely); the result is only used when the return value is true
__device__ __forceinline__ bool bin_fast_nb(float v, float tol, int& h) {
  const float m = floorf(v);
  const float fr = v - m;  // exact (|v| < 2^23)
  h = (int)fminf(fmaxf(m, 0.0f), (float)(kBins - 1));
  return (fr > tol) & (fr < 1.0f - tol);  // also false for NaN
}

__device__ __forceinline__ bool pair_bins_fast(f3 p1, f3 n1, f3 p2, f3 n2, int& h1, int& h2, int& h3) {
  f3 dp = sub3(p2, p1);
  const float s4 = sqn4(dp);
  if (s4 == 0.0f) {  // f4 == 0 in pair_bins
    h1 = bin_of(f1_scaled(0.0));
    h2 = h3 = bin_of((double)kBins * ((0.0 + 1.0) * 0.5));
    return true;
  }
  if (!(isfinite(n1.x) && isfinite(n1.y) && isfinite(n1.z) && isfinite(n2.x) && isfinite(n2.y) && isfinite(n2.z)))
    return false;
  const float d1 = dot4(n1, dp), d2 = dot4(n2, dp);
  const float ad1 = fabsf(d1), ad2 = fabsf(d2);
  const float rf4 = __builtin_amdgcn_rsqf(s4);  // ~ 1 / f4
  if (fmaxf(ad1, ad2) * rf4 < 2e-8f) return false;  // acos_greater's tiny-angle branch
  bool swap;
  if (ad1 < ad2 * (1.0f - 4e-7f)) swap = true;        // |angle1| < |angle2|
  else if (ad1 > ad2 * (1.0f + 4e-7f)) swap = false;
  else return false;
  f3 n1c = n1, n2c = n2;
  float f3a;
  if (swap) {
    n1c = n2; n2c = n1;
    dp = scale3(dp, -1.0f);
    f3a = -d2 * rf4;
  } else {
    f3a = d1 * rf4;
  }
  const f3 v = cross3(dp, n1c);
  const float sv = sqn4(v);
  if (sv == 0.0f) {  // v_norm == 0 in pair_bins
    h1 = bin_of(f1_scaled(0.0));
    h2 = h3 = bin_of((double)kBins * ((0.0 + 1.0) * 0.5));
    return true;
  }
  const f3 vh = scale3(v, __builtin_amdgcn_rsqf(sv));
  const f3 w = cross3(n1c, vh);
  const float f2a = dot4(vh, n2c);
  const float y = dot4(w, n2c), x = dot4(n1c, n2c);
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  if (!(mx > 1e-20f)) return false;
  float t = atan_poly(mn * __builtin_amdgcn_rcpf(mx));
  if (ay > ax) t = 1.57079637f - t;
  if (x < 0.0f) t = 3.14159274f - t;
  const float f1a = y < 0.0f ? -t : t;
  const float d_pi = 1.0f / (2.0f * 3.14159265358979323846f);
  const float tol1 = (1e-6f + 8e-6f * __builtin_amdgcn_rcpf(mx)) * (1.01f * (float)kBins * d_pi) + kBinMapSlack;
  return bin_fast_f((f1a + 3.14159265358979323846f) * ((float)kBins * d_pi), tol1, h1) &&
         bin_fast_f((f2a + 1.0f) * (0.5f * kBins), 4e-6f * 0.5f * kBins + kBinMapSlack, h2) &&
         bin_fast_f((f3a + 1.0f) * (0.5f * kBins), 1e-6f * 0.5f * kBins + kBinMapSlack, h3);
}

// pair_bins_fast for two pairs (p1, p2a) and (p1, p2b) at once: the same float operations
// component by component, the element-wise arithmetic on packed FP32 (v_pk_mul/add_f32: one
// instruction for both pairs, each half rounded exactly as the scalar op), the decisions,
// transcendental approximations and bin maps per component.  p1 / n1 are the S point's
// (wave-uniform, n1 finite: the caller checked).  ok[c] == false: pair c needs the exact path.
typedef float fv2 __attribute__((ext_vector_type(2)));
struct v32 { fv2 x, y, z; };
__device__ __forceinline__ fv2 dot4v(const v32& a, const v32& b) { return (a.x * b.x + a.z * b.z) + (a.y * b.y + 0.0f); }
__device__ __forceinline__ v32 cross3v(const v32& a, const v32& b) {
  return v32{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ fv2 sel2(bool c0, bool c1, fv2 a, fv2 b) { return fv2{c0 ? a.x : b.x, c1 ? a.y : b.y}; }

__device__ __forceinline__ void pair_bins_fast2(f3 p1, f3 n1, bool n1fin, const v32& p2, const v32& n2, int h1[2],
                                                int h2[2], int h3[2], bool ok[2]) {
  const int bz1 = bin_of(f1_scaled(0.0)), bz = bin_of((double)kBins * ((0.0 + 1.0) * 0.5));
  const v32 dp0{p2.x - p1.x, p2.y - p1.y, p2.z - p1.z};
  const fv2 s4 = (dp0.x * dp0.x + dp0.z * dp0.z) + (dp0.y * dp0.y + 0.0f);
  const v32 n1v{fv2(n1.x), fv2(n1.y), fv2(n1.z)};
  const fv2 d1 = dot4v(n1v, dp0), d2 = dot4v(n2, dp0);
  bool sw[2], live[2];
  fv2 rf4;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const bool fin = n1fin && isfinite(n2.x[c]) && isfinite(n2.y[c]) && isfinite(n2.z[c]);
    const float ad1 = fabsf(d1[c]), ad2 = fabsf(d2[c]);
    rf4[c] = __builtin_amdgcn_rsqf(s4[c]);
    sw[c] = ad1 < ad2 * (1.0f - 4e-7f);
    const bool decided = sw[c] || ad1 > ad2 * (1.0f + 4e-7f);
    live[c] = fin && !(fmaxf(ad1, ad2) * rf4[c] < 2e-8f) && decided;
  }
  const fv2 f3a = sel2(sw[0], sw[1], -d2 * rf4, d1 * rf4);
  const v32 n1c{sel2(sw[0], sw[1], n2.x, n1v.x), sel2(sw[0], sw[1], n2.y, n1v.y), sel2(sw[0], sw[1], n2.z, n1v.z)};
  const v32 n2c{sel2(sw[0], sw[1], n1v.x, n2.x), sel2(sw[0], sw[1], n1v.y, n2.y), sel2(sw[0], sw[1], n1v.z, n2.z)};
  const v32 dp{sel2(sw[0], sw[1], -dp0.x, dp0.x), sel2(sw[0], sw[1], -dp0.y, dp0.y), sel2(sw[0], sw[1], -dp0.z, dp0.z)};
  const v32 v = cross3v(dp, n1c);
  const fv2 sv = (v.x * v.x + v.z * v.z) + (v.y * v.y + 0.0f);
  const fv2 rsv{__builtin_amdgcn_rsqf(sv.x), __builtin_amdgcn_rsqf(sv.y)};
  const v32 vh{v.x * rsv, v.y * rsv, v.z * rsv};
  const v32 w = cross3v(n1c, vh);
  const fv2 f2a = dot4v(vh, n2c), y = dot4v(w, n2c), x = dot4v(n1c, n2c);
  fv2 mn, rmx;
  bool big[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float ax = fabsf(x[c]), ay = fabsf(y[c]);
    const float mx = fmaxf(ax, ay);
    mn[c] = fminf(ax, ay);
    big[c] = mx > 1e-20f;
    rmx[c] = __builtin_amdgcn_rcpf(mx);
  }
  // atan_poly on both
  const fv2 a = mn * rmx;
  const fv2 z = a * a;
  fv2 pp = fv2(-0.00405456405133009f);
  pp = pp * z + 0.021862948313355446f;
  pp = pp * z + -0.0559123195707798f;
  pp = pp * z + 0.0964219719171524f;
  pp = pp * z + -0.1390862911939621f;
  pp = pp * z + 0.19946566224098206f;
  pp = pp * z + -0.33329859375953674f;
  pp = pp * z + 0.9999993443489075f;
  fv2 t = pp * a;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float tc = t[c];
    if (fabsf(y[c]) > fabsf(x[c])) tc = 1.57079637f - tc;
    if (x[c] < 0.0f) tc = 3.14159274f - tc;
    t[c] = y[c] < 0.0f ? -tc : tc;
  }
  const float d_pi = 1.0f / (2.0f * 3.14159265358979323846f);
  const fv2 tol1 = (fv2(1e-6f) + 8e-6f * rmx) * (1.01f * (float)kBins * d_pi) + kBinMapSlack;
  const fv2 b1 = (t + 3.14159265358979323846f) * ((float)kBins * d_pi);
  const fv2 b2 = (f2a + 1.0f) * (0.5f * kBins), b3 = (f3a + 1.0f) * (0.5f * kBins);
  // branch-free: every bin map evaluated, the outcome selected (short-circuit && and the
  // if/else chain made the compiler nest exec-mask branches with register copies per level)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    int a1, a2, a3;
    const bool k1 = bin_fast_nb(b1[c], tol1[c], a1);
    const bool k2 = bin_fast_nb(b2[c], 4e-6f * 0.5f * kBins + kBinMapSlack, a2);
    const bool k3 = bin_fast_nb(b3[c], 1e-6f * 0.5f * kBins + kBinMapSlack, a3);
    // f4 == 0, or v_norm == 0, in pair_bins: the zero-feature bins
    const bool zero = (s4[c] == 0.0f) | (live[c] & (sv[c] == 0.0f));
    ok[c] = zero | (live[c] & big[c] & k1 & k2 & k3);
    h1[c] = zero ? bz1 : a1;
    h2[c] = zero ? bz : a2;
    h3[c] = zero ? bz : a3;
  }
}

// the exact path out of line (rare), bins packed h1 | h2 << 8 | h3 << 16
__device__ __attribute__((noinline)) int pair_bins_exact(float p1x, float p1y, float p1z, float n1x, float n1y,
                                                         float n1z, float p2x, float p2y, float p2z, float n2x,
                                                         float n2y, float n2z) {
  int h1, h2, h3;
  pair_bins(mk3(p1x, p1y, p1z), mk3(n1x, n1y, n1z), mk3(p2x, p2y, p2z), mk3(n2x, n2y, n2z), h1, h2, h3);
  return h1 | (h2 << 8) | (h3 << 16);
}

// support (nullable): only the points FPFH reads are copied -- the others may still be being
// written by a concurrent normal-estimation pass (pfx_normals_chains_dev on another stream)
__global__ void k_sorted_normals(const int32_t* __restrict__ perm, int64_t n, const float* __restrict__ nx,
                                 const float* __restrict__ ny, const float* __restrict__ nz,
                                 const uint8_t* __restrict__ support, float4* __restrict__ out,
                                 int* __restrict__ zero9) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (zero9 && i < 9) zero9[i] = 0;
  if (i >= n) return;
  const int32_t p = perm[i];
  if (support && !support[p]) {
    out[i] = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), 0.0f);
    return;
  }
  out[i] = make_float4(nx[p], ny[p], nz[p], 0.0f);
}

// S membership by sorted position
__global__ void __launch_bounds__(256) k_fpfh_mark(GridView g, const float* __restrict__ qx,
                                                   const float* __restrict__ qy, const float* __restrict__ qz,
                                                   int64_t nq, float rr, uint8_t* __restrict__ flags) {
  for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
    Runs R;
    const float x = qx[q], y = qy[q], z = qz[q];
    query_runs(g, x, y, z, R);
    for (int32_t t = threadIdx.x; t < R.pref[9]; t += blockDim.x) {
      const int32_t p = run_pos(R, t);
      const float4 c = g.sp[p];
      if (flann_d2(x, y, z, c.x, c.y, c.z) < rr) flags[p] = 1;
    }
  }
}

// Normals the SPFH stage reads: every r-neighbour of every S point (S = the r-neighbourhoods of
// the queries), by caller index.  One workgroup per S point (sorted positions, device count).
__global__ void __launch_bounds__(256) k_fpfh_mark_support(GridView g, const int32_t* __restrict__ plist,
                                                           const int64_t* __restrict__ n_ptr, float rr,
                                                           uint8_t* __restrict__ mask) {
  const int64_t n = *n_ptr;
  for (int64_t w = blockIdx.x; w < n; w += gridDim.x) {
    Runs R;
    const float4 q = g.sp[plist[w]];
    query_runs(g, q.x, q.y, q.z, R);
    for (int32_t t = threadIdx.x; t < R.pref[9]; t += blockDim.x) {
      const int32_t p = run_pos(R, t);
      const float4 c = g.sp[p];
      if (flann_d2(q.x, q.y, q.z, c.x, c.y, c.z) < rr) mask[g.perm[p]] = 1;
    }
  }
}

// Conservative support: every surface point within 2r of a query (the r-neighbours of the
// r-neighbours lie there).  One workgroup per query over the 5 x 5 x 5 cells around it (cells are
// >= r, so the 2r ball is inside); a superset of k_fpfh_mark_support's set at a fraction of its
// cost (no pass over the SPFH points).
__global__ void __launch_bounds__(256) k_fpfh_mark_ball(GridView g, const float* __restrict__ qx,
                                                        const float* __restrict__ qy, const float* __restrict__ qz,
                                                        int64_t nq, float rr4, uint8_t* __restrict__ mask) {
  for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const float x = qx[q], y = qy[q], z = qz[q];
    if (!(isfinite(x) && isfinite(y) && isfinite(z))) continue;
    const int64_t cx = (int64_t)floor(((double)x - g.ox) * g.inv);
    const int64_t cy = (int64_t)floor(((double)y - g.oy) * g.inv);
    const int64_t cz = (int64_t)floor(((double)z - g.oz) * g.inv);
    const int64_t z0 = max<int64_t>(cz - 2, 0), z1 = min<int64_t>(cz + 2, g.nz - 1);
    if (z0 > z1) continue;
    for (int c = 0; c < 25; ++c) {
      const int64_t ix = cx + c / 5 - 2, iy = cy + c % 5 - 2;
      if (ix < 0 || ix >= g.nx || iy < 0 || iy >= g.ny) continue;
      const int64_t base = (ix * g.ny + iy) * g.nz;
      const int32_t p0 = g.cell_start[base + z0], p1 = g.cell_start[base + z1 + 1];
      for (int32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const float4 c4 = g.sp[p];
        if (flann_d2(x, y, z, c4.x, c4.y, c4.z) <= rr4) mask[g.perm[p]] = 1;
      }
    }
  }
}

__global__ void k_all_finite(const uint32_t* __restrict__ skeys, int64_t n, uint64_t ncells,
                             uint8_t* __restrict__ flags) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (uint64_t)skeys[i] < ncells;
}

// One wave per S point (sorted position, slist[w]): candidates tested in runs, hits other than
// the point itself compacted into a wave-private LDS queue and binned 64 pairs at a time by the
// fast path.  Pairs the fast path cannot bin with certainty go to a global queue for
// k_fpfh_exact (no call to the double-precision path here: fewer registers, more waves); the
// integer bin counts and |N| go to hcount / kcount, k_fpfh_finalize turns them into PCL's floats.
// register budget: 7 waves per SIMD (73 VGPRs; the grid below keeps 16 waves per CU resident):
// fewer spills of the packed-pair code than at 8 (64 VGPRs): SPFH 0.91 -> 0.89 ms, headline
// 182.8 -> 185.0 Mpoints/s over three A/B rounds (6: 183.9, 8 + one run loop: 184.1)
#ifndef PFX_SPFH_WPE
#define PFX_SPFH_WPE 7
#endif
__global__ void __launch_bounds__(256, PFX_SPFH_WPE) k_fpfh_spfh(GridView g, const float4* __restrict__ snp,
                                                      const int32_t* __restrict__ slist,
                                                      const int64_t* __restrict__ count_ptr, float rr,
                                                      int* __restrict__ hcount, int* __restrict__ kcount,
                                                      int2* __restrict__ slowq, unsigned* __restrict__ n_slow,
                                                      unsigned slow_cap, unsigned long long* __restrict__ pairs) {
  __shared__ uint32_t queue[4][192];  // < 128 pending + one 64-candidate push
  // 16 copies of each wave's counters (lane & 15): pairs of a planar patch pile into a few bins,
  // and same-address LDS atomics serialise
  __shared__ int hist[4][kHistCopies][kDesc];
  // wave-uniform values pinned to SGPRs (readfirstlane): the pair path needs the VGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t count = *count_ptr;
  const int64_t stride = (int64_t)gridDim.x * 4;
  unsigned long long wpairs = 0;
  for (int64_t w = xcd_block(blockIdx.x, gridDim.x) * 4 + wv; w < count; w += stride) {
    const int32_t s = __builtin_amdgcn_readfirstlane(slist[w]);
    float4 pc = g.sp[s], pnc = snp[s];
    pc.x = uniformf(pc.x); pc.y = uniformf(pc.y); pc.z = uniformf(pc.z);
    pnc.x = uniformf(pnc.x); pnc.y = uniformf(pnc.y); pnc.z = uniformf(pnc.z);
    const f3 pp = mk3(pc.x, pc.y, pc.z), pn = mk3(pnc.x, pnc.y, pnc.z);
    for (int i = lane; i < kHistCopies * kDesc; i += 64) (&hist[wv][0][0])[i] = 0;
    Runs R;
    query_runs(g, pc.x, pc.y, pc.z, R);
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      R.start[r] = __builtin_amdgcn_readfirstlane(R.start[r]);
      R.pref[r + 1] = __builtin_amdgcn_readfirstlane(R.pref[r + 1]);
    }
    const bool pn_fin = isfinite(pn.x) && isfinite(pn.y) && isfinite(pn.z);
    int k = 0, qn = 0;
    int* hc = hist[wv][lane & (kHistCopies - 1)];
    // a pair the fast path cannot bin goes to the exact-pair queue (or, past its capacity, through
    // the exact path right here, so no pass ever reruns)
    auto defer = [&](bool fast, uint32_t q) {
      const uint64_t m = __ballot(!fast);
      if (m) {
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(n_slow, (unsigned)__popcll(m));
        base = __shfl(base, 0);
        const unsigned slot = base + __popcll(m & lanemask_lt());
        if (!fast) {
          if (slot < slow_cap) {
            slowq[slot] = make_int2((int)w, (int)q);
          } else {
            const float4 qc = g.sp[q], qnv = snp[q];
            const int hb = pair_bins_exact(pp.x, pp.y, pp.z, pn.x, pn.y, pn.z, qc.x, qc.y, qc.z, qnv.x, qnv.y, qnv.z);
            atomicAdd(&hc[hb & 0xff], 1);
            atomicAdd(&hc[kBins + ((hb >> 8) & 0xff)], 1);
            atomicAdd(&hc[2 * kBins + (hb >> 16)], 1);
          }
        }
      }
    };
    // up to 128 queued pairs, two per lane (entries lane and lane + 64) on packed FP32
    auto process = [&](int nvalid) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const bool ina = lane < nvalid, inb = lane + 64 < nvalid;
      const uint32_t qa = ina ? queue[wv][lane] : 0u, qb = inb ? queue[wv][lane + 64] : 0u;
      bool fa = true, fb = true;
      if (ina) {
        const uint32_t qb2 = inb ? qb : qa;
        const float4 ca = g.sp[qa], na = snp[qa], cb = g.sp[qb2], nb = snp[qb2];
        const v32 p2{fv2{ca.x, cb.x}, fv2{ca.y, cb.y}, fv2{ca.z, cb.z}};
        const v32 n2{fv2{na.x, nb.x}, fv2{na.y, nb.y}, fv2{na.z, nb.z}};
        int h1[2], h2[2], h3[2];
        bool ok[2];
        pair_bins_fast2(pp, pn, pn_fin, p2, n2, h1, h2, h3, ok);
        fa = ok[0];
        fb = !inb || ok[1];
        if (fa) {
          atomicAdd(&hc[h1[0]], 1);
          atomicAdd(&hc[kBins + h2[0]], 1);
          atomicAdd(&hc[2 * kBins + h3[0]], 1);
        }
        if (inb && ok[1]) {
          atomicAdd(&hc[h1[1]], 1);
          atomicAdd(&hc[kBins + h2[1]], 1);
          atomicAdd(&hc[2 * kBins + h3[1]], 1);
        }
      }
      defer(fa, qa);
      defer(fb, qb);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    };
    // candidates run by run (contiguous positions: no per-candidate run lookup)
    // (measured and rejected: the run loop not unrolled, runs read by readlane -- one copy of the
    // candidate scan and the pair code, 1.23 -> 1.42 ms)
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int32_t rs = R.start[r], rn = R.pref[r + 1] - R.pref[r];
      for (int32_t t0 = 0; t0 < rn; t0 += 64) {
        const int32_t t = t0 + lane;
        bool hit = false;
        const int32_t pos = rs + t;
        if (t < rn) {
          const float4 c = g.sp[pos];
          hit = flann_d2(pc.x, pc.y, pc.z, c.x, c.y, c.z) < rr;
        }
        k += __popcll(__ballot(hit));
        const bool push = hit && pos != s;
        const uint64_t m = __ballot(push);
        if (push) queue[wv][qn + __popcll(m & lanemask_lt())] = (uint32_t)pos;
        qn += __popcll(m);
        if (qn >= 128) {
          process(128);
          const uint32_t rest = (lane + 128 < qn) ? queue[wv][lane + 128] : 0u;
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
          if (lane + 128 < qn) queue[wv][lane] = rest;
          qn -= 128;
        }
      }
    }
    process(qn);
    if (lane < kDesc) {
      int c = 0;
      for (int j = 0; j < kHistCopies; ++j) c += hist[wv][j][lane];
      hcount[w * kDesc + lane] = c;
    }
    if (lane == 0) kcount[w] = k;
    wpairs += (unsigned long long)(k - 1);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && wpairs) atomicAdd(pairs, wpairs);  // once per wave (same-address atomics serialise)
}

// the deferred pairs through the exact path (double precision), one lane each
__global__ void __launch_bounds__(256) k_fpfh_exact(GridView g, const float4* __restrict__ snp,
                                                    const int32_t* __restrict__ slist,
                                                    const int2* __restrict__ slowq, const unsigned* __restrict__ n_slow,
                                                    unsigned slow_cap, int* __restrict__ hcount,
                                                    unsigned long long* __restrict__ pairs) {
  const unsigned n = min(*n_slow, slow_cap);  // past capacity k_fpfh_spfh took the exact path itself
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) atomicAdd(pairs + 1, (unsigned long long)n);
  for (unsigned j = i; j < n; j += gridDim.x * 256) {
    const int2 e = slowq[j];
    const int32_t s = slist[e.x];
    const float4 pc = g.sp[s], pnc = snp[s], qc = g.sp[e.y], qnv = snp[e.y];
    const int hb = pair_bins_exact(pc.x, pc.y, pc.z, pnc.x, pnc.y, pnc.z, qc.x, qc.y, qc.z, qnv.x, qnv.y, qnv.z);
    int* hc = hcount + (int64_t)e.x * kDesc;
    atomicAdd(&hc[hb & 0xff], 1);
    atomicAdd(&hc[kBins + ((hb >> 8) & 0xff)], 1);
    atomicAdd(&hc[2 * kBins + (hb >> 16)], 1);
  }
}

// PCL's float histogram: hist[b] += 100 / (|N| - 1) once per pair (repeated_add), per S point
__global__ void __launch_bounds__(256) k_fpfh_finalize(GridView g, const int32_t* __restrict__ slist,
                                                       const int64_t* __restrict__ count_ptr,
                                                       const int* __restrict__ hcount,
                                                       const int* __restrict__ kcount, float* __restrict__ spfh) {
  const int64_t count = *count_ptr;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < count * kDesc; e += (int64_t)gridDim.x * 256) {
    const int64_t w = e / kDesc;
    const int b = (int)(e - w * kDesc);
    const float incr = 100.0f / (float)(kcount[w] - 1);
    spfh[(int64_t)g.perm[slist[w]] * kDesc + b] = repeated_add(incr, hcount[e]);
  }
}

// exponent of the least significant set bit of a finite nonzero float; 1000 for non-finite
__device__ __forceinline__ int lsb_exp(float v) {
  const uint32_t b = __float_as_uint(v);
  const int e = (int)((b >> 23) & 0xff);
  if (e == 255) return 1000;
  const uint32_t m = (b & 0x7fffffu) | (e ? 0x800000u : 0u);
  return (e ? e : 1) - 150 + __builtin_ctz(m);
}

// A lower bound of lsb_exp for the per-neighbour step of k_fpfh_weight_lists: a float of biased
// exponent e is a multiple of 2^(max(e, 1) - 150), so the block-sum test stays sufficient (every
// addend a multiple of 2^L, total below 2^(L + 52)) with the exponent alone -- two instructions
// instead of the trailing-zero count; only its margin shrinks, by the addends' trailing zeros
// (1000 for a non-finite value, as lsb_exp)
__device__ __forceinline__ int lsb_exp_bound(float v) {
  const int e = (int)((__float_as_uint(v) >> 23) & 0xff);
  return e == 255 ? 1000 : (e ? e : 1) - 150;
}

// Weighting: one 1024-thread workgroup per query.  The 33 float chains (strict FLANN order)
// run one per lane over SPFH rows staged in LDS.  The three double block sums are formed in
// parallel: every value is a non-negative float, so when all of them are multiples of 2^L and
// the total is below 2^(L+52) every partial sum -- of the sequential loop or of any other order
// -- is exact and the parallel sum is bit-identical to PCL's loop; otherwise the block sum is
// recomputed sequentially.
// GLOBAL = false: the sorted keys in LDS (kCapW); a query with more neighbours is pushed to
// `ovf`.  GLOBAL = true: the overflow queries (count read on the device), keys in a
// per-workgroup global scratch slice of gcap (PCL has no neighbour limit; kCapWGlobal here).
template <bool GLOBAL>
__global__ void __launch_bounds__(kWT) k_fpfh_weight(GridView g, const float* __restrict__ qx,
                                                     const float* __restrict__ qy, const float* __restrict__ qz,
                                                     int64_t nq, float rr, const float* __restrict__ spfh,
                                                     float* __restrict__ out, int* __restrict__ err,
                                                     int32_t* __restrict__ ovf, int* __restrict__ n_ovf,
                                                     uint64_t* __restrict__ scratch, int gcap) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys_lds[];  // kCapW keys + kCapW sort scratch
  __shared__ BucketLdsT<kWT> SB;
  uint64_t* keys = GLOBAL ? scratch + (size_t)blockIdx.x * gcap : keys_lds;
  const int kcap = GLOBAL ? gcap : kCapW;
  __shared__ float rows[kChunkW][kDesc + 1];
  __shared__ float wts[kChunkW];
  __shared__ double red_s[3][kWT / 64];
  __shared__ int red_l[3][kWT / 64];
  __shared__ int s_count;
  __shared__ double s_sum[3];
  const int tid = threadIdx.x;
  const int64_t count = GLOBAL ? (int64_t)*n_ovf : nq;
  for (int64_t w = blockIdx.x; w < count; w += gridDim.x) {
    const int64_t q = GLOBAL ? (int64_t)ovf[w] : w;
    // LDS: bucketed sort (a few barrier phases); global scratch: the bitonic network
    const int k = GLOBAL ? sorted_neighbors(g, qx[q], qy[q], qz[q], rr, keys, kcap, &s_count)
                         : sorted_neighbors_bucketed<kWT>(g, qx[q], qy[q], qz[q], rr, keys, keys + kCapW, kcap,
                                                          &s_count, SB);
    if (k > kcap) {
      const bool give_up = GLOBAL || !ovf;
      if (tid == 0) {
        if (give_up) atomicMax(err, k);
        else ovf[atomicAdd(n_ovf, 1)] = (int32_t)q;  // weighted by the global-scratch pass
      }
      // beyond every capacity: a NaN row (never the previous call's contents); the sticky word
      // reports PFX_ERR_CAPACITY after the next synchronisation
      if (give_up && tid < kDesc) out[q * kDesc + tid] = __builtin_nanf("");
      continue;
    }
    if (k == 0) {
      if (tid < kDesc) out[q * kDesc + tid] = __builtin_nanf("");
      __syncthreads();
      continue;
    }
    float fh = 0.0f;
    double ps0 = 0.0, ps1 = 0.0, ps2 = 0.0;
    int pl0 = 1 << 20, pl1 = 1 << 20, pl2 = 1 << 20;
    // rows of a chunk (+ its weights in column kDesc); LDS path: two buffers in the freed sort
    // scratch, so waves 1.. stage chunk c + 1 (and form chunk c's block partial sums) while wave 0
    // runs the 33 float chains over chunk c -- one barrier per chunk, the chains never wait for
    // a gather.  Global-scratch path: one buffer, stage then chain.
    constexpr int RS = kDesc + 1;
    float* rb0 = GLOBAL ? &rows[0][0] : reinterpret_cast<float*>(keys_lds + kCapW);
    float* rb1 = GLOBAL ? rb0 : rb0 + kChunkW * RS;
    const int nch = (k + kChunkW - 1) / kChunkW;
    auto stage = [&](int c, float* rbuf, int t0, int nt) {
      const int c0 = c * kChunkW, m = min(kChunkW, k - c0), tot = m * kDesc;
      // every row load first (clamped index: all issued back to back), then the LDS stores -- a
      // load-then-store loop waited for each load in turn, one global latency per element a
      // thread stages, on the critical path of the slowest query's chunk sequence
      constexpr int PER = (kChunkW * kDesc + (kWT - 64) - 1) / (kWT - 64);
      float v[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = min(t0 + u * nt, tot - 1);
        const int j = e / kDesc, b = e - j * kDesc;
        v[u] = spfh[(int64_t)key_idx(keys[c0 + j]) * kDesc + b];
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = t0 + u * nt;
        if (e < tot) {
          const int j = e / kDesc, b = e - j * kDesc;
          rbuf[j * RS + b] = v[u];
        }
      }
      for (int j = t0; j < m; j += nt) {
        const float d2 = key_d2(keys[c0 + j]);
        rbuf[j * RS + kDesc] = d2 == 0.0f ? 0.0f : 1.0f / d2;  // 0 marks a skipped neighbour (d2 == 0)
      }
    };
    stage(0, rb0, tid, kWT);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      const int c0 = c * kChunkW, m = min(kChunkW, k - c0);
      const float* cur = (c & 1) ? rb1 : rb0;
      if (!GLOBAL && tid >= 64 && c + 1 < nch) stage(c + 1, (c & 1) ? rb0 : rb1, tid - 64, kWT - 64);
      if (tid < kDesc) {
        // skipped neighbours have w = 0: SPFH rows are finite and fh >= +0, so adding the +0
        // product leaves fh unchanged bit for bit (== PCL's `continue`)
#pragma unroll 8
        for (int j = 0; j < m; ++j) fh = fh + cur[j * RS + tid] * cur[j * RS + kDesc];
      }
      const int pt0 = GLOBAL ? tid : tid - 64, pnt = GLOBAL ? kWT : kWT - 64;
      if (pt0 >= 0) {
        for (int e = pt0; e < m * kDesc; e += pnt) {
          const int j = e / kDesc, b = e - j * kDesc;
          const float w = cur[j * RS + kDesc];
          if (w == 0.0f) continue;
          const float v = cur[j * RS + b] * w;
          if (v != 0.0f) {
            const int l = lsb_exp(v);
            if (b < kBins) { ps0 += (double)v; pl0 = min(pl0, l); }
            else if (b < 2 * kBins) { ps1 += (double)v; pl1 = min(pl1, l); }
            else { ps2 += (double)v; pl2 = min(pl2, l); }
          }
        }
      }
      __syncthreads();
      if (GLOBAL && c + 1 < nch) {
        stage(c + 1, rb0, tid, kWT);
        __syncthreads();
      }
    }
    // block reduction (any order: only used when every partial sum is exact)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ps0 += __shfl_xor(ps0, o); ps1 += __shfl_xor(ps1, o); ps2 += __shfl_xor(ps2, o);
      pl0 = min(pl0, __shfl_xor(pl0, o)); pl1 = min(pl1, __shfl_xor(pl1, o)); pl2 = min(pl2, __shfl_xor(pl2, o));
    }
    if ((tid & 63) == 0) {
      const int wv = tid >> 6;
      red_s[0][wv] = ps0; red_s[1][wv] = ps1; red_s[2][wv] = ps2;
      red_l[0][wv] = pl0; red_l[1][wv] = pl1; red_l[2][wv] = pl2;
    }
    __syncthreads();
    if (tid < 3) {
      double t = 0.0;
      int l = 1 << 20;
      for (int wv = 0; wv < kWT / 64; ++wv) { t += red_s[tid][wv]; l = min(l, red_l[tid][wv]); }
      red_s[tid][0] = t;
      red_l[tid][0] = l;
    }
    __shared__ int s_inexact;
    if (tid == 0) {
      s_inexact = 0;
      atomicMax(err + 1, k);
    }
    __syncthreads();
    if (tid < 3) {
      const int blk = tid;
      const double sum = red_s[blk][0];
      const int L = red_l[blk][0];
      const bool exact = sum == 0.0 || (L < 1000 && sum < ldexp(1.0, L + 52));
      s_sum[blk] = sum;
      if (!exact) atomicOr(&s_inexact, 1 << blk);
    }
    __syncthreads();
    const int inexact = s_inexact;
    if (tid == 0 && inexact) atomicAdd(err + 2, 1);
    if (inexact) {  // PCL's sequential double loop for the blocks that need it, rows staged in LDS
      double seq = 0.0;
      for (int c0 = 0; c0 < k; c0 += kChunkW) {
        const int m = min(kChunkW, k - c0);
        for (int e = tid; e < m * kDesc; e += kWT) {
          const int j = e / kDesc, b = e - j * kDesc;
          rows[j][b] = spfh[(int64_t)key_idx(keys[c0 + j]) * kDesc + b];
        }
        if (tid < m) {
          const float d2 = key_d2(keys[c0 + tid]);
          wts[tid] = d2 == 0.0f ? 0.0f : 1.0f / d2;
        }
        __syncthreads();
        if (tid < 3 && ((inexact >> tid) & 1)) {
          for (int j = 0; j < m; ++j) {
            const float w = wts[j];
            if (w == 0.0f) continue;
#pragma unroll
            for (int b = 0; b < kBins; ++b) seq = seq + (double)(rows[j][tid * kBins + b] * w);
          }
        }
        __syncthreads();
      }
      if (tid < 3 && ((inexact >> tid) & 1)) s_sum[tid] = seq;
      __syncthreads();
    }
    if (tid < 3) {
      double sum = s_sum[tid];
      if (sum != 0.0) sum = 100.0 / sum;
      s_sum[tid] = sum;
    }
    __syncthreads();
    if (tid < kDesc) out[q * kDesc + tid] = fh * (float)s_sum[tid / kBins];
    __syncthreads();
  }
}

// Weighting for input == surface (PCL's all-points branch): the queries are the surface's grid
// points, so their FLANN-ordered neighbour lists come from build_lists (pfx_nblist.hip).  One
// wave per query: 64 list entries at a time are resolved by the lanes (position, caller index,
// w = 1/d2), then lane b < 33 runs bin b's float chain over them in list order, reading the
// neighbours' SPFH rows 8 at a time (loads in flight together).  Block sums: each lane's double
// partial sum + smallest binade, combined in any order when exact (as k_fpfh_weight), else PCL's
// sequential loop by one lane per block.
#ifndef PFX_WL_PIPE
#define PFX_WL_PIPE 2
#endif
#ifndef PFX_W_BLOCKS  // workgroups launched for the keypoint weighting (static query stride, one per CU resident)
#define PFX_W_BLOCKS 512
#endif
#ifndef PFX_WL_GRID  // workgroups per CU launched for the all-points weighting (static query stride)
#define PFX_WL_GRID 32
#endif
__device__ __forceinline__ int32_t entry_pos(uint32_t e, const int32_t (&rs)[9]) {
  const int r = entry_run(e);
  int32_t s = rs[0];
#pragma unroll
  for (int i = 1; i < 9; ++i) s = r == i ? rs[i] : s;
  return s + (int32_t)entry_off(e);
}

template <bool BUF>  // BUF: ns * 132 B < 2^31, the SPFH rows read through a buffer descriptor
__global__ void __launch_bounds__(256) k_fpfh_weight_lists(GridView g, const int32_t* __restrict__ qpos,
                                                           const int64_t* __restrict__ loff,
                                                           const int32_t* __restrict__ lcnt,
                                                           const uint8_t* __restrict__ llg,
                                                           const uint32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ skeys, int64_t nq,
                                                           const float* __restrict__ spfh, float* __restrict__ out,
                                                           int* __restrict__ err) {
  __shared__ double s_ps[4][kDesc];
  __shared__ int s_pl[4][kDesc];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int kmax = 0;  // added to err[1] once per wave (same-address atomics serialise)
#if PFX_WL_PIPE == 2
  // the SPFH rows through a buffer descriptor (32-bit offsets; the caller keeps ns * 132 B below
  // 2^31): lanes >= 33 read bin 0 of the row (in range; their values are never stored)
  const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(spfh), 0, 0x7fffffff,
                                                                          0x00020000);
  const int vlane = (lane < kDesc ? lane : 0) * 4;
#endif
  for (int64_t j = (int64_t)blockIdx.x * 4 + wv; j < nq; j += nw) {
    // (wave-uniform: scalar registers, so the per-neighbour bounds stay scalar)
    const int32_t qp = __builtin_amdgcn_readfirstlane(qpos[j]);
    const int k = __builtin_amdgcn_readfirstlane(lcnt[j]);
    const int64_t off = loff[j];
    const int lg = __builtin_amdgcn_readfirstlane(llg[j]);
    Runs R;
    block_runs(g, skeys[qp], R);
    int32_t rs[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) rs[r] = R.start[r];
    const float4 q = g.sp[qp];
    const int32_t qi = g.perm[qp];
    float fh = 0.0f;
    double ps = 0.0;
    int pl = 1 << 20;
#if PFX_WL_PIPE == 2
    // Round 6: the per-neighbour step without branches or 64-bit address arithmetic.  The SPFH
    // row load is a buffer load (descriptor built once, the row offset id * 132 B in an SGPR, the
    // lane's bin offset in a VGPR); the double block partial sum adds every value (all are
    // non-negative floats -- SPFH percentages times 1/d2 -- and a skipped neighbour's is +0, which
    // leaves a non-negative double sum unchanged), and only the smallest set-bit exponent is
    // selected per value.  The branchy form spent ~16 scalar instructions per neighbour on the exec
    // mask (k_fpfh_weight_lists: 24 VALU + 16 SALU per neighbour step).
    for (int c0 = 0; c0 < k; c0 += 64) {
      const int m = min(64, k - c0);
      const int32_t pos = lane < m ? entry_pos(list_entry(list, off, lg, c0 + lane), rs) : qp;
      const int32_t idx = g.perm[pos];
      const float4 p = g.sp[pos];
      const float d2 = flann_d2(q.x, q.y, q.z, p.x, p.y, p.z);
      const float w = (d2 == 0.0f || lane >= m) ? 0.0f : 1.0f / d2;  // 0: the query itself, or past m
      for (int j0 = 0; j0 < m; j0 += 8) {
        float v[8], wu[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int jj = j0 + u < m ? j0 + u : m - 1;
          const int id = __builtin_amdgcn_readlane(idx, jj);
          wu[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), j0 + u < 64 ? j0 + u : 63));
          if constexpr (BUF) v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(srsrc, vlane, id * (kDesc * 4), 0));
          else v[u] = spfh[(int64_t)id * kDesc + (vlane >> 2)];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          // w = 0 adds +0 (rows finite, fh >= +0): PCL's `continue`, bit for bit
          const float val = v[u] * wu[u];
          fh = fh + val;
          ps += (double)val;
          pl = val != 0.0f ? min(pl, lsb_exp_bound(val)) : pl;
        }
      }
    }
#elif PFX_WL_PIPE
    // Software-pipelined over batches of 8 neighbours (round 6): the SPFH rows of batch b + 1 are
    // loaded while batch b is summed, and each 64-entry chunk's entries are resolved (position,
    // caller index, 1/d2) one chunk ahead -- the loop used to wait one L2 latency per batch.
    auto resolve = [&](int c0, int32_t& idx, float& w) {
      const int m = min(64, k - c0);
      const int32_t pos = lane < m ? entry_pos(list_entry(list, off, lg, c0 + lane), rs) : qp;
      idx = g.perm[pos];
      const float4 p = g.sp[pos];
      const float d2 = flann_d2(q.x, q.y, q.z, p.x, p.y, p.z);
      w = d2 == 0.0f ? 0.0f : 1.0f / d2;  // 0 marks a skipped neighbour (the query itself)
    };
    const int nbat = (k + 7) >> 3;
    int32_t idxA = qi, idxB = qi;  // the chunk of the batch being loaded, and the chunk after it
    float wA = 0.0f, wB = 0.0f;
    if (k > 0) resolve(0, idxA, wA);
    if (k > 64) resolve(64, idxB, wB);
    auto load_batch = [&](int b, int32_t idx, float w, float (&v)[8], float (&wu)[8]) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = 8 * b + u;  // neighbour index in the list
        const int jj = e < k ? (e & 63) : ((k - 1) & 63);
        const int id = __builtin_amdgcn_readlane(idx, jj);
        wu[u] = e < k ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), jj)) : 0.0f;
        v[u] = lane < kDesc ? spfh[(int64_t)id * kDesc + lane] : 0.0f;
      }
    };
    float v[8], wu[8];
    if (nbat > 0) load_batch(0, idxA, wA, v, wu);
    for (int b = 0; b < nbat; ++b) {
      float vn[8], wn[8];
      const int b1 = b + 1;
      if ((b1 & 7) == 0 && b1 < nbat) {  // batch b + 1 opens the next chunk: rotate, resolve one more
        idxA = idxB;
        wA = wB;
        if (64 * (b1 / 8 + 1) < k) resolve(64 * (b1 / 8 + 1), idxB, wB);
      }
      if (b1 < nbat) load_batch(b1, idxA, wA, vn, wn);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        // w = 0 adds +0 (rows finite, fh >= +0): PCL's `continue`, bit for bit
        const float val = v[u] * wu[u];
        fh = fh + val;
        if (wu[u] != 0.0f && val != 0.0f) {
          ps += (double)val;
          pl = min(pl, lsb_exp(val));
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = vn[u];
        wu[u] = wn[u];
      }
    }
#else
    for (int c0 = 0; c0 < k; c0 += 64) {
      const int m = min(64, k - c0);
      const int32_t pos = lane < m ? entry_pos(list_entry(list, off, lg, c0 + lane), rs) : qp;
      const int32_t idx = g.perm[pos];
      const float4 p = g.sp[pos];
      const float d2 = flann_d2(q.x, q.y, q.z, p.x, p.y, p.z);
      const float w = d2 == 0.0f ? 0.0f : 1.0f / d2;  // 0 marks a skipped neighbour (the query itself)
      for (int j0 = 0; j0 < m; j0 += 8) {
        float v[8], wu[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int jj = j0 + u < m ? j0 + u : m - 1;
          const int id = __builtin_amdgcn_readlane(idx, jj);
          wu[u] = j0 + u < m ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), jj)) : 0.0f;
          v[u] = lane < kDesc ? spfh[(int64_t)id * kDesc + lane] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          // w = 0 adds +0 (rows finite, fh >= +0): PCL's `continue`, bit for bit
          const float val = v[u] * wu[u];
          fh = fh + val;
          if (wu[u] != 0.0f && val != 0.0f) {
            ps += (double)val;
            pl = min(pl, lsb_exp(val));
          }
        }
      }
    }
#endif
    if (lane < kDesc) {
      s_ps[wv][lane] = ps;
      s_pl[wv][lane] = pl;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    double scale = 0.0;
    if (lane < 3) {
      double sum = 0.0;
      int L = 1 << 20;
      for (int b = 0; b < kBins; ++b) {
        sum += s_ps[wv][lane * kBins + b];
        L = min(L, s_pl[wv][lane * kBins + b]);
      }
      if (!(sum == 0.0 || (L < 1000 && sum < ldexp(1.0, L + 52)))) {  // PCL's sequential loop
        atomicAdd(err + 2, 1);
        sum = 0.0;
        for (int c = 0; c < k; ++c) {
          const int32_t pos = entry_pos(list_entry(list, off, lg, c), rs);
          const float4 p = g.sp[pos];
          const float d2 = flann_d2(q.x, q.y, q.z, p.x, p.y, p.z);
          if (d2 == 0.0f) continue;
          const float wc = 1.0f / d2;
          const float* row = spfh + (int64_t)g.perm[pos] * kDesc + lane * kBins;
          for (int b = 0; b < kBins; ++b) sum = sum + (double)(row[b] * wc);
        }
      }
      scale = sum != 0.0 ? 100.0 / sum : 0.0;
      s_ps[wv][lane] = scale;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < kDesc) out[(int64_t)qi * kDesc + lane] = fh * (float)s_ps[wv][lane / kBins];
    kmax = max(kmax, k);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && kmax) atomicMax(err + 1, kmax);
}

// NaN rows for the non-finite surface points (PCL: no neighbours -> NaN); the finite ones are
// written by k_fpfh_weight_lists
__global__ void k_nan_rows_nonfinite(const float* __restrict__ x, const float* __restrict__ y,
                                     const float* __restrict__ z, int64_t n, float* __restrict__ out) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= n * kDesc) return;
  const int64_t i = e / kDesc;
  if (!(isfinite(x[i]) && isfinite(y[i]) && isfinite(z[i]))) out[e] = __builtin_nanf("");
}

}  // namespace

void fpfh_prepare_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns, double r) {
  ctx->prep_x = nullptr;
  ctx->prep_n = -1;
  ctx->prep_qx = nullptr;
  ctx->prep_nq = -1;
  if (ns == 0) return;
  // on the previous scan's widened bounds (no bounds readback, so the call queues without a host
  // wait); the first consumer validates it (fpfh_validate_grid) and rebuilds exactly if needed
  build_grid(ctx, ctx->grid_b, sx, sy, sz, ns, r, /*use_hint=*/true);
  if (ctx->grid_b.oob) {
    if (!ctx->grid_b_hoob) PFX_HIP(hipHostMalloc((void**)&ctx->grid_b_hoob, 64, hipHostMallocDefault));
    if (!ctx->grid_b_oob_ev) PFX_HIP(hipEventCreateWithFlags(&ctx->grid_b_oob_ev, hipEventDisableTiming));
    PFX_HIP(hipMemcpyAsync(ctx->grid_b_hoob, ctx->grid_b.oob, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    PFX_HIP(hipEventRecord(ctx->grid_b_oob_ev, ctx->stream));
  }
  ctx->prep_x = sx;
  ctx->prep_n = ns;
  ctx->prep_r = r;
}

bool fpfh_validate_grid(pfx_ctx* ctx) {
  Grid& G = ctx->grid_b;
  if (!G.oob) return false;
  G.oob = nullptr;
  PFX_HIP(hipEventSynchronize(ctx->grid_b_oob_ev));
  if (*ctx->grid_b_hoob == 0) return false;
  ctx->stats["fpfh_speculative_reruns"] += 1;
  // exact rebuild (bounds readback; refreshes the hint); the preparation still describes it
  const float* x = ctx->prep_x;
  const int64_t n = ctx->prep_n;
  const double r = ctx->prep_r;
  build_grid(ctx, G, G.ux, G.uy, G.uz, G.n, r);
  ctx->prep_x = x;
  ctx->prep_n = n;
  ctx->prep_r = r;
  return true;
}

// S of the next fpfh_dev (input != surface) marked and compacted ahead of time: it needs only the
// coordinates and the queries, so it can run while the normals are still being computed.
void fpfh_prepare_queries_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                              const float* qx, const float* qy, const float* qz, int64_t nq, double r) {
  PFX_CHECK(r > 0.0, "fpfh_prepare_queries: radius must be > 0");
  ctx->prep_qx = nullptr;
  ctx->prep_nq = -1;
  if (ns == 0 || nq == 0) return;
  if (!(ctx->prep_x == sx && ctx->prep_n == ns && ctx->prep_r == r)) fpfh_prepare_dev(ctx, sx, sy, sz, ns, r);
  fpfh_validate_grid(ctx);
  hipStream_t st = ctx->stream;
  const Grid& G = ctx->grid_b;
  uint8_t* flags = ctx->buf("fpfh_flags").as<uint8_t>(ns);
  int32_t* slist = ctx->buf("fpfh_list").as<int32_t>(ns);
  int64_t* d_sel = ctx->buf("fpfh_nsel").as<int64_t>(1);
  size_t tmp_bytes = 0;
  PFX_HIP(rocprim::select(nullptr, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel,
                          (size_t)ns, st));
  void* tmp = ctx->buf("fpfh_tmp").get(tmp_bytes + 16);
  TimeScope ts(ctx, "fpfh_prepare_queries");
  PFX_HIP(hipMemsetAsync(flags, 0, ns, st));
  k_fpfh_mark<<<(unsigned)std::min<int64_t>(nq, 8192), 256, 0, st>>>(view(G), qx, qy, qz, nq, (float)(r * r), flags);
  check_launch("k_fpfh_mark");
  PFX_HIP(rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel, (size_t)ns,
                          st));
  ctx->prep_qx = qx;
  ctx->prep_nq = nq;
}

void fpfh_support_mask_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                           const float* qx, const float* qy, const float* qz, int64_t nq, double r, uint8_t* mask) {
  PFX_CHECK(r > 0.0, "fpfh support: radius must be > 0");
  ctx->fpfh_support = nullptr;
  if (ns == 0) return;
  hipStream_t st = ctx->stream;
  PFX_HIP(hipMemsetAsync(mask, 0, ns, st));
  if (nq == 0) return;
  if (!(ctx->prep_x == sx && ctx->prep_n == ns && ctx->prep_r == r)) fpfh_prepare_dev(ctx, sx, sy, sz, ns, r);
  fpfh_validate_grid(ctx);
  TimeScope ts(ctx, "fpfh_support");
  const Grid& G = ctx->grid_b;
  const GridView g = view(G);
  const float rr = (float)(r * r);
  uint8_t* flags = ctx->buf("fpfh_sflags").as<uint8_t>(ns);
  int32_t* slist = ctx->buf("fpfh_slist").as<int32_t>(ns);
  int64_t* d_sel = ctx->buf("fpfh_snsel").as<int64_t>(1);
  size_t tmp_bytes = 0;
  PFX_HIP(rocprim::select(nullptr, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel,
                          (size_t)ns, st));
  void* tmp = ctx->buf("fpfh_stmp").get(tmp_bytes + 16);
  PFX_HIP(hipMemsetAsync(flags, 0, ns, st));
  k_fpfh_mark<<<(unsigned)std::min<int64_t>(nq, 8192), 256, 0, st>>>(g, qx, qy, qz, nq, rr, flags);
  PFX_HIP(rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel, (size_t)ns,
                          st));
  k_fpfh_mark_support<<<8192, 256, 0, st>>>(g, slist, d_sel, rr, mask);
  check_launch("k_fpfh_mark_support");
  ctx->fpfh_support = mask;  // consumed by the next fpfh_dev on this context
}

void fpfh_support_ball_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                           const float* qx, const float* qy, const float* qz, int64_t nq, double r, uint8_t* mask) {
  PFX_CHECK(r > 0.0, "fpfh support: radius must be > 0");
  ctx->fpfh_support = nullptr;
  if (ns == 0) return;
  hipStream_t st = ctx->stream;
  PFX_HIP(hipMemsetAsync(mask, 0, ns, st));
  if (nq == 0) return;
  if (!(ctx->prep_x == sx && ctx->prep_n == ns && ctx->prep_r == r)) fpfh_prepare_dev(ctx, sx, sy, sz, ns, r);
  fpfh_validate_grid(ctx);
  TimeScope ts(ctx, "fpfh_support");
  // (2r)^2 with a relative margin far above the float rounding of the squared distance
  const float rr4 = (float)(4.0 * r * r * (1.0 + 1e-5));
  k_fpfh_mark_ball<<<(unsigned)std::min<int64_t>(nq, 8192), 256, 0, st>>>(view(ctx->grid_b), qx, qy, qz, nq, rr4,
                                                                          mask);
  check_launch("k_fpfh_mark_ball");
  ctx->fpfh_support = mask;  // consumed by the next fpfh_dev on this context
}

void fpfh_dev(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, const float* snx,
              const float* sny, const float* snz, int64_t ns, const float* qx, const float* qy, const float* qz,
              int64_t nq, int same, double r, float* out, bool reuse_normal_lists) {
  PFX_CHECK(r > 0.0, "fpfh: radius must be > 0");
  if (nq == 0) return;
  hipStream_t st = ctx->stream;
  if (ns == 0) {
    // no surface: every query has an empty neighbourhood -> NaN rows (PCL fills NaN)
    std::vector<float> nanrow((size_t)nq * kDesc, __builtin_nanf(""));
    PFX_HIP(hipMemcpyAsync(out, nanrow.data(), sizeof(float) * nanrow.size(), hipMemcpyHostToDevice, st));
    PFX_HIP(hipStreamSynchronize(st));
    return;
  }
  const bool grid_ready = ctx->prep_x == sx && ctx->prep_n == ns && ctx->prep_r == r;
  if (!grid_ready) build_grid(ctx, ctx->grid_b, sx, sy, sz, ns, r);
  const bool rebuilt = grid_ready && fpfh_validate_grid(ctx);
  // S marked ahead (fpfh_prepare_queries_dev on this grid and these queries)?
  const bool s_ready = grid_ready && !rebuilt && !same && ctx->prep_qx == qx && ctx->prep_nq == nq;
  ctx->prep_x = nullptr;  // one-shot
  ctx->prep_n = -1;
  ctx->prep_qx = nullptr;
  ctx->prep_nq = -1;
  const Grid& G = ctx->grid_b;
  GridView g = view(G);
  const float rr = (float)(r * r);
  float* spfh = ctx->buf("fpfh_spfh").as<float>(ns * kDesc);
  float4* snp = ctx->buf("fpfh_snp").as<float4>(ns);
  uint8_t* flags = ctx->buf("fpfh_flags").as<uint8_t>(ns);
  int32_t* slist = ctx->buf("fpfh_list").as<int32_t>(ns);
  int64_t* d_sel = ctx->buf("fpfh_nsel").as<int64_t>(1);
  size_t tmp_bytes = 0;
  PFX_HIP(rocprim::select(nullptr, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel,
                          (size_t)ns, st));
  void* tmp = ctx->buf("fpfh_tmp").get(tmp_bytes + 16);
  const unsigned nb = (unsigned)ceil_div(ns, 256);
  // [0] k over capacity, [1] max k, [2] inexact sums, [3] deferred pairs, [4..7] pairs,
  // [8] queries over the LDS capacity (weighted by the global-scratch pass)
  DevBuf& eb = ctx->buf("fpfh_err");
  const bool fresh = !eb.ptr;
  int* err = eb.as<int>(10);
  if (fresh) PFX_HIP(hipMemsetAsync(err, 0, 10 * sizeof(int), st));  // the sticky word starts clear
  {
    TimeScope ts(ctx, "fpfh_mark");
    // (also zeroes the per-call statistics words err[1..9]: err[0] (neighbourhood beyond
    // capacity) is sticky until the check after the next synchronisation, fpfh_resolve)
    k_sorted_normals<<<nb, 256, 0, st>>>(G.perm, ns, snx, sny, snz, same ? nullptr : ctx->fpfh_support, snp,
                                         err + 1);
    ctx->fpfh_support = nullptr;  // one-shot
    if (!s_ready) {
      if (same) {
        k_all_finite<<<nb, 256, 0, st>>>(G.skeys, ns, (uint64_t)G.ncells, flags);
      } else {
        PFX_HIP(hipMemsetAsync(flags, 0, ns, st));
        k_fpfh_mark<<<(unsigned)std::min<int64_t>(nq, 8192), 256, 0, st>>>(g, qx, qy, qz, nq, rr, flags);
      }
      check_launch("k_fpfh_mark");
      PFX_HIP(rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flags, slist, d_sel,
                              (size_t)ns, st));
    }
  }
  // a neighbourhood can only outgrow the LDS keys when the surface has more than kCapW points
  const bool overflow_pass = ns > kCapW;
  int32_t* ovf = overflow_pass ? ctx->buf("fpfh_wovf").as<int32_t>(nq) : nullptr;
  const int gcap = overflow_pass ? (int)std::min<int64_t>(kCapWGlobal, (int64_t)1 << (64 - __builtin_clzll((unsigned long long)ns - 1))) : 0;
  uint64_t* wscratch = overflow_pass ? ctx->buf("fpfh_wscratch").as<uint64_t>((size_t)kWOvfBlocks * gcap) : nullptr;
  unsigned long long* d_pairs = reinterpret_cast<unsigned long long*>(err + 4);
  unsigned* n_slow = reinterpret_cast<unsigned*>(err + 3);
  int* hcount = ctx->buf("fpfh_hcount").as<int>(ns * kDesc);
  int* kcount = ctx->buf("fpfh_kcount").as<int>(ns);
  // pairs the fast path cannot bin go to a queue for the exact path; past its capacity
  // k_fpfh_spfh runs the exact path in place (PFX_FPFH_SLOW_CAP: test hook for that branch)
  const char* cap_env = getenv("PFX_FPFH_SLOW_CAP");
  const unsigned slow_cap = cap_env ? (unsigned)std::max(1, atoi(cap_env)) : 1u << 20;
  int2* slowq = ctx->buf("fpfh_slowq").as<int2>(slow_cap);
  {
    // the S count stays on the device: grid-stride launches sized for the worst case
    TimeScope ts(ctx, "fpfh_spfh", true);
    // 16 waves per CU (measured, 1M-point room: 8 -> 1.06 ms, 12 -> 1.13, 16 -> 0.94, 20 -> 0.99,
    // 32 -> 1.24, 128 -> 2.45)
    const int64_t waves = std::min<int64_t>(ns, 256 * 4 * 16);
    k_fpfh_spfh<<<(unsigned)std::max<int64_t>(8, ceil_div(waves, 4) & ~7), 256, 0, st>>>(
        g, snp, slist, d_sel, rr, hcount, kcount, slowq, n_slow, slow_cap, d_pairs);
    k_fpfh_exact<<<256, 256, 0, st>>>(g, snp, slist, slowq, n_slow, slow_cap, hcount, d_pairs);
    k_fpfh_finalize<<<(unsigned)std::min<int64_t>(ceil_div(ns * kDesc, 256), 4096), 256, 0, st>>>(
        g, slist, d_sel, hcount, kcount, spfh);
    check_launch("k_fpfh_spfh");
  }
  if (same) {  // input == surface: FLANN-ordered lists of every grid point, a wave per query
    TimeScope ts(ctx, "fpfh_weight", true);
    // Features::compute estimates the normals of the same cloud first (features.h:187-195):
    // when that search had this radius, its lists are this one's (grid_a indexes the same
    // points); otherwise they are built on the FPFH grid
    // (only on the caller's word, pfx_fpfh_after_normals_dev: equal pointers do not prove that
    // the buffers still hold the cloud those lists were built on)
    NormalsState* nst = ctx->normals;
    const bool reuse = reuse_normal_lists && nst && nst->ready && nst->x == sx && nst->y == sy && nst->z == sz &&
                       nst->n == ns && nst->r == r;
    if (nst && reuse_normal_lists) nst->ready = false;  // consumed: a later call cannot vouch for them
    NbLists L;
    if (reuse) L = nst->L;
    else build_lists(ctx, G, nullptr, r, true, L, "fpfh");
    ctx->stats["fpfh_weight_lists_reused"] = reuse ? 1 : 0;
    k_nan_rows_nonfinite<<<(unsigned)ceil_div(ns * kDesc, 256), 256, 0, st>>>(sx, sy, sz, ns, out);
    if (L.nq > 0)
    {
      const unsigned bl = (unsigned)std::min<int64_t>(ceil_div(L.nq, 4), 256 * PFX_WL_GRID);
      const GridView gv = reuse ? view(ctx->grid_a) : g;
      const bool buf = ns * kDesc * 4 < ((int64_t)1 << 31);
      if (buf)
        k_fpfh_weight_lists<true><<<bl, 256, 0, st>>>(gv, L.qpos, L.off, L.cnt, L.lg, L.list, L.skeys, L.nq, spfh, out, err);
      else
        k_fpfh_weight_lists<false><<<bl, 256, 0, st>>>(gv, L.qpos, L.off, L.cnt, L.lg, L.list, L.skeys, L.nq, spfh, out,
                                                       err);
    }
    check_launch("k_fpfh_weight_lists");
  } else {
    TimeScope ts(ctx, "fpfh_weight", true);
    const size_t lds = sizeof(uint64_t) * 2 * kCapW;
    PFX_HIP(hipFuncSetAttribute((const void*)k_fpfh_weight<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const unsigned blocks = (unsigned)std::min<int64_t>(nq, PFX_W_BLOCKS);
    k_fpfh_weight<false><<<blocks, kWT, lds, st>>>(g, qx, qy, qz, nq, rr, spfh, out, err, ovf, err + 8, nullptr, 0);
    if (overflow_pass)
      k_fpfh_weight<true><<<kWOvfBlocks, kWT, 0, st>>>(g, qx, qy, qz, nq, rr, spfh, out, err, ovf, err + 8, wscratch,
                                                        gcap);
    check_launch("k_fpfh_weight");
  }
  // statistics and the sticky error word land in pinned memory in stream order; no host
  // synchronisation here (the step's critical path ends with this call)
  FpfhReadback* rb = ctx->fpfh_rb();
  PFX_HIP(hipMemcpyAsync(rb->h, err, sizeof(rb->h), hipMemcpyDeviceToHost, st));
  PFX_HIP(hipMemcpyAsync(&rb->count, d_sel, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  rb->slow_cap = slow_cap;
  ctx->fpfh_pending = true;
}

// After a synchronisation of ctx's stream: the last fpfh_dev's statistics, and its capacity check
// (PFX_ERR_CAPACITY, reported here for the stream-ordered API; the host API calls this at once).
void fpfh_resolve(pfx_ctx* ctx) {
  if (!ctx->fpfh_pending) return;
  ctx->fpfh_pending = false;
  const FpfhReadback* rb = ctx->fpfh_rb();
  const int* h = rb->h;
  const unsigned n_slow = (unsigned)h[3];
  ctx->stats["fpfh_spfh_points"] = rb->count;
  unsigned long long pr;
  std::memcpy(&pr, h + 4, sizeof(pr));
  ctx->stats["fpfh_spfh_pairs"] = (int64_t)pr;
  std::memcpy(&pr, h + 6, sizeof(pr));
  ctx->stats["fpfh_spfh_exact_pairs"] = (int64_t)pr;
  ctx->stats["fpfh_spfh_deferred"] = n_slow;
  ctx->stats["fpfh_spfh_inline_exact"] = n_slow > rb->slow_cap ? n_slow - rb->slow_cap : 0;
  ctx->stats["fpfh_weight_kmax"] = h[1];
  ctx->stats["fpfh_weight_sequential"] = h[2];
  ctx->stats["fpfh_weight_global"] = h[8];
  if (h[0] > 0) {
    int* err = ctx->buf("fpfh_err").as<int>(10);
    PFX_HIP(hipMemsetAsync(err, 0, sizeof(int), ctx->stream));  // reported once
    throw Error(PFX_ERR_CAPACITY, "fpfh: a query has " + std::to_string(h[0]) + " neighbours (> " +
                                      std::to_string(kCapWGlobal) + " supported)");
  }
}

}  // namespace pfx
