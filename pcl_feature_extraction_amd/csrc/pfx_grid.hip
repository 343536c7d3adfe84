// pfx_grid.hip -- uniform-grid spatial index (replaces the FLANN kd-tree that
// search::KdTree<PointXYZRGB> builds at features.h:192 / tools.h:29).
//
// Layout in HBM (all SoA, 4-byte elements):
//   sx/sy/sz[n]     point coordinates sorted by linear cell key  (coalesced run reads)
//   perm[n]         sorted position -> caller point index         (FLANN tie-break key)
//   cell_start[C+2] first sorted position of each cell (cells in key order), C = nx*ny*nz <= 2^26
// Cells are >= r (r*(1+1e-6)), so the radius ball of a query lies in its 3x3x3 cell block;
// with row-major keys (x, y, z) the block is 9 contiguous runs of 3 z-cells.
// Non-finite points get key C and sort behind every cell (never a neighbour, as PCL's
// kd-tree skips them).
#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_internal.h"

namespace pfx {
namespace {

__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ __forceinline__ float ord2f(uint32_t u) {
  uint32_t b = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  float f;
  memcpy(&f, &b, 4);
  return f;
}

// per-block bounds (ordered-uint encoding: min slots start at 0xffffffff, max at 0), reduced on
// the host -- no device-side initialisation (a pageable H2D copy) before the launch
constexpr int kBboxBlocks = 1024;
__global__ void __launch_bounds__(256) k_bbox(const float* __restrict__ x, const float* __restrict__ y,
                                              const float* __restrict__ z, int64_t n,
                                              uint32_t* __restrict__ mm) {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float p[3] = {x[i], y[i], z[i]};
    if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
#pragma unroll
    for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], p[d]); hi[d] = fmaxf(hi[d], p[d]); }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], off));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off));
    }
  }
  __shared__ float s_lo[3][4], s_hi[3][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int d = 0; d < 3; ++d) { s_lo[d][wv] = lo[d]; s_hi[d][wv] = hi[d]; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float l = fminf(fminf(s_lo[d][0], s_lo[d][1]), fminf(s_lo[d][2], s_lo[d][3]));
      const float h = fmaxf(fmaxf(s_hi[d][0], s_hi[d][1]), fmaxf(s_hi[d][2], s_hi[d][3]));
      const bool any = l <= h;
      mm[blockIdx.x * 6 + d] = any ? f2ord(l) : 0xffffffffu;
      mm[blockIdx.x * 6 + 3 + d] = any ? f2ord(h) : 0u;
    }
  }
}

// the per-block bounds reduced to one (min x, y, z, max x, y, z) record at mm[6 * nblocks]
__global__ void __launch_bounds__(256) k_bbox_reduce(uint32_t* __restrict__ mm, int nblocks) {
  __shared__ uint32_t s[6][256];
  const int t = threadIdx.x;
  uint32_t r[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
  for (int b = t; b < nblocks; b += 256)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      r[d] = min(r[d], mm[b * 6 + d]);
      r[3 + d] = max(r[3 + d], mm[b * 6 + 3 + d]);
    }
#pragma unroll
  for (int d = 0; d < 6; ++d) s[d][t] = r[d];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o)
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        s[d][t] = min(s[d][t], s[d][t + o]);
        s[3 + d][t] = max(s[3 + d][t], s[3 + d][t + o]);
      }
    __syncthreads();
  }
  if (t < 6) mm[nblocks * 6 + t] = s[t][0];
}

// oob (nullable, speculative bounds): counts the finite points outside [lo, hi] (clamped keys
// are then not a valid grid; the caller rebuilds on exact bounds)
__global__ void __launch_bounds__(256) k_cell_keys(const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ z, int64_t n, double inv,
                                                   double ox, double oy, double oz, int32_t nx, int32_t ny,
                                                   int32_t nz, uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals, int* __restrict__ oob,
                                                   double hx, double hy, double hz) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float px = x[i], py = y[i], pz = z[i];
  uint32_t key = (uint32_t)((int64_t)nx * ny * nz);
  if (isfinite(px) && isfinite(py) && isfinite(pz)) {
    // (exactly the points the clamp below would move: cell index outside [0, dims))
    if (oob && ((double)px < ox || (double)py < oy || (double)pz < oz || (double)px > hx || (double)py > hy ||
                (double)pz > hz))
      atomicAdd(oob, 1);
    int64_t ix = (int64_t)floor(((double)px - ox) * inv);
    int64_t iy = (int64_t)floor(((double)py - oy) * inv);
    int64_t iz = (int64_t)floor(((double)pz - oz) * inv);
    ix = ix < 0 ? 0 : (ix >= nx ? nx - 1 : ix);
    iy = iy < 0 ? 0 : (iy >= ny ? ny - 1 : iy);
    iz = iz < 0 ? 0 : (iz >= nz ? nz - 1 : iz);
    key = (uint32_t)((ix * ny + iy) * nz + iz);
  }
  keys[i] = key;
  vals[i] = (uint32_t)i;
}

// cell_start[0, m) = v: a plain kernel launch (hipMemsetD32Async spent ~70 us of host time per
// call in the HIP API trace, on the critical path of the grid build)
__global__ void __launch_bounds__(256) k_fill_i32(int32_t* __restrict__ p, int64_t m, int32_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// first sorted position of every occupied cell (cells are then completed by a suffix minimum)
__global__ void __launch_bounds__(256) k_mark_starts(const uint32_t* __restrict__ skeys, int64_t n,
                                                     int32_t* __restrict__ cell_start) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = skeys[i];
  if (i == 0 || skeys[i - 1] != k) cell_start[k] = (int32_t)i;
}

__global__ void __launch_bounds__(256) k_gather_sorted(const float* __restrict__ x, const float* __restrict__ y,
                                                       const float* __restrict__ z, int64_t n,
                                                       const uint32_t* __restrict__ perm,
                                                       float* __restrict__ sx, float* __restrict__ sy,
                                                       float* __restrict__ sz, float4* __restrict__ sp) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t p = perm[i];
  const float a = x[p], b = y[p], c = z[p];
  sx[i] = a;
  sy[i] = b;
  sz[i] = c;
  sp[i] = make_float4(a, b, c, 0.0f);
}

}  // namespace

// bounds of the finite points: per-block partials read back once (pinned) and reduced here
static bool bbox_dev(pfx_ctx* ctx, Grid& g, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                     double lo[3], double hi[3]) {
  hipStream_t st = ctx->stream;
  uint32_t* mm = g.b_minmax.as<uint32_t>(6 * (kBboxBlocks + 1));
  // ~4 points per thread over up to 1,024 workgroups, reduced on the device (one 24-B readback);
  // 128 workgroups of ~30 points per thread took 28 us alone, 160 us beside NARF's range-image
  // projection (headline A/B: 168.0 vs 168.3 Mpoints/s, within noise)
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(n, 1024), 1), kBboxBlocks);
  {
    TimeScope ts(ctx, "grid_bbox");
    k_bbox<<<blocks, 256, 0, st>>>(d_x, d_y, d_z, n, mm);
    k_bbox_reduce<<<1, 256, 0, st>>>(mm, blocks);
    check_launch("k_bbox");
  }
  uint32_t* h = ctx->readback<uint32_t>();  // pinned
  PFX_HIP(hipMemcpyAsync(h, mm + 6 * blocks, sizeof(uint32_t) * 6, hipMemcpyDeviceToHost, st));
  ctx->sync_spin(st);
  uint32_t r[6];
  for (int d = 0; d < 6; ++d) r[d] = h[d];
  const bool any = r[0] != 0xffffffffu && r[3] != 0u;
  for (int d = 0; d < 3; ++d) {
    lo[d] = any ? ord2f(r[d]) : 0.0;
    hi[d] = any ? ord2f(r[3 + d]) : 0.0;
  }
  return any;
}

void points_bbox(pfx_ctx* ctx, Grid& g, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                 double lo[3], double hi[3]) {
  bbox_dev(ctx, g, d_x, d_y, d_z, n, lo, hi);
}

void build_grid(pfx_ctx* ctx, Grid& g, const float* d_x, const float* d_y, const float* d_z,
                int64_t n, double radius, bool use_hint) {
  PFX_CHECK(n >= 0 && n < (int64_t(1) << 31), "point count must be in [0, 2^31)");
  PFX_CHECK(radius > 0.0, "radius must be > 0");
  if (&g == &ctx->grid_b) {  // a grid prepared ahead for the next fpfh_dev no longer holds
    ctx->prep_x = nullptr;
    ctx->prep_n = -1;
    ctx->prep_qx = nullptr;
    ctx->prep_nq = -1;
  }
  hipStream_t st = ctx->stream;
  ++g.gen;
  g.n = n;
  g.ux = d_x; g.uy = d_y; g.uz = d_z;
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  g.oob = nullptr;
  if (use_hint && g.have_hint && n > 0) {
    // speculative: the previous exact bounds, widened (no bounds pass, no host round trip)
    for (int d = 0; d < 3; ++d) {
      lo[d] = g.hint_lo[d];
      hi[d] = g.hint_hi[d];
    }
    g.oob = g.b_oob.as<int>(1);
  } else if (n > 0) {
    bbox_dev(ctx, g, d_x, d_y, d_z, n, lo, hi);
    // the hint for the next speculative build: 10 % wider on every side, plus two cells (scans of
    // one sensor keep their extent)
    for (int d = 0; d < 3; ++d) {
      const double m = 0.1 * (hi[d] - lo[d]) + 2.0 * radius;
      g.hint_lo[d] = lo[d] - m;
      g.hint_hi[d] = hi[d] + m;
    }
    g.have_hint = true;
  }
  double cell = radius * (1.0 + 1e-6);
  const double max_cells = double(1 << 26);
  int64_t dims[3];
  for (int it = 0; it < 64; ++it) {
    for (int d = 0; d < 3; ++d) dims[d] = (int64_t)std::floor((hi[d] - lo[d]) / cell) + 1;
    double total = double(dims[0]) * double(dims[1]) * double(dims[2]);
    if (total <= max_cells) break;
    cell *= std::cbrt(total / max_cells) * 1.01;
  }
  g.cell = (float)cell;
  g.inv = (float)(1.0 / cell);
  g.ox = (float)lo[0]; g.oy = (float)lo[1]; g.oz = (float)lo[2];
  g.nx = (int32_t)dims[0]; g.ny = (int32_t)dims[1]; g.nz = (int32_t)dims[2];
  g.ncells = dims[0] * dims[1] * dims[2];
  // exact double parameters used by both builder and queries
  const double inv = 1.0 / cell;
  g.inv = (float)inv;
  const int64_t C = g.ncells;

  // onesweep radix sort even at ~1M keys: the default config switches to merge sort below 2^20
  // items (30+ block-merge launches, ~0.4 ms at 1M points on gfx950)
  using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                             rocprim::default_config, 0>;
  int bits = 1;
  while ((int64_t(1) << bits) <= C) ++bits;
  // size every scratch buffer before the first launch (no realloc behind pending work)
  size_t sort_bytes = 0, scan_bytes = 0;
  PFX_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                    (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)std::max<int64_t>(n, 1),
                                    0, bits, st));
  auto rev = rocprim::make_reverse_iterator(static_cast<int32_t*>(nullptr));
  PFX_HIP(rocprim::inclusive_scan(nullptr, scan_bytes, rev, rev, (size_t)(C + 1), rocprim::minimum<int32_t>(), st));
  void* tmp = g.b_tmp.get(std::max(sort_bytes, scan_bytes) + 16);
  uint32_t* keys = g.b_keys.as<uint32_t>(n + 1);
  uint32_t* keys2 = g.b_keys2.as<uint32_t>(n + 1);
  uint32_t* vals = g.b_vals.as<uint32_t>(n + 1);
  g.perm = g.b_perm.as<int32_t>(n + 1);
  g.skeys = keys2;  // radix-sort output: cell key per sorted position
  g.sx = g.b_sx.as<float>(n + 1);
  g.sy = g.b_sy.as<float>(n + 1);
  g.sz = g.b_sz.as<float>(n + 1);
  g.sp = g.b_sp.as<float4>(n + 1);
  g.cell_start = g.b_start.as<int32_t>(C + 2);
  g.dinv = inv;
  g.dox = lo[0]; g.doy = lo[1]; g.doz = lo[2];
  {
    TimeScope ts(ctx, "grid_build");
    // cell_start[c] = first sorted position with key >= c: mark the first position of every
    // occupied cell, then a suffix minimum fills the empty cells (no per-point atomics)
    k_fill_i32<<<(unsigned)std::min<int64_t>(ceil_div(C + 2, 256), 2048), 256, 0, st>>>(g.cell_start, C + 2,
                                                                                       (int32_t)n);
    if (g.oob) k_fill_i32<<<1, 64, 0, st>>>(g.oob, 1, 0);
    if (n > 0) {
      k_cell_keys<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(d_x, d_y, d_z, n, inv, lo[0], lo[1], lo[2],
                                                              g.nx, g.ny, g.nz, keys, vals, g.oob, hi[0], hi[1],
                                                              hi[2]);
      check_launch("k_cell_keys");
      PFX_HIP(rocprim::radix_sort_pairs<SortCfg>(tmp, sort_bytes, keys, keys2, vals,
                                        reinterpret_cast<uint32_t*>(g.perm), (size_t)n, 0, bits, st));
      k_mark_starts<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(keys2, n, g.cell_start);
      auto r = rocprim::make_reverse_iterator(g.cell_start + C + 1);
      PFX_HIP(rocprim::inclusive_scan(tmp, scan_bytes, r, r, (size_t)(C + 1), rocprim::minimum<int32_t>(), st));
      k_gather_sorted<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(
          d_x, d_y, d_z, n, reinterpret_cast<uint32_t*>(g.perm), g.sx, g.sy, g.sz, g.sp);
      check_launch("k_gather_sorted");
    }
  }
}

}  // namespace pfx
