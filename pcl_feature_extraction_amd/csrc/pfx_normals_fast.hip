// pfx_normals_fast.hip -- opt-in fast normal estimation: the covariance accumulation as an MFMA
// contraction (BASELINE north_star).  NOT parity-exact -- see below.
//
// NormalEstimationOMP (tools.h:22-32) sums {x^2, xy, xz, y^2, yz, z^2, x, y, z} over each point's
// radius neighbours in FLANN order, in float; reproducing that bit for bit needs every list sorted
// by (d2, index) and nine strictly sequential chains (pfx_normals.hip: the product path).  Here the
// order is given up and the sums become a dense product: for 16 queries and a candidate stream,
//
//      S (16 queries x 16 features)  =  H (16 x T hit mask, 0 / 1)  .  F (T x 16 features)
//
// with F[c] = {dx^2, dx dy, dx dz, dy^2, dy dz, dz^2, dx, dy, dz, 1, 0...} of candidate c centred
// on the group's first point (|d| <= ~3 r, so the float sums carry ~1000x less rounding than
// PCL's raw-coordinate ones) and H[q][c] = FLANN's test d2(q, c) < (float)(r*r) -- the same
// neighbour set as PCL, no list and no sort.  One v_mfma_f32_16x16x4_f32 per 4 candidates:
// lane l supplies H[l & 15][4s + (l >> 4)] and F[4s + (l >> 4)][l & 15] of candidate step s.
// The covariance is translation invariant, so pcl's formula (sums / k - mean mean^T, eigen33,
// curvature, viewpoint flip: pfx_normal_math.h) runs on the centred sums unchanged.
//
// One wave per 16 consecutive grid points (cell order); the candidates are the union of their
// 3x3x3 blocks per grid column (9 runs over the column's z range), loaded 64 at a time with one
// coalesced float4 load per lane (one chunk ahead); each lane puts its candidate's raw
// coordinates and 10 centred features in LDS, and every MFMA step reads one candidate per 16
// lanes (broadcast) plus one feature per lane, into four accumulators in turn (partial sums added
// at the end).  Rows
// of different columns are processed column by column, each row only against its own column's
// block.
#include <algorithm>

#include "pfx_nblist.h"
#include "pfx_neighbors.h"
#include "pfx_normal_math.h"

namespace pfx {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// feature f of a centred candidate (dx, dy, dz): {dx^2, dx dy, dx dz, dy^2, dy dz, dz^2, dx, dy, dz, 1}
constexpr int kFeat = 10;
constexpr int kFeatStride = 66;  // [feature][candidate]: a step's 16 x 4 reads hit 64 distinct banks
#ifndef PFX_NF_WPE
#define PFX_NF_WPE 8  // waves per SIMD (64 registers incl. the 16 accumulator AGPRs)
#endif

__global__ void __launch_bounds__(256, PFX_NF_WPE) k_normals_mfma(GridView g, float rr, float vpx, float vpy,
                                                                   float vpz, float* __restrict__ nx,
                                                                   float* __restrict__ ny, float* __restrict__ nz,
                                                                   float* __restrict__ curv) {
  // per wave: the 64 candidates of the current chunk (raw coordinates, for FLANN's test) and
  // their centred features; a step reads 4 candidates, each broadcast to 16 lanes
  __shared__ float4 cand[4][64];
  __shared__ float feat[4][(kFeat + 1) * kFeatStride];  // + one zero row for features 10..15
  __shared__ float sums[4][16][17];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int64_t ncells = (int64_t)g.nx * g.ny * g.nz;
  const int64_t nfin = g.cell_start[ncells];  // finite points: sorted positions [0, nfin)
  // natural block order (round-robin over the XCDs): the heavy groups of the dense regions cluster
  // in space, and contiguous per-XCD slices measured 0.99 against 0.66 ms
  const int64_t p0 = ((int64_t)blockIdx.x * 4 + wv) * 16;
  if (p0 >= nfin) return;  // wave-uniform; no workgroup barrier below
  const int nrow = (int)min<int64_t>(16, nfin - p0);
  const bool rowok = r16 < nrow;
  const float4 q = g.sp[p0 + (rowok ? r16 : 0)];
  const float4 o = g.sp[p0];
  const float ox = uniformf(o.x), oy = uniformf(o.y), oz = uniformf(o.z);
  const int cx = (int)floor(((double)q.x - g.ox) * g.inv);
  const int cy = (int)floor(((double)q.y - g.oy) * g.inv);
  const int cz = (int)floor(((double)q.z - g.oz) * g.inv);
  float* fw = &feat[wv][0];
  const int fr = min(r16, kFeat);  // features 10..15 read the zero row
  for (int i = lane; i < kFeatStride; i += 64) fw[kFeat * kFeatStride + i] = 0.0f;
  // four accumulators (steps s mod 4): the 40-cycle dependent latency of the MFMA stays hidden
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  uint32_t done = 0;  // rows handled (wave-uniform)
  const uint32_t rows = (uint32_t)((1u << nrow) - 1u);
  while (done != rows) {
    const int lead = __builtin_ctz(rows & ~done);
    const int lx = __builtin_amdgcn_readlane(cx, lead), ly = __builtin_amdgcn_readlane(cy, lead);
    const bool member = rowok && !((done >> r16) & 1u) && cx == lx && cy == ly;
    const uint32_t mrows = (uint32_t)(__ballot(member) & 0xffffull);  // lanes 0..15 = rows
    done |= mrows;
    int zlo = 1 << 30, zhi = -(1 << 30);
    for (uint32_t m = mrows; m; m &= m - 1) {
      const int zz = __builtin_amdgcn_readlane(cz, __builtin_ctz(m));
      zlo = min(zlo, zz);
      zhi = max(zhi, zz);
    }
    Runs R;
    {
      const int64_t z0 = max(zlo - 1, 0), z1 = min(zhi + 1, g.nz - 1);
      int32_t accn = 0;
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        const int64_t ix = lx + (r / 3) - 1, iy = ly + (r % 3) - 1;
        int32_t st = 0, len = 0;
        if (ix >= 0 && ix < g.nx && iy >= 0 && iy < g.ny && z0 <= z1) {
          const int64_t base = (ix * g.ny + iy) * g.nz;
          st = g.cell_start[base + z0];
          len = g.cell_start[base + z1 + 1] - st;
        }
        R.start[r] = __builtin_amdgcn_readfirstlane(st);
        R.pref[r] = __builtin_amdgcn_readfirstlane(accn);
        accn += len;
      }
      R.pref[9] = __builtin_amdgcn_readfirstlane(accn);
    }
    const int32_t T = R.pref[9];
    // rows outside this column segment never hit: their threshold is -1
    const float rr_row = member ? rr : -1.0f;
    float4 c = g.sp[run_pos(R, min(lane, max(T - 1, 0)))];
    for (int32_t t0 = 0; t0 < T; t0 += 64) {
      {
        // this lane's candidate into LDS: raw coordinates (w = +inf past T: d2 < rr fails) and
        // its centred features
        const bool live = t0 + lane < T;
        const float d0 = c.x - ox, d1 = c.y - oy, d2 = c.z - oz;
        cand[wv][lane] = make_float4(c.x, c.y, c.z, live ? 0.0f : __builtin_inff());
        fw[0 * kFeatStride + lane] = d0 * d0;
        fw[1 * kFeatStride + lane] = d0 * d1;
        fw[2 * kFeatStride + lane] = d0 * d2;
        fw[3 * kFeatStride + lane] = d1 * d1;
        fw[4 * kFeatStride + lane] = d1 * d2;
        fw[5 * kFeatStride + lane] = d2 * d2;
        fw[6 * kFeatStride + lane] = d0;
        fw[7 * kFeatStride + lane] = d1;
        fw[8 * kFeatStride + lane] = d2;
        fw[9 * kFeatStride + lane] = 1.0f;
      }
      // the next chunk's load is issued after the stores, so its latency runs under the steps
      c = g.sp[run_pos(R, min(t0 + 64 + lane, max(T - 1, 0)))];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int ci = 4 * s + kq;
        const float4 cc = cand[wv][ci];
        const float b = fw[fr * kFeatStride + ci];
        // FLANN's d2 (q - p), branch-free; cc.w = +inf past T
        const float d2 = flann_d2(q.x, q.y, q.z, cc.x, cc.y, cc.z) + cc.w;
        const float a = d2 < rr_row ? 1.0f : 0.0f;
        if ((s & 3) == 0) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
        else if ((s & 3) == 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc1, 0, 0, 0);
        else if ((s & 3) == 2) acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc2, 0, 0, 0);
        else acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc3, 0, 0, 0);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();  // the chunk is read before the next one overwrites it
    }
  }
  // D[row = 4 kq + i][col = r16] -> one row of 10 sums per query lane
  const f32x4 acc = (acc0 + acc1) + (acc2 + acc3);
#pragma unroll
  for (int i = 0; i < 4; ++i) sums[wv][4 * kq + i][r16] = acc[i];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < nrow) {
    float a[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) a[i] = sums[wv][lane][i];
    const int k = (int)sums[wv][lane][9];
    float out[4];
    finish_normal(a, k, q.x, q.y, q.z, vpx, vpy, vpz, out);
    const int32_t orig = g.perm[p0 + lane];
    nx[orig] = out[0];
    ny[orig] = out[1];
    nz[orig] = out[2];
    curv[orig] = out[3];
  }
}

__global__ void k_nan_fill4_fast(float* __restrict__ a, float* __restrict__ b, float* __restrict__ c,
                                 float* __restrict__ d, int64_t n) {
  const float v = __builtin_nanf("");  // PCL's quiet_NaN (0x7FC00000), as the product path's fill
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a[i] = v; b[i] = v; c[i] = v; d[i] = v;
  }
}

}  // namespace

void normals_fast_dev(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n, double r,
                      const float vp[3], float* nx, float* ny, float* nz, float* curv) {
  PFX_CHECK(r > 0.0, "normals_fast: radius must be > 0");
  if (n == 0) return;
  TimeScope total(ctx, "normals_fast", true);
  hipStream_t st = ctx->stream;
  build_grid(ctx, ctx->grid_a, x, y, z, n, r);
  if (ctx->normals) ctx->normals->ready = false;  // grid_a no longer matches held lists
  const Grid& G = ctx->grid_a;
  k_nan_fill4_fast<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, st>>>(nx, ny, nz, curv, n);
  {
    TimeScope ts(ctx, "normals_mfma", true);
    // one wave per 16 grid points (all n: waves past the finite count return at once)
    k_normals_mfma<<<(unsigned)ceil_div(ceil_div(n, 16), 4), 256, 0, st>>>(view(G), (float)(r * r), vp[0], vp[1],
                                                                          vp[2], nx, ny, nz, curv);
    check_launch("k_normals_mfma");
  }
}

}  // namespace pfx
