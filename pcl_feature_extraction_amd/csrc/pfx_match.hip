// pfx_match.hip -- descriptor matching of the reference's evaluation loop:
//   Features<T>::getCorrespondences  features.h:255-273  (1-NN through KdTreeFLANN<FeatureT>)
//   Features<T>::findCorrespondences features.h:224-253  (both directions + mutual check)
//
// The reference distance is FLANN's L2_Simple<float>: a sequential float sum of (a_k - b_k)^2
// over the D dimensions (oracle/or_match.cpp).  The 1-NN over all pairs is a dense contraction,
// so it runs on the matrix cores, and exactness is restored afterwards:
//
//   1. prep:   every row -> validity (all finite), fp32 squared norm, and a bf16 split (rows
//              padded to Dp = 32-multiple dims)
//              a = a_hi + a_lo + O(2^-16 |a|), packed as [a_hi | a_hi | a_lo] (source) and
//              [b_hi | b_lo | b_hi] (target), so ONE bf16 MFMA product over K = 3 Dp gives
//              a_hi.b_hi + a_hi.b_lo + a_lo.b_hi (error <= 3.1 2^-16 |a||b|).
//   2. bound:  128x128 workgroup tiles of d^ = |a|^2 + |b|^2 - 2 a.b on v_mfma_f32_32x32x16_bf16;
//              with the rigorous error bound e(a, b) (below) |d^ - L2_Simple(a, b)| <= e, every
//              row keeps U_i = min_j (d^_ij + e_ij) and every column U_j likewise.  A seeding
//              launch over a cross of tiles (4 row tiles x all, all x 4 column tiles) first
//              brings the bounds near their final values.
//   3. prune:  the same launch emits (i, j, d^_ij - e_ij) for the pairs whose d^ - e is within the
//              running bound of the row or the column (running bounds only fall, so no candidate
//              is missed); (i, j) is a candidate of row i iff d^_ij - e_ij <= U_i (the true
//              minimiser always is), of column j iff d^_ij - e_ij <= U_j, tested on that list.
//              A list overflow falls back to a second contraction that tests every pair.
//   4. exact:  one lane per candidate evaluates L2_Simple in the reference's order and keeps the
//              minimum of the 64-bit key (float bits << 32 | row) -- ties go to the lowest row.
//   5. mutual: target2source[source2target[c]] == c, compacted in source order.
//
// Error bound (u = 2^-24, P = (|a| + |b|)^2 >= |a|^2 + |b|^2, Q = |a||b|, S = the real sum of
// squares |a|^2 + |b|^2 - 2 a.b):
//   |L2_Simple - S|         <= (D + 3) u P             (sequential fp32, no FMA)
//   |n2_a - |a|^2| + |n2_b - |b|^2| <= (D + 1) u P     (fp32 sums, any order)
//   2 |MFMA - split dot|    <= 2 * 2 * 3D u 1.016 Q    (exact bf16 products, fp32 accumulation;
//                                                       x2 if the accumulation truncates)
//   2 |split dot - a.b|     <= 2 * 3.1 2^-16 Q
//   the two final roundings <= 2.02 u P
//   => e = 1.5 [(2D + 6.1) u P + (12.2 D u + 6.2 2^-16) Q] + 1e-30 (flushed denormals);
//      x1.5: margin for evaluating e itself in fp32.
#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "pfx_internal.h"

namespace pfx {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kTile = 128;  // workgroup tile (rows x cols); 4 waves of 64 x 64
constexpr uint32_t kInfBits = 0x7f800000u;

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_val(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

#ifndef PFX_MATCH_KC
#define PFX_MATCH_KC 32
#endif
constexpr int kKC = PFX_MATCH_KC;  // K per LDS stage
// packed row length: the three Dp-long parts, zero-padded to whole K stages
__host__ __device__ inline int kp_of(int Dp) { return (3 * Dp + kKC - 1) / kKC * kKC; }

// one wave per row: validity, fp32 squared norm, packed bf16 split (pad rows/dims are zero)
__global__ void __launch_bounds__(256) k_match_prep(const float* __restrict__ X, int64_t n, int64_t stride, int D,
                                                    int Dp, int64_t n_pad, int is_target,
                                                    uint16_t* __restrict__ P, float* __restrict__ n2,
                                                    float* __restrict__ nrm, uint8_t* __restrict__ valid) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_pad) return;
  const int KP = kp_of(Dp);
  uint16_t* row = P + i * KP;
  for (int k = 3 * Dp + lane; k < KP; k += 64) row[k] = 0;
  bool ok = i < n;
  float s = 0.f;
  if (ok) {
    const float* x = X + i * stride;
    bool fin = true;
    for (int k = lane; k < D; k += 64) {
      const float v = x[k];
      fin = fin && isfinite(v);
      s += v * v;
    }
    ok = !__any(!fin);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  for (int k = lane; k < Dp; k += 64) {
    uint16_t hi = 0, lo = 0;
    if (ok && k < D) {
      const float v = X[i * stride + k];
      hi = bf16_rne(v);
      lo = bf16_rne(v - bf16_val(hi));  // exact difference
    }
    row[k] = hi;
    row[Dp + k] = is_target ? lo : hi;
    row[2 * Dp + k] = is_target ? hi : lo;
  }
  if (lane == 0) {
    n2[i] = ok ? s : 0.f;
    nrm[i] = ok ? sqrtf(s) : 0.f;
    valid[i] = ok ? 1 : 0;
  }
}

struct Side {
  const uint16_t* P;
  const float* n2;
  const float* nrm;
  const uint8_t* valid;
  int64_t n;
};

// Slots [base, base + k) of the pair list.  The count is 64-bit, so it cannot wrap back below the
// cap however many pairs near-duplicate sets emit (up to ns x nt; match_pairs_overflowed sees
// count > cap and reruns the second contraction).  (Round 5: a saturating 32-bit count -- an
// atomic load before each add -- slowed the bound pass 0.41 -> 1.0 ms: every wave's reservation
// then made two accesses to the one contended address.)
__device__ __forceinline__ unsigned long long emit_reserve(unsigned long long* nemit, unsigned k) {
  return atomicAdd(nemit, (unsigned long long)k);
}

// PASS 0: row / column upper bounds, and the pruned pair list: after a tile's atomicMin the
// running bound of a row (column) is >= its final U, so a pair with d^ - e above the running
// bound of both its row and its column can never be a candidate; the rest (a few dozen per row:
// the tiles that lowered a bound) are emitted as (row, col, d^ - e) and tested against the final
// bounds by k_match_exact_emit -- no second contraction.  PASS 1 (the fallback when the pair
// list overflows): the contraction again, candidates against the final bounds.
// EMIT = false (PASS 0 only): bounds alone, over the seeding cross (cross = 1: the first sr row
// tiles x every column tile and the first sc column tiles x the other row tiles), so that the
// emitting pass starts from bounds near final ones instead of from +inf.
// Three waves per SIMD requested: the accumulators then live in VGPRs (no AGPR copies), 126 VGPRs,
// four workgroups per CU -- 0.41 -> 0.34 ms for the 10k x 10k bound pass.
template <int PASS, bool EMIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k_match_tiles(Side A, Side B, int D, int Dp, float c1, float c2,
                                                     uint32_t* __restrict__ Urow, uint32_t* __restrict__ Ucol,
                                                     int2* __restrict__ crow, int2* __restrict__ ccol,
                                                     unsigned* __restrict__ ncand, unsigned cap,
                                                     int4* __restrict__ emit, unsigned long long* __restrict__ nemit,
                                                     unsigned ecap, int gx, int gy, int group, int cross,
                                                     int sr, int sc) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so XCD x gets the
  // flat ids x, x + 8, ...; it is handed the x-th contiguous eighth of a grouped tile sequence
  // (group row tiles at a time, column-major inside the group) -- its in-flight tiles then share
  // a few A and B panels in its own L2 instead of streaming every B panel from the MALL.
  int ty, tx;
  {
    const int bid = blockIdx.x, T = gx * gy;
    int seq = bid;
    if (cross) {
      if (seq < sr * gx) {
        ty = seq % sr;
        tx = seq / sr;
      } else {
        seq -= sr * gx;
        ty = sr + seq / sc;
        tx = seq % sc;
      }
    } else if (group > 0) {
      const int xcd = bid & 7, slot = bid >> 3, q = T >> 3, r = T & 7;
      seq = xcd * q + min(xcd, r) + slot;
      const int g = seq / (group * gx), idx = seq - g * group * gx;
      const int rows = min(group, gy - g * group);
      tx = idx / rows;
      ty = g * group + (idx - tx * rows);
    } else {
      ty = seq / gx;
      tx = seq - ty * gx;
    }
  }
  const int64_t r0 = (int64_t)ty * kTile + (wv >> 1) * 64;
  const int64_t q0 = (int64_t)tx * kTile + (wv & 1) * 64;
  const int KP = kp_of(Dp);
  const int h = lane >> 5, l32 = lane & 31;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // K in chunks of KC = 32 (two MFMA k-steps): the workgroup's 128 A rows and 128 B rows of a
  // chunk are staged in LDS (double buffer; rows padded by 16 B so the 32 rows a fragment read
  // touches spread over the banks) and the next chunk's global loads are in flight while the
  // current one is multiplied -- every fragment is read from L2 once per workgroup instead of
  // once per wave.
  constexpr int KC = kKC, RS = KC + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sa[2][kTile * RS];
  __shared__ __attribute__((aligned(16))) uint16_t sb[2][kTile * RS];
  const int tid = threadIdx.x;
  const int64_t ra0 = (int64_t)ty * kTile, qb0 = (int64_t)tx * kTile;
  // 128 rows x 2 KC B per operand = 16 KC 16-B pieces: thread t moves pieces t + 256 i
  constexpr int PARTS = KC / 8, NP = PARTS / 2;
  static_assert(NP == 2 || NP == 4, "KC 32 or 64");
  uint4 va0, va1, va2, va3, vb0, vb1, vb2, vb3;  // (named: an array here went to scratch)
  auto ld = [&](int i, int k0, uint4& x, uint4& y) {
    const int pc = tid + 256 * i, rw = pc / PARTS, pt = pc % PARTS;
    x = *reinterpret_cast<const uint4*>(A.P + (ra0 + rw) * KP + k0 + pt * 8);
    y = *reinterpret_cast<const uint4*>(B.P + (qb0 + rw) * KP + k0 + pt * 8);
  };
  auto st = [&](int i, int buf, const uint4& x, const uint4& y) {
    const int pc = tid + 256 * i, rw = pc / PARTS, pt = pc % PARTS;
    *reinterpret_cast<uint4*>(&sa[buf][rw * RS + pt * 8]) = x;
    *reinterpret_cast<uint4*>(&sb[buf][rw * RS + pt * 8]) = y;
  };
  auto gload = [&](int k0) {
    ld(0, k0, va0, vb0);
    ld(1, k0, va1, vb1);
    if constexpr (NP == 4) {
      ld(2, k0, va2, vb2);
      ld(3, k0, va3, vb3);
    }
  };
  auto sstore = [&](int buf) {
    st(0, buf, va0, vb0);
    st(1, buf, va1, vb1);
    if constexpr (NP == 4) {
      st(2, buf, va2, vb2);
      st(3, buf, va3, vb3);
    }
  };
  const int nch = KP / KC;
  const int ar = (wv >> 1) * 64 + l32, br = (wv & 1) * 64 + l32;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    if (c + 1 < nch) {
      gload((c + 1) * KC);
    }
#pragma unroll
    for (int ks = 0; ks < KC / 16; ++ks) {
      const int ko = 16 * ks + 8 * h;
      const bf16x8 fa0 = *reinterpret_cast<const bf16x8*>(&sa[buf][ar * RS + ko]);
      const bf16x8 fa1 = *reinterpret_cast<const bf16x8*>(&sa[buf][(ar + 32) * RS + ko]);
      const bf16x8 fb0 = *reinterpret_cast<const bf16x8*>(&sb[buf][br * RS + ko]);
      const bf16x8 fb1 = *reinterpret_cast<const bf16x8*>(&sb[buf][(br + 32) * RS + ko]);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb1, acc[1][1], 0, 0, 0);
    }
    if (c + 1 < nch) {  // buf ^ 1 was last read before the previous barrier
      sstore(buf ^ 1);
    }
    __syncthreads();
  }
  // epilogue: C/D map of 32x32 tiles: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float cn2[2], cnr[2];
  bool cval[2];
  uint32_t ucol[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int64_t q = q0 + 32 * b + l32;
    cn2[b] = B.n2[q];
    cnr[b] = B.nrm[q];
    cval[b] = B.valid[q] != 0;
    ucol[b] = Ucol[q];  // PASS 0: the running bound before this tile (>= the final one)
  }
  float cmin[2] = {__uint_as_float(kInfBits), __uint_as_float(kInfBits)};
  // PASS 0: pairs are staged per wave in LDS (free after the main loop: 512 pairs per wave) and
  // flushed with one global atomic per wave; a full stage spills straight to the global list
  constexpr unsigned kStage = 512;
  int4* stage = reinterpret_cast<int4*>(wv < 2 ? &sa[0][0] : &sb[0][0]) + (wv & 1) * kStage;
  unsigned staged = 0;  // wave-uniform
  // the wave's 64 rows (n2, norm, valid, running bound) staged in LDS by one load per lane: the
  // emission branches would otherwise serialise the per-row global loads (one L2 trip per row)
  float4* rowd = reinterpret_cast<float4*>(reinterpret_cast<char*>(wv < 2 ? &sa[0][0] : &sb[0][0]) + 16384) +
                 (wv & 1) * 64;
  if (PASS == 0 && EMIT) {
    const int64_t rl = r0 + lane;
    rowd[lane] = make_float4(A.n2[rl], A.nrm[rl], A.valid[rl] ? 1.f : 0.f, __uint_as_float(Urow[rl]));
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t row = r0 + rr;
      float rn2, rnr;
      bool rval;
      uint32_t urow;
      if (PASS == 0 && EMIT) {
        const float4 rd = rowd[rr];
        rn2 = rd.x;
        rnr = rd.y;
        rval = rd.z != 0.f;
        urow = __float_as_uint(rd.w);
      } else {
        rn2 = A.n2[row];
        rnr = A.nrm[row];
        rval = A.valid[row] != 0;
        urow = Urow[row];
      }
      float rmin = __uint_as_float(kInfBits);
      float dh[2], e[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        dh[b] = (rn2 + cn2[b]) - 2.0f * acc[a][b][r];
        const float s = rnr + cnr[b];
        e[b] = 1.5f * (c1 * (s * s) + c2 * (rnr * cnr[b])) + 1e-30f;
        const bool ok = rval && cval[b];
        if (PASS == 0) {
          const float ub = ok ? fmaxf(dh[b] + e[b], 0.f) : __uint_as_float(kInfBits);
          rmin = fminf(rmin, ub);
          cmin[b] = fminf(cmin[b], ub);
        } else if (ok) {
          const float lb = dh[b] - e[b];
          const int64_t col = q0 + 32 * b + l32;
          if (lb <= __uint_as_float(urow)) {
            const unsigned slot = atomicAdd(&ncand[0], 1u);
            if (slot < cap) crow[slot] = make_int2((int)row, (int)col);
          }
          if (lb <= __uint_as_float(ucol[b])) {
            const unsigned slot = atomicAdd(&ncand[1], 1u);
            if (slot < cap) ccol[slot] = make_int2((int)col, (int)row);
          }
        }
      }
      if (PASS == 0) {
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) rmin = fminf(rmin, __shfl_xor(rmin, o));
        if (l32 == 0 && rmin < __uint_as_float(kInfBits) && row < A.n) atomicMin(&Urow[row], __float_as_uint(rmin));
        // any ub of a row (column) bounds its final U from above: the row's threshold is the
        // running bound read before the tile or this wave's 64-column minimum, the column's the
        // running bound or the minimum over the rows this lane has passed (this one included)
        if (!EMIT) continue;
        const float trow = fminf(__uint_as_float(urow), rmin);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const float lb = dh[b] - e[b];
          const bool em = rval && cval[b] && (lb <= trow || lb <= fminf(__uint_as_float(ucol[b]), cmin[b]));
          const uint64_t m = __ballot(em);
          if (m) {
            const unsigned k = (unsigned)__popcll(m), pre = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            const int4 pr = make_int4((int)row, (int)(q0 + 32 * b + l32), __float_as_int(lb), 0);
            if (staged + k <= kStage) {
              if (em) stage[staged + pre] = pr;
              staged += k;
            } else {
              const int first = __ffsll((long long)m) - 1;
              unsigned long long base = 0;
              if (lane == first) base = emit_reserve(nemit, k);
              base = __shfl(base, first);
              if (em && base + pre < ecap) emit[base + pre] = pr;
            }
          }
        }
      }
    }
  }
  if (PASS == 0) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float v = fminf(cmin[b], __shfl_xor(cmin[b], 32));
      const int64_t q = q0 + 32 * b + l32;
      if (h == 0 && v < __uint_as_float(kInfBits) && q < B.n) atomicMin(&Ucol[q], __float_as_uint(v));
    }
    if (staged) {
      unsigned long long base = 0;
      if (lane == 0) base = emit_reserve(nemit, staged);
      base = __shfl(base, 0);
      for (unsigned i = lane; i < staged; i += 64)
        if (base + i < ecap) emit[base + i] = stage[i];
    }
  }
}

// L2_Simple in the reference order (oracle/or_match.cpp): a sequential fp32 sum, no FMA
template <bool VEC>
__device__ __forceinline__ float l2_simple(const float* __restrict__ a, const float* __restrict__ b, int D) {
  float result = 0.0f;
  if (VEC) {  // 16-B loads, the same sequential sum
#pragma unroll 4
    for (int k = 0; k < D; k += 4) {
      const float4 x = *reinterpret_cast<const float4*>(a + k), y = *reinterpret_cast<const float4*>(b + k);
      const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
      result = result + d0 * d0;
      result = result + d1 * d1;
      result = result + d2 * d2;
      result = result + d3 * d3;
    }
  } else {
    for (int k = 0; k < D; ++k) {
      const float diff = a[k] - b[k];
      result = result + diff * diff;
    }
  }
  return result;
}

// The candidate test of the pruned pairs against the final bounds, fused with the exact pass:
// a pair is a candidate of its row iff d^ - e <= U_row, of its column iff d^ - e <= U_col (the
// tests k_match_tiles<1> makes); (a - b)^2 == (b - a)^2 in fp32, so one L2_Simple serves both.
template <bool VEC>
__global__ void __launch_bounds__(256) k_match_exact_emit(const float* __restrict__ A, int64_t sa,
                                                          const float* __restrict__ B, int64_t sb, int D,
                                                          const int4* __restrict__ emit,
                                                          const unsigned long long* __restrict__ nemit, unsigned ecap,
                                                          const uint32_t* __restrict__ Urow,
                                                          const uint32_t* __restrict__ Ucol,
                                                          unsigned* __restrict__ ncand,
                                                          unsigned long long* __restrict__ bs,
                                                          unsigned long long* __restrict__ bt) {
  const unsigned n = (unsigned)min(*nemit, (unsigned long long)ecap);
  unsigned nr = 0, nc = 0;
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    const int4 p = emit[t];
    const float lb = __int_as_float(p.z);
    const bool pr = lb <= __uint_as_float(Urow[p.x]), pc = lb <= __uint_as_float(Ucol[p.y]);
    if (!(pr || pc)) continue;
    const float d = l2_simple<VEC>(A + (int64_t)p.x * sa, B + (int64_t)p.y * sb, D);
    if (pr) atomicMin(&bs[p.x], ((unsigned long long)__float_as_uint(d) << 32) | (uint32_t)p.y);
    if (pc) atomicMin(&bt[p.y], ((unsigned long long)__float_as_uint(d) << 32) | (uint32_t)p.x);
    nr += pr;
    nc += pc;
  }
  // candidate counts (statistics): one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nr += __shfl_xor(nr, o);
    nc += __shfl_xor(nc, o);
  }
  if ((threadIdx.x & 63) == 0 && (nr | nc)) {
    atomicAdd(&ncand[0], nr);
    atomicAdd(&ncand[1], nc);
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) k_match_exact(const float* __restrict__ A, int64_t sa,
                                                     const float* __restrict__ B, int64_t sb, int D,
                                                     const int2* __restrict__ crow, const int2* __restrict__ ccol,
                                                     const unsigned* __restrict__ ncand, unsigned cap,
                                                     unsigned long long* __restrict__ bs,
                                                     unsigned long long* __restrict__ bt) {
  // both directions in one launch (row candidates, then column candidates); counts past the
  // buffer are clamped here and rerun by the host with a larger buffer
  const unsigned n0 = min(ncand[0], cap), n1 = min(ncand[1], cap);
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < n0 + n1; t += gridDim.x * 256) {
    const bool fwd = t < n0;
    const int2 c = fwd ? crow[t] : ccol[t - n0];
    const float* a = fwd ? A + (int64_t)c.x * sa : B + (int64_t)c.x * sb;
    const float* b = fwd ? B + (int64_t)c.y * sb : A + (int64_t)c.y * sa;
    const float result = l2_simple<VEC>(a, b, D);
    atomicMin(fwd ? &bs[c.x] : &bt[c.x], ((unsigned long long)__float_as_uint(result) << 32) | (uint32_t)c.y);
  }
}

__global__ void k_match_finish(const unsigned long long* __restrict__ best, int64_t n, int32_t* __restrict__ idx,
                               float* __restrict__ dist) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long k = best[i];
  const bool found = k != ~0ull;
  idx[i] = found ? (int32_t)(uint32_t)(k & 0xffffffffu) : -1;
  if (dist) dist[i] = found ? __uint_as_float((uint32_t)(k >> 32)) : __builtin_nanf("");
}

__global__ void k_match_mutual(const int32_t* __restrict__ s2t, int64_t ns, const int32_t* __restrict__ t2s,
                               uint8_t* __restrict__ flags) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= ns) return;
  const int32_t m = s2t[c];
  flags[c] = (m >= 0 && t2s[m] == (int32_t)c) ? 1 : 0;
}

__global__ void k_match_gather(const int32_t* __restrict__ q, const int64_t* __restrict__ nsel,
                               const int32_t* __restrict__ s2t, int32_t* __restrict__ m) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < *nsel) m[t] = s2t[q[t]];
}

struct Prepared {
  Side side;
  int64_t n_pad;
};

Prepared prep(pfx_ctx* ctx, const char* tag, const float* X, int64_t n, int64_t stride, int D, int Dp,
              bool target) {
  const int64_t n_pad = std::max<int64_t>(ceil_div(n, kTile), 1) * kTile;
  const std::string t(tag);
  uint16_t* P = ctx->buf((t + "_pk").c_str()).as<uint16_t>((size_t)n_pad * kp_of(Dp));
  float* n2 = ctx->buf((t + "_n2").c_str()).as<float>(n_pad);
  float* nr = ctx->buf((t + "_nr").c_str()).as<float>(n_pad);
  uint8_t* v = ctx->buf((t + "_v").c_str()).as<uint8_t>(n_pad);
  k_match_prep<<<(unsigned)ceil_div(n_pad, 4), 256, 0, ctx->stream>>>(X, n, stride, D, Dp, n_pad, target ? 1 : 0, P,
                                                                       n2, nr, v);
  check_launch("k_match_prep");
  return Prepared{Side{P, n2, nr, v, n}, n_pad};
}

}  // namespace

// Both directions at once (the tiles serve rows and columns): s2t[i] = nearest target row of
// source row i, t2s[j] = nearest source row of target row j (-1: no finite row / no target).
bool match_pairs_overflowed(pfx_ctx* ctx) {
  const unsigned* h = ctx->readback<unsigned>();  // (written by the deferred call's copy)
  const unsigned long long emitted = (unsigned long long)h[2] | ((unsigned long long)h[3] << 32);
  ctx->stats["match_pairs_emitted"] = (int64_t)emitted;
  ctx->stats["match_candidates_rows"] = h[0];
  ctx->stats["match_candidates_cols"] = h[1];
  return (int64_t)emitted > ctx->stats["match_pair_cap"];
}

bool match_nearest_dev(pfx_ctx* ctx, const float* src, int64_t ns, int64_t ss, const float* tgt, int64_t nt,
                       int64_t ts, int D, int32_t* s2t, float* ds2t, int32_t* t2s, float* dt2s, int mode) {
  PFX_CHECK(D > 0 && ns >= 0 && nt >= 0 && ss >= D && ts >= D, "match: invalid dimensions");
  PFX_CHECK(ns < (int64_t(1) << 31) && nt < (int64_t(1) << 31), "match: too many rows");
  hipStream_t st = ctx->stream;
  if (ns == 0 && nt == 0) return false;
  if (ns == 0 || nt == 0) {  // nothing to match against
    if (ns) PFX_HIP(hipMemsetAsync(s2t, 0xff, sizeof(int32_t) * ns, st));
    if (nt && t2s) PFX_HIP(hipMemsetAsync(t2s, 0xff, sizeof(int32_t) * nt, st));
    if (ns && ds2t) PFX_HIP(hipMemsetAsync(ds2t, 0xff, sizeof(float) * ns, st));
    if (nt && dt2s) PFX_HIP(hipMemsetAsync(dt2s, 0xff, sizeof(float) * nt, st));
    return false;
  }
  TimeScope total(ctx, "match", true);
  const int Dp = (D + 31) / 32 * 32;  // K = 3 Dp: whole 32-deep LDS chunks
  const Prepared a = prep(ctx, "match_a", src, ns, ss, D, Dp, false);
  const Prepared b = prep(ctx, "match_b", tgt, nt, ts, D, Dp, true);
  uint32_t* Urow = ctx->buf("match_urow").as<uint32_t>(a.n_pad);
  uint32_t* Ucol = ctx->buf("match_ucol").as<uint32_t>(b.n_pad);
  unsigned long long* bs = ctx->buf("match_bs").as<unsigned long long>(ns);
  unsigned long long* bt = ctx->buf("match_bt").as<unsigned long long>(nt);
  // [0] row candidates, [1] column candidates, [2..3] the 64-bit pair count
  unsigned* ncand = ctx->buf("match_ncand").as<unsigned>(4);
  PFX_HIP(hipMemsetAsync(Urow, 0x7f, sizeof(uint32_t) * a.n_pad, st));  // 0x7f7f7f7f: above any bound
  PFX_HIP(hipMemsetAsync(Ucol, 0x7f, sizeof(uint32_t) * b.n_pad, st));
  const float u = 5.9604645e-8f;  // 2^-24
  const float c1 = (2.0f * (float)D + 6.1f) * u, c2 = 12.2f * (float)D * u + 6.2f / 65536.0f;
  const int gx = (int)(b.n_pad / kTile), gy = (int)(a.n_pad / kTile);
  const unsigned grid = (unsigned)gx * (unsigned)gy;
  constexpr int group = 8;  // row tiles per XCD group of the tile order
  const bool vec = D % 4 == 0 && ss % 4 == 0 && ts % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)tgt & 15) == 0;
  unsigned* h = ctx->readback<unsigned>();
  // the pruned pair list: a few dozen pairs per row normally (an overflow takes the two-contraction
  // fallback: test_match_pair_list_overflow)
  const unsigned ecap =
      mode == 2 ? 0u : (unsigned)std::min<int64_t>(64 * (ns + nt) + (1 << 16), int64_t(1) << 28);
  ctx->stats["match_pair_cap"] = ecap;
  int4* emit = ctx->buf("match_emit").as<int4>(std::max(ecap, 1u));
  unsigned long long* nemit = reinterpret_cast<unsigned long long*>(ncand + 2);
  PFX_HIP(hipMemsetAsync(ncand, 0, 4 * sizeof(unsigned), st));
  PFX_HIP(hipMemsetAsync(bs, 0xff, sizeof(unsigned long long) * ns, st));
  PFX_HIP(hipMemsetAsync(bt, 0xff, sizeof(unsigned long long) * nt, st));
  if (gx > 16 && gy > 16) {
    // seed the bounds over the cross of the first sr row tiles and sc column tiles, a tenth of the
    // tiles at any size (at least 4 each): a pair then passes a seeded bound with probability
    // ~ 1 / (128 s), so the pair list stays at a few dozen pairs per row as the sets grow
    TimeScope ts0(ctx, "match_seed");
    const int sr = std::min(gy, std::max(4, (gy + 19) / 20)), sc = std::min(gx, std::max(4, (gx + 19) / 20));
    const unsigned ncross = (unsigned)(sr * gx + sc * (gy - sr));
    k_match_tiles<0, false><<<ncross, 256, 0, st>>>(a.side, b.side, D, Dp, c1, c2, Urow, Ucol, nullptr, nullptr,
                                                    nullptr, 0, nullptr, nullptr, 0, gx, gy, 0, 1, sr, sc);
    check_launch("k_match_tiles<0, false>");
  }
  {
    TimeScope ts1(ctx, "match_bound");
    k_match_tiles<0, true><<<grid, 256, 0, st>>>(a.side, b.side, D, Dp, c1, c2, Urow, Ucol, nullptr, nullptr, nullptr,
                                                 0, emit, nemit, ecap, gx, gy, group, 0, 0, 0);
    check_launch("k_match_tiles<0, true>");
  }
  {
    TimeScope ts3(ctx, "match_exact");
    auto* ke = vec ? k_match_exact_emit<true> : k_match_exact_emit<false>;
    ke<<<1024, 256, 0, st>>>(src, ss, tgt, ts, D, emit, nemit, ecap, Urow, Ucol, ncand, bs, bt);
    check_launch("k_match_exact_emit");
  }
  k_match_finish<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(bs, ns, s2t, ds2t);
  if (t2s) k_match_finish<<<(unsigned)ceil_div(nt, 256), 256, 0, st>>>(bt, nt, t2s, dt2s);
  check_launch("k_match_finish");
  PFX_HIP(hipMemcpyAsync(h, ncand, 4 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
  if (mode == 1) return true;  // the caller synchronises once for everything it launched
  PFX_HIP(hipStreamSynchronize(st));  // the one host round trip of a normal call
  if (!match_pairs_overflowed(ctx)) return false;
  // fallback: the pair list overflowed (near-duplicate descriptors) -- the contraction again,
  // candidates against the final bounds, exact pass over the candidate lists
  DevBuf& cb = ctx->buf("match_cand");
  unsigned cap = (unsigned)std::min<int64_t>(std::max<int64_t>(8 * (ns + nt), 1 << 20), int64_t(1) << 30);
  for (int attempt = 0; attempt < 2; ++attempt) {
    int2* crow = static_cast<int2*>(cb.get(sizeof(int2) * 2 * (size_t)cap));
    int2* ccol = crow + cap;
    PFX_HIP(hipMemsetAsync(ncand, 0, 2 * sizeof(unsigned), st));
    PFX_HIP(hipMemsetAsync(bs, 0xff, sizeof(unsigned long long) * ns, st));
    PFX_HIP(hipMemsetAsync(bt, 0xff, sizeof(unsigned long long) * nt, st));
    {
      TimeScope ts2(ctx, "match_filter");
      k_match_tiles<1, false><<<grid, 256, 0, st>>>(a.side, b.side, D, Dp, c1, c2, Urow, Ucol, crow, ccol, ncand,
                                                    cap, nullptr, nullptr, 0, gx, gy, group, 0, 0, 0);
      check_launch("k_match_tiles<1>");
    }
    {
      TimeScope ts3(ctx, "match_exact");
      auto* ke = vec ? k_match_exact<true> : k_match_exact<false>;
      ke<<<1024, 256, 0, st>>>(src, ss, tgt, ts, D, crow, ccol, ncand, cap, bs, bt);
      check_launch("k_match_exact");
    }
    k_match_finish<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(bs, ns, s2t, ds2t);
    if (t2s) k_match_finish<<<(unsigned)ceil_div(nt, 256), 256, 0, st>>>(bt, nt, t2s, dt2s);
    check_launch("k_match_finish");
    PFX_HIP(hipMemcpyAsync(h, ncand, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    ctx->stats["match_candidates_rows"] = h[0];
    ctx->stats["match_candidates_cols"] = h[1];
    if (std::max(h[0], h[1]) > cap) {
      PFX_CHECK(attempt == 0, "match: candidate buffer growth failed");
      cap = std::max(h[0], h[1]);
      continue;
    }
    break;
  }
  return false;
}

int64_t correspondences_dev(pfx_ctx* ctx, const float* src, int64_t ns, int64_t ss, const float* tgt, int64_t nt,
                            int64_t ts, int D, int32_t* query, int32_t* match, int64_t cap) {
  hipStream_t st = ctx->stream;
  int32_t* s2t = ctx->buf("match_s2t").as<int32_t>(ns + 1);
  int32_t* t2s = ctx->buf("match_t2s").as<int32_t>(nt + 1);
  if (ns == 0 || nt == 0) {
    match_nearest_dev(ctx, src, ns, ss, tgt, nt, ts, D, s2t, nullptr, t2s, nullptr);
    return 0;
  }
  uint8_t* flags = ctx->buf("match_flags").as<uint8_t>(ns);
  int32_t* qsel = ctx->buf("match_qsel").as<int32_t>(ns);
  int64_t* nsel = ctx->buf("match_nsel").as<int64_t>(1);
  int32_t* msel = ctx->buf("match_msel").as<int32_t>(ns);
  int64_t n = 0;
  // the nearest search deferred: one stream synchronisation for the whole chain; a pair-list
  // overflow (seen after it) reruns the chain on the two-contraction path
  for (int mode = 1; mode <= 2; ++mode) {
    const bool check = match_nearest_dev(ctx, src, ns, ss, tgt, nt, ts, D, s2t, nullptr, t2s, nullptr, mode);
    k_match_mutual<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(s2t, ns, t2s, flags);
    check_launch("k_match_mutual");
    size_t tb = 0;
    PFX_HIP(rocprim::select(nullptr, tb, rocprim::counting_iterator<int32_t>(0), flags, qsel, nsel, (size_t)ns, st));
    void* tmp = ctx->buf("match_tmp").get(tb + 16);
    PFX_HIP(rocprim::select(tmp, tb, rocprim::counting_iterator<int32_t>(0), flags, qsel, nsel, (size_t)ns, st));
    k_match_gather<<<(unsigned)ceil_div(ns, 256), 256, 0, st>>>(qsel, nsel, s2t, msel);
    check_launch("k_match_gather");
    PFX_HIP(hipMemcpyAsync(&n, nsel, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PFX_HIP(hipStreamSynchronize(st));
    if (!(check && match_pairs_overflowed(ctx))) break;
  }
  if (n > 0 && n <= cap) {
    PFX_HIP(hipMemcpyAsync(query, qsel, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
    PFX_HIP(hipMemcpyAsync(match, msel, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
  }
  ctx->stats["match_correspondences"] = n;
  return n;
}

}  // namespace pfx
