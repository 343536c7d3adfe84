// pfx_normals_tile.h -- the tiled neighbour-gather + ordered-covariance kernel of pfx_normals.hip.
//
// One 256-thread workgroup per tile = up to Q consecutive points of one grid cell.  The tile's
// queries share the 3x3x3 candidate block (9 contiguous runs of the cell-sorted SoA copy):
//   1. the block's candidates are staged once into LDS (coalesced run loads, T <= TCAP);
//   2. wave w owns queries w, w+4, ... (Q/4 per wave): it streams the candidates from LDS and
//      tests them against its queries (wave-uniform cursors: no atomics, no block barrier),
//      keeping hits as u16 candidate indices;
//   3. each list is ordered by an LDS bucket sort on d2 (NB buckets, exact (d2, index) rank
//      inside a bucket -- FLANN's result order);
//   4. the 9 strictly sequential float chains of each query run one per lane over the sorted
//      list (coordinates from LDS), then eigen33 + flip per query.
// A query with more than LCAP neighbours is handed to the per-query path (overflow list).
#pragma once
#include "pfx_neighbors.h"

namespace pfx {

__device__ __forceinline__ float chain_term(int a, float px, float py, float pz) {
  float u = (a == 0 || a == 1 || a == 2 || a == 6) ? px : ((a == 3 || a == 4 || a == 7) ? py : pz);
  float v = (a == 0) ? px : ((a == 1 || a == 3) ? py : pz);
  return (a < 6) ? u * v : u;
}

__device__ __forceinline__ void finish_normal(const float accu_in[9], int k, float px, float py, float pz,
                                              float vpx, float vpy, float vpz, float out[4]) {
  if (k < 3) {
    out[0] = out[1] = out[2] = out[3] = __builtin_nanf("");
    return;
  }
  float a[9];
  const float cnt = (float)k;
#pragma unroll
  for (int i = 0; i < 9; ++i) a[i] = accu_in[i] / cnt;
  Sym3 C;
  C.a00 = a[0] - a[6] * a[6];
  C.a01 = a[1] - a[6] * a[7];
  C.a02 = a[2] - a[6] * a[8];
  C.a11 = a[3] - a[7] * a[7];
  C.a12 = a[4] - a[7] * a[8];
  C.a22 = a[5] - a[8] * a[8];
  C.a10 = C.a01; C.a20 = C.a02; C.a21 = C.a12;
  float lambda;
  f3 n;
  eigen33_min(C, lambda, n);
  float eig_sum = C.a00 + C.a11 + C.a22;
  float curv = (eig_sum != 0.0f) ? fabsf(lambda / eig_sum) : 0.0f;
  float ax = vpx - px, ay = vpy - py, az = vpz - pz;
  float cos_theta = (ax * n.x + ay * n.y) + az * n.z;
  if (cos_theta < 0.0f) { n.x *= -1.0f; n.y *= -1.0f; n.z *= -1.0f; }
  out[0] = n.x; out[1] = n.y; out[2] = n.z; out[3] = curv;
}

// runs of the 3x3 column block around cell `key`
__device__ __forceinline__ void cell_runs(const GridView& g, uint32_t key, int r, int32_t& s, int32_t& len) {
  const int64_t iz = key % g.nz, iy = (key / g.nz) % g.ny, ix = key / ((uint64_t)g.nz * g.ny);
  const int64_t bx = ix + (r / 3) - 1, by = iy + (r % 3) - 1;
  const int64_t z0 = iz - 1 < 0 ? 0 : iz - 1, z1 = iz + 1 >= g.nz ? g.nz - 1 : iz + 1;
  s = 0;
  len = 0;
  if (bx >= 0 && bx < g.nx && by >= 0 && by < g.ny) {
    const int64_t base = (bx * g.ny + by) * g.nz;
    s = g.cell_start[base + z0];
    len = g.cell_start[base + z1 + 1] - s;
  }
}

template <int Q, int LCAP, int NB, int TCAP>
__global__ void __launch_bounds__(256) k_normals_tile(GridView g, const uint32_t* __restrict__ skeys,
                                                      const int32_t* __restrict__ tiles,
                                                      const int* __restrict__ ntiles_ptr, float rr,
                                                      float bscale, float vpx, float vpy, float vpz,
                                                      float* __restrict__ nx, float* __restrict__ ny,
                                                      float* __restrict__ nz, float* __restrict__ curv,
                                                      int32_t* __restrict__ overflow, int* __restrict__ n_overflow,
                                                      unsigned long long* __restrict__ total_nb) {
  constexpr int QW = Q / 4;  // queries per wave
  __shared__ float cx[TCAP], cy[TCAP], cz[TCAP];
  __shared__ uint16_t lists[Q][LCAP];
  __shared__ uint16_t tmp[4][LCAP];
  __shared__ int bcount[4][NB], bstart[4][NB], bfill[4][NB];
  __shared__ int run_start[9], run_pref[10];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned long long my_total = 0;
  const int64_t vb = xcd_block(blockIdx.x, gridDim.x);
  const int ntiles = *ntiles_ptr;
  for (int64_t tile = vb; tile < ntiles; tile += gridDim.x) {
    const int32_t start = tiles[tile];
    if (start < 0) continue;  // second half of a dense tile whose cell run ended
    const uint32_t key = skeys[start];
    const int qn = min(Q, g.cell_start[key + 1] - start);
    if (tid < 9) {
      int32_t s, len;
      cell_runs(g, key, tid, s, len);
      run_start[tid] = s;
      run_pref[tid] = len;
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int r = 0; r < 9; ++r) { int l = run_pref[r]; run_pref[r] = acc; acc += l; }
      run_pref[9] = acc;
    }
    __syncthreads();
    Runs R;
#pragma unroll
    for (int r = 0; r < 9; ++r) { R.start[r] = run_start[r]; R.pref[r] = run_pref[r]; }
    const int T = run_pref[9];
    R.pref[9] = T;
    if (T > TCAP) {  // classification guarantees T <= TCAP; keep the kernel safe regardless
      if (tid < qn) overflow[atomicAdd(n_overflow, 1)] = start + tid;
      __syncthreads();
      continue;
    }
    for (int t = tid; t < T; t += 256) {
      const int32_t pos = run_pos(R, t);
      cx[t] = g.sx[pos];
      cy[t] = g.sy[pos];
      cz[t] = g.sz[pos];
    }
    __syncthreads();
    // ---- test: wave wv owns queries wv + 4*u ----
    float qx[QW], qy[QW], qz[QW];
    int cursor[QW];
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const int j = wv + 4 * u;
      cursor[u] = 0;
      qx[u] = qy[u] = qz[u] = 0.f;
      if (j < qn) { qx[u] = g.sx[start + j]; qy[u] = g.sy[start + j]; qz[u] = g.sz[start + j]; }
    }
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + lane;
      const bool in = t < T;
      const float px = in ? cx[t] : 0.f, py = in ? cy[t] : 0.f, pz = in ? cz[t] : 0.f;
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const int j = wv + 4 * u;
        const bool hit = in && j < qn && flann_d2(qx[u], qy[u], qz[u], px, py, pz) < rr;
        const uint64_t m = __ballot(hit);
        if (hit) {
          const int slot = cursor[u] + __popcll(m & lanemask_lt());
          if (slot < LCAP) lists[j][slot] = (uint16_t)t;
        }
        cursor[u] += __popcll(m);
      }
    }
    // ---- per-query bucket sort (wave-local; LDS ops of one wave are ordered) ----
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const int j = wv + 4 * u;
      const int k = cursor[u];
      if (j >= qn) continue;  // wave-uniform
      if (k > LCAP) {
        if (lane == 0) overflow[atomicAdd(n_overflow, 1)] = start + j;
        continue;
      }
      for (int b = lane; b < NB; b += 64) { bcount[wv][b] = 0; bfill[wv][b] = 0; }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int e = lane; e < k; e += 64) {
        const int t = lists[j][e];
        int b = (int)(flann_d2(qx[u], qy[u], qz[u], cx[t], cy[t], cz[t]) * bscale);
        atomicAdd(&bcount[wv][b < NB ? b : NB - 1], 1);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      {
        constexpr int PER = NB / 64;
        int c[PER], s = 0;
#pragma unroll
        for (int v = 0; v < PER; ++v) { c[v] = bcount[wv][lane * PER + v]; s += c[v]; }
        int inc = s;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int o = __shfl_up(inc, off);
          if (lane >= off) inc += o;
        }
        int ex = inc - s;
#pragma unroll
        for (int v = 0; v < PER; ++v) { bstart[wv][lane * PER + v] = ex; ex += c[v]; }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int e = lane; e < k; e += 64) {
        const int t = lists[j][e];
        int b = (int)(flann_d2(qx[u], qy[u], qz[u], cx[t], cy[t], cz[t]) * bscale);
        b = b < NB ? b : NB - 1;
        tmp[wv][bstart[wv][b] + atomicAdd(&bfill[wv][b], 1)] = (uint16_t)t;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int s = lane; s < k; s += 64) {
        const int t = tmp[wv][s];
        const float d2 = flann_d2(qx[u], qy[u], qz[u], cx[t], cy[t], cz[t]);
        int b = (int)(d2 * bscale);
        b = b < NB ? b : NB - 1;
        const int st = bstart[wv][b], en = st + bcount[wv][b];
        int rank = 0;
        for (int v = st; v < en; ++v) {
          if (v == s) continue;
          const int tv = tmp[wv][v];
          const float dv = flann_d2(qx[u], qy[u], qz[u], cx[tv], cy[tv], cz[tv]);
          if (dv < d2) ++rank;
          else if (dv == d2 && g.perm[run_pos(R, tv)] < g.perm[run_pos(R, t)]) ++rank;
        }
        lists[j][st + rank] = (uint16_t)t;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // ---- 9 ordered chains per query: lane = 9*u + a ----
    float acc = 0.0f;
    int myk = 0;
    {
      const int u = lane / 9, a = lane - 9 * (lane / 9);
      const int j = wv + 4 * u;
      int k = 0;
#pragma unroll
      for (int v = 0; v < QW; ++v)
        if (v == u) k = cursor[v];
      if (u < QW && j < qn && k <= LCAP) {
        const uint16_t* L = lists[j];
#pragma unroll 8
        for (int m = 0; m < k; ++m) {
          const int t = L[m];
          acc = acc + chain_term(a, cx[t], cy[t], cz[t]);
        }
      }
      myk = k;
    }
    float accu[9];
#pragma unroll
    for (int a = 0; a < 9; ++a) accu[a] = __shfl(acc, min(63, 9 * lane + a));
    const int k_of_lane = __shfl(myk, min(63, 9 * lane));
    if (lane < QW) {
      const int j = wv + 4 * lane;
      if (j < qn && k_of_lane <= LCAP) {
        float o[4];
        finish_normal(accu, k_of_lane, g.sx[start + j], g.sy[start + j], g.sz[start + j], vpx, vpy, vpz, o);
        const int32_t orig = g.perm[start + j];
        nx[orig] = o[0]; ny[orig] = o[1]; nz[orig] = o[2]; curv[orig] = o[3];
        my_total += (unsigned long long)k_of_lane;
      }
    }
    __syncthreads();  // LDS (candidates, lists) is reused by the next tile
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) my_total += __shfl_xor(my_total, off);
  if (lane == 0 && my_total) atomicAdd(total_nb, my_total);
}

}  // namespace pfx
