// Microbenchmark (development aid, not product): per-query neighbour-list sorts of the list
// builder (pfx_nblist.hip) on synthetic lists -- each wave sorts one query's k candidate slots by
// d2 = |q - c[t]|^2 recomputed from LDS-staged float4 candidates, as the tile kernels do.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off scripts/sortbench.hip -o sortbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int TC = 1024;  // staged candidates per workgroup
constexpr int LC = 1024;  // list capacity

__device__ __forceinline__ float d2f(float qx, float qy, float qz, float4 c) {
  float dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
  return ((0.0f + dx * dx) + dy * dy) + dz * dz;
}
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ int excl_scan(int v, int lane) {
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(inc, o);
    if (lane >= o) inc += x;
  }
  return inc - v;
}

// ---- V0: round-1 wave_sort_regs (count atomics, scan, slot atomics, rank with 4 reads) ----
template <int NB, int E>
__device__ void sort_old(uint16_t* L, int k, float qx, float qy, float qz, const float4* cs, float bscale,
                         uint32_t* Sd, uint16_t* St, int* bcount, int* bpos, int lane) {
  for (int b = lane; b < NB; b += 64) bcount[b] = 0;
  int t[E], b[E];
  uint32_t d[E];
#pragma unroll
  for (int i = 0; i < E; ++i) t[i] = lane + 64 * i < k ? L[lane + 64 * i] : 0;
  wsync();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const float dd = d2f(qx, qy, qz, cs[t[i]]);
    d[i] = __float_as_uint(dd);
    const int bb = (int)(dd * bscale);
    b[i] = bb < NB ? bb : NB - 1;
    if (lane + 64 * i < k) atomicAdd(&bcount[b[i]], 1);
  }
  wsync();
  {
    constexpr int PER = NB / 64;
    int c[PER], sum = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bcount[lane * PER + v]; sum += c[v]; }
    int ex = excl_scan(sum, lane);
#pragma unroll
    for (int v = 0; v < PER; ++v) { bpos[lane * PER + v] = ex; ex += c[v]; }
  }
  wsync();
  int slot[E];
#pragma unroll
  for (int i = 0; i < E; ++i) slot[i] = lane + 64 * i < k ? atomicAdd(&bpos[b[i]], 1) : 0;
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (lane + 64 * i < k) { Sd[slot[i]] = d[i]; St[slot[i]] = (uint16_t)t[i]; }
  wsync();
  int st[E], en[E], rank[E];
#pragma unroll
  for (int i = 0; i < E; ++i) { en[i] = bpos[b[i]]; st[i] = en[i] - bcount[b[i]]; }
#pragma unroll
  for (int i = 0; i < E; ++i) {
    uint32_t dv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dv[j] = st[i] + j < en[i] ? Sd[st[i] + j] : 0xffffffffu;
    int r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) r += dv[j] < d[i];
    for (int v = st[i] + 4; v < en[i]; ++v) r += Sd[v] < d[i];
    rank[i] = r;
  }
  wsync();
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (lane + 64 * i < k) L[st[i] + rank[i]] = (uint16_t)t[i];
  wsync();
}

// ---- V1/V2: counting sort with arrival indices from ds_add_rtn; W = rank-window reads ----
template <int NB, int E, int W, int STOP = 9>
__device__ void sort_count(uint16_t* L, int k, float qx, float qy, float qz, const float4* cs, float bscale,
                           uint32_t* Sd, uint16_t* St, int* bcount, int* boff, int lane) {
  for (int b = lane; b < NB; b += 64) bcount[b] = 0;
  wsync();
  uint32_t d[E], tb[E];
  int s[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    const bool v = lane + 64 * i < k;
    const int t = v ? L[lane + 64 * i] : 0;
    const float dd = d2f(qx, qy, qz, cs[t]);
    int b = (int)(dd * bscale);
    b = b < NB ? b : NB - 1;
    d[i] = __float_as_uint(dd);
    tb[i] = (uint32_t)t | ((uint32_t)b << 16);
    s[i] = v ? atomicAdd(&bcount[b], 1) : 0;
  }
  wsync();
  if (STOP == 1) { if (lane == 0) L[0] = (uint16_t)(s[0] + tb[0] + d[0]); return; }
  {
    constexpr int PER = NB / 64;
    int c[PER], sum = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bcount[lane * PER + v]; sum += c[v]; }
    int ex = excl_scan(sum, lane);
#pragma unroll
    for (int v = 0; v < PER; ++v) { boff[lane * PER + v] = ex; ex += c[v]; }
  }
  wsync();
  if (STOP == 2) { if (lane == 0) L[0] = (uint16_t)(s[0] + tb[0] + d[0]); return; }
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    if (lane + 64 * i < k) {
      const int b = tb[i] >> 16;
      const int pos = boff[b] + s[i];
      Sd[pos] = d[i];
      St[pos] = (uint16_t)(tb[i] & 0xffffu);
      s[i] = pos;
    }
  }
  wsync();
  if (STOP == 3) { if (lane == 0) L[0] = (uint16_t)(s[0] + tb[0] + d[0]); return; }
  int fin[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    fin[i] = 0;
    if (lane + 64 * i < k) {
      const int b = tb[i] >> 16;
      const int st = boff[b], c = bcount[b];
      int rank = 0;
      if (W == 0) {
        if (c > 1)
          for (int v = st; v < st + c; ++v) rank += Sd[v] < d[i];
      } else {
        uint32_t dv[W > 0 ? W : 1];
#pragma unroll
        for (int j = 0; j < W; ++j) dv[j] = Sd[st + j < k ? st + j : st];
#pragma unroll
        for (int j = 0; j < W; ++j) rank += (j < c) & (dv[j] < d[i]);
        for (int v = st + W; v < st + c; ++v) rank += Sd[v] < d[i];
      }
      fin[i] = st + rank;
    }
  }
  wsync();
  if (STOP == 4) { if (lane == 0) L[0] = (uint16_t)(fin[0] + tb[0] + d[0]); return; }
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    if (lane + 64 * i < k) L[fin[i]] = (uint16_t)(tb[i] & 0xffffu);
  }
  wsync();
}

// ---- V10: counting sort, one packed (offset << 16 | count) word per bucket; singleton buckets
// place directly, only multi-element buckets are scattered and ranked (W-wide window) ----
template <int NB, int E, int MODE = 0>
__device__ void sort_pack(uint16_t* L, int k, float qx, float qy, float qz, const float4* cs, float bscale,
                          uint32_t* Sd, uint16_t* St, uint32_t* bw, int lane) {
#pragma unroll
  for (int b = lane; b < NB; b += 64) bw[b] = 0;
  wsync();
  uint32_t d[E], tb[E];
  int s[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    const bool v = lane + 64 * i < k;
    const int t = v ? L[lane + 64 * i] : 0;
    const float dd = d2f(qx, qy, qz, cs[t]);
    int b = (int)(dd * bscale);
    b = b < NB ? b : NB - 1;
    d[i] = __float_as_uint(dd);
    tb[i] = (uint32_t)t | ((uint32_t)b << 16);
    s[i] = v ? (int)atomicAdd(&bw[b], 1u) : 0;
  }
  wsync();
  {
    constexpr int PER = NB / 64;
    uint32_t c[PER];
    int sum = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bw[lane * PER + v]; sum += (int)c[v]; }
    int ex = excl_scan(sum, lane);
#pragma unroll
    for (int v = 0; v < PER; ++v) { bw[lane * PER + v] = ((uint32_t)ex << 16) | c[v]; ex += (int)c[v]; }
  }
  wsync();
  int fin[E];
  bool multi = false;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    fin[i] = -1;
    if (lane + 64 * i < k) {
      const uint32_t w = bw[tb[i] >> 16];
      const int st = (int)(w >> 16), c = (int)(w & 0xffffu);
      if (c == 1) fin[i] = st;
      else {
        Sd[st + s[i]] = d[i];
        multi = true;
        s[i] = st | (c << 16);
      }
    }
  }
  if (MODE != 2 && __builtin_amdgcn_ballot_w64(multi)) {
    wsync();
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (64 * i >= k) break;
      if (lane + 64 * i < k && fin[i] < 0) {
        const int st = s[i] & 0xffff, c = s[i] >> 16;
        uint32_t a0 = Sd[st], a1 = Sd[st + 1];
        int rank = (a0 < d[i]) + (a1 < d[i]);
        for (int v = st + 2; v < st + c; ++v) rank += Sd[v] < d[i];
        fin[i] = st + rank;
      }
    }
  }
  wsync();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    if (lane + 64 * i < k) L[MODE == 1 ? lane + 64 * i : fin[i]] = (uint16_t)(tb[i] & 0xffffu);
  }
  wsync();
}

// ---- V13/14: as V10 with no divergent branch around any LDS access: invalid slots count into
// a trash bucket, all window reads of all slots are issued before any is used ----
template <int NB, int E>
__device__ void sort_pack2(uint16_t* L, int k, float qx, float qy, float qz, const float4* cs, float bscale,
                           uint32_t* Sd, uint32_t* bw, int lane) {
#pragma unroll
  for (int b = lane; b <= NB; b += 64) bw[b] = 0;
  wsync();
  uint32_t d[E], tb[E];
  int s[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    const int e = lane + 64 * i;
    const bool v = e < k;
    const int t = L[v ? e : k - 1];
    const float dd = d2f(qx, qy, qz, cs[t]);
    int b = (int)(dd * bscale);
    b = b < NB ? b : NB - 1;
    b = v ? b : NB;  // trash bucket
    d[i] = __float_as_uint(dd);
    tb[i] = (uint32_t)t | ((uint32_t)b << 16);
    s[i] = (int)atomicAdd(&bw[b], 1u);
  }
  wsync();
  {
    constexpr int PER = NB / 64;
    uint32_t c[PER];
    int sum = 0;
#pragma unroll
    for (int v = 0; v < PER; ++v) { c[v] = bw[lane * PER + v]; sum += (int)c[v]; }
    int ex = excl_scan(sum, lane);
#pragma unroll
    for (int v = 0; v < PER; ++v) { bw[lane * PER + v] = ((uint32_t)ex << 16) | c[v]; ex += (int)c[v]; }
  }
  wsync();
  uint32_t w[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    w[i] = bw[tb[i] >> 16];
  }
  bool multi = false;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    const bool v = lane + 64 * i < k;
    const int st = (int)(w[i] >> 16), c = (int)(w[i] & 0xffffu);
    const bool m = v && c > 1;
    if (m) Sd[st + s[i]] = d[i];
    multi |= m;
    s[i] = st;
  }
  if (__builtin_amdgcn_ballot_w64(multi)) {
    wsync();
    uint32_t a0[E], a1[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (64 * i >= k) break;
      const int st = s[i] < k ? s[i] : 0;
      a0[i] = Sd[st];
      a1[i] = Sd[st + 1 < k ? st + 1 : st];
    }
    bool more = false;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (64 * i >= k) break;
      const int c = (int)(w[i] & 0xffffu);
      const int r = c > 1 ? (int)(a0[i] < d[i]) + (int)(a1[i] < d[i]) : 0;
      more |= (lane + 64 * i < k) && c > 2;
      s[i] += r;
    }
    if (__builtin_amdgcn_ballot_w64(more)) {
#pragma unroll
      for (int i = 0; i < E; ++i) {
        if (64 * i >= k) break;
        const int c = (int)(w[i] & 0xffffu), st = (int)(w[i] >> 16);
        if (lane + 64 * i < k && c > 2)
          for (int v = st + 2; v < st + c; ++v) s[i] += Sd[v] < d[i];
      }
    }
  }
  wsync();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (64 * i >= k) break;
    if (lane + 64 * i < k) L[s[i]] = (uint16_t)(tb[i] & 0xffffu);
  }
  wsync();
}

// ---- V3: bitonic sort of 64-bit keys (d2 bits, t) in registers, element e = lane * E + i ----
template <int E>
__device__ void sort_bitonic(uint16_t* L, int k, float qx, float qy, float qz, const float4* cs, int lane) {
  uint64_t key[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = lane * E + i;
    if (e < k) {
      const int t = L[e];
      key[i] = ((uint64_t)__float_as_uint(d2f(qx, qy, qz, cs[t])) << 32) | (uint32_t)t;
    } else {
      key[i] = ~0ull;
    }
  }
  constexpr int N = 64 * E;
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int j = size >> 1; j > 0; j >>= 1) {
      if (j < E) {
#pragma unroll
        for (int i = 0; i < E; ++i) {
          if (i & j) continue;
          const int e = lane * E + i;
          const bool asc = (e & size) == 0;
          const uint64_t a = key[i], b = key[i | j];
          const bool sw = asc ? (a > b) : (a < b);
          key[i] = sw ? b : a;
          key[i | j] = sw ? a : b;
        }
      } else {
        const int lm = j / E;
        const bool lower = (lane & lm) == 0;
#pragma unroll
        for (int i = 0; i < E; ++i) {
          const int e = lane * E + i;
          const bool asc = (e & size) == 0;
          const uint64_t o = __shfl_xor(key[i], lm);
          const bool takemin = asc == lower;
          key[i] = takemin ? (o < key[i] ? o : key[i]) : (o > key[i] ? o : key[i]);
        }
      }
    }
  }
  wsync();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = lane * E + i;
    if (e < k) L[e] = (uint16_t)(key[i] & 0xffffu);
  }
  wsync();
}

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float u01(uint32_t x) { return (hsh(x) >> 8) * (1.0f / 16777216.0f); }

template <int V>
__global__ void __launch_bounds__(256, 3) k_bench(const int* __restrict__ kk, int nq, int* __restrict__ next,
                                                  int* __restrict__ errs, unsigned long long* __restrict__ sink) {
  __shared__ float4 cs[TC];
  __shared__ uint16_t lists[4][LC + 2];
  __shared__ uint32_t sd[4][LC];
  __shared__ uint16_t stt[4][LC];
  __shared__ int bc[4][513], bo[4][256];
  __shared__ int bx[V == 14 ? 4 : 1][1025];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int t = tid; t < TC; t += 256) {  // candidates in a ball of radius 1 (r^2 = 1)
    float x, y, z;
    uint32_t h = blockIdx.x * 7919u + t * 104729u;
    do { x = 2 * u01(h) - 1; y = 2 * u01(h + 1) - 1; z = 2 * u01(h + 2) - 1; h += 3; } while (x * x + y * y + z * z >= 0.999f);
    cs[t] = make_float4(x, y, z, 1.0f);
  }
  __syncthreads();
  unsigned long long acc = 0;
  int bad = 0;
  const int nw = gridDim.x * 4;
  for (int q = blockIdx.x * 4 + wv; q < nq; q += nw) {  // static: a queue atomic per query would bound it
    const int k = kk[q];
    const float qx = 0.02f * (u01(q * 3u) - 0.5f), qy = 0.02f * (u01(q * 3u + 1) - 0.5f),
                qz = 0.02f * (u01(q * 3u + 2) - 0.5f);
    uint16_t* L = lists[wv];
    const uint32_t rot = hsh(q) % TC;
    for (int e = lane; e < k; e += 64) L[e] = (uint16_t)((e * 7u + rot) % TC);  // distinct candidates
    wsync();
    const float bs = (V == 1 ? 128.0f : 256.0f) / 1.25f;  // d2 < (1 + 0.02 * sqrt 3)^2 < 1.25
    if (V == 0) {
      if (k <= 128) sort_old<256, 2>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else if (k <= 256) sort_old<256, 4>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else if (k <= 512) sort_old<256, 8>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else sort_old<256, 16>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
    } else if (V == 1 || V == 2 || (V >= 6 && V <= 9)) {
      constexpr int NB = V == 1 ? 128 : 256;
      constexpr int W = V == 1 ? 0 : 4;
      constexpr int SP = V >= 6 ? V - 5 : 9;
      if (k <= 64) sort_count<NB, 1, W, SP>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else if (k <= 128) sort_count<NB, 2, W, SP>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else if (k <= 256) sort_count<NB, 4, W, SP>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else if (k <= 512) sort_count<NB, 8, W, SP>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
      else sort_count<NB, 16, W, SP>(L, k, qx, qy, qz, cs, bs, sd[wv], stt[wv], bc[wv], bo[wv], lane);
    } else if (V >= 13) {
      constexpr int NB2 = V == 13 ? 512 : 1024;
      const float b5 = NB2 / 1.25f;
      uint32_t* bw = reinterpret_cast<uint32_t*>(V == 13 ? &bc[wv][0] : &bx[wv][0]);
      if (k <= 64) sort_pack2<NB2, 1>(L, k, qx, qy, qz, cs, b5, sd[wv], bw, lane);
      else if (k <= 128) sort_pack2<NB2, 2>(L, k, qx, qy, qz, cs, b5, sd[wv], bw, lane);
      else if (k <= 256) sort_pack2<NB2, 4>(L, k, qx, qy, qz, cs, b5, sd[wv], bw, lane);
      else if (k <= 512) sort_pack2<NB2, 8>(L, k, qx, qy, qz, cs, b5, sd[wv], bw, lane);
      else sort_pack2<NB2, 16>(L, k, qx, qy, qz, cs, b5, sd[wv], bw, lane);
    } else if (V >= 10) {
      constexpr int M = V - 10;
      const float b5 = 512.0f / 1.25f;
      uint32_t* bw = reinterpret_cast<uint32_t*>(&bc[wv][0]);  // 256 ints + 256 ints of bo: 512 words
      if (k <= 64) sort_pack<512, 1, M>(L, k, qx, qy, qz, cs, b5, sd[wv], stt[wv], bw, lane);
      else if (k <= 128) sort_pack<512, 2, M>(L, k, qx, qy, qz, cs, b5, sd[wv], stt[wv], bw, lane);
      else if (k <= 256) sort_pack<512, 4, M>(L, k, qx, qy, qz, cs, b5, sd[wv], stt[wv], bw, lane);
      else if (k <= 512) sort_pack<512, 8, M>(L, k, qx, qy, qz, cs, b5, sd[wv], stt[wv], bw, lane);
      else sort_pack<512, 16, M>(L, k, qx, qy, qz, cs, b5, sd[wv], stt[wv], bw, lane);
    } else if (V == 3) {
      if (k <= 64) sort_bitonic<1>(L, k, qx, qy, qz, cs, lane);
      else if (k <= 128) sort_bitonic<2>(L, k, qx, qy, qz, cs, lane);
      else if (k <= 256) sort_bitonic<4>(L, k, qx, qy, qz, cs, lane);
      else if (k <= 512) sort_bitonic<8>(L, k, qx, qy, qz, cs, lane);
      else sort_bitonic<16>(L, k, qx, qy, qz, cs, lane);
    } else {
      // V4: no sort (harness overhead); V5: d2 + one LDS atomic per element only
      if (V == 5)
        for (int e = lane; e < k; e += 64) {
          int b = (int)(d2f(qx, qy, qz, cs[L[e]]) * bs);
          atomicAdd(&bc[wv][b < 256 ? b : 255], 1);
        }
    }
    // check: d2 non-decreasing along the list
    if ((q & 63) == 0)
      for (int e = lane; e + 1 < k; e += 64)
        bad += d2f(qx, qy, qz, cs[L[e]]) > d2f(qx, qy, qz, cs[L[e + 1]]);
    if (lane < k) acc += L[lane] * (unsigned long long)(lane + 1);
    wsync();
  }
  if (bad) atomicAdd(errs, bad);
  atomicAdd(sink, acc);
}

int main(int argc, char** argv) {
  const int nq = argc > 1 ? atoi(argv[1]) : 1000000;
  std::mt19937 rng(7);
  std::lognormal_distribution<double> ln(std::log(150.0), 0.8);
  std::vector<int> hk(nq);
  double sum = 0;
  for (int i = 0; i < nq; ++i) {
    hk[i] = std::min(1024, std::max(2, (int)ln(rng)));
    sum += hk[i];
  }
  // neighbouring queries have similar k (cell order): sort blocks of 64 queries
  for (int i = 0; i + 64 <= nq; i += 64) std::sort(hk.begin() + i, hk.begin() + i + 64);
  int *dk, *dn, *de;
  unsigned long long* ds;
  CK(hipMalloc(&dk, sizeof(int) * nq));
  CK(hipMalloc(&dn, sizeof(int)));
  CK(hipMalloc(&de, sizeof(int)));
  CK(hipMalloc(&ds, sizeof(unsigned long long)));
  CK(hipMemcpy(dk, hk.data(), sizeof(int) * nq, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("queries %d, mean k %.1f\n", nq, sum / nq);
  const char* names[] = {"old bucket (r01)", "count NB128 loop", "count NB256 win4", "bitonic regs", "no sort",
                         "d2 + atomic only", "count: phase1", "count: +scan", "count: +scatter", "count: +rank", "packed NB512", "packed, linear write", "packed, no rank", "pack2 NB512", "pack2 NB1024"};
  for (int v = 0; v < 15; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(dn, 0, sizeof(int)));
      CK(hipMemset(de, 0, sizeof(int)));
      CK(hipEventRecord(a));
      const int grid = 256 * 3 * 2;
      if (v == 0) k_bench<0><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 1) k_bench<1><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 2) k_bench<2><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 3) k_bench<3><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 4) k_bench<4><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 5) k_bench<5><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 6) k_bench<6><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 7) k_bench<7><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 8) k_bench<8><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 9) k_bench<9><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 10) k_bench<10><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 11) k_bench<11><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 12) k_bench<12><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 13) k_bench<13><<<grid, 256>>>(dk, nq, dn, de, ds);
      if (v == 14) k_bench<14><<<grid, 256>>>(dk, nq, dn, de, ds);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      int errs;
      CK(hipMemcpy(&errs, de, sizeof(int), hipMemcpyDeviceToHost));
      if (rep == 2) printf("%-20s %8.3f ms  errors %d\n", names[v], ms, errs);
    }
  }
  return 0;
}
