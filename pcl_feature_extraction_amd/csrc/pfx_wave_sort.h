// pfx_wave_sort.h -- one wavefront sorts up to kWaveSortCap 64-bit keys held in its own LDS
// region (ascending; keys distinct).  k <= 64: rank sort (one key per lane); else bitonic over
// the next power of two, padded with ~0.  Every lane of the wave calls it with the same k.
#pragma once
#include <cstdint>

namespace pfx {

constexpr int kWaveSortCap = 512;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ inline void wave_sort_keys(uint64_t* key, int k, int lane) {
  wave_lds_sync();
  if (k <= 64) {
    const uint64_t mine = lane < k ? key[lane] : ~0ull;
    int rank = 0;
    for (int m = 0; m < k; ++m) rank += key[m] < mine ? 1 : 0;
    wave_lds_sync();
    if (lane < k) key[rank] = mine;
    wave_lds_sync();
    return;
  }
  int P = 64;
  while (P < k) P <<= 1;
  for (int m = k + lane; m < P; m += 64) key[m] = ~0ull;
  wave_lds_sync();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int c = lane; c < (P >> 1); c += 64) {
        const int a = 2 * stride * (c / stride) + (c % stride), b = a + stride;
        const uint64_t ka = key[a], kb = key[b];
        if ((ka > kb) == ((a & size) == 0)) {
          key[a] = kb;
          key[b] = ka;
        }
      }
      wave_lds_sync();
    }
  }
}

}  // namespace pfx
