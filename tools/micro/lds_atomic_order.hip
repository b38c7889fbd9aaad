// Microbenchmark (dev tool): do the lanes of one ds_add_rtn_u32 that hit the same LDS address get
// their return values in lane order?  Random bucket patterns (few buckets: many lanes per
// address), many trials; counts order violations.  Also the cycles of one dependent atomic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k(uint32_t* bad, uint64_t* cyc, int trials, int nb) {
  __shared__ uint32_t cur[4][64];
  __shared__ uint32_t got[4][64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t nbad = 0;
  uint64_t c0 = 0, c1 = 0;
  for (int i = 0; i < trials; i++) {
    if (lane < 64) cur[wv][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t x = (uint32_t)(i * 2654435761u) ^ (uint32_t)(blockIdx.x * 40503u) ^ (uint32_t)(lane * 2246822519u);
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    const int h = (int)(x % (uint32_t)nb);
    c0 = __builtin_amdgcn_s_memtime();
    const uint32_t r = atomicAdd(&cur[wv][h], 1u);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    c1 = __builtin_amdgcn_s_memtime();
    got[wv][lane] = r;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // lane order: every lower lane with the same bucket got a smaller value
    for (int l = 0; l < lane; l++) {
      const uint32_t y0 = (uint32_t)(i * 2654435761u) ^ (uint32_t)(blockIdx.x * 40503u) ^ (uint32_t)(l * 2246822519u);
      uint32_t y = y0 ^ (y0 >> 13);
      y *= 0x5bd1e995u;
      y ^= y >> 15;
      if ((int)(y % (uint32_t)nb) == h && got[wv][l] > r) nbad++;
    }
    __builtin_amdgcn_wave_barrier();
  }
  atomicAdd(bad, nbad);
  if (t == 0 && blockIdx.x == 0) cyc[0] = c1 - c0;
}

int main() {
  uint32_t* bad;
  uint64_t* cyc;
  hipMalloc(&bad, 4);
  hipMalloc(&cyc, 8);
  for (int nb : {1, 2, 4, 16, 64}) {
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, bad, cyc, 64, nb);
    hipDeviceSynchronize();
    uint32_t h;
    uint64_t c;
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("buckets %2d: %u lane-order violations in %d atomics (2048 x 4 waves x 64 trials x 64 lanes); one atomic %llu cycles\n",
           nb, h, 2048 * 4 * 64 * 64, (unsigned long long)c);
  }
  return 0;
}
