// Microbenchmark: issue cost (cycles per wave64 instruction, per SIMD) of the integer VALU
// instructions the record hash (splitmix64 finalizer per 8-byte word) is made of, with 1 and 4
// waves per SIMD and 8 independent chains per lane (no dependency stalls).
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/valu_rates tools/micro/valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITER = 512;

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t a[8];
  uint64_t w[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    a[j] = seed + threadIdx.x * 8 + j;
    w[j] = ((uint64_t)a[j] << 32) | (a[j] * 3u);
  }
  const uint32_t b = seed | 1u;
  __syncthreads();
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 3) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[j]), "=s"(c) : "v"(a[j]), "v"(b));
      }
      if (OP == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 5) asm volatile("v_lshrrev_b64 %0, 27, %0" : "+v"(w[j]));
      if (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 27" : "+v"(a[j]) : "v"(b));
      if (OP == 7) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
    }
  }
  const unsigned long long t1 = clock64();
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += a[j] + (uint32_t)w[j] + (uint32_t)(w[j] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
double run(int wg_per_cu, uint32_t* out, unsigned long long* cyc) {
  const int nwg = 256 * wg_per_cu;  // 256 threads = one wave per SIMD per workgroup
  hipLaunchKernelGGL(k<OP>, dim3(nwg), dim3(256), 0, 0, out, cyc, 7u);
  hipDeviceSynchronize();
  static unsigned long long h[256 * 8 * 4];
  hipMemcpy(h, cyc, sizeof(unsigned long long) * nwg * 4, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < nwg * 4; i++) s += (double)h[i];
  return s / (nwg * 4) / (ITER * 8.0);  // cycles per instruction per wave
}

int main() {
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(uint32_t) * 256 * 256 * 8);
  hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8 * 4);
  const char* names[8] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
                          "v_mul_u32_u24", "v_lshrrev_b64", "v_alignbit_b32", "v_xor_b32"};
  for (int wpc : {1, 4}) {
    double r[8];
    r[0] = run<0>(wpc, out, cyc); r[1] = run<1>(wpc, out, cyc); r[2] = run<2>(wpc, out, cyc);
    r[3] = run<3>(wpc, out, cyc); r[4] = run<4>(wpc, out, cyc); r[5] = run<5>(wpc, out, cyc);
    r[6] = run<6>(wpc, out, cyc); r[7] = run<7>(wpc, out, cyc);
    for (int i = 0; i < 8; i++)  // a wave's elapsed cycles per instruction; x waves/SIMD = SIMD issue cost
      printf("waves/SIMD %d  %-15s %6.2f cyc per instruction per wave  (SIMD: %5.2f)\n", wpc, names[i],
             r[i], r[i] / wpc);
  }
  return 0;
}
