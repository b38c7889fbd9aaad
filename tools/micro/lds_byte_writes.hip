// Microbenchmark (dev tool): LDS cost of 64 lanes writing 64 consecutive bytes with ds_write_b8
// (four lanes per dword) against 16 lanes writing the same 64 bytes as dwords, and of 64 lanes
// reading consecutive bytes (ds_read_u8).  Cycles per instruction by s_memtime over a loop with
// a dependency through LDS; run under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(256) void k(uint64_t* out, int iters) {
  __shared__ uint8_t buf[16384];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint8_t* b = buf + wv * 4096;
  uint32_t acc = t;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    const int base = (i * 64) & 4032;
    if (MODE == 0) {  // 64 byte writes, 4 lanes per dword
      b[base + lane] = (uint8_t)acc;
    } else if (MODE == 1) {  // 16 dword writes
      if ((lane & 3) == 0) *reinterpret_cast<uint32_t*>(b + base + lane) = acc;
    } else if (MODE == 2) {  // 64 u16 writes, 2 lanes per dword (the resolve's next pointers)
      reinterpret_cast<uint16_t*>(b)[(base >> 1) + lane] = (uint16_t)acc;
    } else {  // 64 byte reads of consecutive bytes
      acc += b[base + lane];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): each op completes before the next
    acc ^= i;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[0] = t1 - t0;
  if (acc == 0xdeadbeef) out[1] = acc;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 16);
  const int iters = 4096;
  const char* nm[4] = {"ds_write_b8 x64 (4 lanes/dword)", "ds_write_b32 x16", "ds_write_b16 x64 (2 lanes/dword)", "ds_read_u8 x64"};
  for (int m = 0; m < 4; m++) {
    for (int rep = 0; rep < 2; rep++) {
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1024), dim3(256), 0, 0, d, iters);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1024), dim3(256), 0, 0, d, iters);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1024), dim3(256), 0, 0, d, iters);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(1024), dim3(256), 0, 0, d, iters);
      hipDeviceSynchronize();
    }
    uint64_t h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("%-36s %.1f cycles per op (one wave's dependent chain, 4 waves per CU-SIMD set)\n", nm[m], (double)h[0] / iters);
  }
  return 0;
}
