// Microbenchmark: HBM rates of the access patterns of the records stage on one MI355X --
// (1) a streaming read by global_load_dwordx4, (2) the same read through LDS-DMA pieces
// (global_load_lds_dwordx4, 12 KiB per wave per turn, as decode_records_kernel stages a group),
// (3) (2) plus a 1:5.4 write stream (the SoA rows: 60 B per 330-byte record).
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/hbm_rates tools/micro/hbm_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void rd_kernel(const uint4* __restrict__ a, int64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// one wave per workgroup, STAGE bytes per turn into LDS by LDS-DMA, then a light pass over it
template <int STAGE, bool WRITE>
__global__ __launch_bounds__(64) void dma_kernel(const uint8_t* __restrict__ a, int64_t nbytes, uint32_t* out,
                                                 uint32_t* __restrict__ wout) {
  __shared__ uint4 st[STAGE / 16];
  const int lane = threadIdx.x;
  uint32_t acc = 0;
  const int64_t nturn = nbytes / STAGE;
  for (int64_t t = blockIdx.x; t < nturn; t += gridDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(a + t * STAGE);
    for (int c0 = 0; c0 < STAGE / 16; c0 += 64)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + c0 + lane),
                                       (__attribute__((address_space(3))) void*)(st + c0), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const uint4 v = st[lane * (STAGE / 16 / 64)];
    acc ^= v.x ^ v.w;
    if (WRITE) {  // 60 bytes per 330: 11 fields of the 32 records of a 10.5 KB group, as 32-lane stores
      uint32_t* w = wout + t * (STAGE * 60 / 330 / 4);
      for (int k = lane; k < STAGE * 60 / 330 / 4; k += 64) w[k] = acc + k;
    }
    __syncthreads();
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int64_t nbytes = 6ll << 30;
  uint8_t* a;
  uint32_t *out, *w;
  if (hipMalloc(&a, nbytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess ||
      hipMalloc(&w, nbytes / 4) != hipSuccess)
    return 1;
  (void)hipMemset(a, 1, nbytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch, double bytes) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-48s %8.3f ms  %7.2f TB/s\n", name, best, bytes / best / 1e9);
  };
  time("read, global_load_dwordx4, 256x8192 grid", [&] {
    hipLaunchKernelGGL(rd_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)a, nbytes / 16, out);
  }, (double)nbytes);
  for (int g : {3328, 8192, 16384})
    for (int pass = 0; pass < 2; pass++) {
      char nm[96];
      snprintf(nm, sizeof nm, "LDS-DMA 12 KiB turns, %d waves%s", g, pass ? " + SoA-like writes" : "");
      const double wbytes = pass ? (double)(nbytes / 12288) * (12288 * 60 / 330 / 4) * 4 : 0;
      time(nm, [&] {
        if (pass)
          hipLaunchKernelGGL((dma_kernel<12288, true>), dim3(g), dim3(64), 0, 0, a, nbytes, out, w);
        else
          hipLaunchKernelGGL((dma_kernel<12288, false>), dim3(g), dim3(64), 0, 0, a, nbytes, out, w);
      }, (double)nbytes + wbytes);
    }
  return 0;
}
