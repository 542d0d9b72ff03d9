// mall_probe.hip -- development probe: does the 256 MiB Infinity Cache (MALL)
// serve a buffer that was just written by another kernel?  Measures
//   (1) plain streaming copy bandwidth (HBM roof as achieved by a trivial kernel)
//   (2) read bandwidth of a B-byte buffer right after a kernel wrote it (hot)
//   (3) the same read after 1 GiB of unrelated streaming traffic (cold)
// Build: hipcc --offload-arch=gfx950 -O3 -o mall_probe mall_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}
__global__ void k_write(float4* __restrict__ b, size_t n, float v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = make_float4(v, v + 1, v + 2, v + 3);
}
__global__ void k_read(const float4* __restrict__ a, size_t n, float* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (; i < n; i += s) { float4 v = a[i]; acc += v.x + v.y + v.z + v.w; }
  if (acc == 1234.5f) *out = acc;
}

int main() {
  const size_t big = 4ull << 30;   // 4 GiB
  float4 *a, *b, *c;
  float* o;
  CK(hipMalloc(&a, big)); CK(hipMalloc(&b, big)); CK(hipMalloc(&c, 1ull << 30)); CK(hipMalloc(&o, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grid = 256 * 16, blk = 256;
  float ms;
  // (1) copy
  size_t n = big / 16;
  hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("copy 4 GiB -> 4 GiB: %.1f GB/s (read+write)\n", 5 * 2.0 * big / (ms * 1e-3) / 1e9);
  // write-only and read-only streaming
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_write, grid, blk, 0, 0, b, n, 1.f);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("write 4 GiB: %.1f GB/s\n", 5.0 * big / (ms * 1e-3) / 1e9);
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, n, o);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("read 4 GiB: %.1f GB/s\n", 5.0 * big / (ms * 1e-3) / 1e9);
  // (2)/(3) hot vs cold re-read of B bytes
  for (size_t mb : {8, 16, 32, 64, 96, 128, 192, 256, 384, 512, 1024}) {
    const size_t B = mb << 20, m = B / 16;
    float hot = 0, cold = 0, wr = 0;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_write, grid, blk, 0, 0, b, m, (float)r);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) wr += ms;
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_read, grid, blk, 0, 0, b, m, o);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) hot += ms;
      hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, (size_t)(1ull << 30) / 16, o);   // 1 GiB of other traffic
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_read, grid, blk, 0, 0, b, m, o);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) cold += ms;
    }
    printf("B=%5zu MiB  write %.1f GB/s  read-after-write %.1f GB/s  read-after-1GiB-other %.1f GB/s\n", mb,
           5.0 * B / (wr / 1e3) / 1e9, 5.0 * B / (hot / 1e3) / 1e9, 5.0 * B / (cold / 1e3) / 1e9);
  }
  return 0;
}
