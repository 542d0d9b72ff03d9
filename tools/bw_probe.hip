// bw_probe.hip -- development probe: HBM streaming ceilings on MI355X for the
// access shapes the FMCW kernels use.  Each "chirp" is a 1024-element row of
// complex float (8 KB); a wave owns one row, lane t touches t + 64*m.
//   copy8   : 16 x 8-byte loads per lane, then 16 x 8-byte stores (K1 shape)
//   copy16  : 8 x 16-byte loads per lane, then 8 x 16-byte stores
//   copy8nt : copy8 with nontemporal stores
//   rows/wave: each wave walks `cpw` rows (persistent-ish) vs one row per wave
// Build: hipcc --offload-arch=gfx950 -O3 -o bw_probe bw_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int NT>
__global__ __launch_bounds__(256) void k_copy8(const float2* __restrict__ a, float2* __restrict__ b, long rows, int cpw) {
  const int lane = threadIdx.x & 63;
  const long w0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * cpw;
  for (int c = 0; c < cpw; ++c) {
    const long r = w0 + c;
    if (r >= rows) return;
    const float2* s = a + r * 1024;
    float2* d = b + r * 1024;
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = s[lane + 64 * m];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (NT) __builtin_nontemporal_store(v[m].x, &d[lane + 64 * m].x), __builtin_nontemporal_store(v[m].y, &d[lane + 64 * m].y);
      else d[lane + 64 * m] = v[m];
    }
  }
}

__global__ __launch_bounds__(256) void k_copy16(const float4* __restrict__ a, float4* __restrict__ b, long rows, int cpw) {
  const int lane = threadIdx.x & 63;
  const long w0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * cpw;
  for (int c = 0; c < cpw; ++c) {
    const long r = w0 + c;
    if (r >= rows) return;
    const float4* s = a + r * 512;
    float4* d = b + r * 512;
    float4 v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = s[lane + 64 * m];
#pragma unroll
    for (int m = 0; m < 8; ++m) d[lane + 64 * m] = v[m];
  }
}

// software-pipelined copy8: loads of row c+1 issued before the stores of row c
__global__ __launch_bounds__(256) void k_copy8_pf(const float2* __restrict__ a, float2* __restrict__ b, long rows, int cpw) {
  const int lane = threadIdx.x & 63;
  const long w0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * cpw;
  if (w0 >= rows) return;
  float2 cur[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) cur[m] = a[w0 * 1024 + lane + 64 * m];
  for (int c = 0; c < cpw; ++c) {
    const long r = w0 + c;
    if (r >= rows) return;
    const long rn = (c + 1 < cpw && r + 1 < rows) ? r + 1 : r;
    float2 nxt[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) nxt[m] = a[rn * 1024 + lane + 64 * m];
#pragma unroll
    for (int m = 0; m < 16; ++m) b[r * 1024 + lane + 64 * m] = cur[m];
#pragma unroll
    for (int m = 0; m < 16; ++m) cur[m] = nxt[m];
  }
}

int main() {
  const long rows = 262144;                      // 2 GiB per buffer
  const size_t bytes = (size_t)rows * 1024 * 8;
  float2 *a, *b;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %7.1f GB/s (read+write)\n", name, 5 * 2.0 * bytes / (ms * 1e-3) / 1e9);
    return 0;
  };
  for (int cpw : {1, 2, 4, 8, 16}) {
    const unsigned grid = (unsigned)((rows + 4L * cpw - 1) / (4L * cpw));
    char nm[64];
    snprintf(nm, 64, "copy8   rows/wave=%d", cpw);
    if (run(nm, [&] { hipLaunchKernelGGL(k_copy8<0>, grid, 256, 0, 0, a, b, rows, cpw); })) return 1;
    snprintf(nm, 64, "copy8nt rows/wave=%d", cpw);
    if (run(nm, [&] { hipLaunchKernelGGL(k_copy8<1>, grid, 256, 0, 0, a, b, rows, cpw); })) return 1;
    snprintf(nm, 64, "copy16  rows/wave=%d", cpw);
    if (run(nm, [&] { hipLaunchKernelGGL(k_copy16, grid, 256, 0, 0, (const float4*)a, (float4*)b, rows, cpw); })) return 1;
    snprintf(nm, 64, "copy8pf rows/wave=%d", cpw);
    if (run(nm, [&] { hipLaunchKernelGGL(k_copy8_pf, grid, 256, 0, 0, a, b, rows, cpw); })) return 1;
  }
  return 0;
}
