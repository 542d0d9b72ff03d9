// mall_chain.hip -- development probe for the two-pass schedule: can a small
// ring of intermediate buffers (the range cube of a chunk of frames) live in
// the 256 MiB Infinity Cache, so that HBM only sees the input reads and the
// output writes?
//
//   direct : copy X -> Y                                   (16 GiB of HBM traffic)
//   chain  : copy X_i -> R[i % S], then R[i % S] -> Y_i    (two streams, S ring slots)
//
// If the ring stays on die, `chain` approaches `direct`; if not, it takes ~2x.
// Build: hipcc --offload-arch=gfx950 -O3 -o mall_chain mall_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t ck_e = (x); if (ck_e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(ck_e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t s = (size_t)gridDim.x * blockDim.x;
  // 4 loads in flight per lane
  for (; i + 3 * s < n; i += 4 * s) {
    const float4 v0 = a[i], v1 = a[i + s], v2 = a[i + 2 * s], v3 = a[i + 3 * s];
    b[i] = v0; b[i + s] = v1; b[i + 2 * s] = v2; b[i + 3 * s] = v3;
  }
  for (; i < n; i += s) b[i] = a[i];
}

int main(int argc, char** argv) {
  const size_t frame = 2ull << 20;            // one config-3 frame (2 MiB)
  const int F = 4096;
  const size_t big = frame * F;               // 8 GiB
  float4 *X, *Y, *R;
  CK(hipMalloc(&X, big));
  CK(hipMalloc(&Y, big));
  CK(hipMalloc(&R, 1ull << 30));
  CK(hipMemset(X, 0x3c, big));
  CK(hipMemset(Y, 0, big));
  CK(hipMemset(R, 0, 1ull << 30));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int grid_cap = 256 * 8;
  auto launch = [&](const float4* a, float4* b, size_t bytes, hipStream_t s) {
    const size_t n = bytes / 16;
    size_t g = (n + 256 * 4 - 1) / (256 * 4);
    if (g > (size_t)grid_cap) g = grid_cap;
    hipLaunchKernelGGL(k_copy, dim3((unsigned)g), dim3(256), 0, s, a, b, n);
  };
  float ms;
  // direct copy, whole 8 GiB, and in chunks
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(t0, s1));
    launch(X, Y, big, s1);
    CK(hipEventRecord(t1, s1));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    if (rep) printf("direct  8 GiB one launch        : %7.3f ms  %6.1f GB/s (rd+wr)\n", ms, 2.0 * big / ms / 1e6);
  }
  for (int c : {8, 16, 32, 64}) {
    const size_t cb = frame * c;
    CK(hipEventRecord(t0, s1));
    for (int i = 0; i < F / c; ++i) launch(X + i * cb / 16, Y + i * cb / 16, cb, s1);
    CK(hipEventRecord(t1, s1));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("direct  chunks of %3d frames     : %7.3f ms  %6.1f GB/s (rd+wr)\n", c, ms, 2.0 * big / ms / 1e6);
  }
  // chain through a ring
  std::vector<hipEvent_t> e1(4096), e2(4096);
  for (auto& e : e1) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : e2) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int c : {4, 8, 16, 32, 64, 128}) {
    for (int S : {2, 3, 4}) {
      const size_t cb = frame * c;
      if (cb * S > (1ull << 30)) continue;
      const int n = F / c;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(t0, s1));
        CK(hipStreamWaitEvent(s2, t0, 0));
        for (int i = 0; i < n; ++i) {
          if (i >= S) CK(hipStreamWaitEvent(s1, e2[i - S], 0));
          launch(X + i * cb / 16, R + (i % S) * cb / 16, cb, s1);
          CK(hipEventRecord(e1[i], s1));
          CK(hipStreamWaitEvent(s2, e1[i], 0));
          launch(R + (i % S) * cb / 16, Y + i * cb / 16, cb, s2);
          CK(hipEventRecord(e2[i], s2));
        }
        CK(hipStreamWaitEvent(s1, e2[n - 1], 0));
        CK(hipEventRecord(t1, s1));
        CK(hipEventSynchronize(t1));
        CK(hipEventElapsedTime(&ms, t0, t1));
      }
      printf("chain   chunk %3d frames, ring %d (%5zu MiB): %7.3f ms  %6.1f GB/s of X+Y traffic\n", c, S,
             cb * S >> 20, ms, 2.0 * big / ms / 1e6);
    }
  }
  // sequential chain on one stream (no overlap)
  for (int c : {16, 64}) {
    const size_t cb = frame * c;
    const int n = F / c;
    CK(hipEventRecord(t0, s1));
    for (int i = 0; i < n; ++i) {
      launch(X + i * cb / 16, R + (i % 2) * cb / 16, cb, s1);
      launch(R + (i % 2) * cb / 16, Y + i * cb / 16, cb, s1);
    }
    CK(hipEventRecord(t1, s1));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("serial  chunk %3d frames, one stream         : %7.3f ms  %6.1f GB/s of X+Y traffic\n", c, ms,
           2.0 * big / ms / 1e6);
  }
  return 0;
}
