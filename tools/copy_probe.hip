// copy_probe.hip -- development probe: the HBM copy floor for k_rdx's bytes
// (4096 config-3 frames: 8.59 GB of IQ read, 8.59 GB of RD written).
//
// Variants: (a) grid-stride, one 16-byte load per thread in flight (the old
// tools/xcd_probe k_copy); (b) U 16-byte loads per thread issued before their
// U stores, grid of G blocks x 256 threads, plain or nontemporal; (c) a
// persistent 256 x 512 grid shaped like k_rdx (one workgroup per CU, every
// wave moving 8 KiB chunks = 8 loads per lane) with D chunks in flight per
// wave (register double buffer).
//
//   hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o tools/copy_probe.bin && tools/copy_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

__global__ __launch_bounds__(256) void k_copy1(const f4v* __restrict__ a, f4v* __restrict__ o, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), o + i);
}

// U loads in flight per thread; consecutive threads take consecutive 16-byte words
template <int U, int NT>
__global__ __launch_bounds__(256) void k_copyU(const f4v* __restrict__ a, f4v* __restrict__ o, long n) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = blockIdx.x * 256L * U + threadIdx.x; base < n; base += stride) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n) v[u] = NT & 1 ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n) {
        if (NT & 2) __builtin_nontemporal_store(v[u], o + i);
        else o[i] = v[u];
      }
    }
  }
}

// persistent, k_rdx-shaped: 8 waves per CU, each wave moves 8 KiB chunks (8 x 16 B per lane);
// chunk c of wave (b, w) is chunk index ((c * 256 + b) * 8 + w); D chunks loaded ahead
template <int D, int NT>
__global__ __launch_bounds__(512, 1) void k_copyP(const f4v* __restrict__ a, f4v* __restrict__ o, long nchunks) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long per = (long)gridDim.x * 8;
  const long first = (long)blockIdx.x * 8 + w;
  f4v v[D][8];
  long c = first;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const long cc = c + d * per;
    if (cc < nchunks)
#pragma unroll
      for (int i = 0; i < 8; ++i) v[d][i] = NT & 1 ? __builtin_nontemporal_load(a + cc * 512 + lane + 64 * i) : a[cc * 512 + lane + 64 * i];
  }
  for (; c < nchunks; c += D * per) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const long cc = c + d * per;
      if (cc < nchunks) {
        f4v t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = v[d][i];
        const long nx = cc + D * per;
        if (nx < nchunks)
#pragma unroll
          for (int i = 0; i < 8; ++i) v[d][i] = NT & 1 ? __builtin_nontemporal_load(a + nx * 512 + lane + 64 * i) : a[nx * 512 + lane + 64 * i];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (NT & 2) __builtin_nontemporal_store(t[i], o + cc * 512 + lane + 64 * i);
          else o[cc * 512 + lane + 64 * i] = t[i];
        }
      }
    }
  }
}

template <typename L>
float timeit(L launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) { best = ms < best ? ms : best; sum += ms; }
  }
  return best;
}

int main() {
  const int F = 4096;
  const long nin = (long)F * 256 * 1024 / 2;      // f4v per direction (8.59 GB)
  f4v *a, *o;
  CK(hipMalloc(&a, nin * 16));
  CK(hipMalloc(&o, nin * 16));
  CK(hipMemset(a, 0, nin * 16));
  CK(hipMemset(o, 0, nin * 16));
  const double gb = (double)F * 4198400 / 1e9;    // k_rdx algorithmic bytes per 4096 frames
  auto rep = [&](const char* name, float ms) {
    printf("%-34s %.3f ms  %.2f TB/s (in+out)  frac %.3f of 8 TB/s (k_rdx bytes)\n", name, ms, 2.0 * nin * 16 / ms / 1e9,
           gb / ms / 8.0);
  };
  rep("grid-stride x1 nt (4096 blk)", timeit([&] { hipLaunchKernelGGL(k_copy1, dim3(4096), dim3(256), 0, 0, a, o, nin); }));
  for (int G : {2048, 8192, 65536}) {
    char nm[64];
    snprintf(nm, 64, "U4 plain G%d", G);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copyU<4, 0>), dim3(G), dim3(256), 0, 0, a, o, nin); }));
    snprintf(nm, 64, "U4 nt G%d", G);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copyU<4, 3>), dim3(G), dim3(256), 0, 0, a, o, nin); }));
    snprintf(nm, 64, "U8 nt G%d", G);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copyU<8, 3>), dim3(G), dim3(256), 0, 0, a, o, nin); }));
    snprintf(nm, 64, "U8 ntload G%d", G);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copyU<8, 1>), dim3(G), dim3(256), 0, 0, a, o, nin); }));
    snprintf(nm, 64, "U2 nt G%d", G);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copyU<2, 3>), dim3(G), dim3(256), 0, 0, a, o, nin); }));
  }
  const long nch = nin / 512;
  rep("persistent 256x512 D1 nt", timeit([&] { hipLaunchKernelGGL((k_copyP<1, 3>), dim3(256), dim3(512), 0, 0, a, o, nch); }));
  rep("persistent 256x512 D2 nt", timeit([&] { hipLaunchKernelGGL((k_copyP<2, 3>), dim3(256), dim3(512), 0, 0, a, o, nch); }));
  rep("persistent 256x512 D2 plain", timeit([&] { hipLaunchKernelGGL((k_copyP<2, 0>), dim3(256), dim3(512), 0, 0, a, o, nch); }));
  rep("persistent 256x512 D3 nt", timeit([&] { hipLaunchKernelGGL((k_copyP<3, 3>), dim3(256), dim3(512), 0, 0, a, o, nch); }));
  rep("persistent 256x512 D2 ntload", timeit([&] { hipLaunchKernelGGL((k_copyP<2, 1>), dim3(256), dim3(512), 0, 0, a, o, nch); }));
  rep("persistent 512x512 D1 nt", timeit([&] { hipLaunchKernelGGL((k_copyP<1, 3>), dim3(512), dim3(512), 0, 0, a, o, nch); }));
  return 0;
}
