// l2_probe.hip -- development probe: how fast can the 8 range tiles of a frame
// re-read the frame from the XCD's L2 (the single-pass kernel's read pattern)?
//
// Each workgroup = one tile of one frame (blocks 64j + 8t + x: the 8 tiles of
// frame 8j + x on XCD x), NW waves, each wave streams chirps w + NW k2 of the
// frame (8 x 16-byte loads per lane per chirp), DEPTH chirps in flight, and
// sums what it loads; WORK extra packed FMAs per chirp stand in for the
// range-FFT arithmetic.  Optional stagger: tile t starts STAG*t chirps later
// (mod C).  Prints the L2->CU read rate (8 reads per frame) and the frame rate.
//
//   hipcc --offload-arch=gfx950 -O3 tools/l2_probe.hip -o tools/l2_probe.bin && tools/l2_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int NW, int DEPTH, int LDSKB, int WORK>
__global__ __launch_bounds__(64 * NW, 1) void k_read(const f4v* __restrict__ iq, int F, int C, int stag, float* out) {
  __shared__ float pad[LDSKB * 256];             // occupancy as the real kernel (1 workgroup per CU)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.x;
  const long f = (long)(b >> 6) * 8 + (b & 7);
  const int t = (b >> 3) & 7;
  if (f >= F) return;
  constexpr int cpw = 256 / NW;                  // C = 256
  const f4v* fr = iq + f * (long)C * 512;
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  f4v buf[DEPTH][8];
  auto ld = [&](int i, f4v (&x)[8]) {
    const int k = (w + NW * ((i + stag * t) % cpw)) % C;
    const f4v* q = fr + (long)k * 512;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = q[lane + 64 * j];
  };
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i) ld(i, buf[i]);
#pragma unroll
  for (int i = 0; i < cpw; ++i) {
    if (i + DEPTH - 1 < cpw) ld(i + DEPTH - 1, buf[(i + DEPTH - 1) % DEPTH]);
    f4v s = buf[i % DEPTH][0];
#pragma unroll
    for (int j = 1; j < 8; ++j) s += buf[i % DEPTH][j];
    // WORK packed FMAs per chirp in 4 independent chains (2 per f4v op)
    f4v u0 = s, u1 = s * 1.5f;
#pragma unroll
    for (int q = 0; q < WORK / 4; ++q) {
      u0 = u0 * 0.999f + 0.5f;
      u1 = u1 * 0.998f + 0.25f;
    }
    acc += u0 + u1;
  }
  if (acc.x == 1234.5f) { pad[threadIdx.x] = acc.y; out[b] = pad[(threadIdx.x + 1) % 64]; }
}

template <int NW, int DEPTH, int LDSKB, int WORK>
void run(const char* name, const f4v* d, int F, int C, int stag, float* o) {
  const int blocks = ((F + 7) / 8) * 64;
  hipEvent_t a, e;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&e);
  k_read<NW, DEPTH, LDSKB, WORK><<<blocks, 64 * NW>>>(d, F, C, stag, o);
  (void)hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_read<NW, DEPTH, LDSKB, WORK><<<blocks, 64 * NW>>>(d, F, C, stag, o);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, e);
  ms /= reps;
  const double bytes = (double)F * C * 8192.0;
  printf("%-28s stag %d: %.3f ms  L2->CU %.1f TB/s  frames %.3f M/s (HBM-once %.2f TB/s)\n", name, stag, ms,
         8 * bytes / ms / 1e9, F / ms / 1e3, bytes / ms / 1e9);
}

__global__ void k_fill(f4v* d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = f4v{(float)(i & 1023), 1.f, -0.5f, (float)(i >> 20)};
}

int main() {
  const int F = 4096, C = 256;
  f4v* d;
  float* o;
  (void)hipMalloc(&d, (size_t)F * C * 8192);
  (void)hipMalloc(&o, 1 << 20);
  k_fill<<<4096, 256>>>(d, (size_t)F * C * 512);
  run<8, 3, 128, 0>("nw8 depth3", d, F, C, 0, o);
  run<8, 3, 128, 64>("nw8 depth3 work64", d, F, C, 0, o);
  run<8, 3, 128, 160>("nw8 depth3 work160", d, F, C, 0, o);
  run<8, 3, 128, 320>("nw8 depth3 work320", d, F, C, 0, o);
  run<8, 3, 128, 0>("nw8 depth3 F=32", d, 32, C, 0, o);
  run<8, 3, 128, 160>("nw8 depth3 work160 F=32", d, 32, C, 0, o);
  run<8, 3, 128, 0>("nw8 depth3 stag1", d, F, C, 1, o);
  run<8, 3, 60, 0>("nw8 depth3 2 WG/CU", d, F, C, 0, o);
  return 0;
}
