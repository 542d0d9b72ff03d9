// xlane_probe.hip -- development probe: issue cost of the cross-lane moves the
// single-pass FFT uses (DPP movs, v_permlane16/32_swap) against plain packed
// FMAs, at 2 waves per SIMD (8 waves per workgroup, 1 workgroup per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/xlane_probe.hip -o tools/xlane_probe.bin && tools/xlane_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2v __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(512, 1) void k_op(float* out, int iters) {
  __shared__ float pad[128 * 256];
  float a = threadIdx.x * 0.001f, b = a + 1.f, c = a + 2.f, d = a + 3.f;
  f2v p = {a, b}, q = {c, d}, r = {b, c}, s = {d, a};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (KIND == 0) {          // 4 independent v_pk_fma_f32
        p = p * 0.999f + q; q = q * 0.998f + r; r = r * 0.997f + s; s = s * 0.996f + p;
      } else if constexpr (KIND == 1) {   // 4 independent fused DPP adds (row_ror 8)
        a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x128, 0xF, 0xF, true));
        b += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b), 0x128, 0xF, 0xF, true));
        c += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c), 0x128, 0xF, 0xF, true));
        d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x128, 0xF, 0xF, true));
      } else if constexpr (KIND == 2) {   // 4 independent v_permlane32_swap (+ add to consume)
        auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
        auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(d), false, false);
        a = __uint_as_float(x[0]); b = __uint_as_float(x[1]); c = __uint_as_float(y[0]); d = __uint_as_float(y[1]);
        a += 1.f; c += 1.f;
      } else if constexpr (KIND == 3) {   // 4 independent v_permlane16_swap (+ add)
        auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
        auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(c), __float_as_uint(d), false, false);
        a = __uint_as_float(x[0]); b = __uint_as_float(x[1]); c = __uint_as_float(y[0]); d = __uint_as_float(y[1]);
        a += 1.f; c += 1.f;
      } else if constexpr (KIND == 4) {   // 4 independent v_add_f32
        a = a + 1.001f; b = b + 1.002f; c = c + 1.003f; d = d + 1.004f;
      } else {                            // 4 DPP movs + 2 pk_fma (an FFT exchange+butterfly pair)
        const float o0 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(p.x), 0x4E, 0xF, 0xF, true));
        const float o1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(p.y), 0x4E, 0xF, 0xF, true));
        const float o2 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q.x), 0x4E, 0xF, 0xF, true));
        const float o3 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q.y), 0x4E, 0xF, 0xF, true));
        p = __builtin_elementwise_fma(r, p, f2v{o0, o1});
        q = __builtin_elementwise_fma(s, q, f2v{o2, o3});
      }
    }
  }
  const float v = a + b + c + d + p.x + p.y + q.x + q.y + r.x + s.y;
  if (v == 1234.5f) { pad[threadIdx.x] = v; out[blockIdx.x] = pad[(threadIdx.x + 1) & 511]; }
}

template <int KIND>
void run(const char* name, float* o, int ops_per_unroll) {
  const int iters = 2000, blocks = 256;
  hipEvent_t a, e;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&e);
  k_op<KIND><<<blocks, 512>>>(o, iters);
  (void)hipEventRecord(a);
  k_op<KIND><<<blocks, 512>>>(o, iters);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, e);
  // per SIMD: 2 waves x iters x 16 x ops instructions
  const double instr = 2.0 * iters * 16 * ops_per_unroll;
  printf("%-34s %.3f ms  %.2f ns per wave-instruction per SIMD (%.2f cyc at 2.4 GHz)\n", name, ms,
         ms * 1e6 / instr, ms * 1e6 / instr * 2.4);
}

int main() {
  float* o;
  (void)hipMalloc(&o, 1 << 20);
  run<4>("v_add_f32 x4", o, 4);
  run<0>("v_pk_fma_f32 x4", o, 4);
  run<1>("v_add_f32_dpp x4", o, 4);
  run<2>("v_permlane32_swap x2 + 2 add", o, 4);
  run<3>("v_permlane16_swap x2 + 2 add", o, 4);
  run<5>("4 dpp mov + 2 pk_fma", o, 6);
  return 0;
}
