// xchg_probe.hip -- checks the lane-exchange primitives k_rd1p relies on
// (DPP quad_perm / row_ror / mirrors, v_permlane16/32_swap) on the device.
// Prints OK or the first mismatching lane; exit status 0 only when all hold.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL> __device__ int dpp(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }

__global__ void probe(int* out) {
  const int l = threadIdx.x;
  out[0 * 64 + l] = dpp<0xB1>(l);      // expect l ^ 1
  out[1 * 64 + l] = dpp<0x4E>(l);      // expect l ^ 2
  out[2 * 64 + l] = dpp<0x128>(l);     // expect l ^ 8
  out[3 * 64 + l] = dpp<0x12C>(l);     // expect row base + ((l + 4) & 15)
  out[4 * 64 + l] = dpp<0x124>(l);     // expect row base + ((l - 4) & 15)
  out[5 * 64 + l] = dpp<0x141>(l);     // expect 8-group base + 7 - (l & 7)
  out[6 * 64 + l] = dpp<0x140>(l);     // expect row base + 15 - (l & 15)
  auto r32 = __builtin_amdgcn_permlane32_swap((unsigned)l, (unsigned)l, false, false);
  out[7 * 64 + l] = (int)r32[0];       // expect l & 31          (lo half value)
  out[8 * 64 + l] = (int)r32[1];       // expect (l & 31) + 32   (hi half value)
  auto r16 = __builtin_amdgcn_permlane16_swap((unsigned)l, (unsigned)l, false, false);
  out[9 * 64 + l] = (int)r16[0];       // expect l & ~16
  out[10 * 64 + l] = (int)r16[1];      // expect l | 16
}

int main() {
  int* d;
  int h[11 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* name[11] = {"xor1", "xor2", "ror8", "ror12", "ror4", "half_mirror", "mirror", "p32_lo", "p32_hi",
                          "p16_lo", "p16_hi"};
  int bad = 0;
  for (int k = 0; k < 11; ++k)
    for (int l = 0; l < 64; ++l) {
      const int rb = l & ~15;
      int e = 0;
      switch (k) {
        case 0: e = l ^ 1; break;
        case 1: e = l ^ 2; break;
        case 2: e = l ^ 8; break;
        case 3: e = rb + ((l + 4) & 15); break;
        case 4: e = rb + ((l - 4) & 15); break;
        case 5: e = (l & ~7) + 7 - (l & 7); break;
        case 6: e = rb + 15 - (l & 15); break;
        case 7: e = l & 31; break;
        case 8: e = (l & 31) + 32; break;
        case 9: e = l & ~16; break;
        case 10: e = l | 16; break;
      }
      if (h[k * 64 + l] != e) {
        if (!bad) printf("MISMATCH %s lane %d: got %d want %d\n", name[k], l, h[k * 64 + l], e);
        bad++;
      }
    }
  printf(bad ? "xchg_probe: %d mismatches\n" : "xchg_probe: OK%d\n", bad);
  return bad ? 1 : 0;
}
