// xcd_probe2.hip -- development probe: the memory pattern of k_rdx's XCD-team schedule
// (kernels_xcd.hip) without the DSP, to price the hand-off unit and the Doppler lag.
//
// One persistent 512-thread workgroup per CU, team = the 32 CUs of one XCD (HW_REG_XCC_ID
// + ticket, as k_rdx).  A "unit" is UC chirps x 1024 samples (UC = 256: a config-3 frame;
// UC = 128: the half-frame unit of a design that hands half the range bins over per step).
// Member k loads its UC/32 chirps (nt loads), stores them into the unit's slot as 32 groups
// of [UC chirps][32 bins] (plain buffer stores: kept in the XCD's L2), publishes with one
// agent-scope add after vmcnt + barrier; LAG units later it reads group k (sc1 buffer loads,
// L1 bypassed) and writes 32 rows of UC x 8 bytes (sc1 stores).  Step order as k_rdx: publish
// R(j-1), wait ready(j-LAG), group loads, R(j) stores, wait group, next unit's loads, D stores.
// WORK_R / WORK_D packed FMAs per step stand in for the FFTs.
//
//   hipcc --offload-arch=gfx950 -O3 tools/xcd_probe2.hip -o tools/xcd_probe2.bin && tools/xcd_probe2.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

constexpr int NK = 32, NR = 1024;
constexpr int CTR_TICKET = 8 * 8 * 32;   // [8 XCC][8 slots][32] ready counters, then 16 tickets (x32), then abort

__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  unsigned v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ void wait_ge(const unsigned* p, unsigned v, unsigned* err) {
  for (int it = 0; it < (1 << 20); ++it) {
    if (ld_flag(p) >= v) return;
    if ((it & 63) == 63 && ld_flag(err)) return;
    __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) atomicOr(err, 1u);
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int UC, int LAG, int WORK_R, int WORK_D, int W8 = 0>
__global__ __launch_bounds__(512, 1) void k_probe(const char* __restrict__ iq, char* __restrict__ cube, char* __restrict__ rd,
                                                  unsigned* ctr, long nunits, int NS, unsigned* err) {
  constexpr int NL = UC / 32;                 // 16-byte loads per thread per unit (input, group)
  constexpr long UB = (long)UC * NR * 8;      // bytes per unit
  __shared__ int team[2];
  const int tid = threadIdx.x;
  if (tid == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    team[0] = (int)xcc;
    team[1] = (int)__hip_atomic_fetch_add(ctr + CTR_TICKET + xcc * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int x = __builtin_amdgcn_readfirstlane(team[0]), k = __builtin_amdgcn_readfirstlane(team[1]);
  if (k >= NK) { atomicOr(err, 2u); return; }
  const int nj = (int)((nunits - x + 7) / 8);
  unsigned* ready = ctr + x * 8 * 32;
  char* slots0 = cube + (long)x * NS * UB;
  // member k's input: chirps k*UC/32 .. +UC/32 of the unit, contiguous (UC/32 * 8 KiB)
  auto ld_in = [&](long j, f4v (&v)[NL]) __attribute__((always_inline)) {
    const f4v* q = reinterpret_cast<const f4v*>(iq + (x + 8 * j) * UB + (long)k * (UC / 32) * NR * 8);
#pragma unroll
    for (int i = 0; i < NL; ++i) v[i] = __builtin_nontemporal_load(q + tid + 512 * i);
  };
  f4v xin[NL], acc{0.f, 0.f, 0.f, 0.f};
  ld_in(0, xin);
  auto body = [&](int j, bool dj, bool rj, bool pub, auto CNT, bool next) __attribute__((always_inline)) {
    if (pub) vm_wait<decltype(CNT)::value>();
    if (dj && tid < 64) wait_ge(&ready[((j - LAG) % NS) * 32], (unsigned)(NK * ((j - LAG) / NS + 1)), err + 1);
    if (pub || dj) __syncthreads();
    if (pub && tid == 0) __hip_atomic_fetch_add(&ready[((j - 1) % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f4v grp[NL];
    if (dj) {
      const char* g = slots0 + (long)((j - LAG) % NS) * UB + (long)k * UC * 256;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(g), (short)0, UC * 256, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) grp[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 512 * i) * 16, 0, 16);
    }
    if (rj) {
      f4v u = xin[0];
#pragma unroll
      for (int r = 0; r < WORK_R; ++r)
#pragma unroll
        for (int i = 0; i < NL; ++i) xin[i] = xin[i] * 0.999f + u;
      // chirp c = k*UC/32 + (tid*NL... : thread's 16-byte piece e = tid + 512 i of the member's
      // input is chirp ch = e / 512 (of UC/32), sample pair p = e % 512 -> bins 2p, 2p+1 of group p / 16
      char* s = slots0 + (long)(j % NS) * UB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, (short)0, (int)UB, 0x00020000);
      if constexpr (W8 == 2) {   // k_rdx's exact slot-store shape: wave w = chirp 8k + w, lane = (half, position)
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const int lane = tid & 63, w = tid >> 6, c = k * (UC / 32) + w;   // (UC = 256: one chirp per wave)
        const int o = (((lane >> 5) * UC + c) * 32 + (lane & 31)) * 8;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, xin[s2].xy), rs, o + 4 * s2 * UC * 32 * 8, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, xin[s2].zw), rs, o + (4 * s2 + 2) * UC * 32 * 8, 0, 0);
        }
      } else if constexpr (W8) {   // 8-byte stores, each half-wave one 256-byte row
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int e = tid + 512 * i, ch = k * (UC / 32) + (e >> 9), p = e & 511;
          const int lo = ((p >> 4) * UC + ch) * 256, hi = lo + 128;   // the row's two 128-byte halves
          typedef unsigned u2 __attribute__((ext_vector_type(2)));
          const u2 v0 = __builtin_bit_cast(u2, xin[i].xy), v1 = __builtin_bit_cast(u2, xin[i].zw);
          __builtin_amdgcn_raw_buffer_store_b64(v0, rs, lo + (p & 15) * 8, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(v1, rs, hi + (p & 15) * 8, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int e = tid + 512 * i, ch = k * (UC / 32) + (e >> 9), p = e & 511;
          __builtin_amdgcn_raw_buffer_store_b128(xin[i], rs, (((p >> 4) * UC + ch) * 16 + (p & 15)) * 16, 0, 0);
        }
      }
    }
    if (rj) vm_wait<(W8 ? 2 : 1) * NL>();
    else vm_wait<0>();
    __syncthreads();
    if (next) ld_in(j + 1 < nj ? j + 1 : nj - 1, xin);
    if (dj) {
      f4v u = grp[0];
#pragma unroll
      for (int r = 0; r < WORK_D; ++r)
#pragma unroll
        for (int i = 0; i < NL; ++i) grp[i] = grp[i] * 0.998f + u;
      const long f = x + 8L * (j - LAG);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rd + f * UB + (long)k * 32 * UC * 8, (short)0, 32 * UC * 8, 0x00020000);
      if constexpr (W8 == 2) {   // k_rdx's exact RD shape: wave w rows 4w + pp, lane (pp, q) positions q + 16 d1s
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const int lane = tid & 63, w = tid >> 6, pp = lane >> 4, q = lane & 15, row = 4 * w + pp;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, grp[d].xy), rr, (row * UC + q + 32 * d) * 8, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, grp[d].zw), rr, (row * UC + q + 32 * d + 16) * 8, 0, 16);
        }
      } else if constexpr (W8) {   // 8-byte sc1 stores, 16 lanes per 128-byte row segment
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int e = tid + 512 * i;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, grp[i].xy), rr, e * 8, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, grp[i].zw), rr, (e + 512 * NL) * 8, 0, 16);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) __builtin_amdgcn_raw_buffer_store_b128(grp[i], rr, (tid + 512 * i) * 16, 0, 16);
      }
      acc += u;
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using CS = std::integral_constant<int, NL + (W8 ? 2 : 1) * NL>;   // after R(j-1)'s stores: next loads + D's RD stores
  using C1 = std::integral_constant<int, NL>;       // step 1: only the next loads
  if (nj >= LAG + 1) {
    body(0, false, true, false, C0{}, true);
    for (int j = 1; j < LAG; ++j) body(j, false, true, true, C1{}, true);
    body(LAG, true, true, true, C1{}, true);
    for (int j = LAG + 1; j < nj; ++j) body(j, true, true, true, CS{}, true);
    body(nj, true, false, true, CS{}, false);
    for (int j = nj + 1; j < nj + LAG; ++j) body(j, true, false, false, C0{}, false);
  }
  if (acc.x == 1234.5f) rd[tid] = 1;
}

template <int UC, int LAG, int WR, int WD, int W8 = 0>
float run(const char* iq, char* cube, char* rd, unsigned* ctr, unsigned* err, long F, int NS) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  const long nunits = F * 256 / UC;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(ctr, 0, 4096 * 4));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_probe<UC, LAG, WR, WD, W8>), dim3(256), dim3(512), 0, 0, iq, cube, rd, ctr, nunits, NS, err);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best = ms < best ? ms : best;
  }
  unsigned h[2] = {0, 0};
  CK(hipMemcpy(h, err, 8, hipMemcpyDeviceToHost));
  if (h[0] | h[1]) printf("  (err %x %x)\n", h[0], h[1]);
  CK(hipMemset(err, 0, 8));
  return best;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  if (p.multiProcessorCount != 256) { printf("needs 256 CUs, have %d\n", p.multiProcessorCount); return 3; }
  const long F = 4096, B = F * 256L * NR * 8;
  char *iq, *rd, *cube;
  unsigned *ctr, *err;
  CK(hipMalloc(&iq, B));
  CK(hipMalloc(&rd, B));
  CK(hipMalloc(&cube, 8L * 8 * 256 * NR * 8));
  CK(hipMalloc(&ctr, 4096 * 4));
  CK(hipMalloc(&err, 8));
  CK(hipMemset(err, 0, 8));
  CK(hipMemset(iq, 0, B));
  const double gb = 2.0 * B / 1e9;
  auto pr = [&](const char* what, float ms) { printf("%-40s %.3f ms  frac %.3f of 8 TB/s (in + out)\n", what, ms, gb / ms / 8.0); };
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  if (which == 0 || which == 1) {
    pr("frame unit, lag 2, 4 slots", run<256, 2, 0, 0>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 1, 3 slots", run<256, 1, 0, 0>(iq, cube, rd, ctr, err, F, 3));
    pr("half unit, lag 2, 4 slots", run<128, 2, 0, 0>(iq, cube, rd, ctr, err, F, 4));
    pr("half unit, lag 2, 3 slots", run<128, 2, 0, 0>(iq, cube, rd, ctr, err, F, 3));
    pr("half unit, lag 3, 5 slots", run<128, 3, 0, 0>(iq, cube, rd, ctr, err, F, 5));
    pr("quarter unit, lag 3, 5 slots", run<64, 3, 0, 0>(iq, cube, rd, ctr, err, F, 5));
    pr("quarter unit, lag 4, 6 slots", run<64, 4, 0, 0>(iq, cube, rd, ctr, err, F, 6));
  }
  if (which == 0 || which == 3) {
    pr("frame unit, lag 2, 4 slots", run<256, 2, 0, 0>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 2, 4 slots, 8-B stores", run<256, 2, 0, 0, 1>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 2, 4 slots, work", run<256, 2, 24, 16>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 2, 4 slots, 8-B stores, work", run<256, 2, 24, 16, 1>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 2, 4 slots, k_rdx store shapes", run<256, 2, 0, 0, 2>(iq, cube, rd, ctr, err, F, 4));
    pr("frame unit, lag 2, 4 slots, k_rdx store shapes, work", run<256, 2, 24, 16, 2>(iq, cube, rd, ctr, err, F, 4));
  }
  if (which == 0 || which == 2) {
    pr("frame unit, lag 2, 4 slots, work", run<256, 2, 24, 16>(iq, cube, rd, ctr, err, F, 4));
    pr("half unit, lag 2, 4 slots, work", run<128, 2, 24, 16>(iq, cube, rd, ctr, err, F, 4));
    pr("half unit, lag 3, 5 slots, work", run<128, 3, 24, 16>(iq, cube, rd, ctr, err, F, 5));
  }
  return 0;
}
