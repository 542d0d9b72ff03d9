// r04_probe.hip -- development probe (round 4): what bounds k_rdx's data movement?
//
// Part A (copy ceiling): read-only, write-only and in -> out copies of the
// config-3 byte count (8.59 GB each way) in several shapes, to place the 6.29 TB/s of
// MI355X_MICROARCH.md against this buffer size.
//
// Part B (hand-off): the XCD-team frame-unit schedule of
// tools/xcd_probe2.hip (k_rdx's memory streams without the DSP) with
//   THR     512 or 1024 threads per workgroup (8 or 16 waves: memory-level parallelism),
//   AUX     the slot-store cache policy (0 plain, 1 sc0, 2 nt, 16 sc1),
//   spread  the ring's slot addresses cycle over `spread` x the ring (spread 1: the same
//           4 MiB per XCD every step; spread 64: 256 MiB per XCD, beyond the Infinity Cache),
//   HO      0: no hand-off at all (input copied straight to RD, same team protocol).
// WRITE_SIZE / FETCH_SIZE per variant come from separate rocprofv3 --pmc passes.
//
//   hipcc --offload-arch=gfx950 -O3 tools/r04_probe.hip -o tools/r04_probe.bin && tools/r04_probe.bin [part]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

constexpr int NK = 32, NR = 1024, UC = 256;
constexpr long UB = (long)UC * NR * 8;        // bytes per frame (2 MiB)
constexpr int CTR_TICKET = 8 * 8 * 32;        // [8 XCC][8 slots][32] ready counters, then tickets

// ---------------------------------------------------------------- part A: copy shapes
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
// one block per 256 x U chunk (no grid-stride loop)
template <int U, int NT>
__global__ __launch_bounds__(256) void k_copyB(const f4v* __restrict__ a, f4v* __restrict__ o) {
  const long base = blockIdx.x * 256L * U + threadIdx.x;
  f4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = NT & 1 ? __builtin_nontemporal_load(a + base + 256L * u) : a[base + 256L * u];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (NT & 2) __builtin_nontemporal_store(v[u], o + base + 256L * u);
    else o[base + 256L * u] = v[u];
  }
}
template <int U>
__global__ __launch_bounds__(256) void k_read(const f4v* __restrict__ a, long n, float* sink) {
  f4v s{0.f, 0.f, 0.f, 0.f};
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = blockIdx.x * 256L * U + threadIdx.x; base < n; base += stride) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + 256L * u < n ? __builtin_nontemporal_load(a + base + 256L * u) : f4v{};
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  if (s.x == 1234.5f) sink[threadIdx.x] = s.y;
}
template <int U>
__global__ __launch_bounds__(256) void k_write(f4v* __restrict__ o, long n) {
  const long stride = (long)gridDim.x * 256 * U;
  const f4v v{1.f, 2.f, 3.f, (float)threadIdx.x};
  for (long base = blockIdx.x * 256L * U + threadIdx.x; base < n; base += stride)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + 256L * u < n) __builtin_nontemporal_store(v, o + base + 256L * u);
}

// ---------------------------------------------------------------- part H: K1's access shape
// config 2's K1 (k_range<512>) moves 4 KiB per chirp in and 4 KiB out: 32-thread teams, 8 per
// 256-thread block, each team walking CPT chirps; lane t of a team holds elements t + 32 m
// (m = 0..15, 8 bytes each).  W = 8: that shape, copied; W = 16: the same chirps as 8 loads of
// 16 bytes per lane (elements 2t + 64 m', 2t + 1 + 64 m').  A data-movement ceiling for K1.
template <int W, int CPT, int NT>
__global__ __launch_bounds__(256, 3) void k_k1shape(const char* __restrict__ in, char* __restrict__ out, long nchirps) {
  const int t = threadIdx.x & 31, team = threadIdx.x >> 5;
  const long c0 = ((long)blockIdx.x * 8 + team) * CPT;
  typedef float f2 __attribute__((ext_vector_type(2)));
  for (int c = 0; c < CPT; ++c) {
    const long ch = c0 + c;
    if (ch >= nchirps) break;
    if constexpr (W == 8) {
      const f2* src = reinterpret_cast<const f2*>(in + ch * 4096);
      f2* dst = reinterpret_cast<f2*>(out + ch * 4096);
      f2 v[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = NT ? __builtin_nontemporal_load(src + t + 32 * m) : src[t + 32 * m];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (NT) __builtin_nontemporal_store(v[m], dst + t + 32 * m);
        else dst[t + 32 * m] = v[m];
      }
    } else {
      const f4v* src = reinterpret_cast<const f4v*>(in + ch * 4096);
      f4v* dst = reinterpret_cast<f4v*>(out + ch * 4096);
      f4v v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = NT ? __builtin_nontemporal_load(src + t + 32 * m) : src[t + 32 * m];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (NT) __builtin_nontemporal_store(v[m], dst + t + 32 * m);
        else dst[t + 32 * m] = v[m];
      }
    }
  }
}

// ---------------------------------------------------------------- part B: the hand-off
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

// frame unit, Doppler LAG 2 steps behind, NS slots per XCD; member k: chirps 8k..8k+7 in,
// group k (32 bins x 256 chirps) out of the slot, 32 RD rows written
template <int THR, int AUX, int HO, int INAUX = 2, int RDAUX = 2, int UC = 256>
__global__ __launch_bounds__(THR, 1) void k_team(const char* __restrict__ iq, char* __restrict__ cube, char* __restrict__ rd,
                                                 unsigned* ctr, long nunits, int NS, int spread, unsigned* err) {
  constexpr int LAG = 2;
  constexpr long UB = (long)UC * NR * 8;      // bytes per unit (UC = 256: a frame)
  constexpr int NL = UC * 16 / THR;           // 16-byte pieces per thread (member share UC/4 KiB)
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
  char* slots0 = cube + (long)x * NS * spread * UB;
  auto slotp = [&](int j) { return slots0 + ((long)(j % NS) + (long)NS * ((j / NS) % spread)) * UB; };
  auto ld_in = [&](long j, f4v (&v)[NL]) __attribute__((always_inline)) {
    const char* q = iq + (x + 8 * j) * UB + (long)k * (UC / 32) * NR * 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(q), (short)0, (UC / 32) * NR * 8, 0x00020000);
#pragma unroll
    for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, INAUX);
  };
  f4v xin[NL], acc{0.f, 0.f, 0.f, 0.f};
  ld_in(0, xin);
  f4v hold[NL];                                // HO == 0: the input handed to D directly (same member)
  auto body = [&](int j, bool dj, bool rj, bool pub, auto CNT, bool next) __attribute__((always_inline)) {
    if (pub) vm_wait<decltype(CNT)::value>();
    constexpr bool SYNC = HO == 1 || HO == 3, TRAF = HO == 1 || HO == 2;
    if (SYNC && dj && tid < 64) wait_ge(&ready[((j - LAG) % NS) * 32], (unsigned)(NK * ((j - LAG) / NS + 1)), err + 1);
    if (pub || dj) __syncthreads();
    if (SYNC && pub && tid == 0) __hip_atomic_fetch_add(&ready[((j - 1) % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f4v grp[NL];
    if (dj) {
      if (TRAF) {
        const char* g = slotp(j - LAG) + (long)k * UC * 256;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(g), (short)0, UC * 256, 0x00020000);
#pragma unroll
        for (int i = 0; i < NL; ++i) grp[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 16);
      } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) grp[i] = hold[i];
      }
    }
    if (rj) {
      if (TRAF) {
        char* s = slotp(j);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, (short)0, (int)UB, 0x00020000);
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int e = tid + THR * i, ch = k * (UC / 32) + (e >> 9), p = e & 511;   // piece p of chirp ch
          __builtin_amdgcn_raw_buffer_store_b128(xin[i], rs, (((p >> 4) * UC + ch) * 16 + (p & 15)) * 16, 0, AUX);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) hold[i] = xin[i];
      }
    }
    if (TRAF) {
      if (rj) vm_wait<NL>();
      else vm_wait<0>();
    }
    __syncthreads();
    if (next) ld_in(j + 1 < nj ? j + 1 : nj - 1, xin);
    if (dj) {
      const long f = x + 8L * (j - LAG);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rd + f * UB + (long)k * 32 * UC * 8, (short)0, 32 * UC * 8, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) __builtin_amdgcn_raw_buffer_store_b128(grp[i], rr, (tid + THR * i) * 16, 0, RDAUX);
      acc += grp[0];
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using CS = std::integral_constant<int, NL + NL>;   // after R(j-1)'s stores: next loads + D's RD stores
  using C1 = std::integral_constant<int, NL>;
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

// k_rdx's own protocol with the group consumed one step after it is loaded: step j publishes
// R(j-1) (after its slot stores completed), stores D(j-2)'s rows from the group loaded in step
// j-1, polls ready(j-1) and loads group k of unit j-1, writes R(j)'s slot (after that poll: every
// read of the slot's previous unit is done), then loads the next unit's input.  2 slots.
// LAGP: the unit polled and loaded in step j is j - LAGP (1: k_rdx); NS >= 2 LAGP slots (a member
// that sees ready(j - LAGP) knows every member has read unit j - 2 LAGP)
// BURN (part M, round 5): v_pk_fma_f32 per wave and full-frame step (scaled by UC / 256) after
// R(j)'s slot stores, with the next input loads in flight -- k_rdx's DSP energy without its data
template <int UC, int LAGP = 1, int NS = 2, int HB = 1, int BURN = 0, int BURNK = 0>   // HB 2: every stream at half the bytes (fp16 storage, part K)
__global__ __launch_bounds__(512, 1) void k_team_def(const char* __restrict__ iq, char* __restrict__ cube, char* __restrict__ rd,
                                                     unsigned* ctr, long nunits, unsigned* err) {
  constexpr int THR = 512;
  static_assert(NS >= 2 * LAGP && NS <= 8, "slot reuse: seeing ready(j - LAGP) proves unit j - 2 LAGP read");
  constexpr long UB = (long)UC * NR * 8 / HB;
  constexpr int NL = UC * 16 / THR / HB;
  __shared__ int team[2];
  __shared__ unsigned gflag;
  const int tid = threadIdx.x;
  if (tid == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    team[0] = (int)xcc;
    team[1] = (int)__hip_atomic_fetch_add(ctr + CTR_TICKET + xcc * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gflag = 0;
  }
  __syncthreads();
  const int x = __builtin_amdgcn_readfirstlane(team[0]), k = __builtin_amdgcn_readfirstlane(team[1]);
  if (k >= NK) { atomicOr(err, 2u); return; }
  const int nj = (int)((nunits - x + 7) / 8);
  unsigned* ready = ctr + x * 8 * 32;
  char* slots0 = cube + (long)x * NS * UB;
  auto ld_in = [&](long j, f4v (&v)[NL]) __attribute__((always_inline)) {
    const char* q = iq + (x + 8 * j) * UB + (long)k * (UC / 32) * NR * 8 / HB;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(q), (short)0, (UC / 32) * NR * 8 / HB, 0x00020000);
#pragma unroll
    for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 2);
  };
  f4v xin[NL], grp[NL], acc{0.f, 0.f, 0.f, 0.f};
  if (nj > 0) ld_in(0, xin);
  for (int j = 0; j < nj + LAGP + 1; ++j) {
    const bool pub = j >= 1 && j - 1 < nj, dj = j >= LAGP + 1, gj = j >= LAGP && j - LAGP < nj, rj = j < nj;
    if (pub) vm_wait<NL>();                       // R(j-1)'s slot stores; the next input loads may fly
    else vm_wait<0>();
    __syncthreads();
    if (pub && tid == 0) __hip_atomic_fetch_add(&ready[((j - 1) % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dj) {                                     // D(j-1-LAGP): rows from the group loaded in step j-1
      const long f = x + 8L * (j - 1 - LAGP);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rd + f * UB + (long)k * 32 * UC * 8 / HB, (short)0, 32 * UC * 8 / HB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) __builtin_amdgcn_raw_buffer_store_b128(grp[i], rr, (tid + THR * i) * 16, 0, 2);
      acc += grp[0];
    }
    if (gj) {                                     // poll ready(j-LAGP), then load group k of unit j-LAGP
      if (tid < 64) {
        wait_ge(&ready[((j - LAGP) % NS) * 32], (unsigned)(NK * ((j - LAGP) / NS + 1)), err + 1);
        if (tid == 0) *reinterpret_cast<volatile unsigned*>(&gflag) = (unsigned)j;
      } else {
        while (*reinterpret_cast<volatile unsigned*>(&gflag) < (unsigned)j) __builtin_amdgcn_s_sleep(1);
      }
      const char* g = slots0 + (long)((j - LAGP) % NS) * UB + (long)k * UC * 256 / HB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(g), (short)0, UC * 256 / HB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) grp[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 16);
    }
    if (rj) {                                     // R(j): the slot's previous unit j - NS <= j - 2 LAGP was read by all
      if (j >= 1) vm_wait<NL>();                  // xin of unit j (the group loads may fly)
      else vm_wait<0>();
      char* s = slots0 + (long)(j % NS) * UB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, (short)0, (int)UB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int e = tid + THR * i, ch = k * (UC / 32) + (e / (512 / HB)), p = e % (512 / HB);
        __builtin_amdgcn_raw_buffer_store_b128(xin[i], rs, (((p >> 4) * UC + ch) * 16 + (p & 15)) * 16, 0, 0);
      }
      if (j + 1 < nj) ld_in(j + 1, xin);
      if constexpr (BURN > 0) {
        // BURNK 0: u = 0.999 u + c (converges: constant bits, little switching); 1: u = -0.5 u + g with
        // g the random samples of the group (every mantissa bit toggles, as in the FFTs)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 u[8], g[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          u[i] = f2{acc.x + (float)i, acc.y - (float)i};
          const f4v gi = grp[i % NL];
          g[i] = i & 1 ? f2{gi.z, gi.w} : f2{gi.x, gi.y};
        }
        const f2 m = BURNK ? f2{-0.5f, -0.5f} : f2{acc.z * 1e-30f + 0.999f, acc.w * 1e-30f + 0.998f};
        constexpr int IT = BURN * UC / 256 / 8;
#pragma unroll 4
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int i = 0; i < 8; ++i) u[i] = __builtin_elementwise_fma(u[i], m, BURNK ? g[(i + it) & 7] : f2{1e-3f, 2e-3f});
#pragma unroll
        for (int i = 0; i < 8; ++i) acc.x += u[i].x + u[i].y;
      }
    }
  }
  if (acc.x == 1234.5f) rd[tid] = 1;
}

// Part J: slot reuse proven by done counters instead of a later ready counter.  Step j: wait
// until every member has read the slot's previous unit (done(j - NS)), store R(j), publish
// ready(j); store D's RD rows of the group loaded in step j - 1; poll ready(j - NS + 1), load group
// k of that unit, wait for the loads, publish done.  NS = 1: the unit is written and read in the
// same step, so a slot line lives one step (2 MiB of ring per XCD at the frame unit) at the price
// of a serial store -> ready -> load -> done chain per step.
constexpr int CTR_DONE = 4096;                // [8 XCC][8 slots][32] done counters
template <int UC, int NS>
__global__ __launch_bounds__(512, 1) void k_team_done(const char* __restrict__ iq, char* __restrict__ cube, char* __restrict__ rd,
                                                      unsigned* ctr, long nunits, unsigned* err) {
  constexpr int THR = 512, LAGD = NS - 1;
  constexpr long UB = (long)UC * NR * 8;
  constexpr int NL = UC * 16 / THR;
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
  unsigned* done = ctr + CTR_DONE + x * 8 * 32;
  char* slots0 = cube + (long)x * NS * UB;
  auto ld_in = [&](long j, f4v (&v)[NL]) __attribute__((always_inline)) {
    const char* q = iq + (x + 8 * j) * UB + (long)k * (UC / 32) * NR * 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(q), (short)0, (UC / 32) * NR * 8, 0x00020000);
#pragma unroll
    for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 2);
  };
  f4v xin[NL], grp[NL], acc{0.f, 0.f, 0.f, 0.f};
  if (nj > 0) ld_in(0, xin);
  for (int j = 0; j < nj + LAGD + 1; ++j) {
    if (j < nj) {
      if (j >= NS && tid < 64) wait_ge(&done[(j % NS) * 32], (unsigned)(NK * ((j - NS) / NS + 1)), err + 1);
      vm_wait<0>();                               // xin of unit j
      __syncthreads();
      char* s = slots0 + (long)(j % NS) * UB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, (short)0, (int)UB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int e = tid + THR * i, ch = k * (UC / 32) + (e >> 9), p = e & 511;
        __builtin_amdgcn_raw_buffer_store_b128(xin[i], rs, (((p >> 4) * UC + ch) * 16 + (p & 15)) * 16, 0, 0);
      }
      if (j + 1 < nj) {
        ld_in(j + 1, xin);
        vm_wait<NL>();                            // the slot stores (the next input may fly)
      } else {
        vm_wait<0>();
      }
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&ready[(j % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (j >= 1 && j - 1 - LAGD >= 0 && j - 1 - LAGD < nj) {   // D(u'): rows of the group loaded in step j - 1
      const long f = x + 8L * (j - 1 - LAGD);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rd + f * UB + (long)k * 32 * UC * 8, (short)0, 32 * UC * 8, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) __builtin_amdgcn_raw_buffer_store_b128(grp[i], rr, (tid + THR * i) * 16, 0, 2);
      acc += grp[0];
    }
    const int u = j - LAGD;
    if (u >= 0 && u < nj) {
      if (tid < 64) wait_ge(&ready[(u % NS) * 32], (unsigned)(NK * (u / NS + 1)), err + 1);
      __syncthreads();
      const char* g = slots0 + (long)(u % NS) * UB + (long)k * UC * 256;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(g), (short)0, UC * 256, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) grp[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 16);
      vm_wait<0>();
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&done[(u % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (acc.x == 1234.5f) rd[tid] = 1;
}

// Part L: role split.  Members 0-15 of an XCD team only transform (R: 16 chirps of each frame in,
// their 128 KiB into the slot), members 16-31 only Doppler (D: 2 groups = 128 KiB of the slot in,
// 128 KiB of RD rows out).  R rewrites slot j % NS once every D member has counted frame j - NS out
// (done), D reads frame j once every R member has published it (ready): the two roles run decoupled
// by NS frames of ring.
template <int NS>
__global__ __launch_bounds__(512, 1) void k_team_role(const char* __restrict__ iq, char* __restrict__ cube, char* __restrict__ rd,
                                                      unsigned* ctr, long nunits, unsigned* err) {
  constexpr int THR = 512, NL = 16;           // 16 x 16 B per thread = 128 KiB per member and frame
  constexpr long UB = (long)256 * NR * 8;
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
  unsigned* done = ctr + CTR_DONE + x * 8 * 32;
  char* slots0 = cube + (long)x * NS * UB;
  f4v v[NL], acc{0.f, 0.f, 0.f, 0.f};
  if (k < 16) {                               // R
    const int r = k;
    auto ld_in = [&](long j) __attribute__((always_inline)) {
      const char* q = iq + (x + 8 * j) * UB + (long)r * 16 * NR * 8;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(q), (short)0, 16 * NR * 8, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 2);
    };
    if (nj > 0) ld_in(0);
    for (int j = 0; j < nj; ++j) {
      if (j >= NS && tid < 64) wait_ge(&done[(j % NS) * 32], (unsigned)(16 * ((j - NS) / NS + 1)), err + 1);
      vm_wait<0>();
      __syncthreads();
      char* s = slots0 + (long)(j % NS) * UB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, (short)0, (int)UB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int e = tid + THR * i, ch = r * 16 + (e >> 9), p = e & 511;   // piece p of chirp ch
        __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, (((p >> 4) * 256 + ch) * 16 + (p & 15)) * 16, 0, 0);
      }
      if (j + 1 < nj) {
        ld_in(j + 1);
        vm_wait<NL>();
      } else {
        vm_wait<0>();
      }
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&ready[(j % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {                                    // D: groups 2d, 2d + 1
    const int d = k - 16;
    for (int j = 0; j < nj; ++j) {
      if (tid < 64) wait_ge(&ready[(j % NS) * 32], (unsigned)(16 * (j / NS + 1)), err + 1);
      __syncthreads();
      const char* g = slots0 + (long)(j % NS) * UB + (long)d * 2 * 256 * 256;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(g), (short)0, 2 * 256 * 256, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + THR * i) * 16, 0, 16);
      vm_wait<0>();
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&done[(j % NS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const long f = x + 8L * j;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rd + f * UB + (long)d * 64 * 256 * 8, (short)0, 64 * 256 * 8, 0x00020000);
#pragma unroll
      for (int i = 0; i < NL; ++i) __builtin_amdgcn_raw_buffer_store_b128(v[i], rr, (tid + THR * i) * 16, 0, 2);
      acc += v[0];
    }
  }
  if (acc.x == 1234.5f) rd[tid] = 1;
}

// ---------------------------------------------------------------- part C: stores leaving the L2
// every CU rewrites its own R-byte region `passes` times with policy AUX (16-byte stores);
// WRITE_SIZE / bytes stored says whether each pass leaves the XCD's L2
template <int AUX>
__global__ __launch_bounds__(512, 1) void k_rewrite(char* __restrict__ buf, int region, int passes) {
  char* my = buf + (long)blockIdx.x * region;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(my, (short)0, region, 0x00020000);
  const f4v v{1.f, 2.f, 3.f, (float)threadIdx.x};
  for (int p = 0; p < passes; ++p)
    for (int o = threadIdx.x * 16; o < region; o += 512 * 16) __builtin_amdgcn_raw_buffer_store_b128(v + (float)p, rs, o, 0, AUX);
}

template <typename L>
float timeit(L launch, int reps = 6) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < reps; ++rep) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best = ms < best ? ms : best;
  }
  return best;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  if (p.multiProcessorCount != 256) { printf("needs 256 CUs, have %d\n", p.multiProcessorCount); return 3; }
  const int part = argc > 1 ? atoi(argv[1]) : 0;
  const long F = 4096, B = F * UB, n = B / 16;
  char *iq, *rd, *cube;
  unsigned *ctr, *err;
  float* sink;
  CK(hipMalloc(&iq, B));
  CK(hipMalloc(&rd, B));
  const long cube_bytes = 8L * 2 * 64 * UB;   // 8 XCDs x NS 2 x spread up to 64
  // CUBE_ALLOC: 0 hipMalloc (coarse-grained, default), 1 fine-grained, 3 uncached (the hand-off
  // ring's memory type: part G)
  const int calloc_flag = getenv("CUBE_ALLOC") ? atoi(getenv("CUBE_ALLOC")) : 0;
  if (calloc_flag) CK(hipExtMallocWithFlags((void**)&cube, cube_bytes, (unsigned)calloc_flag));
  else CK(hipMalloc(&cube, cube_bytes));
  CK(hipMalloc(&ctr, 8192 * 4));
  CK(hipMalloc(&err, 8));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(err, 0, 8));
  CK(hipMemset(iq, 0, B));
  CK(hipMemset(rd, 0, B));
  CK(hipMemset(cube, 0, cube_bytes));
  const double gb1 = B / 1e9, algo = F * 4198400.0 / 1e9;
  if (part == 0 || part == 1) {
    printf("== part A: copy ceiling (8.59 GB each way; frac = k_rdx's 17.2 GB / time / 8 TB/s)\n");
    auto rc = [&](const char* nm, float ms) { printf("%-34s %.3f ms  %.2f TB/s in+out  frac %.3f\n", nm, ms, 2 * gb1 / ms / 1e3, algo / ms / 8.0); };
    auto r1 = [&](const char* nm, float ms) { printf("%-34s %.3f ms  %.2f TB/s one way\n", nm, ms, gb1 / ms / 1e3); };
    r1("read-only U4 G8192", timeit([&] { hipLaunchKernelGGL((k_read<4>), dim3(8192), dim3(256), 0, 0, (const f4v*)iq, n, sink); }));
    r1("read-only U8 G8192", timeit([&] { hipLaunchKernelGGL((k_read<8>), dim3(8192), dim3(256), 0, 0, (const f4v*)iq, n, sink); }));
    r1("read-only U4 G65536", timeit([&] { hipLaunchKernelGGL((k_read<4>), dim3(65536), dim3(256), 0, 0, (const f4v*)iq, n, sink); }));
    r1("write-only U4 G8192", timeit([&] { hipLaunchKernelGGL((k_write<4>), dim3(8192), dim3(256), 0, 0, (f4v*)rd, n); }));
    r1("write-only U4 G65536", timeit([&] { hipLaunchKernelGGL((k_write<4>), dim3(65536), dim3(256), 0, 0, (f4v*)rd, n); }));
    rc("copy U4 nt G65536", timeit([&] { hipLaunchKernelGGL((k_copyU<4, 3>), dim3(65536), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd, n); }));
    rc("copy U4 plain G65536", timeit([&] { hipLaunchKernelGGL((k_copyU<4, 0>), dim3(65536), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd, n); }));
    rc("copy U4 ntstore G65536", timeit([&] { hipLaunchKernelGGL((k_copyU<4, 2>), dim3(65536), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd, n); }));
    rc("copy blocks U4 nt", timeit([&] { hipLaunchKernelGGL((k_copyB<4, 3>), dim3(n / 1024), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd); }));
    rc("copy blocks U2 nt", timeit([&] { hipLaunchKernelGGL((k_copyB<2, 3>), dim3(n / 512), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd); }));
    rc("copy blocks U1 nt", timeit([&] { hipLaunchKernelGGL((k_copyB<1, 3>), dim3(n / 256), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd); }));
    rc("copy blocks U1 plain", timeit([&] { hipLaunchKernelGGL((k_copyB<1, 0>), dim3(n / 256), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd); }));
    // a 1 GiB copy (the size a quick copy benchmark often uses: part of it can sit in the 256 MiB Infinity Cache)
    const long n1 = (1L << 30) / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const float ms1 = timeit([&] { hipLaunchKernelGGL((k_copyB<1, 0>), dim3(n1 / 256), dim3(256), 0, 0, (const f4v*)iq, (f4v*)rd); });
    printf("%-34s %.3f ms  %.2f TB/s in+out\n", "copy 1 GiB blocks U1 plain", ms1, 2.0 * (1L << 30) / ms1 / 1e9);
  }
  auto rb = [&](const char* nm, float ms) {
    unsigned h[2] = {0, 0};
    CK(hipMemcpy(h, err, 8, hipMemcpyDeviceToHost));
    printf("%-44s %.3f ms  frac %.3f%s\n", nm, ms, algo / ms / 8.0, (h[0] | h[1]) ? "  (ERR)" : "");
    CK(hipMemset(err, 0, 8));
  };
  auto team = [&](auto kern, int thr, int NS, int spread) {
    return timeit([&] {
      CK(hipMemsetAsync(ctr, 0, 4096 * 4));
      hipLaunchKernelGGL(kern, dim3(256), dim3(thr), 0, 0, (const char*)iq, cube, rd, ctr, F, NS, spread, err);
    }, 5);
  };
  if (part == 0 || part == 2) {
    printf("== part B: XCD-team frame unit, lag 2 (k_rdx's streams, no DSP)\n");
    rb("512 thr, plain slots, 2 slots", team(k_team<512, 0, 1>, 512, 2, 1));
    rb("512 thr, plain slots, 4 slots", team(k_team<512, 0, 1>, 512, 4, 1));
    rb("512 thr, sc0 slots, 2 slots", team(k_team<512, 1, 1>, 512, 2, 1));
    rb("512 thr, nt slots, 2 slots", team(k_team<512, 2, 1>, 512, 2, 1));
    rb("512 thr, sc1 slots, 2 slots", team(k_team<512, 16, 1>, 512, 2, 1));
    rb("512 thr, plain slots, 2 slots, spread 8", team(k_team<512, 0, 1>, 512, 2, 8));
    rb("512 thr, plain slots, 2 slots, spread 64", team(k_team<512, 0, 1>, 512, 2, 64));
    rb("1024 thr, plain slots, 2 slots", team(k_team<1024, 0, 1>, 1024, 2, 1));
    rb("1024 thr, nt slots, 2 slots", team(k_team<1024, 2, 1>, 1024, 2, 1));
    rb("512 thr, no hand-off (in -> RD)", team(k_team<512, 0, 0>, 512, 2, 1));
    rb("1024 thr, no hand-off (in -> RD)", team(k_team<1024, 0, 0>, 1024, 2, 1));
  }
  auto teamu = [&](auto kern, int NS, int UCv) {
    return timeit([&] {
      CK(hipMemsetAsync(ctr, 0, 4096 * 4));
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, (const char*)iq, cube, rd, ctr, F * 256 / UCv, NS, 1, err);
    }, 5);
  };
  if (part == 0 || part == 4) {
    printf("== part D: cache policies of the input loads / RD stores (plain slots, 2 slots), unit size\n");
    rb("in nt, RD nt (part B row 1)", teamu(k_team<512, 0, 1, 2, 2>, 2, 256));
    rb("in nt, RD sc1", teamu(k_team<512, 0, 1, 2, 16>, 2, 256));
    rb("in nt, RD sc0 sc1", teamu(k_team<512, 0, 1, 2, 17>, 2, 256));
    rb("in nt, RD sc1 nt", teamu(k_team<512, 0, 1, 2, 18>, 2, 256));
    rb("in sc1, RD sc1", teamu(k_team<512, 0, 1, 16, 16>, 2, 256));
    rb("in sc0 sc1, RD sc1", teamu(k_team<512, 0, 1, 17, 16>, 2, 256));
    rb("in sc1 nt, RD sc1", teamu(k_team<512, 0, 1, 18, 16>, 2, 256));
    rb("in plain, RD sc1", teamu(k_team<512, 0, 1, 0, 16>, 2, 256));
    rb("half unit, in nt, RD nt, 2 slots", teamu(k_team<512, 0, 1, 2, 2, 128>, 2, 128));
    rb("half unit, in nt, RD sc1, 2 slots", teamu(k_team<512, 0, 1, 2, 16, 128>, 2, 128));
    rb("half unit, in nt, RD sc1, 3 slots", teamu(k_team<512, 0, 1, 2, 16, 128>, 3, 128));
    rb("quarter unit, in nt, RD sc1, 2 slots", teamu(k_team<512, 0, 1, 2, 16, 64>, 2, 64));
    rb("quarter unit, in nt, RD nt, 2 slots", teamu(k_team<512, 0, 1, 2, 2, 64>, 2, 64));
  }
  if (part == 0 || part == 5) {
    printf("== part E: the hand-off split into its traffic and its synchronisation (frame unit, 2 slots)\n");
    rb("full hand-off", teamu(k_team<512, 0, 1, 2, 2>, 2, 256));
    rb("traffic only (no publish / poll)", teamu(k_team<512, 0, 2, 2, 2>, 2, 256));
    rb("sync only (no slot stores / loads)", teamu(k_team<512, 0, 3, 2, 2>, 2, 256));
    rb("no hand-off", teamu(k_team<512, 0, 0, 2, 2>, 2, 256));
    rb("quarter: full", teamu(k_team<512, 0, 1, 2, 2, 64>, 2, 64));
    rb("quarter: traffic only", teamu(k_team<512, 0, 2, 2, 2, 64>, 2, 64));
    rb("quarter: sync only", teamu(k_team<512, 0, 3, 2, 2, 64>, 2, 64));
    rb("quarter: no hand-off", teamu(k_team<512, 0, 0, 2, 2, 64>, 2, 64));
  }
  auto teamd = [&](auto kern, int UCv) {
    return timeit([&] {
      CK(hipMemsetAsync(ctr, 0, 4096 * 4));
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, (const char*)iq, cube, rd, ctr, F * 256 / UCv, err);
    }, 5);
  };
  if (part == 0 || part == 6) {
    printf("== part F: k_rdx's protocol, group consumed one step after its loads (2 slots)\n");
    rb("frame unit, deferred group", teamd(k_team_def<256>, 256));
    rb("half unit, deferred group", teamd(k_team_def<128>, 128));
    rb("quarter unit, deferred group", teamd(k_team_def<64>, 64));
    rb("eighth unit, deferred group", teamd(k_team_def<32>, 32));
    rb("(part B) frame unit, full", teamu(k_team<512, 0, 1, 2, 2>, 2, 256));
    rb("(part B) no hand-off", teamu(k_team<512, 0, 0, 2, 2>, 2, 256));
  }
  if (part == 8) {
    printf("== part H: K1's access shape (config 2: 524288 chirps of 4 KiB in and out; frac on K1's 4.30 GB)\n");
    const long nch = 4096L * 128;
    const double k1b = 4096.0 * 1050624 / 1e9;
    auto rk = [&](const char* nm, float ms) { printf("%-40s %.3f ms  frac %.3f\n", nm, ms, k1b / ms / 8.0); };
    rk("8-byte lanes, cpt 16, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<8, 16, 1>), dim3(nch / 128), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("16-byte lanes, cpt 16, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<16, 16, 1>), dim3(nch / 128), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("8-byte lanes, cpt 4, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<8, 4, 1>), dim3(nch / 32), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("16-byte lanes, cpt 4, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<16, 4, 1>), dim3(nch / 32), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("8-byte lanes, cpt 1, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<8, 1, 1>), dim3(nch / 8), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("16-byte lanes, cpt 1, nt", timeit([&] { hipLaunchKernelGGL((k_k1shape<16, 1, 1>), dim3(nch / 8), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
    rk("8-byte lanes, cpt 16, plain", timeit([&] { hipLaunchKernelGGL((k_k1shape<8, 16, 0>), dim3(nch / 128), dim3(256), 0, 0, (const char*)iq, rd, nch); }));
  }
  if (part == 9) {
    printf("== part I: k_rdx's protocol with a deeper poll lag (the unit polled was published LAGP steps earlier)\n");
    rb("frame, lag 1, 2 slots (part F)", teamd(k_team_def<256, 1, 2>, 256));
    rb("frame, lag 2, 4 slots", teamd(k_team_def<256, 2, 4>, 256));
    rb("half, lag 1, 2 slots", teamd(k_team_def<128, 1, 2>, 128));
    rb("half, lag 2, 4 slots", teamd(k_team_def<128, 2, 4>, 128));
    rb("quarter, lag 2, 4 slots", teamd(k_team_def<64, 2, 4>, 64));
    rb("quarter, lag 3, 6 slots", teamd(k_team_def<64, 3, 6>, 64));
    rb("quarter, lag 4, 8 slots", teamd(k_team_def<64, 4, 8>, 64));
    rb("eighth, lag 4, 8 slots", teamd(k_team_def<32, 4, 8>, 32));
  }
  auto teamx = [&](auto kern, int UCv) {
    return timeit([&] {
      CK(hipMemsetAsync(ctr, 0, 8192 * 4));
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, (const char*)iq, cube, rd, ctr, F * 256 / UCv, err);
    }, 5);
  };
  if (part == 10) {
    printf("== part J: slot reuse by done counters (NS slots; NS = 1: written and read in one step)\n");
    rb("frame, lag 1, 2 slots (part F)", teamd(k_team_def<256, 1, 2>, 256));
    rb("frame, done, 1 slot", teamx(k_team_done<256, 1>, 256));
    rb("frame, done, 2 slots", teamx(k_team_done<256, 2>, 256));
    rb("half, done, 1 slot", teamx(k_team_done<128, 1>, 128));
    rb("half, done, 2 slots", teamx(k_team_done<128, 2>, 128));
    rb("half, done, 3 slots", teamx(k_team_done<128, 3>, 128));
    rb("quarter, done, 2 slots", teamx(k_team_done<64, 2>, 64));
    rb("quarter, done, 4 slots", teamx(k_team_done<64, 4>, 64));
  }
  if (part == 12) {
    printf("== part L: role split (16 range members, 16 Doppler members per XCD; NS frames of ring)\n");
    rb("frame, lag 1, 2 slots (part F)", teamd(k_team_def<256, 1, 2>, 256));
    rb("roles, 2 slots", teamx(k_team_role<2>, 256));
    rb("roles, 3 slots", teamx(k_team_role<3>, 256));
    rb("roles, 4 slots", teamx(k_team_role<4>, 256));
  }
  if (part == 13) {
    printf("== part M: k_rdx's protocol under a VALU burn (v_pk_fma_f32 per wave and frame step; k_rdx: ~1,000 VALU)\n");
    rb("frame, lag 1, 2 slots, burn 0", teamd(k_team_def<256, 1, 2, 1, 0>, 256));
    rb("half, lag 2, 4 slots, burn 0", teamd(k_team_def<128, 2, 4, 1, 0>, 128));
    rb("frame, lag 1, 2 slots, burn 768", teamd(k_team_def<256, 1, 2, 1, 768>, 256));
    rb("half, lag 2, 4 slots, burn 768", teamd(k_team_def<128, 2, 4, 1, 768>, 128));
    rb("frame, lag 1, 2 slots, burn 1536", teamd(k_team_def<256, 1, 2, 1, 1536>, 256));
    rb("half, lag 2, 4 slots, burn 1536", teamd(k_team_def<128, 2, 4, 1, 1536>, 128));
  }
  if (part == 14) {
    printf("== part M2: the same under a toggling burn (u = -u/2 + random samples)\n");
    rb("frame, lag 1, 2 slots, tburn 384", teamd(k_team_def<256, 1, 2, 1, 384, 1>, 256));
    rb("half, lag 2, 4 slots, tburn 384", teamd(k_team_def<128, 2, 4, 1, 384, 1>, 128));
    rb("frame, lag 1, 2 slots, tburn 768", teamd(k_team_def<256, 1, 2, 1, 768, 1>, 256));
    rb("half, lag 2, 4 slots, tburn 768", teamd(k_team_def<128, 2, 4, 1, 768, 1>, 128));
    rb("frame, lag 1, 2 slots, tburn 1152", teamd(k_team_def<256, 1, 2, 1, 1152, 1>, 256));
    rb("half, lag 2, 4 slots, tburn 1152", teamd(k_team_def<128, 2, 4, 1, 1152, 1>, 128));
  }
  if (part == 11) {
    printf("== part K: k_rdx's protocol at fp16-storage bytes (input, RD and slots halved; frac on 8.6 GB)\n");
    auto rh = [&](const char* nm, float ms) { printf("%-44s %.3f ms  frac %.3f (fp16 bytes)\n", nm, ms, algo / 2 / ms / 8.0); };
    rh("frame, lag 1, 2 slots, fp16 bytes", teamd(k_team_def<256, 1, 2, 2>, 256));
    rh("frame, lag 2, 4 slots, fp16 bytes", teamd(k_team_def<256, 2, 4, 2>, 256));
    rb("frame, lag 1, 2 slots, fp32 bytes (part F)", teamd(k_team_def<256, 1, 2>, 256));
  }
  if (part == 7) {
    printf("== part G: the hand-off ring's memory type (CUBE_ALLOC=%d)\n", calloc_flag);
    rb("frame unit, full (part B protocol)", teamu(k_team<512, 0, 1, 2, 2>, 2, 256));
    rb("frame unit, deferred group (part F protocol)", teamd(k_team_def<256>, 256));
    rb("half unit, deferred group", teamd(k_team_def<128>, 128));
  }
  if (part == 0 || part == 3) {
    printf("== part C: a region rewritten in place, 16-B stores (WRITE_SIZE per byte from the pmc pass)\n");
    for (int region : {32 * 1024, 128 * 1024}) {   // per CU: 1 / 4 MiB per XCD
      const int passes = 64;
      const double bytes = 256.0 * region * passes;
      auto rw = [&](const char* nm, float ms) { printf("region %4d KiB/CU %-10s %.3f ms  %.2f TB/s stored (%.3f GB)\n", region / 1024, nm, ms, bytes / ms / 1e9, bytes / 1e9); };
      rw("plain", timeit([&] { hipLaunchKernelGGL((k_rewrite<0>), dim3(256), dim3(512), 0, 0, cube, region, passes); }));
      rw("sc0", timeit([&] { hipLaunchKernelGGL((k_rewrite<1>), dim3(256), dim3(512), 0, 0, cube, region, passes); }));
      rw("nt", timeit([&] { hipLaunchKernelGGL((k_rewrite<2>), dim3(256), dim3(512), 0, 0, cube, region, passes); }));
      rw("sc1", timeit([&] { hipLaunchKernelGGL((k_rewrite<16>), dim3(256), dim3(512), 0, 0, cube, region, passes); }));
    }
  }
  return 0;
}
