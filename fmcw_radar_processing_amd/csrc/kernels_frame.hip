// kernels_frame.hip -- per-frame stages of the FMCW path on gfx950.
//
//   k_range    (K1)  radar_processing.m:203-205 (+:207 store, +:210 profile in
//                    range-only mode): calibration subtract, IF scale, per-chirp
//                    mean removal, 2*blackman window, Nr-point range FFT.
//   k_doppler  (K2)  :210/:265 range profile (max over chirps) and :216-219
//                    Doppler mean removal, 2*chebwin window, Nd-point FFT
//                    (truncating when Nd < PN), fftshift -- for every range row.
//   k_detect   (K3)  :211 f_search_peak rule, :227-239 Doppler
//                    index with threshold/fallback, :257-259 slow-time row,
//                    :410-411 probe column.
//
// HBM layouts (C order, last index fastest):
//   iq    [frame][chirp][sample]   complex (MATLAB cat(3, frame.Chirp(:,:,1)))
//   cube  [frame][chirp][range]    complex (= range_tx1rx1_complete, Nr x PN x F)
//   rd    [frame][range][doppler]  complex, fftshift-ed along doppler
//   prof  [frame][range]           float  (= range_tx1rx1_max_abs, Nr x F)
#include "frame_ops.h"
#include "../../include/fmcw.h"

#include <climits>
#include <cstdlib>

namespace fmcw {

// ---------------------------------------------------------------------------
// K1: fast-time conditioning + range FFT.  One team of T = Nr/16 threads per
// chirp; a 256-thread workgroup holds 256/T teams; each team walks `cpt`
// consecutive chirps.  Thread t loads samples t + T*m (coalesced), keeps them
// in registers through the FFT and stores range bins t + T*m (coalesced).
//
// Streaming: the {cal, IF*w} taps sit in LDS (loaded once per workgroup); three
// workgroups per CU (3 waves per SIMD) keep loads in flight while other waves
// transform (K1_PREFETCH: the round-3 form, the next chirp's samples requested
// before this chirp's FFT, at 2 waves per SIMD).
// ---------------------------------------------------------------------------
// Occupancy over prefetch (config 2, 4096 frames, one box, 3 alternating rounds,
// tools/gpu_k1ab.sh): no register prefetch at 3 waves per SIMD (<= 168 VGPRs) 824-827 us;
// the round-3 register prefetch of the next chirp at 2 waves per SIMD 846-849 us; that
// prefetch squeezed into 3 waves per SIMD spills (1637 us).  K1_PREFETCH=1 restores it (A/B).
#ifndef K1_WAVES
#ifdef K1_PREFETCH
#define K1_WAVES 2
#else
#define K1_WAVES 3
#endif
#endif
template <int NR, typename TIn, typename TCube, bool PROFILE>
__global__ __launch_bounds__(256, NR >= 2048 ? 2 : K1_WAVES) void k_range(RangeArgs a) {   // Nr 2048: LDS allows 2
  using Plan = FftPlan<NR>;
  constexpr int P = Plan::P, T = Plan::T;
  constexpr int TEAMS = T >= 256 ? 1 : 256 / T;
  constexpr int LDSN = Plan::STRIDE > 0 ? Plan::STRIDE : 1;
  __shared__ float2 lds[TEAMS * LDSN];
  __shared__ float2 red[TEAMS * (T > 64 ? T / 64 : 1)];
  const int nmax = a.S < NR ? a.S : NR;
#ifdef K1_TAPS_GLOBAL   // A/B: taps read through the L1 from global memory (no per-workgroup LDS prologue)
  const float4* taps = a.calw;
#else
  __shared__ float4 taps[NR];
  {
    constexpr int TP = (NR + 255) / 256;                       // taps per thread, loads issued together
    float4 tp[TP];
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int i = threadIdx.x + 256 * j;
      tp[j] = a.calw[i < nmax ? i : 0];
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < nmax) taps[i] = tp[j];
    }
  }
  __syncthreads();
#endif

  const int team = threadIdx.x / T, t0 = team_index<T>(threadIdx.x % T);   // bank-conflict-free LDS stores
  float2* my = lds + team * LDSN;
  float2* myred = red + team * (T > 64 ? T / 64 : 1);
  const TIn* __restrict__ in = static_cast<const TIn*>(a.iq);
  TCube* __restrict__ out = static_cast<TCube*>(a.cube);
  const int64_t g0 = ((int64_t)blockIdx.x * TEAMS + team) * a.cpt;

  float pm[PROFILE ? P : 1];
#pragma unroll
  for (int m = 0; m < (PROFILE ? P : 1); ++m) pm[m] = 0.f;

  float2 cur[P];
#ifdef K1_GLDS
  // A/B (round 6): the next chirp of every team of the wave is brought into a wave-private LDS buffer by
  // LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction) while this chirp is transformed, so its
  // bytes are in flight without registers; the twiddles are read from an LDS copy (an ordinary global load
  // behind an LDS-DMA would make the compiler drain it).  Full chirps of c64 samples only (S == NR, 128 <=
  // NR <= 1024: a chirp is whole 1 KiB pieces and a team lives in one wave).
  constexpr bool kGlds = std::is_same_v<TIn, float2> && NR >= 128 && NR <= 1024;
  constexpr int kPiece = NR >= 128 ? NR / 128 : 1;             // 1 KiB pieces per chirp
  __shared__ __attribute__((aligned(16))) float2 pf[kGlds ? 4 * 64 * P : 1];
  __shared__ float2 twl[kGlds ? NR : 1];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, tiw = (threadIdx.x & 63) / T;   // team in the wave
  const bool glds = kGlds && a.S == NR;
  auto glds_issue = [&](int c) __attribute__((always_inline)) {   // chirp c of every team of this wave
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) {
      const int s = pc / kPiece;                                // wave-uniform: the piece's team
      const int64_t gs = ((int64_t)blockIdx.x * TEAMS + wv * (64 / T) + s) * a.cpt + c;
      const float2* src = reinterpret_cast<const float2*>(in) + (gs < a.nchirps ? gs : 0) * a.S + (pc % kPiece) * 128 + 2 * ln;
      // as inline asm: hipcc's own bookkeeping of a builtin LDS-DMA waits vmcnt(0) before every ds_read of the
      // FFT (it cannot tell pf from the exchange buffer), draining the prefetch; the waits here are explicit
      typedef __attribute__((address_space(3))) float2 lf2;
      const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lf2*)&pf[wv * 64 * P + pc * 128]);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    }
  };
  if constexpr (kGlds) {
    if (glds) {
      for (int i = threadIdx.x; i < NR; i += 256) twl[i] = a.tw[i];
      __syncthreads();
      glds_issue(0);
    }
  }
  if (!glds)
#endif
  chirp_load<NR>(in + (g0 < a.nchirps ? g0 : 0) * a.S, g0 < a.nchirps, nmax, t0, cur);
#ifdef K1_GLDS
  // a loop of its own: sharing the register-load loop would make the compiler wait for that path's
  // (never pending) chirp loads before every ds_read into the same registers
  if (kGlds && glds) {
    for (int c = 0; c < a.cpt; ++c) {
      const int64_t g = g0 + c;
      const bool valid = g < a.nchirps;
      int t = t0;
      asm volatile("" : "+v"(t));
      float2 tb[FftPasses<NR>::NB];
      // chirp c's DMA is the oldest VMEM operation after the previous chirp's stores (P of them when that
      // chirp was valid): wait for it, read this thread's samples, retire the reads, then reuse the buffer
      if (c > 0 && g - 1 < a.nchirps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      load_tw_bases<NR>(tb, t, twl);
#pragma unroll
      for (int m = 0; m < P; ++m) cur[m] = pf[wv * 64 * P + tiw * NR + t + T * m];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (c + 1 < a.cpt) glds_issue(c + 1);
      chirp_finish<NR>(cur, in + (valid ? g : 0) * a.S, valid, out + g * NR, a.S, taps, a.cal_sum, a.cube_scale, tb,
                       my, myred, t);
      if constexpr (PROFILE) {
#pragma unroll
        for (int m = 0; m < P; ++m) pm[m] = fmaxf(pm[m], cabs2(cur[m]));
      }
    }
  } else
#endif
  for (int c = 0; c < a.cpt; ++c) {
    const int64_t g = g0 + c;
    const bool valid = g < a.nchirps;
    // Opaque copy of the lane index: stops the compiler hoisting the per-lane
    // LDS addresses and twiddle products of every pass out of the chirp loop
    // (that hoisting costs ~100 VGPRs and halves occupancy).
    int t = t0;
    asm volatile("" : "+v"(t));
    float2 tb[FftPasses<NR>::NB];
    const bool vn = (c + 1 < a.cpt) && (g + 1 < a.nchirps);
    load_tw_bases<NR>(tb, t, a.tw);                            // before the prefetch below
#ifndef K1_PREFETCH   // the next chirp is loaded after this one's stores; the other waves of the SIMD cover it
    chirp_finish<NR>(cur, in + (valid ? g : 0) * a.S, valid, out + g * NR, a.S, taps, a.cal_sum, a.cube_scale, tb,
                     my, myred, t);
    if constexpr (PROFILE) {
#pragma unroll
      for (int m = 0; m < P; ++m) pm[m] = fmaxf(pm[m], cabs2(cur[m]));
    }
    chirp_load<NR>(in + (vn ? g + 1 : 0) * a.S, vn, nmax, t, cur);
#else
    float2 nxt[P];
    chirp_load<NR>(in + (vn ? g + 1 : 0) * a.S, vn, nmax, t, nxt);
    chirp_finish<NR>(cur, in + (valid ? g : 0) * a.S, valid, out + g * NR, a.S, taps, a.cal_sum, a.cube_scale, tb,
                     my, myred, t);
    if constexpr (PROFILE) {
#pragma unroll
      for (int m = 0; m < P; ++m) pm[m] = fmaxf(pm[m], cabs2(cur[m]));
    }
#pragma unroll
    for (int m = 0; m < P; ++m) cur[m] = nxt[m];
#endif
  }
  if constexpr (PROFILE) {                                     // :210 max over chirps
    constexpr bool kLdsCombine = Plan::STRIDE > 0 && (size_t)TEAMS * NR * 4 <= sizeof(lds);
    if constexpr (kLdsCombine) {
      // The block's teams combine their maxima in LDS (the FFT exchange region is free after the
      // chirp loop): one plain store per (frame, bin) when the block's teams hold the whole frame
      // (config 2: 8 teams x 16 chirps = 128), else one atomicMax per block and bin -- not one per
      // team and bin (16.8 M atomics per config-2 launch).
      __syncthreads();
      float* pl = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int m = 0; m < P; ++m) pl[team * NR + t0 + T * m] = pm[m];
      __syncthreads();
      const int64_t gb = (int64_t)blockIdx.x * TEAMS * a.cpt;   // the block's first chirp
      for (int b = threadIdx.x; b < NR; b += 256) {
        float acc = 0.f;
        int64_t fcur = -1;
        int nteam = 0;
        for (int i = 0; i <= TEAMS; ++i) {
          const int64_t gi = gb + (int64_t)i * a.cpt;
          const bool vi = i < TEAMS && gi < a.nchirps;
          const int64_t fi = vi ? gi / a.C : -2;
          if (fi != fcur && fcur >= 0) {                      // flush the previous frame's group
            float* dst = a.profile + fcur * NR + b;
            const int64_t span = (int64_t)nteam * a.cpt;      // chirps of frame fcur in this block
            if (span == a.C) {
              *dst = sqrtf(acc);                              // the whole frame: this block alone
            } else if (a.parts > 1 && span * a.parts == a.C) {
              // one of the frame's `parts` equal workgroups: its maximum goes to its own slot
              const int64_t g_start = gb + (int64_t)(i - nteam) * a.cpt;   // the group's first chirp
              const int64_t part = (g_start - fcur * a.C) / span;
              a.prof_part[(fcur * a.parts + part) * NR + b] = sqrtf(acc);
            } else {
              atomicMax(reinterpret_cast<unsigned*>(dst), __float_as_uint(sqrtf(acc)));
            }
            acc = 0.f;
            nteam = 0;
          }
          if (!vi) break;
          fcur = fi;
          acc = fmaxf(acc, pl[i * NR + b]);
          ++nteam;
        }
      }
    } else {
      if (g0 >= a.nchirps) return;
      const int64_t f = g0 / a.C;
      unsigned* pb = reinterpret_cast<unsigned*>(a.profile) + f * NR;
#pragma unroll
      for (int m = 0; m < P; ++m) atomicMax(pb + t0 + T * m, __float_as_uint(sqrtf(pm[m])));
    }
  }
}

// profile[f][b] = max over K1's per-workgroup maxima of frame f (cpt chosen so that several
// workgroups share a frame: plain stores there, this reduction instead of atomics)
__global__ __launch_bounds__(256) void k_profile_reduce(const float* __restrict__ part, int parts, int64_t n, int nr,
                                                        float* __restrict__ profile) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t f = i / nr, b = i - f * nr;
    const float* p = part + f * parts * (int64_t)nr + b;
    float m = p[0];
    for (int q = 1; q < parts; ++q) m = fmaxf(m, p[(int64_t)q * nr]);
    profile[i] = m;
  }
}

hipError_t launch_profile_reduce(const float* part, int parts, int64_t frames, int nr, float* profile, hipStream_t s) {
  const int64_t n = frames * nr;
  if (n <= 0) return hipSuccess;
  int64_t b = (n + 1023) / 1024;
  if (b > 65536) b = 65536;
  hipLaunchKernelGGL(k_profile_reduce, dim3((unsigned)b), dim3(256), 0, s, part, parts, n, nr, profile);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K2: range profile + Doppler FFT for every range row; a workgroup owns RB
// consecutive rows of one frame (doppler_tile in frame_ops.h).
// ---------------------------------------------------------------------------
template <int ND, typename TCube, typename TRd, bool PAIR>
__global__ __launch_bounds__(256) void k_doppler(DopplerArgs a) {
  using L = DopplerLds<ND, PAIR>;
  __shared__ __attribute__((aligned(16))) float2 lds[L::N];
  __shared__ float2 red_s[256];
  __shared__ float red_m[256];
  const int tiles = (a.NR + L::RB - 1) / L::RB;
  const int f = blockIdx.x / tiles, tile = blockIdx.x - f * tiles;
  doppler_tile<ND, PAIR, false>(static_cast<const TCube*>(a.cube) + (int64_t)f * a.C * a.NR, a.C, a.NR,
                                tile * L::RB, a.cube_unscale, a.wd, a.tw,
                                static_cast<TRd*>(a.rd) + (int64_t)f * a.NR * a.ND, a.rd_scale,
                                a.profile + (int64_t)f * a.NR, lds, red_s, red_m, threadIdx.x);
}

// ---------------------------------------------------------------------------
// K3: detection, one wave per frame (detect_frame in frame_ops.h).
// ---------------------------------------------------------------------------
template <int NR, typename TRd, typename TCube>
__global__ __launch_bounds__(256) void k_detect(DetectArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f = (int64_t)blockIdx.x * 4 + w;
  if (f >= a.nframes) return;            // wave-uniform exit; no block barriers below
  DetectParams q{a.ND, a.C, a.M, a.range_thr, a.doppler_thr, a.min_d, a.max_d, a.dist_per_bin, a.fallback,
                 a.cube_unscale, a.rd_unscale};
  detect_frame<NR, false>(q, lane, a.profile + f * NR, static_cast<const TRd*>(a.rd) + f * NR * (int64_t)a.ND,
                          static_cast<const TCube*>(a.cube) + f * a.C * (int64_t)NR, a.count + f, a.ridx + f * a.M,
                          a.rmag + f * a.M, a.didx + f * a.M, a.slow_mag + f * a.C, f == a.probe_frame,
                          a.probe_chirp, a.probe_mag);
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
// 16-byte lane-pair access in K2 (FMCW_PAIR=1).  Off by default: on MI355X the
// 8-byte cyclic path measured slightly faster.
static bool pair_access_enabled() {
  const char* e = getenv("FMCW_PAIR");
  return e && e[0] == '1';
}
template <int NR, typename TIn, typename TCube>
static hipError_t go_range(const RangeArgs& a, hipStream_t s) {
  constexpr int T = FftPlan<NR>::T;
  constexpr int TEAMS = T >= 256 ? 1 : 256 / T;
  const int64_t per_block = (int64_t)TEAMS * a.cpt;
  const int64_t blocks = (a.nchirps + per_block - 1) / per_block;
  if (a.profile) hipLaunchKernelGGL((k_range<NR, TIn, TCube, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_range<NR, TIn, TCube, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int NR>
static hipError_t go_range_t(const RangeArgs& a, hipStream_t s) {
  if (a.in_dtype == FMCW_C64 && a.cube_dtype == FMCW_C64) return go_range<NR, float2, float2>(a, s);
  if (a.in_dtype == FMCW_C32H && a.cube_dtype == FMCW_C64) return go_range<NR, __half2, float2>(a, s);
  if (a.in_dtype == FMCW_C32H && a.cube_dtype == FMCW_C32H) return go_range<NR, __half2, __half2>(a, s);
  if (a.in_dtype == FMCW_C64 && a.cube_dtype == FMCW_C32H) return go_range<NR, float2, __half2>(a, s);
  return hipErrorInvalidValue;
}

bool range_size_supported(int nr) { return nr >= 16 && nr <= 2048 && (nr & (nr - 1)) == 0; }
bool doppler_size_supported(int nd) { return nd >= 2 && nd <= 1024 && (nd & (nd - 1)) == 0; }

hipError_t launch_range(const RangeArgs& a, hipStream_t s) {
  if (a.nchirps <= 0) return hipSuccess;
  switch (a.NR) {
    case 16: return go_range_t<16>(a, s);
    case 32: return go_range_t<32>(a, s);
    case 64: return go_range_t<64>(a, s);
    case 128: return go_range_t<128>(a, s);
    case 256: return go_range_t<256>(a, s);
    case 512: return go_range_t<512>(a, s);
    case 1024: return go_range_t<1024>(a, s);
    case 2048: return go_range_t<2048>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int ND, typename TCube, typename TRd>
static hipError_t go_doppler(const DopplerArgs& a, hipStream_t s) {
  constexpr int RB = 256 / FftPlan<ND>::T;
  const int tiles = (a.NR + RB - 1) / RB;
  const int64_t blocks = (int64_t)tiles * a.nframes;
  if (pair_access_enabled())
    hipLaunchKernelGGL((k_doppler<ND, TCube, TRd, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_doppler<ND, TCube, TRd, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int ND>
static hipError_t go_doppler_t(const DopplerArgs& a, hipStream_t s) {
  if (a.cube_dtype == FMCW_C64 && a.rd_dtype == FMCW_C64) return go_doppler<ND, float2, float2>(a, s);
  if (a.cube_dtype == FMCW_C64 && a.rd_dtype == FMCW_C32H) return go_doppler<ND, float2, __half2>(a, s);
  if (a.cube_dtype == FMCW_C32H && a.rd_dtype == FMCW_C32H) return go_doppler<ND, __half2, __half2>(a, s);
  if (a.cube_dtype == FMCW_C32H && a.rd_dtype == FMCW_C64) return go_doppler<ND, __half2, float2>(a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_doppler(const DopplerArgs& a, hipStream_t s) {
  if (a.nframes <= 0) return hipSuccess;
  switch (a.ND) {
    case 2: return go_doppler_t<2>(a, s);
    case 4: return go_doppler_t<4>(a, s);
    case 8: return go_doppler_t<8>(a, s);
    case 16: return go_doppler_t<16>(a, s);
    case 32: return go_doppler_t<32>(a, s);
    case 64: return go_doppler_t<64>(a, s);
    case 128: return go_doppler_t<128>(a, s);
    case 256: return go_doppler_t<256>(a, s);
    case 512: return go_doppler_t<512>(a, s);
    case 1024: return go_doppler_t<1024>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int NR>
static hipError_t go_detect(const DetectArgs& a, hipStream_t s) {
  const unsigned blocks = (unsigned)((a.nframes + 3) / 4);
  if (a.rd_dtype == FMCW_C64 && a.cube_dtype == FMCW_C64)
    hipLaunchKernelGGL((k_detect<NR, float2, float2>), dim3(blocks), dim3(256), 0, s, a);
  else if (a.rd_dtype == FMCW_C32H && a.cube_dtype == FMCW_C64)
    hipLaunchKernelGGL((k_detect<NR, __half2, float2>), dim3(blocks), dim3(256), 0, s, a);
  else if (a.rd_dtype == FMCW_C32H && a.cube_dtype == FMCW_C32H)
    hipLaunchKernelGGL((k_detect<NR, __half2, __half2>), dim3(blocks), dim3(256), 0, s, a);
  else if (a.rd_dtype == FMCW_C64 && a.cube_dtype == FMCW_C32H)
    hipLaunchKernelGGL((k_detect<NR, float2, __half2>), dim3(blocks), dim3(256), 0, s, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_detect(const DetectArgs& a, hipStream_t s) {
  if (a.nframes <= 0) return hipSuccess;
  switch (a.NR) {
    case 16: return go_detect<16>(a, s);
    case 32: return go_detect<32>(a, s);
    case 64: return go_detect<64>(a, s);
    case 128: return go_detect<128>(a, s);
    case 256: return go_detect<256>(a, s);
    case 512: return go_detect<512>(a, s);
    case 1024: return go_detect<1024>(a, s);
    case 2048: return go_detect<2048>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fmcw
