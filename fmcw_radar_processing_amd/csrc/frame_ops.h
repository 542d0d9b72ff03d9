// frame_ops.h -- per-frame stage bodies of the streams schedule
// (kernels_frame.hip: K1/K2/K3 launched as a 3-stream chunk pipeline); the
// peak rule is shared with the single pass (kernels_onepass.hip).
//
//   range_team     radar_processing.m:203-205 (+:207 store): one chirp per team
//   doppler_tile   :210/:265 profile, :216-219 Doppler (mean over all PN,
//                  2*chebwin, fft(., Nd, 2) truncating, fftshift) for RB rows
//   detect_frame   :211 f_search_peak rule, :227-239 Doppler
//                  index, :257-259 slow-time row, :410-411 probe column
//
// Load policy NT (template flag): `nt` loads bypass the CU's vector L1 and are
// served by the XCD's L2 (MI355X_MICROARCH.md, visibility table).  The
// stand-alone kernels read data written by an earlier launch and use plain loads.
#pragma once
#include <type_traits>
#include <climits>

#include "fft_team.h"
#include "fmcw_internal.h"

namespace fmcw {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT> __device__ __forceinline__ float2 ldp(const float2* p, int64_t i) {
  if constexpr (NT) {
    const f2v v = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p + i));
    return make_float2(v.x, v.y);
  } else {
    return p[i];
  }
}
template <bool NT> __device__ __forceinline__ float2 ldp(const __half2* p, int64_t i) {
  if constexpr (NT) {
    const unsigned v = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p + i));
    return __half22float2(*reinterpret_cast<const __half2*>(&v));
  } else {
    return __half22float2(p[i]);
  }
}
template <bool NT> __device__ __forceinline__ float ldf(const float* p, int64_t i) {
  if constexpr (NT) return __builtin_nontemporal_load(p + i);
  else return p[i];
}

// Sum over aligned groups of W lanes (W = 2..64) by DPP and the half-wave swaps -- no
// LDS (a __shfl_xor is a ds_bpermute through the LDS crossbar).  xor 1, xor 2, then
// the row mirrors on group-uniform values (xor 4, xor 8), then the 16- and 32-lane
// swaps; symmetric pairings, so every lane of a group gets the same bits.
template <int W> __device__ __forceinline__ float group_sum(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, true));
  };
  if constexpr (W >= 2) v += dpp(v, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
  if constexpr (W >= 4) v += dpp(v, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
  if constexpr (W >= 8) v += dpp(v, std::integral_constant<int, 0x141>{});   // row_half_mirror
  if constexpr (W >= 16) v += dpp(v, std::integral_constant<int, 0x140>{});  // row_mirror
  if constexpr (W >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if constexpr (W >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return v;
}

// team-wide sum of a complex value over T threads that are consecutive lanes
template <int T>
__device__ __forceinline__ float2 team_sum(float2 s, float2* red, int t) {
  constexpr int W = T < 64 ? T : 64;
  s.x = group_sum<W>(s.x);
  s.y = group_sum<W>(s.y);
  if constexpr (T > 64) {
    // teams span T/64 waves (T = 128 for Nr = 2048): combine through LDS
    if ((t & 63) == 0) red[t >> 6] = s;
    __syncthreads();
    float2 r = red[0];
#pragma unroll
    for (int i = 1; i < T / 64; ++i) r = cadd(r, red[i]);
    __syncthreads();
    return r;
  } else {
    return s;
  }
}

// ---------------------------------------------------------------------------
// range_team: one chirp by one team of T = Nr/16 threads (K1 body).
// x: the chirp's S samples (a readable address even when `valid` is false);
// o: its Nr range bins.  `valid` false keeps the team in lock-step (barriers)
// without stores.  Leaves the spectrum in v (cyclic layout) for the caller's
// profile accumulation.
//
// Every global load of the chirp -- samples and the {cal, IF*w} taps -- is
// issued branch-free (clamped index, value selected afterwards) before the
// first use, so a chirp costs ONE memory round trip; guarding each load with
// `if` makes the compiler wait after every load (16 serial trips).
// ---------------------------------------------------------------------------
template <int NR, bool PAIR, typename TIn, typename TCube>
__device__ __forceinline__ void range_team(const TIn* __restrict__ x, bool valid, TCube* __restrict__ o, int S,
                                           const float4* __restrict__ calw, float2 cal_sum, float if_scale,
                                           float cube_scale, const float2* __restrict__ tw, float2* my,
                                           float2* myred, int t, float2 (&v)[FftPlan<NR>::P]) {
  using Plan = FftPlan<NR>;
  constexpr int P = Plan::P, T = Plan::T;
  using Sync = typename TeamSync<T>::type;
  const int nmax = S < NR ? S : NR;      // fft(x, Nr): zero-pad (S < Nr) or truncate (S > Nr)
  const bool odd = (t & 1) != 0;
  (void)if_scale;
  if constexpr (PAIR) {
    // 16-byte loads: lane pair (2i, 2i+1) reads samples 2i, 2i+1 of blocks 2j
    // and 2j+1 (T samples each), then swaps one element (pair_xchg)
#pragma unroll
    for (int j = 0; j < P / 2; ++j) {
      const int e0 = T * (2 * j + (t & 1)) + 2 * (t >> 1);
      const bool ok = valid && e0 < nmax;                    // nmax even: e0+1 < nmax too
      float2 u0, u1;
      ld_c2(x, ok ? e0 : 0, u0, u1);
      if (!ok) u0 = u1 = make_float2(0.f, 0.f);
      pair_xchg(odd, u0, u1);
      v[2 * j] = u0;
      v[2 * j + 1] = u1;
    }
  } else {
#pragma unroll
    for (int m = 0; m < P; ++m) {
      const int n = t + T * m;
      v[m] = ld_c(x, (valid && n < nmax) ? n : 0);
    }
  }
  // taps {cal.re, cal.im, IF_scale*w}: issued with the samples
  float cr[P], ci[P], cw[P];
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int n = t + T * m;
    const float* cp = reinterpret_cast<const float*>(calw + (n < nmax ? n : 0));
    cr[m] = cp[0];
    ci[m] = cp[1];
    cw[m] = cp[2];
  }
  float2 s = make_float2(0.f, 0.f);
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int n = t + T * m;
    if (!(valid && n < nmax)) v[m] = make_float2(0.f, 0.f);
    s = cadd(s, v[m]);
  }
  if (S > NR && valid) {                                     // samples beyond Nr still enter the mean
    for (int n = NR + t; n < S; n += T) s = cadd(s, ld_c(x, n));
  }
  s = team_sum<T>(s, myred, t);
  // :203-205  ((x - cal)*IF - mean((x - cal)*IF)) .* w  ==  (x - cal - mu) * (IF*w),
  // mu = mean(x - cal) over all S samples
  const float2 mu = cscale(csub(s, cal_sum), 1.0f / (float)S);
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int n = t + T * m;
    const float2 d = make_float2(v[m].x - cr[m] - mu.x, v[m].y - ci[m] - mu.y);
    v[m] = n < nmax ? cscale(d, cw[m]) : make_float2(0.f, 0.f);
  }
  team_fft<NR>(v, my, t, tw, Sync{});                       // :205 fft(., Nr, 1)
  if constexpr (PAIR) {
#pragma unroll
    for (int j = 0; j < P / 2; ++j) {                        // :207, 16-byte stores
      float2 p0 = cscale(v[2 * j], cube_scale), p1 = cscale(v[2 * j + 1], cube_scale);
      pair_xchg(odd, p0, p1);
      if (valid) st_c2(o, T * (2 * j + (t & 1)) + 2 * (t >> 1), p0, p1);
    }
  } else if (valid) {
#pragma unroll
    for (int m = 0; m < P; ++m) st_c(o, t + T * m, cscale(v[m], cube_scale));    // :207
  }
}

// ---------------------------------------------------------------------------
// Streaming form of range_team for K1 (k_range): the caller keeps the next
// chirp's loads in flight while this chirp is transformed.
//   chirp_load    issues the P sample loads of one chirp (branch-free)
//   chirp_finish  mean removal, calibration (taps from LDS), window, FFT with
//                 preloaded twiddles, store.  Same arithmetic, in the same
//                 order, as range_team.
// ---------------------------------------------------------------------------
template <int NR, typename TIn>
__device__ __forceinline__ void chirp_load(const TIn* __restrict__ x, bool valid, int nmax, int t,
                                           float2 (&v)[FftPlan<NR>::P]) {
  using Plan = FftPlan<NR>;
  if (nmax == NR) {
    // whole chirp in range (S >= Nr): one base address + immediate offsets.
    // x is a readable chirp even when !valid; chirp_finish zeroes those.
    // read-once samples: `nt` loads, paired with the `nt` cube stores of chirp_finish (config 2,
    // 4096 frames: 818-833 us vs 857-872 plain; nt loads alone 908-914)
    const TIn* __restrict__ xb = x + t;
#pragma unroll
    for (int m = 0; m < Plan::P; ++m) v[m] = ldp<true>(xb, Plan::T * m);
  } else {
#pragma unroll
    for (int m = 0; m < Plan::P; ++m) {
      const int n = t + Plan::T * m;
      v[m] = ld_c(x, (valid && n < nmax) ? n : 0);
    }
  }
}

template <int NR, typename TIn, typename TCube>
__device__ __forceinline__ void chirp_finish(float2 (&v)[FftPlan<NR>::P], const TIn* __restrict__ x, bool valid,
                                             TCube* __restrict__ o, int S, const float4* taps, float2 cal_sum,
                                             float cube_scale, const float2* tb, float2* my, float2* myred, int t) {
  using Plan = FftPlan<NR>;
  constexpr int P = Plan::P, T = Plan::T;
  using Sync = typename TeamSync<T>::type;
  const int nmax = S < NR ? S : NR;
  float2 s = make_float2(0.f, 0.f);
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int n = t + T * m;
    if (!(valid && n < nmax)) v[m] = make_float2(0.f, 0.f);
    s = cadd(s, v[m]);
  }
  if (S > NR && valid) {
    for (int n = NR + t; n < S; n += T) s = cadd(s, ld_c(x, n));
  }
  s = team_sum<T>(s, myred, t);
  const float2 mu = cscale(csub(s, cal_sum), 1.0f / (float)S);
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int n = t + T * m;
    const float4 c = taps[n < nmax ? n : 0];
    const float2 d = make_float2(v[m].x - c.x - mu.x, v[m].y - c.y - mu.y);
    v[m] = n < nmax ? cscale(d, c.z) : make_float2(0.f, 0.f);
  }
#ifndef K1_NOFFT     // diagnostic builds only (tools/ab_build.sh k1nofft -DK1_NOFFT): K1's data movement without its FFT
  team_fft_pre<NR>(v, my, t, tb, Sync{});                   // :205 fft(., Nr, 1)
#endif
  if (valid) {
#pragma unroll
    for (int m = 0; m < P; ++m) {                            // :207, write-once cube: `nt` stores
      const float2 c = cscale(v[m], cube_scale);
      if constexpr (std::is_same_v<TCube, float2>)
        __builtin_nontemporal_store(f2v{c.x, c.y}, reinterpret_cast<f2v*>(o + t + T * m));
      else
        st_c(o, t + T * m, c);
    }
  }
}

// ---------------------------------------------------------------------------
// doppler_tile: RB = 256/T rows [r0, r0+RB) of one frame (K2 body, 256 threads).
// Thread (b, u) = (tid % RB, tid / RB) is member u of row b's Nd-point team.
// ---------------------------------------------------------------------------
template <int ND, bool PAIR> struct DopplerLds {
  using Plan = FftPlan<ND>;
  static constexpr int T = Plan::T, RB = 256 / T;
  static constexpr int SROW = PAIR ? ND + 2 : ND + 1;   // staging row (PAIR: 16-byte aligned)
  static constexpr int FFTL = RB * Plan::STRIDE, STGL = RB * SROW;
  static constexpr int N = FFTL > STGL ? FFTL : STGL;
};

template <int ND, bool PAIR, bool NT, typename TCube, typename TRd>
__device__ __forceinline__ void doppler_tile(const TCube* __restrict__ cube, int C, int NR, int r0,
                                             float cube_unscale, const float* __restrict__ wd,
                                             const float2* __restrict__ tw, TRd* __restrict__ rd_frame,
                                             float rd_scale, float* __restrict__ prof_frame, float2* lds,
                                             float2* red_s, float* red_m, int tid) {
  using L = DopplerLds<ND, PAIR>;
  using Plan = FftPlan<ND>;
  constexpr int P = Plan::P, T = Plan::T, RB = L::RB, SROW = L::SROW;
  static_assert(RB % 2 == 0 && P % 2 == 0, "pair access needs even tiles");
  const int b = tid % RB, u = tid / RB;
  const int r = r0 + b;
  const bool vb = r < NR;
  const bool odd = (b & 1) != 0;         // = hardware lane parity (RB even)
  const int kfft = C < ND ? C : ND;      // fft(., Nd, 2) truncates to the first Nd chirps
  const int r2 = r0 + 2 * (b >> 1);

  // All loads of the tile (cube column block + window taps) are issued
  // branch-free before the first use: one memory round trip per tile.
  float2 v[P];
  float wdv[P];
  float2 s = make_float2(0.f, 0.f);
  float pm = 0.f;
  if constexpr (PAIR && !NT) {
    // 16-byte loads: lane pair (2i, 2i+1) reads bins r2, r2+1 of chirps
    // u + T*2j (even lane) and u + T*(2j+1) (odd lane), then swaps one element
#pragma unroll
    for (int j = 0; j < P / 2; ++j) {
      const int k = u + T * (2 * j + (b & 1));
      const bool ok = r2 < NR && k < kfft;
      float2 u0, u1;
      ld_c2(cube, ok ? (int64_t)k * NR + r2 : (int64_t)r0, u0, u1);
      if (!ok) u0 = u1 = make_float2(0.f, 0.f);
      pair_xchg(odd, u0, u1);
      v[2 * j] = u0;
      v[2 * j + 1] = u1;
    }
  } else {
#pragma unroll
    for (int m = 0; m < P; ++m) {
      const int k = u + T * m;
      v[m] = ldp<NT>(cube, (vb && k < kfft) ? (int64_t)k * NR + r : (int64_t)r0);
    }
  }
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int k = u + T * m;
    wdv[m] = wd[k < kfft ? k : 0];
  }
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int k = u + T * m;
    const bool ok = PAIR && !NT ? k < kfft : (vb && k < kfft);
    v[m] = ok ? cscale(v[m], cube_unscale) : make_float2(0.f, 0.f);
    s = cadd(s, v[m]);
    pm = fmaxf(pm, cabs2(v[m]));
  }
  if (C > ND && vb) {                    // chirps beyond Nd: profile and mean only
    for (int k = ND + u; k < C; k += T) {
      const float2 x = cscale(ldp<NT>(cube, (int64_t)k * NR + r), cube_unscale);
      s = cadd(s, x);
      pm = fmaxf(pm, cabs2(x));
    }
  }
  red_s[tid] = s;
  red_m[tid] = pm;
  __syncthreads();
  if (u == 0) {
#pragma unroll 4
    for (int i = 1; i < T; ++i) {
      s = cadd(s, red_s[b + RB * i]);
      pm = fmaxf(pm, red_m[b + RB * i]);
    }
    red_s[b] = s;
    if (vb) prof_frame[r] = sqrtf(pm);                       // :210 / :265 abs(max(X,[],2))
  }
  __syncthreads();
  const float2 mean = cscale(red_s[b], 1.0f / (float)C);    // :217 mean over ALL chirps
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int k = u + T * m;
    v[m] = (k < kfft) ? cscale(csub(v[m], mean), wdv[m]) : make_float2(0.f, 0.f);  // :218-219
  }
  team_fft<ND>(v, lds + b * Plan::STRIDE, u, tw, BlockSync{}); // :219 fft(., Nd, 2)
  __syncthreads();
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int e = u + T * m;
    lds[b * SROW + ((e + ND / 2) & (ND - 1))] = v[m];        // :219 fftshift(., 2)
  }
  __syncthreads();
  const int nrows = (NR - r0) < RB ? (NR - r0) : RB;
  TRd* __restrict__ out = rd_frame + (int64_t)r0 * ND;
  if constexpr (PAIR) {
    for (int e2 = tid; e2 < nrows * (ND / 2); e2 += 256) {   // RB whole rows, 16-byte stores
      const int e = 2 * e2, bb = e / ND, d = e & (ND - 1);
      const float4 q = *reinterpret_cast<const float4*>(&lds[bb * SROW + d]);
      st_c2(out, e, cscale(make_float2(q.x, q.y), rd_scale), cscale(make_float2(q.z, q.w), rd_scale));
    }
  } else {
    for (int e = tid; e < nrows * ND; e += 256) {
      const int bb = e / ND, d = e & (ND - 1);
      st_c(out, e, cscale(lds[bb * SROW + d], rd_scale));
    }
  }
}

// ---------------------------------------------------------------------------
// detect_frame: one wave (lane = 0..63) on one frame (K3 body).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o);
    const int oi = __shfl_xor(i, o);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// f_search_peak (radar_processing.m:211; helper absent from the reference,
// rule of SURVEY 8a a9): local maxima above range_thr inside [min_d, max_d];
// the max_targets largest, ties -> lower index.  One wave; every lane ends
// with the same sel[0..n-1] (0-based bins) and their magnitudes.
template <int NR, bool NT>
__device__ __forceinline__ int select_peaks(const DetectParams& a, int lane, const float* __restrict__ prof,
                                            int (&sel)[8], float (&selv)[8]) {
  constexpr int PPL = NR >= 64 ? NR / 64 : 1;
  const int M = a.M;
  const double dpb = a.dist_per_bin, lo = a.min_d, hi = a.max_d;
  float cv[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int i = lane + 64 * j;
    float v = -1.f;
    if (i >= 1 && i <= NR - 2) {                        // 1-based 2..Nr-1
      const double rng = (double)i * dpb;               // (idx-1)*dist_per_bin
      const float pc = ldf<NT>(prof, i), pl = ldf<NT>(prof, i - 1), pr = ldf<NT>(prof, i + 1);
      if (rng >= lo && rng <= hi && pc > a.range_thr && pc >= pl && pc > pr) v = pc;
    }
    cv[j] = v;
  }
  int n = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) { sel[q] = -1; selv[q] = 0.f; }
  for (int jt = 0; jt < M; ++jt) {
    float bv = -1.f;
    int bi = INT_MAX;
#pragma unroll
    for (int j = 0; j < PPL; ++j)
      if (cv[j] > bv) { bv = cv[j]; bi = lane + 64 * j; }   // ascending i: first max kept
    wave_argmax(bv, bi);
    if (bv < 0.f) break;                                // wave-uniform
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q == n) { sel[q] = bi; selv[q] = bv; }
#pragma unroll
    for (int j = 0; j < PPL; ++j)
      if (lane + 64 * j == bi) cv[j] = -1.f;            // exclude from the next round
    ++n;
  }
  return n;
}

// Latency-shaped: every load a lane needs in a phase is issued together
// (profile + both neighbours; then the target's Doppler row and slow-time
// row), so a frame costs two dependent memory round trips.
template <int NR, bool NT, typename TRd, typename TCube>
__device__ __forceinline__ void detect_frame(const DetectParams& a, int lane, const float* __restrict__ prof,
                                             const TRd* __restrict__ rd, const TCube* __restrict__ cube,
                                             int32_t* count, int32_t* ridx, float* rmag, int32_t* didx,
                                             float* __restrict__ slow, bool probe, int probe_chirp,
                                             float* __restrict__ probe_mag) {
  const int ND = a.ND, C = a.C, M = a.M;
  int sel[8];
  float selv[8];
  const int n = select_peaks<NR, NT>(a, lane, prof, sel, selv);
  // :257-259 slow-time row of the strongest target, from the stored cube;
  // issued before the Doppler rows so both round trips overlap
  {
    const int row = n > 0 ? sel[0] : 0;
    for (int k = lane; k < C; k += 64)
      slow[k] = n > 0 ? sqrtf(cabs2(ldp<NT>(cube, (int64_t)k * NR + row))) * a.cube_unscale : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j >= M) break;
    int di = 0, ri = 0;
    float rm = 0.f;
    if (j < n) {
      // :233 [val, idx] = max(abs(range_Doppler(tgt_range_idx(j), :)))
      const TRd* __restrict__ row = rd + (int64_t)sel[j] * ND;
      float bv = -1.f;
      int bi = INT_MAX;
      for (int d = lane; d < ND; d += 64) {
        const float mag = sqrtf(cabs2(ldp<NT>(row, d))) * a.rd_unscale;
        if (mag > bv) { bv = mag; bi = d; }
      }
      wave_argmax(bv, bi);
      di = bi + 1;
      if (!(bv >= a.doppler_thr && di != a.fallback)) di = a.fallback;   // :234-238
      ri = sel[j] + 1;
      rm = selv[j];
    }
    if (lane == 0) {
      ridx[j] = ri;
      rmag[j] = rm;
      didx[j] = di;
    }
  }
  if (lane == 0) count[0] = n;
  // :410-411 abs(range_tx1rx1_complete(:, fr_idx)) for one linear column
  if (probe && probe_mag) {
    for (int i = lane; i < NR; i += 64)
      probe_mag[i] = sqrtf(cabs2(ldp<NT>(cube, (int64_t)probe_chirp * NR + i))) * a.cube_unscale;
  }
}

}  // namespace fmcw
