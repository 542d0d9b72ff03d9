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
#include "fft_team.h"
#include "fmcw_internal.h"
#include "../../include/fmcw.h"

#include <climits>

namespace fmcw {

// ---------------------------------------------------------------------------
// team-wide sum of a complex value over T threads that are consecutive lanes
// ---------------------------------------------------------------------------
template <int T>
__device__ __forceinline__ float2 team_sum(float2 s, float2* red, int t) {
  constexpr int W = T < 64 ? T : 64;
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) {
    s.x += __shfl_xor(s.x, o);
    s.y += __shfl_xor(s.y, o);
  }
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
// K1: fast-time conditioning + range FFT.  One team of T = Nr/16 threads per
// chirp; a 256-thread workgroup holds 256/T teams; each team walks `cpt`
// consecutive chirps.  Thread t loads samples t + T*m (coalesced), keeps them
// in registers through the FFT and stores range bins t + T*m (coalesced).
// ---------------------------------------------------------------------------
template <int NR, typename TIn, typename TCube, bool PROFILE, bool PAIR>
__global__ __launch_bounds__(256, 2) void k_range(RangeArgs a) {
  using Plan = FftPlan<NR>;
  constexpr int P = Plan::P, T = Plan::T;
  constexpr int TEAMS = T >= 256 ? 1 : 256 / T;
  constexpr int LDSN = Plan::STRIDE > 0 ? Plan::STRIDE : 1;
  static_assert(!PAIR || (T % 2 == 0 && P % 2 == 0), "pair access needs an even team");
  __shared__ float2 lds[TEAMS * LDSN];
  __shared__ float2 red[TEAMS * (T > 64 ? T / 64 : 1)];

  const int team = threadIdx.x / T, t0 = threadIdx.x % T;
  float2* my = lds + team * LDSN;
  float2* myred = red + team * (T > 64 ? T / 64 : 1);
  const TIn* __restrict__ in = static_cast<const TIn*>(a.iq);
  TCube* __restrict__ out = static_cast<TCube*>(a.cube);
  const int S = a.S;
  const int nmax = S < NR ? S : NR;      // fft(x, Nr): zero-pad (S < Nr) or truncate (S > Nr)
  const float inv_s = 1.0f / (float)S;
  const int64_t g0 = ((int64_t)blockIdx.x * TEAMS + team) * a.cpt;

  float pm[PROFILE ? P : 1];
#pragma unroll
  for (int m = 0; m < (PROFILE ? P : 1); ++m) pm[m] = 0.f;
  using Sync = typename TeamSync<T>::type;

  for (int c = 0; c < a.cpt; ++c) {
    const int64_t g = g0 + c;
    const bool valid = g < a.nchirps;
    // Opaque copy of the lane index: stops the compiler hoisting the per-lane
    // LDS addresses and twiddles of every pass out of the chirp loop (that
    // hoisting costs ~100 VGPRs and halves occupancy).
    int t = t0;
    asm volatile("" : "+v"(t));
    const bool odd = (t & 1) != 0;
    const TIn* __restrict__ x = in + g * S;
    float2 v[P];
    float2 s = make_float2(0.f, 0.f);
    if constexpr (PAIR) {
      // 16-byte loads: lane pair (2i, 2i+1) reads samples 2i, 2i+1 of blocks
      // 2j and 2j+1 (T samples each), then swaps one element (pair_xchg)
#pragma unroll
      for (int j = 0; j < P / 2; ++j) {
        const int e0 = T * (2 * j + (t & 1)) + 2 * (t >> 1);
        float2 u0 = make_float2(0.f, 0.f), u1 = u0;
        if (valid && e0 < nmax) ld_c2(x, e0, u0, u1);    // nmax even: e0+1 < nmax too
        pair_xchg(odd, u0, u1);
        v[2 * j] = u0;
        v[2 * j + 1] = u1;
        s = cadd(s, cadd(u0, u1));
      }
    } else {
#pragma unroll
      for (int m = 0; m < P; ++m) {
        const int n = t + T * m;
        float2 xv = make_float2(0.f, 0.f);
        if (valid && n < nmax) xv = ld_c(x, n);
        v[m] = xv;
        s = cadd(s, xv);
      }
    }
    if (S > NR && valid) {                                     // samples beyond Nr still enter the mean
      for (int n = NR + t; n < S; n += T) s = cadd(s, ld_c(x, n));
    }
    s = team_sum<T>(s, myred, t);
    // :203-204  y = (x - cal)*IF_scale ; y -= mean(y)   (mean over all S samples)
    const float2 mean = cscale(csub(s, a.cal_sum), a.if_scale * inv_s);
#pragma unroll
    for (int m = 0; m < P; ++m) {
      const int n = t + T * m;
      if (n < nmax) {
        const float4 cw = a.calw[n];
        // :205 (.) .* w  ==  (x - cal)*(IF_scale*w) - mean*w
        const float2 d = csub(v[m], make_float2(cw.x, cw.y));
        v[m] = make_float2(fmaf(d.x, cw.z, -mean.x * cw.w), fmaf(d.y, cw.z, -mean.y * cw.w));
      } else {
        v[m] = make_float2(0.f, 0.f);
      }
    }
    team_fft<NR>(v, my, t, a.tw, Sync{});                     // :205 fft(., Nr, 1)
    if constexpr (PROFILE) {
#pragma unroll
      for (int m = 0; m < P; ++m) pm[m] = fmaxf(pm[m], cabs2(v[m]));
    }
    TCube* __restrict__ o = out + g * NR;
    if constexpr (PAIR) {
#pragma unroll
      for (int j = 0; j < P / 2; ++j) {                        // :207, 16-byte stores
        float2 p0 = cscale(v[2 * j], a.cube_scale), p1 = cscale(v[2 * j + 1], a.cube_scale);
        pair_xchg(odd, p0, p1);
        if (valid) st_c2(o, T * (2 * j + (t & 1)) + 2 * (t >> 1), p0, p1);
      }
    } else if (valid) {
#pragma unroll
      for (int m = 0; m < P; ++m) st_c(o, t + T * m, cscale(v[m], a.cube_scale));    // :207
    }
  }
  if constexpr (PROFILE) {
    if (g0 >= a.nchirps) return;                               // :210 max over chirps
    const int64_t f = g0 / a.C;
    unsigned* pb = reinterpret_cast<unsigned*>(a.profile) + f * NR;
#pragma unroll
    for (int m = 0; m < P; ++m) atomicMax(pb + t0 + T * m, __float_as_uint(sqrtf(pm[m])));
  }
}

// ---------------------------------------------------------------------------
// K2: range profile + Doppler FFT for every range row.  A workgroup owns RB
// consecutive range rows of one frame; thread (b, u) = (tid % RB, tid / RB) is
// member u of the Nd-point FFT team of row b and loads chirps u + T*m, so each
// load instruction reads RB contiguous bins of T/4 chirp rows.  The shifted
// spectrum is staged in LDS and written back as RB contiguous rows.
// ---------------------------------------------------------------------------
template <int ND, typename TCube, typename TRd>
__global__ __launch_bounds__(256) void k_doppler(DopplerArgs a) {
  using Plan = FftPlan<ND>;
  constexpr int P = Plan::P, T = Plan::T;
  constexpr int RB = 256 / T;
  constexpr int SROW = ND + 2;           // staging row: 16-byte aligned rows for float4 reads
  constexpr int FFTL = RB * Plan::STRIDE, STGL = RB * SROW;
  constexpr int LDSN = FFTL > STGL ? FFTL : STGL;
  static_assert(RB % 2 == 0 && P % 2 == 0, "pair access needs even tiles");
  __shared__ __attribute__((aligned(16))) float2 lds[LDSN];
  __shared__ float2 red_s[256];
  __shared__ float red_m[256];

  const int NR = a.NR, C = a.C;
  const int tiles = (NR + RB - 1) / RB;
  const int f = blockIdx.x / tiles, tile = blockIdx.x - f * tiles;
  const int b = threadIdx.x % RB, u = threadIdx.x / RB;
  const int r = tile * RB + b;
  const bool vb = r < NR;
  const bool odd = (b & 1) != 0;         // = hardware lane parity (RB even)
  const TCube* __restrict__ cube = static_cast<const TCube*>(a.cube) + (int64_t)f * C * NR;
  const int kfft = C < ND ? C : ND;      // fft(., Nd, 2) truncates to the first Nd chirps
  const int r2 = tile * RB + 2 * (b >> 1);

  float2 v[P];
  float2 s = make_float2(0.f, 0.f);
  float pm = 0.f;
  // 16-byte loads: lane pair (2i, 2i+1) reads bins r2, r2+1 of chirps
  // u + T*2j (even lane) and u + T*(2j+1) (odd lane), then swaps one element
#pragma unroll
  for (int j = 0; j < P / 2; ++j) {
    const int k = u + T * (2 * j + (b & 1));
    float2 u0 = make_float2(0.f, 0.f), u1 = u0;
    if (r2 < NR && k < kfft) {
      ld_c2(cube, (int64_t)k * NR + r2, u0, u1);
      u0 = cscale(u0, a.cube_unscale);
      u1 = cscale(u1, a.cube_unscale);
    }
    pair_xchg(odd, u0, u1);
    v[2 * j] = u0;
    v[2 * j + 1] = u1;
    s = cadd(s, cadd(u0, u1));
    pm = fmaxf(pm, fmaxf(cabs2(u0), cabs2(u1)));
  }
  if (C > ND && vb) {                    // chirps beyond Nd: profile and mean only
    for (int k = ND + u; k < C; k += T) {
      const float2 x = cscale(ld_c(cube, (int64_t)k * NR + r), a.cube_unscale);
      s = cadd(s, x);
      pm = fmaxf(pm, cabs2(x));
    }
  }
  red_s[threadIdx.x] = s;
  red_m[threadIdx.x] = pm;
  __syncthreads();
  if (u == 0) {
#pragma unroll 4
    for (int i = 1; i < T; ++i) {
      s = cadd(s, red_s[b + RB * i]);
      pm = fmaxf(pm, red_m[b + RB * i]);
    }
    red_s[b] = s;
    if (vb) a.profile[(int64_t)f * NR + r] = sqrtf(pm);       // :210 / :265 abs(max(X,[],2))
  }
  __syncthreads();
  const float2 mean = cscale(red_s[b], 1.0f / (float)C);      // :217 mean over ALL chirps
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int k = u + T * m;
    v[m] = (k < kfft) ? cscale(csub(v[m], mean), a.wd[k]) : make_float2(0.f, 0.f);  // :218-219
  }
  team_fft<ND>(v, lds + b * Plan::STRIDE, u, a.tw, BlockSync{}); // :219 fft(., Nd, 2)
  __syncthreads();
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int e = u + T * m;
    lds[b * SROW + ((e + ND / 2) & (ND - 1))] = v[m];          // :219 fftshift(., 2)
  }
  __syncthreads();
  const int nrows = (NR - tile * RB) < RB ? (NR - tile * RB) : RB;
  TRd* __restrict__ out = static_cast<TRd*>(a.rd) + ((int64_t)f * NR + (int64_t)tile * RB) * ND;
  for (int e2 = threadIdx.x; e2 < nrows * (ND / 2); e2 += 256) {   // RB whole rows, 16-byte stores
    const int e = 2 * e2, bb = e / ND, d = e & (ND - 1);
    const float4 q = *reinterpret_cast<const float4*>(&lds[bb * SROW + d]);
    st_c2(out, e, cscale(make_float2(q.x, q.y), a.rd_scale), cscale(make_float2(q.z, q.w), a.rd_scale));
  }
}

// ---------------------------------------------------------------------------
// K3: detection.  One wave per frame.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o);
    const int oi = __shfl_xor(i, o);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

template <int NR, typename TRd, typename TCube>
__global__ __launch_bounds__(256) void k_detect(DetectArgs a) {
  // One wave per frame.  Latency-shaped: every load a lane needs in a phase is
  // issued together (profile + both neighbours; then the target's Doppler row
  // and slow-time row), so a frame costs two dependent memory round trips.
  constexpr int PPL = NR >= 64 ? NR / 64 : 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f = (int64_t)blockIdx.x * 4 + w;
  if (f >= a.nframes) return;            // wave-uniform exit; no block barriers below
  const int ND = a.ND, C = a.C, M = a.M;
  const float* __restrict__ prof = a.profile + f * NR;
  const double dpb = a.dist_per_bin, lo = a.min_d, hi = a.max_d;

  // f_search_peak: local maxima above range_thr inside
  // [min_d, max_d]; the max_targets largest, ties -> lower index.
  float cv[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int i = lane + 64 * j;
    float v = -1.f;
    if (i >= 1 && i <= NR - 2) {                        // 1-based 2..Nr-1
      const double rng = (double)i * dpb;               // (idx-1)*dist_per_bin
      const float pc = prof[i], pl = prof[i - 1], pr = prof[i + 1];
      if (rng >= lo && rng <= hi && pc > a.range_thr && pc >= pl && pc > pr) v = pc;
    }
    cv[j] = v;
  }
  int sel[8];
  float selv[8];
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

  // :257-259 slow-time row of the strongest target, from the stored cube;
  // issued before the Doppler rows so both round trips overlap
  const TCube* __restrict__ cube = static_cast<const TCube*>(a.cube) + f * C * (int64_t)NR;
  float* __restrict__ slow = a.slow_mag + f * C;
  {
    const int row = n > 0 ? sel[0] : 0;
    for (int k = lane; k < C; k += 64)
      slow[k] = n > 0 ? sqrtf(cabs2(ld_c(cube, (int64_t)k * NR + row))) * a.cube_unscale : 0.f;
  }

  const TRd* __restrict__ rd = static_cast<const TRd*>(a.rd);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j >= M) break;
    int di = 0, ri = 0;
    float rm = 0.f;
    if (j < n) {
      // :233 [val, idx] = max(abs(range_Doppler(tgt_range_idx(j), :)))
      const TRd* __restrict__ row = rd + ((int64_t)f * NR + sel[j]) * ND;
      float bv = -1.f;
      int bi = INT_MAX;
      for (int d = lane; d < ND; d += 64) {
        const float mag = sqrtf(cabs2(ld_c(row, d))) * a.rd_unscale;
        if (mag > bv) { bv = mag; bi = d; }
      }
      wave_argmax(bv, bi);
      di = bi + 1;
      if (!(bv >= a.doppler_thr && di != a.fallback)) di = a.fallback;   // :234-238
      ri = sel[j] + 1;
      rm = selv[j];
    }
    if (lane == 0) {
      a.ridx[f * M + j] = ri;
      a.rmag[f * M + j] = rm;
      a.didx[f * M + j] = di;
    }
  }
  if (lane == 0) a.count[f] = n;

  // :410-411 abs(range_tx1rx1_complete(:, fr_idx)) for one linear column
  if (f == a.probe_frame && a.probe_mag) {
    for (int i = lane; i < NR; i += 64)
      a.probe_mag[i] = sqrtf(cabs2(ld_c(cube, (int64_t)a.probe_chirp * NR + i))) * a.cube_unscale;
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
template <int NR, typename TIn, typename TCube>
static hipError_t go_range(const RangeArgs& a, hipStream_t s) {
  constexpr int T = FftPlan<NR>::T;
  constexpr int TEAMS = T >= 256 ? 1 : 256 / T;
  const int64_t per_block = (int64_t)TEAMS * a.cpt;
  const int64_t blocks = (a.nchirps + per_block - 1) / per_block;
  // 16-byte (pair) access needs an even team and 16-byte-aligned chirp rows
  constexpr bool kPairOk = (T % 2 == 0);
  const bool pair = kPairOk && (a.S % 2 == 0);
  if (a.profile) {
    if (pair) hipLaunchKernelGGL((k_range<NR, TIn, TCube, true, kPairOk>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_range<NR, TIn, TCube, true, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  } else {
    if (pair) hipLaunchKernelGGL((k_range<NR, TIn, TCube, false, kPairOk>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_range<NR, TIn, TCube, false, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  }
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
  hipLaunchKernelGGL((k_doppler<ND, TCube, TRd>), dim3((unsigned)blocks), dim3(256), 0, s, a);
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
