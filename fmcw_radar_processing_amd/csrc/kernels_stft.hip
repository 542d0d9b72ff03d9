// kernels_stft.hip -- slow-time compaction, STFT, dB/log-frequency stages and
// the synthetic IQ generator.
//
//   k_compact     radar_processing.m:257-260  (which frames feed slow_time_signal)
//   k_stft_power  :270-276  spectrogram(|slow|, win, noverlap, nfft, 1/PRT):
//                 one-sided PSD P of every hop-spaced, window-long segment,
//                 zero-padded to nfft, plus the running max of P
//   k_stft_db     :279-283 psd = 20*log10(P/max(P(:)))  and  :293-299
//                 interp1 onto 1024 logspace bins (table from the host)
//   k_synth       SURVEY.md 8d synthetic frames (bench/test input only)
#include "fft_team.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include "fmcw_internal.h"
#include "../../include/fmcw.h"

namespace fmcw {

// max(P) of a block into the launch-wide maximum.  P >= 0, so the bit order of the floats is
// their value order and an unsigned atomicMax combines them.  Thousands of blocks adding to ONE
// word serialise at the memory side (~12 ns each, MI355X_MICROARCH.md fanin: ~44 us for the
// 3,661 blocks of a config-4 step), so a block first reads the current maximum (an agent-scope
// load, served by the L2) and skips the atomic when it cannot raise it; a stale read only costs
// an unneeded atomic, never a wrong maximum.
__device__ __forceinline__ void max_into(float* pmax, float m) {
  unsigned* p = reinterpret_cast<unsigned*>(pmax);
  const unsigned cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__float_as_uint(m) > cur) atomicMax(p, __float_as_uint(m));
}

// psd = 20 log10(P / max) (:283) as 20 log10(2) log2(v): the hardware log2 (v_log_f32) and one
// multiply, 3 instructions against log10f's 13 (which scales denormals and splits log10(2) for an
// extra-precise product: < 1e-5 dB apart down to -200 dB, against the 1e-3 dB bar of SURVEY 8d).
// A denormal v (below -759 dB) is scaled into the normal range first; v = 0 gives -Inf as MATLAB's
// G = 0 guard (:551).  Every dB kernel uses it, so the matrix-core and VALU forms stay bit-identical.
__device__ __forceinline__ float db20(float v) {
  // branch-free: a denormal v is scaled by 2^32 into the normal range first (as OCML's log does)
  const bool dn = v < 1.17549435e-38f;
  const float l2 = __log2f(dn ? v * 4294967296.0f : v);
  return fmaf(6.0205999132796239f, l2, dn ? -192.65919722494796f : 0.0f);
}

// ---------------------------------------------------------------------------
// exclusive scan of (count > 0) over F frames in one 1024-thread workgroup
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_compact(const int32_t* __restrict__ count, int64_t F, int pn,
                                                  int32_t* __restrict__ list, int64_t* __restrict__ len) {
  __shared__ int wsum[16];
  __shared__ long long carry;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < F; base += 1024) {
    const int64_t i = base + tid;
    const bool flag = i < F && count[i] > 0;
    const unsigned long long bal = __ballot(flag);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int wpre = 0;
    for (int q = 0; q < wid; ++q) wpre += wsum[q];
    if (flag) list[carry + wpre + pre] = (int32_t)i;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int q = 0; q < 16; ++q) tot += wsum[q];
      carry += tot;
    }
    __syncthreads();
  }
  if (tid == 0) *len = (int64_t)carry * pn;
}

// ---------------------------------------------------------------------------
// STFT power.  A workgroup owns `seg_tile` consecutive segments; it stages the
// samples they cover (through the compaction indirection) in LDS, then each
// thread evaluates S(seg, bin) = sum_m x[seg*hop+m] w[m] e^{-2 pi i bin m/nfft}
// by Horner's rule in z = e^{-2 pi i bin/nfft} (wlen-1 complex FMAs).
// ---------------------------------------------------------------------------
constexpr int STFT_MAX_SAMPLES = 8192;
constexpr int STFT_MAX_WLEN = 256;

__global__ __launch_bounds__(256) void k_stft_power(StftArgs a, int seg_tile) {
  __shared__ float xs[STFT_MAX_SAMPLES];
  __shared__ float ws[STFT_MAX_WLEN];
  __shared__ float bmax[4];
  __shared__ float wss;
  const int64_t L = *a.len;
  const int64_t H = a.halo_len ? *a.halo_len : a.n_halo;
  const int64_t Lx = L + H;
  const int noverlap = a.wlen - a.hop;
  int64_t nseg = Lx - noverlap >= 0 ? (Lx - noverlap) / a.hop : 0;   // fix((L-noverlap)/hop)
  if (nseg > a.max_seg) nseg = a.max_seg;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.nseg_out = nseg;
  const int64_t s0 = (int64_t)blockIdx.x * seg_tile;
  if (s0 >= nseg) return;                                           // block-uniform
  const int64_t s1 = (s0 + seg_tile < nseg) ? s0 + seg_tile : nseg;
  const int nsamp = (int)((s1 - 1 - s0) * a.hop + a.wlen);
  const int64_t q0 = s0 * a.hop;
  for (int i = threadIdx.x; i < nsamp; i += 256) {
    const int64_t q = q0 + i;
    float x;
    if (q < L) {
      const int64_t fr = a.frame_list[q / a.pn];
      x = a.slow_mag[fr * a.pn + (q % a.pn)];
    } else {
      x = a.halo[q - L];
    }
    xs[i] = x;
  }
  for (int i = threadIdx.x; i < a.wlen; i += 256) ws[i] = a.win[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    float u = 0.f;
    for (int i = 0; i < a.wlen; ++i) u = fmaf(ws[i], ws[i], u);
    wss = a.inv_fs / u;                                             // 1/(fs*sum(w.^2))
  }
  __syncthreads();
  const float p_scale = wss;

  const int nb = a.nfft / 2 + 1;
  const int64_t total = (s1 - s0) * nb;
  const float two_over_nfft = 2.0f / (float)a.nfft;
  float lmax = 0.f;
  for (int64_t o = threadIdx.x; o < total; o += 256) {
    const int sl = (int)(o / nb), bin = (int)(o - (int64_t)sl * nb);
    float sn, cs;
    sincospif((float)bin * two_over_nfft, &sn, &cs);
    const float2 z = make_float2(cs, -sn);
    const float* xp = xs + sl * a.hop;
    float2 acc = make_float2(xp[a.wlen - 1] * ws[a.wlen - 1], 0.f);
    for (int m = a.wlen - 2; m >= 0; --m) {
      acc = cmul(acc, z);
      acc.x = fmaf(xp[m], ws[m], acc.x);
    }
    const float k = (bin == 0 || 2 * bin == a.nfft) ? 1.f : 2.f;  // one-sided 'psd'
    const float p = cabs2(acc) * p_scale * k;
    if (a.P) a.P[(s0 + sl) * nb + bin] = p;
    lmax = fmaxf(lmax, p);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
  if ((threadIdx.x & 63) == 0) bmax[threadIdx.x >> 6] = lmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(bmax[0], bmax[1]), fmaxf(bmax[2], bmax[3]));
    max_into(a.pmax, m);
  }
}

// ---------------------------------------------------------------------------
// STFT fast path for the reference's 20-tap window (:276 kaiser(20,3); config 4
// Hann(20)).  One thread per segment, 256 segments per workgroup:
//   S(seg, bin) = sum_m x[seg hop + m] * W[bin][m],  W[bin][m] = w[m] e^{-2 pi i bin m/nfft}
// x[0..19] in registers; W read as wave-uniform scalar loads (every lane of a
// wave evaluates the same bin), so each complex MAC of a real sample is two
// v_fma_f32 with an SGPR operand -- no per-output sincos, no Horner chain, no
// 64-bit division.  Output tiles of 256 segments x 32 bins go through LDS so the
// stores are coalesced.  MODE 0: P (one-sided 'psd') + max(P); MODE 1: max(P)
// only; MODE 2: psd = 20 log10(P / max) (:283) written directly (the P of a
// second pass, recomputed instead of stored and re-read); MODE 3: P of the
// listed bins only (the host call's second pass: the bins the log-frequency
// interp1 of :299 and the picture read, not all nfft/2+1).
// blockIdx.y splits the columns into chunks of col_chunk (a multiple of 32), so a
// call with few segments and a large nfft (the reference's nextpow2 rule on a
// long signal) still fills the chip.
// ---------------------------------------------------------------------------
constexpr int STFT_W = 20;

// W[k][m] = w[m] e^{-2 pi i k m / nfft}: exact phase reduction, fp64, rounded once
__device__ __forceinline__ float2 stft_w(float wm, int k, int m, int nfft) {
  double sn, cs;
  sincospi(2.0 * (double)((int64_t)k * m % nfft) / (double)nfft, &sn, &cs);
  return make_float2((float)(wm * cs), (float)(-wm * sn));
}

// The table [nfft/2+1][20], followed by the 20 window taps it was built from (the nfft-64 kernel
// checks them against the window of its call, so a cached table is never used stale)
__global__ __launch_bounds__(256) void k_stft_table(const float* __restrict__ win, int nfft, float2* __restrict__ tab) {
  const int nb = nfft / 2 + 1;
  const int64_t n = (int64_t)nb * STFT_W;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i / STFT_W), m = (int)(i - (int64_t)k * STFT_W);
    tab[i] = stft_w(win[m], k, m, nfft);
  }
  if (blockIdx.x == 0 && threadIdx.x < STFT_W) reinterpret_cast<float*>(tab + n)[threadIdx.x] = win[threadIdx.x];
}

template <int MODE>
__global__ __launch_bounds__(256) void k_stft20(StftArgs a, const float2* __restrict__ tab, float* __restrict__ dst,
                                                int col_chunk) {
  constexpr int TS = 256, KC = 32;
  __shared__ float xs[TS * 4 + STFT_W];         // hop <= 4 (the reference's is 1): 38 KiB of LDS, 4 blocks per CU
  __shared__ float tile[TS][KC + 1];
  __shared__ float bmax[4];
  const int64_t L = *a.len;
  const int64_t H = a.halo_len ? *a.halo_len : a.n_halo;
  const int64_t Lx = L + H;
  const int noverlap = STFT_W - a.hop;
  int64_t nseg = Lx - noverlap >= 0 ? (Lx - noverlap) / a.hop : 0;   // fix((L-noverlap)/hop)
  if (nseg > a.max_seg) nseg = a.max_seg;
  if (MODE < 2 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.nseg_out = nseg;
  const int64_t s0 = (int64_t)blockIdx.x * TS;
  if (s0 >= nseg) return;                                           // block-uniform
  const int ns = (int)(nseg - s0 < TS ? nseg - s0 : TS);
  const int nsamp = (ns - 1) * a.hop + STFT_W;
  const int64_t q0 = s0 * a.hop;
  for (int i = threadIdx.x; i < nsamp; i += 256) {
    const int64_t q = q0 + i;
    xs[i] = q < L ? a.slow_mag[(int64_t)a.frame_list[q / a.pn] * a.pn + (q % a.pn)] : a.halo[q - L];
  }
  __syncthreads();
  const int sl = threadIdx.x;
  const bool valid = sl < ns;
  float x[STFT_W];
#pragma unroll
  for (int m = 0; m < STFT_W; ++m) x[m] = valid ? xs[sl * a.hop + m] : 0.f;
  typedef float f2t __attribute__((ext_vector_type(2)));
  const __attribute__((address_space(4))) f2t* T = (const __attribute__((address_space(4))) f2t*)(const void*)tab;
  float u = 0.f;                                                    // sum(w.^2): |W[0][m]|^2
#pragma unroll
  for (int m = 0; m < STFT_W; ++m) u = fmaf(T[m].x, T[m].x, u);
  const float scale = a.inv_fs / u;                                 // 1/(fs*sum(w.^2))
  float inv = 0.f;
  if constexpr (MODE == 2) {
    const float pm = *a.pmax;
    inv = pm > 0.f ? 1.0f / pm : 0.f;                               // all-zero P: -Inf dB (MATLAB G = 0)
  }
  const int nb = a.nfft / 2 + 1;
  const int ncol = MODE == 3 ? a.ncol : nb;                         // output row length
  const int c_lo = blockIdx.y * col_chunk;
  const int c_hi = ncol - c_lo < col_chunk ? ncol : c_lo + col_chunk;
  const __attribute__((address_space(4))) int* B = (const __attribute__((address_space(4))) int*)(const void*)a.bins;
  float lmax = 0.f;
  for (int k0 = c_lo; k0 < c_hi; k0 += KC) {                        // uniform: columns k0 .. k0+KC-1
    const int kn = c_hi - k0 < KC ? c_hi - k0 : KC;
#pragma unroll 4
    for (int kk = 0; kk < kn; ++kk) {             // unrolled: the scalar table loads of 4 bins issue together
      const int k = MODE == 3 ? B[k0 + kk] : k0 + kk;
      const auto* Wk = T + (int64_t)k * STFT_W;
      // (re, im) as one packed accumulator: one v_pk_fma_f32 per tap (the same two fmas)
      f2t acc = {0.f, 0.f};
#pragma unroll
      for (int m = 0; m < STFT_W; ++m) acc = __builtin_elementwise_fma(f2t{x[m], x[m]}, Wk[m], acc);
      const float re = acc.x, im = acc.y;
      const float g = (k == 0 || 2 * k == a.nfft) ? 1.f : 2.f;     // one-sided 'psd'
      const float p = fmaf(re, re, im * im) * scale * g;
      if (valid) lmax = fmaxf(lmax, p);
      if constexpr (MODE == 0 || MODE == 3) tile[sl][kk] = p;
      if constexpr (MODE == 2) tile[sl][kk] = db20(p * inv);
    }
    if constexpr (MODE != 1) {
      __syncthreads();
      float* out = MODE == 0 ? a.P : dst;
      for (int i = threadIdx.x; i < ns * kn; i += 256) {            // row-major [seg][col] chunk, coalesced per row
        const int r = i / kn, c = i - r * kn;
        out[(s0 + r) * ncol + k0 + c] = tile[r][c];
      }
      __syncthreads();
    }
  }
  if constexpr (MODE < 2) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    if ((threadIdx.x & 63) == 0) bmax[threadIdx.x >> 6] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(bmax[0], bmax[1]), fmaxf(bmax[2], bmax[3]));
      max_into(a.pmax, m);
    }
  }
}

// ---------------------------------------------------------------------------
// The nfft-64 case of k_stft20 MODE 0 / 1 / 2 (config 4's hop-1 Hann(20) STFT at nfft 64, 33
// one-sided bins) on the matrix cores: per 16 segments, the [16 seg x 20 tap] window-sample
// matrix (a Hankel matrix of the slow-time signal: row s = x[s .. s+19]) times the [20 x 64]
// table of W[bin][m] = w[m] e^{-2 pi i bin m / 64}, as 4 x 5 v_mfma_f32_16x16x4_f32:
//   tile 0: Re W of bins 0-15; tile 1: Im W of bins 1-15, column 0 = Re W of bin 32 (Nyquist:
//   its Im W and bin 0's are exactly -0, so that column is free); tile 2 / 3: Re / Im W of
//   bins 16-31.
// An f32 MFMA is a k-ordered chain of f32 fmas (cdna_hip_programming.md, FP32-input MFMA), so
// each S(seg, bin) is the same chain over m = 0..19 as k_stft20's v_pk_fma_f32 loop: P, max(P)
// and the direct dB are bit-identical (tests/test_gpu_stft_mfma.py).  Lane l of a wave: A = x[seg_base +
// (l & 15) + 4 q + (l >> 4)], B = its tile's W[col = l & 15][m = 4 q + (l >> 4)]; result
// register r: segment seg_base + 4 (l >> 4) + r, column l & 15.  Persistent over 256-segment
// tiles (round 4: one tile per block, 3,661 blocks whose start-up and two-load gather latency
// were not covered: 52 us for the max(P) pass, 3x its matrix work); outputs through an LDS tile
// and whole-line 16-byte stores (4-byte stores straight from the accumulators leave partial
// lines: 2x slower in the round-5 A/B).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_stft64m(StftArgs a, const float2* __restrict__ tab, float* __restrict__ dst) {
  constexpr int TS = 256, NB = 33, RS = 36, NX = TS * 4 + STFT_W, NPT = (NX + 255) / 256;
  typedef float f4t __attribute__((ext_vector_type(4)));
  __shared__ float xs[NX];
  // the tile of outputs [seg][RS]: 4 RS = 16 (mod 64 banks), so the 4 segment rows of one MFMA
  // result register (16 columns each) land on disjoint banks (round 4's stride 33: 4-way conflicts)
  __shared__ __attribute__((aligned(16))) float tile[MODE == 1 ? 4 : TS * RS];
  __shared__ float bmax[4];
  const int64_t L = *a.len;
  const int64_t H = a.halo_len ? *a.halo_len : a.n_halo;
  const int64_t Lx = L + H;
  const int noverlap = STFT_W - a.hop;
  int64_t nseg = Lx - noverlap >= 0 ? (Lx - noverlap) / a.hop : 0;   // fix((L-noverlap)/hop)
  if (nseg > a.max_seg) nseg = a.max_seg;
  if (MODE < 2 && blockIdx.x == 0 && threadIdx.x == 0) *a.nseg_out = nseg;
  const int64_t ntiles = (nseg + TS - 1) / TS;
  if ((int64_t)blockIdx.x >= ntiles) return;                        // block-uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, kq = lane >> 4;
  const int nx = TS * a.hop + STFT_W;
  // the tiles this block covers: t = blockIdx.x + k gridDim.x
  const int64_t t_first = blockIdx.x;
  // sample q of the tile starting at q0: q < L is slow_mag[frame_list[q / pn]][q % pn] (one 64-bit
  // division per tile, uniform; 32-bit ones per sample)
  const unsigned upn = (unsigned)a.pn;
  auto gather = [&](int64_t t, float (&v)[NPT]) __attribute__((always_inline)) {
    const int64_t s0 = t * TS;
    const int ns = (int)(nseg - s0 < TS ? nseg - s0 : TS);
    const int nsamp = (ns - 1) * a.hop + STFT_W;
    const int64_t q0 = s0 * a.hop;
    const int64_t fq0 = q0 / a.pn;
    const unsigned r0 = (unsigned)(q0 - fq0 * a.pn);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int i = threadIdx.x + 256 * k;
      float x = 0.f;                                                // zero past the last segment's samples
      if (i < nsamp) {
        const int64_t q = q0 + i;
        if (q < L) {
          const unsigned rr = r0 + (unsigned)i, df = rr / upn;
          x = a.slow_mag[(int64_t)a.frame_list[fq0 + df] * a.pn + (rr - df * upn)];
        } else {
          x = a.halo[q - L];
        }
      }
      v[k] = x;
    }
  };
  float pre[NPT];
  if (t_first < ntiles) gather(t_first, pre);                       // the first tile's samples in flight
  // the table may be cached across calls (fmcw_api.cpp stft_tab64): it is used only when the 20
  // taps stored behind it are this call's window, else every lane forms its W entries itself
  // (the same fp64 expression as k_stft_table, so the same bits)
  const float wcall = threadIdx.x < STFT_W ? a.win[threadIdx.x] : 0.f;
  const float* tabw = reinterpret_cast<const float*>(tab + NB * STFT_W);
  const bool fresh = __syncthreads_and(threadIdx.x >= STFT_W || tabw[threadIdx.x] == wcall);
  // the B operands of the 4 column tiles x 5 k-steps (loaded once per block), and sum(w.^2)
  float bw[4][5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int m = 4 * q + kq;
    float2 e0, eN, e1;
    if (fresh) {
      e0 = tab[col * STFT_W + m]; eN = tab[32 * STFT_W + m]; e1 = tab[(16 + col) * STFT_W + m];
    } else {
      const float wm = a.win[m];
      e0 = stft_w(wm, col, m, 64); eN = stft_w(wm, 32, m, 64); e1 = stft_w(wm, 16 + col, m, 64);
    }
    bw[0][q] = e0.x;
    bw[1][q] = col == 0 ? eN.x : e0.y;
    bw[2][q] = e1.x;
    bw[3][q] = e1.y;
  }
  float u = 0.f;
#pragma unroll
  for (int m = 0; m < STFT_W; ++m) {
    const float wm = fresh ? tab[m].x : a.win[m];                   // W[0][m] = w[m] exactly
    u = fmaf(wm, wm, u);
  }
  const float scale = a.inv_fs / u;                                 // 1/(fs*sum(w.^2))
  float inv = 0.f;
  if constexpr (MODE == 2) {
    const float pm = *a.pmax;
    inv = pm > 0.f ? 1.0f / pm : 0.f;                               // all-zero P: -Inf dB (MATLAB G = 0)
  }
  auto emit = [&](int sl, int b, float p) __attribute__((always_inline)) {
    if constexpr (MODE == 0) tile[sl * RS + b] = p;
    if constexpr (MODE == 2) tile[sl * RS + b] = db20(p * inv);    // :283
  };
  // P = |S|^2 * scale * g (g = 2 inside the one-sided spectrum, 1 at DC and Nyquist) as one multiply
  // by scale * g: a power-of-two factor commutes with the rounding, so these are k_stft20's bits
  const float sg0 = col == 0 ? scale : 2.f * scale, sg1 = 2.f * scale;
  // max(P) of MODE 0 / 1 from the raw |S|^2 per lane (the scaling is monotonic: the same bits)
  float m0 = 0.f, m1 = 0.f, mN = 0.f;
  // one group's epilogue; FULL: the tile holds 256 segments (every tile but the last), no bounds checks
  auto epilogue = [&](const f4t (&acc)[4], int sb, int ns, auto FULL) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sl = sb + 4 * kq + r;
      const float re0 = acc[0][r], im0 = col == 0 ? 0.f : acc[1][r];
      const float q0 = fmaf(re0, re0, im0 * im0);
      const float re1 = acc[2][r], im1 = acc[3][r];
      const float q1 = fmaf(re1, re1, im1 * im1);
      const float rn = acc[1][r];                                   // column 0: Re S of bin 32
      const float qn = fmaf(rn, rn, 0.f * 0.f);
      if (decltype(FULL)::value || sl < ns) {
        if constexpr (MODE < 2) {
          m0 = fmaxf(m0, q0);
          m1 = fmaxf(m1, q1);
          mN = fmaxf(mN, qn);
        }
        if constexpr (MODE != 1) {
          emit(sl, col, q0 * sg0);
          emit(sl, 16 + col, q1 * sg1);
          if (col == 0) emit(sl, 32, qn * scale);
        }
      }
    }
  };
  // Persistent over tiles of 256 segments (grid: a few blocks per CU): the next tile's samples
  // are loaded while this one is transformed, so the gather's two dependent loads (frame list,
  // samples) and the block's start-up are paid once per block, not per tile
  for (int64_t t = t_first; t < ntiles;) {
    const int64_t s0 = t * TS;
    const int ns = (int)(nseg - s0 < TS ? nseg - s0 : TS);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < nx) xs[i] = pre[k];
    }
    const int64_t tn = t + gridDim.x;
    if (tn < ntiles) gather(tn, pre);
    __syncthreads();                                                // xs holds tile t
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {                                   // 4 groups of 16 segments per wave
      const int sb = w * 64 + 16 * g;
      if (sb >= ns) break;                                          // wave-uniform
      f4t acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const float av = xs[(sb + col) * a.hop + 4 * q + kq];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bw[tt][q], acc[tt], 0, 0, 0);
      }
      if (ns == TS) epilogue(acc, sb, ns, std::true_type{});
      else epilogue(acc, sb, ns, std::false_type{});
    }
    __syncthreads();                                                // xs read out; the tile written
    if constexpr (MODE != 1) {
      // the tile's rows s0 .. s0+ns-1 are one contiguous run of ns x 33 floats, 16-byte aligned
      // (s0 x 33 x 4 = 33792 t bytes): whole-line 16-byte stores
      float* out = (MODE == 0 ? a.P : dst) + s0 * NB;
      const int n = ns * NB, n4 = n >> 2;
      for (int i = threadIdx.x; i < n4; i += 256) {
        f4t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int o = 4 * i + e, rr = o / NB;
          v[e] = tile[rr * RS + (o - rr * NB)];
        }
        reinterpret_cast<f4t*>(out)[i] = v;
      }
      for (int o = 4 * n4 + threadIdx.x; o < n; o += 256) out[o] = tile[(o / NB) * RS + o % NB];
      __syncthreads();                                              // the tile read out
    }
    t = tn;
  }
  if constexpr (MODE < 2) {
    float lmax = fmaxf(m0 * sg0, m1 * sg1);
    if (col == 0) lmax = fmaxf(lmax, mN * scale);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    if (lane == 0) bmax[w] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(bmax[0], bmax[1]), fmaxf(bmax[2], bmax[3]));
      max_into(a.pmax, m);
    }
  }
}

// ---------------------------------------------------------------------------
// The nfft-64 STFT folded about the window's centre (round 5; the default for config 4).  For
// the segment x[s .. s+19] and theta_b = 2 pi b / 64, pairing tap 10+k with tap 9-k (k = 0..9):
//   S(b) e^{i theta_b 9.5} = sum_k (u_k cos(theta_b (k + 1/2)) - i v_k sin(theta_b (k + 1/2))),
//   u_k = w[10+k] x[s+10+k] + w[9-k] x[s+9-k],  v_k = w[10+k] x[s+10+k] - w[9-k] x[s+9-k],
// and P only needs |S|^2, which the phase factor leaves unchanged: two 10-term real sums per bin
// instead of one 20-term complex one, for any window (the taps are applied to the samples).  Per
// 32 segments: [32 seg x 10] x [10 x 32 bins] twice, 2 x 5 v_mfma_f32_32x32x2_f32 (k_stft64m: 20
// v_mfma_f32_16x16x4_f32 per 16 segments, 2.5x the matrix work).  Re from the sums u, Im from the
// differences v; Im of bin 0 is identically 0, so its column carries the Nyquist bin (cos terms
// 0, sin terms (-1)^k, exact).  Not bit-identical to k_stft20 (a different exact identity, the
// same f32 error order: tests/test_gpu_stft_mfma.py holds it to the VALU form and the oracle).
// Lane l: A = u or v of segment sb + (l & 31), k = 2q + (l >> 5); B = cos / sin of bin l & 31 at
// that k; result register r: segment sb + (r & 3) + 8 (r >> 2) + 4 (l >> 5), bin l & 31.
// Each wave is independent (no block barrier in the loop): units of 64 segments, the next unit's
// samples gathered into registers while this one is transformed, its outputs staged in the
// wave's own LDS tile in the output's [seg][33] layout and stored as 16-byte lines.
// ---------------------------------------------------------------------------
// cos(pi m / 64), m = 0..127, correctly rounded (exact zeros at m = 32, 96): the folded form's B
// operands are cos / sin (pi b (2k+1) / 64) = k_cospi64[b (2k+1) mod 128] / k_cospi64[(b (2k+1) - 32) mod 128]
__device__ const float k_cospi64[128] = {
    0x1.0000000000000p+0f, 0x1.ff621e0000000p-1f, 0x1.fd88da0000000p-1f, 0x1.fa75580000000p-1f,
    0x1.f6297c0000000p-1f, 0x1.f0a7f00000000p-1f, 0x1.e9f4160000000p-1f, 0x1.e212100000000p-1f,
    0x1.d906bc0000000p-1f, 0x1.ced7b00000000p-1f, 0x1.c38b300000000p-1f, 0x1.b728340000000p-1f,
    0x1.a9b6620000000p-1f, 0x1.9b3e040000000p-1f, 0x1.8bc8060000000p-1f, 0x1.7b5df20000000p-1f,
    0x1.6a09e60000000p-1f, 0x1.57d6940000000p-1f, 0x1.44cf320000000p-1f, 0x1.30ff800000000p-1f,
    0x1.1c73b40000000p-1f, 0x1.07387a0000000p-1f, 0x1.e2b5d40000000p-2f, 0x1.b5d1000000000p-2f,
    0x1.87de2a0000000p-2f, 0x1.58f9a80000000p-2f, 0x1.2940620000000p-2f, 0x1.f19f980000000p-3f,
    0x1.8f8b840000000p-3f, 0x1.2c81060000000p-3f, 0x1.917a6c0000000p-4f, 0x1.91f6600000000p-5f,
    0.0f, -0x1.91f6600000000p-5f, -0x1.917a6c0000000p-4f, -0x1.2c81060000000p-3f,
    -0x1.8f8b840000000p-3f, -0x1.f19f980000000p-3f, -0x1.2940620000000p-2f, -0x1.58f9a80000000p-2f,
    -0x1.87de2a0000000p-2f, -0x1.b5d1000000000p-2f, -0x1.e2b5d40000000p-2f, -0x1.07387a0000000p-1f,
    -0x1.1c73b40000000p-1f, -0x1.30ff800000000p-1f, -0x1.44cf320000000p-1f, -0x1.57d6940000000p-1f,
    -0x1.6a09e60000000p-1f, -0x1.7b5df20000000p-1f, -0x1.8bc8060000000p-1f, -0x1.9b3e040000000p-1f,
    -0x1.a9b6620000000p-1f, -0x1.b728340000000p-1f, -0x1.c38b300000000p-1f, -0x1.ced7b00000000p-1f,
    -0x1.d906bc0000000p-1f, -0x1.e212100000000p-1f, -0x1.e9f4160000000p-1f, -0x1.f0a7f00000000p-1f,
    -0x1.f6297c0000000p-1f, -0x1.fa75580000000p-1f, -0x1.fd88da0000000p-1f, -0x1.ff621e0000000p-1f,
    -0x1.0000000000000p+0f, -0x1.ff621e0000000p-1f, -0x1.fd88da0000000p-1f, -0x1.fa75580000000p-1f,
    -0x1.f6297c0000000p-1f, -0x1.f0a7f00000000p-1f, -0x1.e9f4160000000p-1f, -0x1.e212100000000p-1f,
    -0x1.d906bc0000000p-1f, -0x1.ced7b00000000p-1f, -0x1.c38b300000000p-1f, -0x1.b728340000000p-1f,
    -0x1.a9b6620000000p-1f, -0x1.9b3e040000000p-1f, -0x1.8bc8060000000p-1f, -0x1.7b5df20000000p-1f,
    -0x1.6a09e60000000p-1f, -0x1.57d6940000000p-1f, -0x1.44cf320000000p-1f, -0x1.30ff800000000p-1f,
    -0x1.1c73b40000000p-1f, -0x1.07387a0000000p-1f, -0x1.e2b5d40000000p-2f, -0x1.b5d1000000000p-2f,
    -0x1.87de2a0000000p-2f, -0x1.58f9a80000000p-2f, -0x1.2940620000000p-2f, -0x1.f19f980000000p-3f,
    -0x1.8f8b840000000p-3f, -0x1.2c81060000000p-3f, -0x1.917a6c0000000p-4f, -0x1.91f6600000000p-5f,
    0.0f, 0x1.91f6600000000p-5f, 0x1.917a6c0000000p-4f, 0x1.2c81060000000p-3f,
    0x1.8f8b840000000p-3f, 0x1.f19f980000000p-3f, 0x1.2940620000000p-2f, 0x1.58f9a80000000p-2f,
    0x1.87de2a0000000p-2f, 0x1.b5d1000000000p-2f, 0x1.e2b5d40000000p-2f, 0x1.07387a0000000p-1f,
    0x1.1c73b40000000p-1f, 0x1.30ff800000000p-1f, 0x1.44cf320000000p-1f, 0x1.57d6940000000p-1f,
    0x1.6a09e60000000p-1f, 0x1.7b5df20000000p-1f, 0x1.8bc8060000000p-1f, 0x1.9b3e040000000p-1f,
    0x1.a9b6620000000p-1f, 0x1.b728340000000p-1f, 0x1.c38b300000000p-1f, 0x1.ced7b00000000p-1f,
    0x1.d906bc0000000p-1f, 0x1.e212100000000p-1f, 0x1.e9f4160000000p-1f, 0x1.f0a7f00000000p-1f,
    0x1.f6297c0000000p-1f, 0x1.fa75580000000p-1f, 0x1.fd88da0000000p-1f, 0x1.ff621e0000000p-1f,
};

template <int MODE, bool H1>
__global__ __launch_bounds__(256) void k_stft64f(StftArgs a, float* __restrict__ dst) {
  // US segments per unit; a wave gathers UB units' samples at once (every load of the batch in
  // flight together: the frame-list loads first, then the samples), then transforms them in turn
  constexpr int US = 64, NB = 33, UB = 4, HOPMAX = H1 ? 1 : 4;
  constexpr int NXW = US * HOPMAX + STFT_W, NPW = (NXW + 63) / 64;
  typedef float f16t __attribute__((ext_vector_type(16)));
  typedef float f4t __attribute__((ext_vector_type(4)));
  __shared__ float xs_all[4][UB * NXW];
  __shared__ __attribute__((aligned(16))) float tile_all[MODE == 1 ? 1 : 4][MODE == 1 ? 4 : US * NB];
  __shared__ float bmax[4];
  const int hop = H1 ? 1 : a.hop;
  const int64_t L = *a.len;
  const int64_t H = a.halo_len ? *a.halo_len : a.n_halo;
  const int64_t Lx = L + H;
  const int noverlap = STFT_W - hop;
  int64_t nseg = Lx - noverlap >= 0 ? (Lx - noverlap) / hop : 0;     // fix((L-noverlap)/hop)
  if (nseg > a.max_seg) nseg = a.max_seg;
  if (MODE < 2 && blockIdx.x == 0 && threadIdx.x == 0) *a.nseg_out = nseg;
#ifdef STFT_AB_STAMPS   // development probe (tools/stft_stamps.py): the max(P) pass's s_memtime / s_memrealtime stamps into a caller-sized nseg_out
  unsigned long long* stp = reinterpret_cast<unsigned long long*>(a.nseg_out) + 1;
  const bool stamper = MODE == 1 && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1);
  const int so = blockIdx.x == 0 ? 0 : 16;
  int nst = 0;
#define STAMP() do { if (stamper && nst < 15) { stp[so + nst] = __builtin_amdgcn_s_memtime(); } ++nst; } while (0)
  unsigned long long* rtp = reinterpret_cast<unsigned long long*>(a.nseg_out) + 64 + 3 * (blockIdx.x * 4 + (threadIdx.x >> 6));
  if (MODE == 1 && (threadIdx.x & 63) == 0) { rtp[0] = __builtin_amdgcn_s_memrealtime(); unsigned xcc, hwid; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc)); asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid)); rtp[2] = ((unsigned long long)xcc << 32) | hwid; }
#else
#define STAMP() do {} while (0)
#endif
  STAMP();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 31, kh = lane >> 5;
  float* xs = xs_all[w];
  float* tile = tile_all[MODE == 1 ? 0 : w];
  const int64_t units = (nseg + US - 1) / US;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const unsigned upn = (unsigned)a.pn;
  // sample i of unit u: q = 64 u hop + i; q < L is slow_mag[frame_list[q / pn]][q % pn], L <= q <
  // L + H the halo, past the unit's last segment 0.  q0 / pn once per unit from a double reciprocal
  // (exact after one correction step: q0 < 2^53), (q0 % pn + i) / pn per sample from a float one
  // (exact after one correction step: the dividend is below pn + 276 < 2^24); no integer division
  const double inv_pn_d = 1.0 / (double)a.pn;
  const float inv_pn_f = 1.0f / (float)a.pn;
  auto locate = [&](int64_t u, int (&f)[NPW], unsigned (&c)[NPW]) __attribute__((always_inline)) {
    const int64_t s0 = u * US;
    const int ns = (int)(nseg - s0 < US ? nseg - s0 : US);
    const int nsamp = u < units ? (ns - 1) * hop + STFT_W : 0;
    const int64_t q0 = s0 * hop;
    int64_t fq0 = (int64_t)((double)q0 * inv_pn_d);
    int64_t r0 = q0 - fq0 * a.pn;
    if (r0 < 0) { --fq0; r0 += a.pn; }
    if (r0 >= a.pn) { ++fq0; r0 -= a.pn; }
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int i = lane + 64 * k;
      f[k] = -2;
      c[k] = 0;
      if (i < nsamp) {
        const int64_t q = q0 + i;
        if (q < L) {
          const unsigned rr = (unsigned)r0 + (unsigned)i;
          unsigned df = (unsigned)((float)rr * inv_pn_f);
          int d = (int)(rr - df * upn);
          if (d < 0) { --df; d += a.pn; }
          if (d >= a.pn) { ++df; d -= a.pn; }
          f[k] = a.frame_list[fq0 + df];
          c[k] = (unsigned)d;
        } else {
          f[k] = -1;
          c[k] = (unsigned)(q - L);
        }
      }
    }
  };
  // this lane's taps (k = 2q + kh) and B operands
  float wp[5], wn[5], bc[5], bs[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int k = 2 * q + kh;
    wp[q] = a.win[10 + k];
    wn[q] = a.win[9 - k];
    const int m = (col * (2 * k + 1)) & 127;
    bc[q] = k_cospi64[m];
    bs[q] = col == 0 ? ((k & 1) ? -1.f : 1.f) : k_cospi64[(m + 96) & 127];   // column 0: the Nyquist bin's sin terms
  }
  float usum = 0.f;
#pragma unroll
  for (int m = 0; m < STFT_W; ++m) usum = fmaf(a.win[m], a.win[m], usum);
  const float scale = a.inv_fs / usum;                              // 1/(fs*sum(w.^2))
  float inv = 0.f;
  if constexpr (MODE == 2) {
    const float pm = *a.pmax;
    inv = pm > 0.f ? 1.0f / pm : 0.f;                               // all-zero P: -Inf dB (MATLAB G = 0)
  }
  // P = |S|^2 * scale * g (g = 2 inside the one-sided spectrum, 1 at DC and Nyquist); MODE 2 writes
  // P / max(P) = |S|^2 * (scale g / max(P)) into the tile and takes 20 log10 in the store phase
  const float sg = col == 0 ? scale : 2.f * scale;
  const float fz = col == 0 ? 0.f : 1.f;                            // column 0: Im S of bin 0 is 0
  const int nyo = col == 0 ? 32 : col;                              // column 0 also writes the Nyquist bin
  const float so = MODE == 2 ? sg * inv : sg, sn = MODE == 2 ? scale * inv : scale;
  // max of the raw |S|^2 as unsigned bits (|S|^2 >= 0: the order of the bits is the order of the
  // values, one v_max_u32 and no NaN quieting); the scaling is monotonic, so max(P) = max(|S|^2) g scale
  unsigned m0 = 0u, mN = 0u;
  // one group's epilogue; FULL: all 64 segments of the unit exist (every unit but the last), no checks
  auto epilogue = [&](const f16t& re, const f16t& im, int sb, int ns, auto FULL) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int sl = sb + (r & 3) + 8 * (r >> 2) + 4 * kh;
      const float rv = re[r], iv = im[r];
      const float t = iv * iv;                                      // column 0: |S|^2 of the Nyquist bin
      const float q = fmaf(rv, rv, t * fz);                         // |S|^2 of bin col
      if (decltype(FULL)::value || sl < ns) {
        if constexpr (MODE < 2) {
          m0 = max(m0, __float_as_uint(q));
          mN = max(mN, __float_as_uint(t));
        }
        if constexpr (MODE != 1) {
          const float p = q * so;
          tile[sl * NB + col] = p;
          tile[sl * NB + nyo] = col == 0 ? t * sn : p;              // column 0: the Nyquist bin, else p again
        }
      }
    }
  };
  STAMP();
  for (int64_t ub = (int64_t)blockIdx.x * 4 + w; ub < units; ub += UB * nw) {
    int fr[UB][NPW];
    unsigned cc[UB][NPW];
    float xv[UB][NPW];
#pragma unroll
    for (int b = 0; b < UB; ++b) locate(ub + b * nw, fr[b], cc[b]);
#pragma unroll
    for (int b = 0; b < UB; ++b)
#pragma unroll
      for (int k = 0; k < NPW; ++k) {
        const int f = fr[b][k];
        xv[b][k] = f >= 0 ? a.slow_mag[(int64_t)f * a.pn + cc[b][k]] : f == -1 ? a.halo[cc[b][k]] : 0.f;
      }
#pragma unroll
    for (int b = 0; b < UB; ++b)
#pragma unroll
      for (int k = 0; k < NPW; ++k) {
        const int i = lane + 64 * k;
        if (i < NXW) xs[b * NXW + i] = xv[b][k];
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");          // xs written before any lane reads it
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    STAMP();
#pragma unroll 1
    for (int b = 0; b < UB; ++b) {
      const int64_t u = ub + b * nw;
      if (u >= units) break;                                        // wave-uniform
      const int64_t s0 = u * US;
      const int ns = (int)(nseg - s0 < US ? nseg - s0 : US);
      const float* xb = xs + b * NXW;
#pragma unroll 1
      for (int g = 0; g < 2; ++g) {
        const int sb = 32 * g;
        if (sb >= ns) break;                                        // wave-uniform
        f16t re = {}, im = {};
        const int base = (sb + col) * hop;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          const int k = 2 * q + kh;
          const float xp = xb[base + 10 + k], xm = xb[base + 9 - k];
          const float t = wn[q] * xm;
          const float uk = fmaf(wp[q], xp, t), vk = fmaf(wp[q], xp, -t);
          re = __builtin_amdgcn_mfma_f32_32x32x2f32(uk, bc[q], re, 0, 0, 0);
          im = __builtin_amdgcn_mfma_f32_32x32x2f32(vk, bs[q], im, 0, 0, 0);
        }
        if (ns == US) epilogue(re, im, sb, ns, std::true_type{});
        else epilogue(re, im, sb, ns, std::false_type{});
      }
      if constexpr (MODE != 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");      // the tile written before it is read out
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rows s0 .. s0+ns-1 are one contiguous run of ns x 33 floats, 16-byte aligned (s0 x 132 = 8448 u bytes)
        float* out = (MODE == 0 ? a.P : dst) + s0 * NB;
        const int n = ns * NB, n4 = n >> 2;
        const f4t* t4 = reinterpret_cast<const f4t*>(tile);
        if constexpr (MODE == 0) {
          for (int i = lane; i < n4; i += 64) reinterpret_cast<f4t*>(out)[i] = t4[i];
          for (int o = 4 * n4 + lane; o < n; o += 64) out[o] = tile[o];
        } else {                                                    // :283 20 log10(P / max(P))
          for (int i = lane; i < n4; i += 64) {
            const f4t v = t4[i];
            // the dB map is the leg's output, not re-read: streamed out with nontemporal stores
            // (0.5-0.9 us of the pass's 38, profiles/r05_stft_fold.txt)
            __builtin_nontemporal_store(f4t{db20(v.x), db20(v.y), db20(v.z), db20(v.w)}, reinterpret_cast<f4t*>(out) + i);
          }
          for (int o = 4 * n4 + lane; o < n; o += 64) out[o] = db20(tile[o]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");      // read out before the next unit rewrites it
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    STAMP();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");          // xs read before the next batch rewrites it
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  STAMP();
#ifdef STFT_AB_STAMPS
  if (MODE == 1 && (threadIdx.x & 63) == 0) rtp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (MODE < 2) {
    float lmax = __uint_as_float(m0) * sg;
    if (col == 0) lmax = fmaxf(lmax, __uint_as_float(mN) * scale);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    if (lane == 0) bmax[w] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(bmax[0], bmax[1]), fmaxf(bmax[2], bmax[3]));
      max_into(a.pmax, m);
    }
  }
}

// ---------------------------------------------------------------------------
// k_stft20 on the matrix cores for any nfft (the host call's reference rule nfft =
// 2^nextpow2(L), :273, e.g. 65536 for 256 config-3 frames): columns in chunks of 32 bins,
// tiles 0 / 1 = Re / Im W of the chunk's bins 0-15, tiles 2 / 3 = bins 16-31, 5 k-steps of
// v_mfma_f32_16x16x4_f32 per 16 segments and chunk.  MODE as k_stft20 (0 P + max, 1 max,
// 2 dB, 3 P of the listed bins a.bins); the same k-ordered fma chain per output, so the
// results are bit-identical to k_stft20's (tests/test_gpu_stft_mfma.py).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_stft_mfma(StftArgs a, const float2* __restrict__ tab, float* __restrict__ dst,
                                                   int col_chunk) {
  constexpr int TS = 256, KC = 32;
  typedef float f4t __attribute__((ext_vector_type(4)));
  __shared__ float xs[TS * 4 + STFT_W];
  __shared__ float tile[MODE == 1 ? 4 : MODE == 4 ? TS : TS * (KC + 1)];   // MODE 4: per-segment max
  __shared__ float bmax[4];
  const int64_t L = *a.len;
  const int64_t H = a.halo_len ? *a.halo_len : a.n_halo;
  const int64_t Lx = L + H;
  const int noverlap = STFT_W - a.hop;
  int64_t nseg = Lx - noverlap >= 0 ? (Lx - noverlap) / a.hop : 0;   // fix((L-noverlap)/hop)
  if (nseg > a.max_seg) nseg = a.max_seg;
  if (MODE < 2 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.nseg_out = nseg;
  const int64_t s0 = (int64_t)(a.tiles ? a.tiles[blockIdx.x] : (int)blockIdx.x) * TS;
  if (s0 >= nseg) return;                                           // block-uniform
  const int ns = (int)(nseg - s0 < TS ? nseg - s0 : TS);
  const int nsamp = (ns - 1) * a.hop + STFT_W;
  const int64_t q0 = s0 * a.hop;
  for (int i = threadIdx.x; i < TS * a.hop + STFT_W; i += 256) {
    const int64_t q = q0 + i;
    xs[i] = i >= nsamp ? 0.f : q < L ? a.slow_mag[(int64_t)a.frame_list[q / a.pn] * a.pn + (q % a.pn)] : a.halo[q - L];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, kq = lane >> 4;
  if constexpr (MODE == 4) tile[threadIdx.x] = 0.f;                 // TS == blockDim (P >= 0)
  float u = 0.f;
#pragma unroll
  for (int m = 0; m < STFT_W; ++m) u = fmaf(tab[m].x, tab[m].x, u);
  const float scale = a.inv_fs / u;                                 // 1/(fs*sum(w.^2))
  float inv = 0.f;
  if constexpr (MODE == 2) {
    const float pm = *a.pmax;
    inv = pm > 0.f ? 1.0f / pm : 0.f;
  }
  const int nb = a.nfft / 2 + 1;
  constexpr bool LISTED = MODE == 3 || MODE == 4;
  const int ncol = LISTED ? a.ncol : nb;
  const int c_lo = blockIdx.y * col_chunk;
  const int c_hi = ncol - c_lo < col_chunk ? ncol : c_lo + col_chunk;
  __syncthreads();
  float lmax = 0.f;
  for (int k0 = c_lo; k0 < c_hi; k0 += KC) {                        // uniform: columns k0 .. k0+KC-1
    const int kn = c_hi - k0 < KC ? c_hi - k0 : KC;
    // this lane's two columns of the chunk (col, 16 + col) and their bins
    const bool v0 = col < kn, v1 = 16 + col < kn;
    const int b0 = v0 ? (LISTED ? a.bins[k0 + col] : k0 + col) : 0;
    const int b1 = v1 ? (LISTED ? a.bins[k0 + 16 + col] : k0 + 16 + col) : 0;
    float bw[4][5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int m = 4 * q + kq;
      const float2 t0 = tab[(int64_t)b0 * STFT_W + m], t1 = tab[(int64_t)b1 * STFT_W + m];
      bw[0][q] = v0 ? t0.x : 0.f;
      bw[1][q] = v0 ? t0.y : 0.f;
      bw[2][q] = v1 ? t1.x : 0.f;
      bw[3][q] = v1 ? t1.y : 0.f;
    }
    const float g0 = (b0 == 0 || 2 * b0 == a.nfft) ? 1.f : 2.f;     // one-sided 'psd'
    const float g1 = (b1 == 0 || 2 * b1 == a.nfft) ? 1.f : 2.f;
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {                                   // 4 groups of 16 segments per wave
      const int sb = w * 64 + 16 * g;
      if (sb >= ns) break;                                          // wave-uniform
      f4t acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const float av = xs[(sb + col) * a.hop + 4 * q + kq];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bw[t][q], acc[t], 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sl = sb + 4 * kq + r;
        const float p0 = fmaf(acc[0][r], acc[0][r], acc[1][r] * acc[1][r]) * scale * g0;
        const float p1 = fmaf(acc[2][r], acc[2][r], acc[3][r] * acc[3][r]) * scale * g1;
        if (sl < ns) {
          if (v0) lmax = fmaxf(lmax, p0);
          if (v1) lmax = fmaxf(lmax, p1);
        }
        if constexpr (MODE == 4) {   // the row's 16 lanes hold this segment's columns; one lane owns it
          float m = fmaxf(v0 ? p0 : 0.f, v1 ? p1 : 0.f);
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
          if (col == 0 && sl < ns) tile[sl] = fmaxf(tile[sl], m);
        }
        if constexpr (MODE == 0 || MODE == 3) {
          tile[sl * (KC + 1) + col] = p0;
          tile[sl * (KC + 1) + 16 + col] = p1;
        }
        if constexpr (MODE == 2) {
          tile[sl * (KC + 1) + col] = db20(p0 * inv);
          tile[sl * (KC + 1) + 16 + col] = db20(p1 * inv);
        }
      }
    }
    if constexpr (MODE != 1 && MODE != 4) {
      __syncthreads();
      float* out = MODE == 0 ? a.P : dst;
      for (int i = threadIdx.x; i < ns * kn; i += 256) {            // row-major [seg][col] chunk, coalesced per row
        const int r = i / kn, c = i - r * kn;
        out[(s0 + r) * ncol + k0 + c] = tile[r * (KC + 1) + c];
      }
      __syncthreads();
    }
  }
  if constexpr (MODE < 2) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    if (lane == 0) bmax[w] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(bmax[0], bmax[1]), fmaxf(bmax[2], bmax[3]));
      max_into(a.pmax, m);
    }
  }
  if constexpr (MODE == 4) {
    __syncthreads();
    if ((int)threadIdx.x < ns) dst[s0 + threadIdx.x] = tile[threadIdx.x];
  }
}

__global__ __launch_bounds__(256) void k_stft_db(StftDbArgs a) {
  const int64_t nseg = *a.nseg;
  const float pm = *a.pmax;
  const float inv = pm > 0.f ? 1.0f / pm : 0.f;   // all-zero P: 20log10(0) = -Inf, as MATLAB's G = 0 guard (:551)
  const int nout = a.nlog > 0 ? a.nlog : a.nbins_in;
  const int64_t total = nseg * nout;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int64_t s = o / nout;
    const int j = (int)(o - s * nout);
    const float* row = a.P + s * a.nbins_in;
    if (a.nlog == 0) {
      a.out[o] = db20(row[j] * inv);                                // :283
    } else {
      const int i0 = a.lidx[j];
      const float w = a.lw[j];
      const float d0 = db20(row[i0] * inv), d1 = db20(row[i0 + 1] * inv);
      a.out[o] = d0 + w * (d1 - d0);                               // :299 interp1 'linear','extrap'
    }
  }
}

// :283 without resampling: P [nseg][nb] and the dB map are the same flat array shape, so the
// map is one elementwise pass, 16 bytes per lane (P and out 16-byte aligned; may alias).
__global__ __launch_bounds__(256) void k_stft_db_flat(StftDbArgs a) {
  typedef float f4t __attribute__((ext_vector_type(4)));
  const int64_t n = *a.nseg * a.nbins_in;
  const float pm = *a.pmax;
  const float inv = pm > 0.f ? 1.0f / pm : 0.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const f4t* in = reinterpret_cast<const f4t*>(a.P);          // not __restrict__: P and out may alias
  f4t* out = reinterpret_cast<f4t*>(a.out);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f4t v = in[i];
    out[i] = f4t{db20(v.x * inv), db20(v.y * inv), db20(v.z * inv), db20(v.w * inv)};
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    a.out[i] = db20(a.P[i] * inv);
}

// ---------------------------------------------------------------------------
// synthetic frames; the same integer hash as oracle/oracle.py
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long hmix(unsigned long long seed, unsigned long long ctr) {
  return splitmix64(seed * 0xD1342543DE82EF95ull + ctr);
}
__device__ __forceinline__ double u24(unsigned long long h, int sh) {
  return ((double)((h >> sh) & 0xFFFFFFull) + 0.5) / 16777216.0;
}

template <typename TOut>
__global__ __launch_bounds__(256) void k_synth(SynthArgs a) {
  const int64_t per_frame = (int64_t)a.C * a.S;
  const int64_t total = a.nframes * per_frame;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  TOut* out = static_cast<TOut*>(a.iq);
  const double dpb = a.dist_per_bin;
  const int rlo = (int)ceil(0.9 / dpb) + 2;
  int rhi = (int)floor(25.0 / dpb) - 2;
  if (rhi < rlo) rhi = rlo;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t fl = e / per_frame;
    const int64_t rem = e - fl * per_frame;
    const int k = (int)(rem / a.S), n = (int)(rem - (int64_t)k * a.S);
    const unsigned long long seed = 0xF3C0ull ^ (unsigned long long)(a.frame0 + fl);
    const double u0 = u24(hmix(seed, 0x1000), 40), u1 = u24(hmix(seed, 0x1001), 40);
    const double u2 = u24(hmix(seed, 0x1002), 40), u3 = u24(hmix(seed, 0x1003), 40);
    const double u4 = u24(hmix(seed, 0x1004), 40), u5 = u24(hmix(seed, 0x1005), 40);
    const bool no_target = u0 < 0.10;
    const double off = u1 < 0.25 ? 0.37 : 0.0;
    int ri = (int)(u2 * (rhi - rlo + 1));
    if (ri > rhi - rlo) ri = rhi - rlo;
    const int r = rlo + ri;
    int d = 0;
    if (a.ND > 1) {
      int di = (int)(u3 * (a.ND - 1));
      if (di > a.ND - 2) di = a.ND - 2;
      d = -a.ND / 2 + 1 + di;
    }
    const double A = no_target ? 0.0 : 0.02 + 0.18 * u4;
    const int dm = ((d % a.ND) + a.ND) % a.ND;
    double ph = (double)(((int64_t)n * r) % a.NR) / a.NR + (double)n * off / a.NR +
                (double)(((int64_t)k * dm) % a.ND) / a.ND + u5;
    ph = ph - floor(ph);
    float sn, cs;
    sincospif((float)(2.0 * ph), &sn, &cs);
    const unsigned long long h = hmix(seed, (unsigned long long)(k * (int64_t)a.S + n) + (1ull << 40));
    const float v1 = (float)u24(h, 40), v2 = (float)u24(h, 16);
    const float rad = sqrtf(-2.0f * logf(v1)) * (1e-3f * 0.70710678118654752f);
    float ns, nc;
    sincospif(2.0f * v2, &ns, &nc);
    const float2 c = a.cal[n];
    const float2 x = make_float2(c.x + (float)A * cs + rad * nc, c.y + (float)A * sn + rad * ns);
    st_c(out, e, x);
  }
}

__global__ void k_fill_u32(uint32_t* p, uint32_t v, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

static unsigned grid_for(int64_t n, int per_thread = 1) {
  int64_t b = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (unsigned)b;
}

hipError_t launch_compact(const int32_t* count, int64_t F, int pn, int32_t* list, int64_t* len, hipStream_t s) {
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, count, F, pn, list, len);
  return hipGetLastError();
}

bool stft_fast_path(int wlen, int hop) { return wlen == STFT_W && hop >= 1 && hop <= 4; }

bool stft64_form(int nfft) {
  const char* mf = std::getenv("FMCW_STFT_MFMA");
  return nfft == 64 && !(mf && mf[0] == '0');
}

hipError_t launch_stft_table(const float* win, int nfft, float2* tab, hipStream_t s) {
  const int64_t n = (int64_t)(nfft / 2 + 1) * STFT_W;
  hipLaunchKernelGGL(k_stft_table, dim3(grid_for(n)), dim3(256), 0, s, win, nfft, tab);
  return hipGetLastError();
}

// CUs of a device, queried once per device (the persistent STFT grids are sized by it)
static int device_cus(int dev) {
  static std::mutex mu;
  static std::map<int, int> cus;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cus.find(dev);
  if (it == cus.end()) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    it = cus.emplace(dev, n).first;
  }
  return it->second;
}

hipError_t launch_stft20(const StftArgs& a, const float2* tab, int mode, float* dst, hipStream_t s, int64_t dst_cap,
                         int64_t tab_cap) {
  if (a.max_seg <= 0) return hipSuccess;
  if (mode < 0 || mode > 4 || !tab) return hipErrorInvalidValue;
  if (!stft_fast_path(a.wlen, a.hop)) return hipErrorInvalidValue;
  if ((mode == 3 || mode == 4) && (!a.bins || a.ncol < 1)) return hipErrorInvalidValue;
  if (a.tiles && (mode != 1 || a.ntiles < 1)) return hipErrorInvalidValue;
  const int64_t blocks = a.tiles ? a.ntiles : (a.max_seg + 255) / 256;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  // What each mode writes, against the capacity the caller states (round 4's GPU fault: a mode-4
  // launch that reached the mode-3 kernel writes [seg][ncol] P columns into the [seg] maxima,
  // DESIGN.md 4.0.2): 0 P [max_seg][nb] at a.P, 2 dB [max_seg][nb] at dst, 3 P [max_seg][ncol]
  // at dst, 4 one maximum per segment at dst; 1 only max(P).  The W table is [nfft/2+1][20].
  const int64_t nb = a.nfft / 2 + 1;
  if (tab_cap < nb * STFT_W) return hipErrorInvalidValue;
  const int64_t need = mode == 0 || mode == 2 ? a.max_seg * nb : mode == 3 ? a.max_seg * a.ncol : mode == 4 ? a.max_seg : 0;
  if (need > 0 && ((mode == 0 ? !a.P : !dst) || dst_cap < need)) return hipErrorInvalidValue;
  // columns per y-block: enough y-blocks for ~2048 workgroups in all, in chunks of 32 columns
  // (mode 4 keeps every column of a segment in one block: its per-segment max is block-local)
  const int ncol = mode == 3 || mode == 4 ? a.ncol : a.nfft / 2 + 1;
  const int64_t chunks = (ncol + 31) / 32;
  int64_t ysplit = (2048 + blocks - 1) / blocks;
  if (ysplit > chunks) ysplit = chunks;
  if (ysplit < 1 || mode == 4) ysplit = 1;
  const int col_chunk = (int)((chunks + ysplit - 1) / ysplit) * 32;
  const dim3 grid((unsigned)blocks, (unsigned)((ncol + col_chunk - 1) / col_chunk));
  // nfft 64 (config 4): P / max(P) on the matrix cores, bit-identical (FMCW_STFT_MFMA=0: VALU)
  const char* mf = std::getenv("FMCW_STFT_MFMA");
  if ((mode == 4 || a.tiles) && mf && mf[0] == '0') return hipErrorInvalidValue;   // matrix-core form only
  // k_stft64f / k_stft64m store 16 bytes per lane at out + 33 s0 (s0 a multiple of 64): an output
  // that is not 16-byte aligned (a caller's slice) takes the table form, whose stores are 4 bytes
  const float* outp = mode == 0 ? a.P : dst;
  const bool out16 = mode == 1 || (reinterpret_cast<uintptr_t>(outp) & 15) == 0;
  if (stft64_form(a.nfft) && mode <= 2 && !a.tiles && !a.table_form && out16) {
    // persistent: a few blocks per CU loop over the tiles (nseg is on the device: the grid covers
    // max_seg's tiles at most, the blocks past the last tile return)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const int cus = device_cus(dev);
    int bpc = 3;
    if (const char* e = std::getenv("FMCW_STFT64_BPC")) bpc = std::max(1, std::min(16, std::atoi(e)));   // A/B
    const char* fe = std::getenv("FMCW_STFT64_FOLD");
    if (!(fe && fe[0] == '0')) {                  // the folded form (default; =0: k_stft64m, bit-identical to k_stft20)
      // persistent: exactly the blocks that are resident at once (the occupancy query of each
      // instantiation, once): a grid past it runs its last blocks as a second round, which cost
      // the first form of this kernel 2x (3 resident blocks per CU against the 4 launched)
      const void* kf = a.hop == 1 ? (mode == 0 ? (const void*)k_stft64f<0, true> : mode == 1 ? (const void*)k_stft64f<1, true>
                                                                                           : (const void*)k_stft64f<2, true>)
                                  : (mode == 0 ? (const void*)k_stft64f<0, false> : mode == 1 ? (const void*)k_stft64f<1, false>
                                                                                              : (const void*)k_stft64f<2, false>);
      static std::mutex mu;
      static std::map<std::pair<int, const void*>, int> occ;   // per (device, instantiation)
      int bpcf;
      {
        std::lock_guard<std::mutex> lk(mu);
        auto it = occ.find({dev, kf});
        if (it == occ.end()) {
          int n = 0;
          if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kf, 256, 0) != hipSuccess || n < 1) n = 1;
          it = occ.emplace(std::make_pair(dev, kf), n).first;
        }
        bpcf = it->second;
      }
      if (const char* e = std::getenv("FMCW_STFT64_BPC")) bpcf = std::max(1, std::min(8, std::atoi(e)));   // A/B
      const int64_t wblocks = (a.max_seg + 255) / 256;                  // 4 waves x 64 segments per block and pass
      const unsigned g = (unsigned)std::min<int64_t>(wblocks, (int64_t)cus * bpcf);
      StftArgs ka = a;
      float* kd = dst;
      void* args[] = {&ka, &kd};
      return hipLaunchKernel(kf, dim3(g), dim3(256), args, 0, s);
    }
    const unsigned g = (unsigned)std::min<int64_t>(blocks, (int64_t)cus * bpc);
    if (mode == 0) hipLaunchKernelGGL(k_stft64m<0>, dim3(g), dim3(256), 0, s, a, tab, dst);
    else if (mode == 1) hipLaunchKernelGGL(k_stft64m<1>, dim3(g), dim3(256), 0, s, a, tab, dst);
    else hipLaunchKernelGGL(k_stft64m<2>, dim3(g), dim3(256), 0, s, a, tab, dst);
    return hipGetLastError();
  }
  if (!(mf && mf[0] == '0')) {      // any other nfft: 32-bin column chunks on the matrix cores
    if (mode == 0) hipLaunchKernelGGL(k_stft_mfma<0>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
    else if (mode == 1) hipLaunchKernelGGL(k_stft_mfma<1>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
    else if (mode == 2) hipLaunchKernelGGL(k_stft_mfma<2>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
    else if (mode == 3) hipLaunchKernelGGL(k_stft_mfma<3>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
    else if (mode == 4) hipLaunchKernelGGL(k_stft_mfma<4>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (mode == 0) hipLaunchKernelGGL(k_stft20<0>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
  else if (mode == 1) hipLaunchKernelGGL(k_stft20<1>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
  else if (mode == 2) hipLaunchKernelGGL(k_stft20<2>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
  else if (mode == 3) hipLaunchKernelGGL(k_stft20<3>, grid, dim3(256), 0, s, a, tab, dst, col_chunk);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_stft_power(const StftArgs& a, hipStream_t s) {
  if (a.max_seg <= 0) return hipSuccess;
  if (a.wlen > STFT_MAX_WLEN || a.hop < 1) return hipErrorInvalidValue;
  const int nb = a.nfft / 2 + 1;
  int seg_tile = 4096 / nb;
  if (seg_tile < 1) seg_tile = 1;
  const int cap = (STFT_MAX_SAMPLES - a.wlen) / a.hop + 1;
  if (seg_tile > cap) seg_tile = cap;
  if (seg_tile > 1024) seg_tile = 1024;
  const int64_t blocks = (a.max_seg + seg_tile - 1) / seg_tile;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stft_power, dim3((unsigned)blocks), dim3(256), 0, s, a, seg_tile);
  return hipGetLastError();
}

hipError_t launch_stft_db(const StftDbArgs& a, hipStream_t s) {
  if (a.max_seg <= 0) return hipSuccess;
  const int nout = a.nlog > 0 ? a.nlog : a.nbins_in;
  const bool aligned = ((reinterpret_cast<uintptr_t>(a.P) | reinterpret_cast<uintptr_t>(a.out)) & 15) == 0;
  if (a.nlog == 0 && aligned) {
    hipLaunchKernelGGL(k_stft_db_flat, dim3(grid_for(a.max_seg * nout, 16)), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_stft_db, dim3(grid_for(a.max_seg * nout, 4)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_synth(const SynthArgs& a, hipStream_t s) {
  const int64_t total = a.nframes * (int64_t)a.C * a.S;
  if (total <= 0) return hipSuccess;
  if (a.dtype == FMCW_C64)
    hipLaunchKernelGGL((k_synth<float2>), dim3(grid_for(total, 4)), dim3(256), 0, s, a);
  else if (a.dtype == FMCW_C32H)
    hipLaunchKernelGGL((k_synth<__half2>), dim3(grid_for(total, 4)), dim3(256), 0, s, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_fill_u32(uint32_t* p, uint32_t v, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(n, 4)), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

}  // namespace fmcw
