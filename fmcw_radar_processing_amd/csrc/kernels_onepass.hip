// kernels_onepass.hip -- single-pass range + Doppler for gfx950: the range
// cube (radar_processing.m:207, `range_tx1rx1_complete`) never leaves the chip.
//
// The two-pass schedule (k_range -> cube in HBM -> k_doppler) moves 8.4 MB per
// config-3 frame for 4.2 MB of algorithmic traffic.  Here a frame is split into
// OP_TILES = 8 range tiles; the workgroup of tile t computes only the bins
// r == t (mod 8), for every chirp, and keeps them on chip (half in VGPRs, half
// in LDS) until its Doppler FFTs are done.  Decimation in frequency makes the
// partial range FFT cheap:
//
//   n = a + 128 b (a < 128, b < 8),  r = t + 8 m (m < 128):
//   X[t + 8m] = sum_a W128^(a m) * [ sum_b y[a + 128 b] W1024^(t (a + 128 b)) ]
//
// i.e. an in-lane 8-term sum ("stage A") and one 128-point FFT per chirp.  The
// price is that each of the 8 tiles reads the whole frame: 1 read from HBM and
// 7 from the XCD's L2.  Blocks b and b+8 share an XCD, so the 8 tiles of a
// frame are blocks 64j + 8t + x (same x): dispatched together, same L2.
//
// The kernel is VALU-issue bound, so the arithmetic is arranged for the fewest
// wave instructions:
// - Calibration and mean removal (:203-204) enter by linearity.  With
//   y[n] = (x[n] - cal[n] - mu) w'[n] (w' = IF_scale * 2 blackman, :205) and
//   mu = mean(x) - mean(cal):
//     X[r] = sum_n x[n] c_t[n] W128^(a m)... - Gh[r] - mean(x) Hh[r],
//     Gh[r] = DFT((cal - mean(cal)) w')[r],  Hh[r] = DFT(w')[r],
//   where c_t[n] = w'[n] W1024^(t n) are 16 per-lane constants and Gh/Hh a
//   per-bin table built on the host in float64 (fmcw_api.cpp).  Stage A is 16
//   complex MACs straight from the loads, and the chirp mean (one wave sum) is
//   applied after the FFT.
// - Complex MACs against per-lane constants are two v_pk_fma_f32 with op_sel /
//   neg_lo modifiers (inline asm: the compiler would keep a rotated copy of
//   every constant), wave sums use DPP-fused adds, the Doppler DFTs run on
//   packed pairs, and the Doppler peak search compares squared magnitudes.
//
// Per chirp (one wave, 16 samples per lane as 8 float4 loads, lane l holds
// a = 2l and 2l+1): stage A, a 64-point cross-lane DIF FFT on each of the two
// sub-sequences (spans 32 and 16 as pair butterflies over v_permlane32/16_swap
// of the two registers, spans 8..1 by DPP, no LDS), one in-lane radix-2 ->
// bins r(l, s) = t + 8 (lane_bin(l) + 64 s), s = 0, 1, then the
// Gh/Hh correction.  Loads run two chirps ahead (a 3-deep register ring).
// Wave w handles chirps k = w + 8 k2 (k2 < 32): slot 0 in VGPRs, slot 1 in LDS.
//
// Doppler (:216-219) for every row of the tile: the mean over chirps and the
// max-abs profile (:210, :265) are reduced across waves in LDS; each lane runs
// a 32-point DFT over its own chirps (k2), a swizzled LDS corner turn (the
// slot-1 region, 128 KiB) hands each (row, d2) column to one thread, which
// applies W256^(w d2) and the 8-point DFT over the waves; fftshift is folded
// into the store index.  Each row's max |D| and its first argmax (:233) are
// kept so detection never reads RD.
//
// Slow-time row (:257-259): the target bin is only known once all 8 tiles'
// profiles exist, so each tile stores |X[r, :]| for its OP_CAND strongest
// in-window bins above range_threshold; k_detect_1p copies the selected row
// from there, and k_slow_fix recomputes the rare row that is not a candidate.
// The fft_data probe (:410-411) is k_probe, a direct DFT of the one chirp.
#include "frame_ops.h"
#include "../../include/fmcw.h"

#include "op_math.h"

namespace fmcw {
namespace op {

constexpr int NW = 8;                  // waves per workgroup (2 per SIMD: 256 VGPRs per lane)
static_assert(NR / OP_TILES == 128, "the lane layout assumes a 128-point sub-FFT");

// LDS image of k_rd1p.
struct Lds1p {
  c2 t1[256 * 64];         // slot-1 tile [chirp][lane]; then the corner turn
  f4v gh[2][64];           // {Gh, Hh} of lane l's bins r0(l), r1(l) (lane order: conflict-free reads)
  float red[2][NW][3][64]; // per-wave {sum.re, sum.im, max |X|^2} of each row over the wave's chirps
  float cand[OP_CAND][256];// candidate rows |X|^2 as [wave][k2] (chirp w + 8 k2), written out coalesced
};

}  // namespace op

// ---------------------------------------------------------------------------
// k_rd1p: one workgroup (8 waves, 2 per SIMD, 256 VGPRs per lane) = one range
// tile of one frame.  FULL: S == NR (no zero padding, no masking).
//
// ---------------------------------------------------------------------------
template <bool FULL, bool H>   // H: fp16 storage (c32h IQ in, c32h RD out), fp32 arithmetic
__global__ __launch_bounds__(64 * op::NW, 1) void k_rd1p(OnePassArgs a) {
  using namespace op;
  constexpr int CPW = 32, C = NW * CPW, ND = C;  // wave w owns chirps w + 8 k2, k2 < 32
  __shared__ __attribute__((aligned(16))) Lds1p L;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar loads / SGPRs
  const int b = blockIdx.x;
  const int64_t f = (int64_t)(b >> 6) * 8 + (b & 7);
  const int t = (b >> 3) & 7;
  if (f >= a.F) return;                          // block-uniform
  const int S = FULL ? NR : a.S;
#ifdef OP_STAMPS2
#ifndef OP_STAMPS
#define OP_STAMPS 1
#endif
#define OP_NST 16
#else
#define OP_NST 8
#endif
#ifdef OP_STAMPS
  if (tid == 0) a.dbg[(int64_t)b * OP_NST] = __builtin_amdgcn_s_memrealtime();
#endif
#ifndef OP_ROT
#define OP_ROT 1
#endif
  // Tile t walks its chirp groups rotated by rs = OP_ROT * t groups (register k2
  // holds chirp w + 8 ((k2 + rs) mod 32)): at any moment the 8 tiles of a frame
  // first-touch 8 different groups instead of all waiting on the same HBM miss,
  // and each group is re-read from L2 within 8 steps (measured: 4 % faster than
  // no rotation; 4 groups per tile overflows the L2 and is 35 % slower).
  const int rs = (OP_ROT * t) & 31;

  // Per-tile tables come from host-built arrays laid out in lane order
  // (fmcw_api.cpp build_onepass_gh), so every table read is a coalesced
  // 512-byte wave access: gathers here would cost the L2 as many requests as
  // the frame itself.
  const c2* __restrict__ tab = reinterpret_cast<const c2*>(a.tab);
  if (tid < 128) L.gh[tid >> 6][lane] = reinterpret_cast<const f4v*>(a.gh)[(2 * t + (tid >> 6)) * 64 + lane];
  // stage-A constants c_t[n] = w'[n] W1024^(t n), n = 2 lane + e + 128 j (0 beyond S: fft(., Nr) zero-padding)
  c2 cst[16];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) cst[2 * j + e] = tab[OP_TAB_CST + ((t * 8 + j) * 2 + e) * 64 + lane];
  c2 twh[5];                                     // spans 32, 16 (every lane), 8, 4, 2 (1 on clear lanes)
  float sg[6];                                   // spans 32 .. 1
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int hh = 32 >> i;
    sg[i] = (lane & hh) ? -1.f : 1.f;
    if (i < 5) twh[i] = tab[OP_TAB_LANE + i * 64 + lane];
  }
  const int m0 = lane_bin(lane);
  const c2 w128 = tab[OP_TAB_LANE + 5 * 64 + lane];
  const int r0 = t + 8 * m0, r1 = r0 + 512;      // this lane's two range bins
#ifdef OP_STAMPS2
  auto stamp2 = [&](int i) { if (tid == 0) a.dbg[(int64_t)b * OP_NST + i] = __builtin_amdgcn_s_memrealtime(); };
#else
  auto stamp2 = [](int) {};
#endif
#ifdef OP_STAMPS
  auto stamp = [&](int i) { if (tid == 0) a.dbg[(int64_t)b * OP_NST + i] = __builtin_amdgcn_s_memrealtime(); };
#else
  auto stamp = [](int) {};
#endif
  stamp(1);
  __syncthreads();

  // ---------------- range phase: :203-205 for chirps w + 8 k2 --------------
  // one load = one sample pair: 16 bytes (c64) or 8 bytes (c32h, half the L2 traffic)
  using TP = std::conditional_t<H, h4v, f4v>;
#ifdef OP_XP_SAMEFR   // diagnostic: every tile of XCD x reads frame x (L2-resident input, no HBM stream)
  const TP* __restrict__ fr = reinterpret_cast<const TP*>(a.iq) + (f & 7) * (int64_t)C * (S >> 1);
#else
  const TP* __restrict__ fr = reinterpret_cast<const TP*>(a.iq) + f * (int64_t)C * (S >> 1);
#endif
  const int S2 = S >> 1;                         // sample pairs per chirp
  const float ninvS = -1.0f / (float)S;
  auto ld_chirp = [&](int k, TP (&x)[8]) {
    const TP* __restrict__ q = fr + (int64_t)k * S2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = lane + 64 * j;               // sample pair: samples 2p, 2p+1
#ifdef OP_XP_NOLOAD  // diagnostic: no input loads (VALU-only range phase)
      x[j] = __builtin_convertvector(f4v{(float)(lane + j), (float)k, (float)(p ^ k), 1.f}, TP);
#else
      if constexpr (FULL) x[j] = (q + 64 * j)[lane];
      else x[j] = q[p < S2 ? p : 0];
#endif
    }
  };
  auto widen = [&](const TP (&bf)[8], f4v (&x)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (H) x[j] = __builtin_convertvector(bf[j], f4v);
      else x[j] = bf[j];
      if constexpr (!FULL)
        if (!(lane + 64 * j < S2)) x[j] = f4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  // 128-point FFT across lanes of (R0, R1) = (a' = 2 lane, 2 lane + 1):
  // spans 32, 16 as pair butterflies, then four 16-point DIFs per register
  auto fft128 = [&](c2& R0, c2& R1) {
    pair_bfly<32>(R0, R1, twh[0]);
    pair_bfly<16>(R0, R1, twh[1]);
    R0 = dif_stage<8>(R0, twh[2], sg[2]);  R1 = dif_stage<8>(R1, twh[2], sg[2]);
    R0 = dif_stage<4>(R0, twh[3], sg[3]);  R1 = dif_stage<4>(R1, twh[3], sg[3]);
    R0 = dif_stage<2>(R0, twh[4], sg[4]);  R1 = dif_stage<2>(R1, twh[4], sg[4]);
    R0 = dif_stage<1>(R0, twh[4], sg[5]);  R1 = dif_stage<1>(R1, twh[4], sg[5]);
    pair_swap32(R0, R1);                          // lane l: E[m], O[m], m = lane_bin(l)
  };
  // :204 the chirp mean, applied to the spectrum: X -= Gh + mean(x) Hh
  auto finish = [&](c2 R0, c2 R1, c2 nmx, f4v g0, f4v g1, c2& X0, c2& X1) {
    const c2 ow = cmv(R1, w128);
    X0 = cmac_a(R0 + ow - g0.xy, nmx, g0.zw);    // bin r0 (slot 0)
    X1 = cmac_a(R0 - ow - g1.xy, nmx, g1.zw);    // bin r1 (slot 1)
  };
#ifndef OP_RING
#define OP_RING 3
#endif
  constexpr int RING = OP_RING;                  // chirps in registers: RING - 1 in flight while one is consumed
                                                 // (3: 1 % over 2 with the rotation; 4 spills)
  c2 tile0[CPW];                                 // slot 1 goes to LDS (L.t1)

  {
    c2 cs7[2];                                   // rotated copies for the last, compiler-visible MAC
    cs7[0] = c2{-cst[14].y, cst[14].x};
    cs7[1] = c2{-cst[15].y, cst[15].x};
    TP buf[RING][8];
#pragma unroll
    for (int i = 0; i < RING - 1; ++i) ld_chirp(w + NW * ((i + rs) & (CPW - 1)), buf[i]);
#ifdef OP_XP_DOPONLY  // diagnostic: no range phase (synthetic tile)
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) {
      tile0[k2] = c2{(float)(lane * k2), (float)(w + k2)};
      L.t1[(w + NW * k2) * 64 + lane] = c2{(float)(lane + k2), (float)(w * k2)};
    }
    if (0)
#endif
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) {
      const int k = w + NW * k2;                 // register order (chirp w + 8 ((k2 + rs) mod 32))
      if (k2 + RING - 1 < CPW) ld_chirp(w + NW * ((k2 + RING - 1 + rs) & (CPW - 1)), buf[(k2 + RING - 1) % RING]);
      f4v x[8];
      widen(buf[k2 % RING], x);
#ifdef OP_XP_NOVALU  // diagnostic: the loads only (a plain sum keeps them live)
      {
        f4v s4 = x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) s4 += x[j];
        tile0[k2] = s4.xy;
        L.t1[k * 64 + lane] = s4.zw;
        continue;
      }
#endif
      // stage A: sum_b x[a + 128 b] c_t[a + 128 b], straight from the loads
      c2 A0 = cmul_a(x[0].xy, cst[0]), A1 = cmul_a(x[0].zw, cst[1]);
      f4v s4 = x[0];
#pragma unroll
      for (int j = 1; j < 7; ++j) {
        A0 = cmac_a(A0, x[j].xy, cst[2 * j]);
        A1 = cmac_a(A1, x[j].zw, cst[2 * j + 1]);
        s4 += x[j];
      }
      A0 = cmacv(A0, x[7].xy, cst[14], cs7[0]);   // compiler-visible producer for the DPP stages
      A1 = cmacv(A1, x[7].zw, cst[15], cs7[1]);
      s4 += x[7];
      fft128(A0, A1);
      const c2 nmx = wave_sum_c(s4.xy + s4.zw) * ninvS;
      c2 X0, X1;
      finish(A0, A1, nmx, L.gh[0][lane], L.gh[1][lane], X0, X1);
      tile0[k2] = X0;
      L.t1[k * 64 + lane] = X1;
    }
  }

#ifdef OP_XP_RANGEONLY  // diagnostic: stop after the range phase (one store keeps it live)
  {
    c2 acc = c2{0.f, 0.f};
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) acc += tile0[k2];
    __syncthreads();
    acc += L.t1[((w + 1) & 7) * 64 + lane];
    a.profile[f * NR + (w * 64 + lane) % NR] = (acc.x + acc.y) * 0.f;   // 0 unless non-finite: no detections downstream
    return;
  }
#endif
  // ---------------- per-row reductions over the 8 waves --------------------
#ifdef OP_STAMPS
  if (lane == 0 && (w == 4 || w == 7)) a.dbg[(int64_t)b * OP_NST + (w == 4 ? 6 : 7)] = __builtin_amdgcn_s_memrealtime();
#endif
  stamp(2);
  __syncthreads();                               // B1: slot 1 complete in LDS
  c2 tile1[CPW];
#pragma unroll
  for (int k2 = 0; k2 < CPW; ++k2) tile1[k2] = L.t1[(w + NW * k2) * 64 + lane];
  {
    c2 s0 = c2{0.f, 0.f}, s1 = c2{0.f, 0.f};
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) {
      s0 += tile0[k2];
      s1 += tile1[k2];
      p0 = fmaxf(p0, abs2v(tile0[k2]));
      p1 = fmaxf(p1, abs2v(tile1[k2]));
    }
    L.red[0][w][0][lane] = s0.x; L.red[0][w][1][lane] = s0.y; L.red[0][w][2][lane] = p0;
    L.red[1][w][0][lane] = s1.x; L.red[1][w][1][lane] = s1.y; L.red[1][w][2][lane] = p1;
  }
  __syncthreads();                               // B2: partials visible; L.t1 read out (free for the corner turn)
  stamp2(8);
  // every wave reduces the 8 partials of its lane's two rows in the same order
  // (identical bits in every wave), so no serial section follows
  c2 mu0 = c2{0.f, 0.f}, mu1 = c2{0.f, 0.f};
  float q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    mu0 += c2{L.red[0][i][0][lane], L.red[0][i][1][lane]};
    mu1 += c2{L.red[1][i][0][lane], L.red[1][i][1][lane]};
    q0 = fmaxf(q0, L.red[0][i][2][lane]);
    q1 = fmaxf(q1, L.red[1][i][2][lane]);
  }
  mu0 *= 1.0f / (float)C;                        // :217 mean over all chirps
  mu1 *= 1.0f / (float)C;
  const float pr0 = sqrtf(q0), pr1 = sqrtf(q1);  // :210 / :265 abs(max(X,[],2))
  stamp(3);
  if (w == 0) {
    a.profile[f * NR + r0] = pr0;
    a.profile[f * NR + r1] = pr1;
  }

  // ---------------- slow-time candidates (:257-259) -------------------------
  int csel[OP_CAND];
  {
    const double dpb = a.dist_per_bin, lo = a.min_d, hi = a.max_d;
    auto key = [&](int r, float p) {
      const double rng = (double)r * dpb;
      return (r >= 1 && r <= NR - 2 && rng >= lo && rng <= hi && p > a.range_thr) ? p : -1.f;
    };
    float v0 = key(r0, pr0), v1 = key(r1, pr1);
#pragma unroll
    for (int c = 0; c < OP_CAND; ++c) {
      float bv = v0;
      int bi = r0;
      if (v1 > bv) { bv = v1; bi = r1; }                           // r0 < r1: ties keep r0
      wave_argmax_dpp(bv, bi);                                      // same result in every wave
      const int sel = (bv < 0.f || a.force_fix) ? -1 : bi;
      if (w == 0 && lane == 0) a.cand_idx[(f * OP_TILES + t) * OP_CAND + c] = sel;
      // |X[sel, k]|^2 of the candidate row (k_detect_1p takes the square root of
      // the one row it keeps); the slot is wave-uniform (r1 = r0 + 512)
      // (staged in LDS by the owning lane, stored coalesced after the next barrier)
      csel[c] = sel;
      f4v* crow = reinterpret_cast<f4v*>(&L.cand[c][w * CPW]);
      if (sel >= 512) {
        if (r1 == sel)
#pragma unroll
          for (int q = 0; q < CPW / 4; ++q)
            crow[q] = f4v{abs2v(tile1[4 * q]), abs2v(tile1[4 * q + 1]), abs2v(tile1[4 * q + 2]), abs2v(tile1[4 * q + 3])};
      } else if (sel >= 0) {
        if (r0 == sel)
#pragma unroll
          for (int q = 0; q < CPW / 4; ++q)
            crow[q] = f4v{abs2v(tile0[4 * q]), abs2v(tile0[4 * q + 1]), abs2v(tile0[4 * q + 2]), abs2v(tile0[4 * q + 3])};
      }
      if (r0 == sel) v0 = -1.f;
      if (r1 == sel) v1 = -1.f;
    }
  }

  stamp2(9);
  // ---------------- Doppler: :217-219 on every row of the tile -------------
  // k = w + 8 k2, d = d2 + 32 d1: each lane's 32-point DFT over its own chirps
  // (W32^(k2 d2)), corner turn through LDS, twiddle W256^(w d2) by the reader,
  // 8-point DFT over the waves (W8^(w d1)).
  auto pre = [&](c2 (&x)[CPW], c2 mu) {
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) x[k2] = (x[k2] - mu) * sload(a.wd, w + NW * ((k2 + rs) & (CPW - 1)));   // :218 (X - mean) .* 2chebwin
    dft32p(x);
  };
  // corner turn [wave][row][d2 ^ sw(row)], sw(row) = 2 (row mod 16): even, so a lane's d2
  // pair (2q, 2q + 1) stays one aligned 16-byte word; conflict-free 8-byte writes
  c2* stg = L.t1;
  const int q2 = tid & 15;                       // the reader's d2 pair: 2 q2, 2 q2 + 1
  // W256^((i + 8 rs) d2): the inter-stage twiddle W256^(i d2) times the W32^(rs d2) of the
  // rotated registers (register r holds chirp group g = r + rs mod 32:
  //   sum_g x_g W32^(g d2) = W32^(rs d2) sum_r x_(r + rs) W32^(r d2)), applied by the reader
  c2 twr[2][NW];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int i = 0; i < NW; ++i) twr[e][i] = tab[OP_TAB_TWR2 + ((i + 8 * rs) & 255) * 32 + 2 * q2 + e];
  // max / min over the 16 lanes of a row (DPP: xor 1, xor 2, then mirrors on group-uniform values)
  auto row_max16 = [&](int v) {
    v = max(v, dppi<0xB1>(v));
    v = max(v, dppi<0x4E>(v));
    v = max(v, dppi<0x141>(v));
    return max(v, dppi<0x140>(v));
  };
  auto row_min16 = [&](int v) {
    v = min(v, dppi<0xB1>(v));
    v = min(v, dppi<0x4E>(v));
    v = min(v, dppi<0x141>(v));
    return min(v, dppi<0x140>(v));
  };
  auto stage = [&](const c2 (&z)[CPW]) {
#pragma unroll
    for (int d2 = 0; d2 < CPW; ++d2) stg[(w * 64 + lane) * CPW + (d2 ^ ((lane & 15) << 1))] = z[d2];
  };
  // Reader: 16 lanes per row, each with a d2 pair and all 8 d1, so it holds the two
  // adjacent elements (2 q2, 2 q2 + 1) of every fftshift-ed column block: 16-byte stores
  // with no lane exchange, 256 contiguous bytes per row and instruction
  auto post = [&](int sl) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {       // 32 rows per pass
      const int lb = (tid >> 4) + 32 * pass;
      const int sw = (lb & 15) << 1;
      c2 v0[NW], v1[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const f4v pr = *reinterpret_cast<const f4v*>(&stg[(i * 64 + lb) * CPW + ((2 * q2) ^ sw)]);
        v0[i] = pr.xy;
        v1[i] = pr.zw;
      }
#pragma unroll
      for (int i = 1; i < NW; ++i) {
        v0[i] = cmul_a(v0[i], twr[0][i]);
        v1[i] = cmul_a(v1[i], twr[1][i]);
      }
      if (rs) {
        v0[0] = cmul_a(v0[0], twr[0][0]);
        v1[0] = cmul_a(v1[0], twr[1][0]);
      }
      dft8p(v0);
      dft8p(v1);
      const int r = t + 8 * lane_bin(lb) + 512 * sl;
      // :219 fftshift(., 2): d1 -> position d1s = (d1 + 4) mod 8, element 2 q2 + e + 32 d1s
      if (a.rd) {                                // RD written: k_detect_1p reads the target rows' peaks from it
        TP* __restrict__ out = reinterpret_cast<TP*>(a.rd) + (f * NR + r) * (int64_t)(ND / 2);
#pragma unroll
        for (int d1s = 0; d1s < NW; ++d1s) {
          const int d1 = (d1s + NW / 2) & (NW - 1);
          const f4v o = f4v{v0[d1].x, v0[d1].y, v1[d1].x, v1[d1].y};
#ifdef OP_XP_NOSTORE  // diagnostic: no RD stores (a never-taken store keeps the values live)
          if (o.x == 1234.5f)
#endif
          // sc0 sc1: write-through stores that drop the line from the XCD's L2, so the RD map
          // (never re-read by this kernel) does not evict input lines the other 7 tiles of the
          // frame still read (measured +1.5 % over plain stores, 2 A/B rounds)
          if constexpr (H) st_wt(out + q2 + 16 * d1s, __builtin_convertvector(o * a.rd_scale, h4v));
          else st_wt(out + q2 + 16 * d1s, o);
        }
        continue;
      }
      // :233 [val, di] = max(abs(.)): exact max of |D|^2 over the row, then its first index
      float qa[NW], qb[NW];
#pragma unroll
      for (int d1s = 0; d1s < NW; ++d1s) {
        qa[d1s] = abs2v(v0[(d1s + NW / 2) & (NW - 1)]);
        qb[d1s] = abs2v(v1[(d1s + NW / 2) & (NW - 1)]);
      }
      float m = fmaxf(qa[0], qb[0]);
#pragma unroll
      for (int d1s = 1; d1s < NW; ++d1s) m = fmaxf(m, fmaxf(qa[d1s], qb[d1s]));
      const float rm = __int_as_float(row_max16(__float_as_int(m)));   // non-negative: int order == float order
      int e = INT_MAX;
#pragma unroll
      for (int d1s = NW - 1; d1s >= 0; --d1s) {
        if (qb[d1s] == rm) e = 2 * q2 + 1 + CPW * d1s;
        if (qa[d1s] == rm) e = 2 * q2 + CPW * d1s;
      }
      e = row_min16(e);
      if (q2 == 0) a.rowpk[f * NR + r] = make_int2(__float_as_int(sqrtf(rm)), e);
    }
  };
  pre(tile0, mu0);
  stage(tile0);                                  // L.t1 was read out before B2; tile0 dies here
  stamp2(10);
  __syncthreads();                               // B3: slot-0 corner turn written (and the candidate rows)
  stamp2(11);
#pragma unroll
  for (int c = 0; c < OP_CAND; ++c)
    if (csel[c] >= 0 && tid < C)
      a.cand_rows[((f * OP_TILES + t) * OP_CAND + c) * (int64_t)C + tid] = L.cand[c][(tid % NW) * CPW + ((tid / NW - rs) & (CPW - 1))];
  post(0);                                       // its LDS reads and stores overlap slot 1's DFT arithmetic
  stamp2(12);
  pre(tile1, mu1);
  stamp2(13);
  __syncthreads();                               // B4: slot-0 corner turn read out
  stage(tile1);
  __syncthreads();                               // B5
  stamp2(14);
  post(1);
  stamp(4);
#ifdef OP_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(5);
#endif
}

// ---------------------------------------------------------------------------
// k_probe: |X[:, k]| of one chirp (radar_processing.m:410-411, fft_data column)
// by a direct DFT: only called when a probe column is requested.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_probe(ProbeArgs a) {
  __shared__ float2 y[1024];
  __shared__ float2 red[16];
  const int tid = threadIdx.x, S = a.S, NR = a.NR;
  const int64_t x0 = (a.frame * (int64_t)a.C + a.chirp) * S;
  auto x = [&](int n) { return op::ld_iq(a.iq, x0 + n, a.h); };
  float2 d = make_float2(0.f, 0.f);
  for (int n = tid; n < S; n += 1024) d = cadd(d, make_float2(x(n).x - a.calw[n].x, x(n).y - a.calw[n].y));
  d = make_float2(op::wave_sum(d.x), op::wave_sum(d.y));
  if ((tid & 63) == 0) red[tid >> 6] = d;
  __syncthreads();
  float2 mu = make_float2(0.f, 0.f);
  for (int i = 0; i < 16; ++i) mu = cadd(mu, red[i]);
  mu = cscale(mu, 1.0f / (float)S);
  for (int n = tid; n < NR; n += 1024) {
    float2 v = make_float2(0.f, 0.f);
    if (n < S) {
      const float4 c = a.calw[n];
      v = cscale(make_float2(x(n).x - c.x - mu.x, x(n).y - c.y - mu.y), c.z);
    }
    y[n] = v;
  }
  __syncthreads();
  for (int r = tid; r < NR; r += 1024) {
    float2 acc = make_float2(0.f, 0.f);
    for (int n = 0; n < NR; ++n) acc = cadd(acc, cmul(y[n], a.tw_nr[((int64_t)n * r) & (NR - 1)]));
    a.probe_mag[r] = sqrtf(cabs2(acc));
  }
}

// ---------------------------------------------------------------------------
// k_detect_1p: one wave per frame.  Peak rule on the profile (:211), Doppler
// index from the row peaks (:227-239), slow-time row from the candidates.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_detect_1p(Detect1pArgs a) {
  constexpr int NR = op::NR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f = (int64_t)blockIdx.x * 4 + w;
  if (f >= a.nframes) return;
  const DetectParams& q = a.det;
  const int C = a.C, M = a.M;
  int sel[8];
  float selv[8];
  const int n = select_peaks<NR, false>(q, lane, a.profile + f * NR, sel, selv);
  float* slow = a.slow_mag + f * C;
  if (n > 0) {
    const int row = sel[0], tt = a.tiles == OP_TILES ? row & (OP_TILES - 1) : xcd_group(row);
    const int32_t* ci = a.cand_idx + (f * a.tiles + tt) * a.ncand;
    int c = -1;
    for (int i = a.ncand - 1; i >= 0; --i)
      if (ci[i] == row) c = i;
    if (c >= 0) {
      const float* src = a.cand_rows + ((f * a.tiles + tt) * a.ncand + c) * (int64_t)C;
      for (int k = lane; k < C; k += 64) slow[k] = sqrtf(src[k]);     // candidates hold |X|^2
    } else if (lane == 0) {
      a.fix_list[atomicAdd(a.fix_count, 1)] = (int32_t)f;
    }
  } else {
    for (int k = lane; k < C; k += 64) slow[k] = 0.f;
  }
  // :233 [val, di] = max(abs(D)) of each target row: from the RD map when it
  // was written (k_rd1p then skips the per-row peak search), else from rowpk
  int2 pkr[8];
  if (a.rd) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < n) {
        const int64_t row = (f * NR + sel[j]) * (int64_t)a.ND;
        float bv = -1.f;
        int bi = INT_MAX;
        for (int e = lane; e < a.ND; e += 64) {
          const float m = sqrtf(cabs2(op::ld_iq(a.rd, row + e, a.rd_h))) * q.rd_unscale;
          if (m > bv) { bv = m; bi = e; }
        }
        wave_argmax(bv, bi);
        pkr[j] = make_int2(__float_as_int(bv), bi);
      }
  }
  if (lane < M) {
    int ri = 0, di = 0;
    float rm = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j == lane && j < n) {
        const int2 pk = a.rd ? pkr[j] : a.rowpk[f * NR + sel[j]];
        di = pk.y + 1;
        if (!(__int_as_float(pk.x) >= q.doppler_thr && di != q.fallback)) di = q.fallback;   // :234-238
        ri = sel[j] + 1;
        rm = selv[j];
      }
    a.ridx[f * M + lane] = ri;
    a.rmag[f * M + lane] = rm;
    a.didx[f * M + lane] = di;
  }
  if (lane == 0) a.count[f] = n;
}

// ---------------------------------------------------------------------------
// k_slow_fix: |X[ridx, k]| by a direct DFT at one bin, for frames whose target
// row was not among the tile's candidates (rare: needs a larger non-peak bin
// of the same tile inside the window).  One wave per chirp.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_slow_fix(SlowFixArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nfix = *a.fix_count;
  const int S = a.S, NR = a.NR, C = a.C;
  const int nmax = S < NR ? S : NR;
  for (int i = blockIdx.x; i < nfix; i += gridDim.x) {
    const int64_t f = a.fix_list[i];
    const int r = a.ridx[f * a.M] - 1;
    for (int k = w; k < C; k += 4) {
      const int64_t x0 = (f * C + k) * (int64_t)S;
      auto xc = [&](int n) { return op::ld_iq(a.iq, x0 + n, a.h); };
      float2 s = make_float2(0.f, 0.f);
      for (int n = lane; n < S; n += 64) {
        const float4 c = a.calw[n];
        s = cadd(s, make_float2(xc(n).x - c.x, xc(n).y - c.y));
      }
      s = make_float2(op::wave_sum(s.x), op::wave_sum(s.y));
      const float2 mu = cscale(s, 1.0f / (float)S);
      float2 acc = make_float2(0.f, 0.f);
      for (int n = lane; n < nmax; n += 64) {
        const float4 c = a.calw[n];
        const float2 y = cscale(make_float2(xc(n).x - c.x - mu.x, xc(n).y - c.y - mu.y), c.z);
        const float2 tw = a.tw_nr[((int64_t)n * r) & (NR - 1)];
        acc = cadd(acc, cmul(y, tw));
      }
      acc = make_float2(op::wave_sum(acc.x), op::wave_sum(acc.y));
      if (lane == 0) a.slow_mag[f * C + k] = sqrtf(cabs2(acc));
    }
  }
}

// ---------------------------------------------------------------------------
bool onepass_supported(int nts, int pn, int nr, int nd) {
  return nr == op::NR && pn == nd && nd == 256 && nts >= 2 && nts <= nr && (nts % 2) == 0;
}

hipError_t launch_onepass(const OnePassArgs& a, hipStream_t s) {
  if (a.F <= 0) return hipSuccess;
  if (!onepass_supported(a.S, a.C, op::NR, a.C)) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)(((a.F + 7) / 8) * 64);
  const dim3 g(blocks), bl(64 * op::NW);
  if (a.S == op::NR) {
    if (a.h) hipLaunchKernelGGL((k_rd1p<true, true>), g, bl, 0, s, a);
    else hipLaunchKernelGGL((k_rd1p<true, false>), g, bl, 0, s, a);
  } else {
    if (a.h) hipLaunchKernelGGL((k_rd1p<false, true>), g, bl, 0, s, a);
    else hipLaunchKernelGGL((k_rd1p<false, false>), g, bl, 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_detect_1p(const Detect1pArgs& a, hipStream_t s) {
  if (a.nframes <= 0) return hipSuccess;
  if (a.NR != op::NR) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_detect_1p, dim3((unsigned)((a.nframes + 3) / 4)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_slow_fix(const SlowFixArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_slow_fix, dim3(64), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_probe(const ProbeArgs& a, hipStream_t s) {
  if (a.S > a.NR || a.NR != op::NR) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

}  // namespace fmcw
