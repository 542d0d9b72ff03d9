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
//   X[t + 8m] = sum_a W128^(a m) * [ W1024^(a t) * sum_b y[a + 128 b] W8^(b t) ]
//
// i.e. an in-lane 8-term sum ("stage A") and one 128-point FFT per chirp.  The
// price is that each of the 8 tiles reads the whole frame: 1 read from HBM and
// 7 from the XCD's L2.  Blocks b and b+8 share an XCD, so the 8 tiles of a
// frame are blocks 64j + 8t + x (same x): dispatched together, same L2.
//
// Calibration and mean removal (:203-204) enter by linearity.  With
// y[n] = (x[n] - cal[n] - mu) w'[n] (w' = IF_scale * 2 blackman, :205) and
// mu = mean(x) - mean(cal):
//   stage A = sum_b x w' W8^(bt) - G_t[a] - mean(x) H_t[a],
//   G_t[a] = sum_b (cal - mean(cal)) w' W8^(bt),  H_t[a] = sum_b w' W8^(bt),
// two per-lane constants per sub-sequence (built once per workgroup, in LDS),
// so a chirp is consumed straight from its loads: no calibrated copy, and the
// chirp mean is one wave sum that is applied after stage A.
//
// Per chirp (one wave, 16 samples per lane as 8 float4 loads, lane l holds
// a = 2l and 2l+1): stage A as the float4s arrive (the next chirp's first half
// is requested as soon as this chirp's first half is consumed: a rolling
// prefetch that keeps >= 4 loads per lane in flight in 32 VGPRs), the mean
// correction, a 64-point cross-lane DIF FFT on each of the two sub-sequences
// (DPP and v_permlane16/32_swap exchanges, no LDS), one in-lane radix-2 ->
// bins r(l, s) = t + 8 (bitrev6(l) + 64 s), s = 0, 1.
// Wave w handles chirps k = w + 16 k2 (k2 < 16): slot 0 in VGPRs, slot 1 in LDS.
//
// Doppler (:216-219) for every row of the tile: the mean over chirps and the
// max-abs profile (:210, :265) are reduced across waves in LDS; each lane runs
// a 16-point DFT over its own chirps (k2), twiddles by W256^(w d2), and the
// last 16-point DFT over the waves goes through an XOR-swizzled LDS corner
// turn (the slot-1 region, 128 KiB), one slot (64 rows) at a time; fftshift
// is folded into the store index.  Each row's max |D| and its first argmax
// (:233) are kept so detection never reads RD.
//
// Slow-time row (:257-259): the target bin is only known once all 8 tiles'
// profiles exist, so each tile stores |X[r, :]| for its OP_CAND strongest
// in-window bins above range_threshold; k_detect_1p copies the selected row
// from there, and k_slow_fix recomputes the rare row that is not a candidate.
#include "frame_ops.h"
#include "../../include/fmcw.h"

namespace fmcw {
namespace op {

constexpr int NR = 1024;
constexpr int NW = 8;                  // waves per workgroup (2 per SIMD: 256 VGPRs per lane)
static_assert(NR / OP_TILES == 128, "the lane layout assumes a 128-point sub-FFT");

using c2 = f2v;                        // complex (re, im) in a packed-fp32 register pair

// a * b in two packed ops: a.re * (b.re, b.im) + a.im * (-b.im, b.re)
__device__ __forceinline__ c2 cmv(c2 a, c2 b) { return __builtin_elementwise_fma(a.yy, c2{-b.y, b.x}, a.xx * b); }
// acc + a * b given bs = (-b.im, b.re)
__device__ __forceinline__ c2 cmacv(c2 acc, c2 a, c2 b, c2 bs) {
  return __builtin_elementwise_fma(a.yy, bs, __builtin_elementwise_fma(a.xx, b, acc));
}
__device__ __forceinline__ c2 tov(float2 v) { return c2{v.x, v.y}; }
__device__ __forceinline__ float2 tof(c2 v) { return make_float2(v.x, v.y); }
__device__ __forceinline__ float abs2v(c2 v) { return fmaf(v.x, v.x, v.y * v.y); }

template <int CTRL> __device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Value of lane ^ H, H < 16, by DPP (FFT data: not uniform inside groups).
template <int H> __device__ __forceinline__ float xpart(float v, int lane) {
  if constexpr (H == 1) return dppf<0xB1>(v);            // quad_perm [1,0,3,2]
  if constexpr (H == 2) return dppf<0x4E>(v);            // quad_perm [2,3,0,1]
  if constexpr (H == 8) return dppf<0x128>(v);           // row_ror:8 == xor 8 inside a row
  const float p = dppf<0x12C>(v), m = dppf<0x124>(v);    // row_ror:12 (l+4), row_ror:4 (l-4)
  return (lane & 4) ? m : p;
}
// (value of the bit-H-clear lane, value of the bit-H-set lane) of this lane's pair, H = 16, 32
template <int H> __device__ __forceinline__ void xhalves(float v, float& lo, float& hi) {
  if constexpr (H == 32) {   // lanes 32-63 of the first operand swap with lanes 0-31 of the second
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
  } else {                   // odd rows of the first operand swap with even rows of the second
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
  }
}

// Wave-wide sum.  Symmetric pairings only (xor 1, xor 2, half-mirror and
// mirror on group-uniform values, then the two half swaps), so a + b == b + a
// gives every lane the same bits.
__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);       // row_half_mirror: quads are uniform, so this is xor 4
  v += dppf<0x140>(v);       // row_mirror: 8-lane groups are uniform, so this is xor 8
  float lo, hi;
  xhalves<16>(v, lo, hi);
  v = lo + hi;
  xhalves<32>(v, lo, hi);
  return lo + hi;
}

// One radix-2 DIF stage of span H across lanes: bit-H-clear lane -> a + b,
// bit-H-set lane -> (a - b) * tw.  sg = -1 on set lanes, +1 on clear lanes.
template <int H>
__device__ __forceinline__ c2 dif_stage(c2 x, int lane, c2 tw, float sg) {
  c2 u;
  if constexpr (H >= 16) {
    float lr, hr, li, hi;
    xhalves<H>(x.x, lr, hr);
    xhalves<H>(x.y, li, hi);
    u = __builtin_elementwise_fma(c2{sg, sg}, c2{hr, hi}, c2{lr, li});
  } else {
    const c2 o = c2{xpart<H>(x.x, lane), xpart<H>(x.y, lane)};   // the partner's value
    u = __builtin_elementwise_fma(c2{sg, sg}, x, o);              // clear: o + x, set: o - x
  }
  return H == 1 ? u : cmv(u, tw);
}

// Wave-uniform table read through the constant address space: an s_load into
// SGPRs instead of a vector load into VGPRs (the index must be wave-uniform).
__device__ __forceinline__ float sload(const float* p, int i) {
  return ((const __attribute__((address_space(4))) float*)p)[i];
}
__device__ __forceinline__ float2 sload(const float2* p, int i) {
  const f2v v = ((const __attribute__((address_space(4))) f2v*)p)[i];
  return make_float2(v.x, v.y);
}

__device__ __forceinline__ int bitrev6(int l) { return (int)(__brev((unsigned)l) >> 26); }


// 32-point forward DFT in registers (natural order): radix-2 over two dft<16>.
__device__ __forceinline__ void dft32(float2 (&v)[32]) {
  constexpr float kc[16] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                            0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                            0.19509032201612826785f, 0.0f, -0.19509032201612826785f, -0.38268343236508977173f,
                            -0.55557023301960222474f, -0.70710678118654752440f, -0.83146961230254523708f,
                            -0.92387953251128675613f, -0.98078528040323044913f};
  constexpr float ks[16] = {0.0f, 0.19509032201612826785f, 0.38268343236508977173f, 0.55557023301960222474f,
                            0.70710678118654752440f, 0.83146961230254523708f, 0.92387953251128675613f,
                            0.98078528040323044913f, 1.0f, 0.98078528040323044913f, 0.92387953251128675613f,
                            0.83146961230254523708f, 0.70710678118654752440f, 0.55557023301960222474f,
                            0.38268343236508977173f, 0.19509032201612826785f};
  float2 e[16], o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    e[i] = v[2 * i];
    o[i] = v[2 * i + 1];
  }
  dft<16>(e);
  dft<16>(o);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float2 ot = k == 0 ? o[0] : cmul(o[k], make_float2(kc[k], -ks[k]));   // W32^k
    v[k] = cadd(e[k], ot);
    v[k + 16] = csub(e[k], ot);
  }
}

// LDS image of k_rd1p.
struct Lds1p {
  c2 t1[256 * 64];         // slot-1 tile [chirp][lane]; then the reduction scratch; then the corner turn
  c2 w[8 * 64];            // {w'[2l + 128j], w'[2l + 1 + 128j]} at [j][l]
  c2 g[128], h[128];       // G'_t[a], H'_t[a] (times W1024^(a t))
  c2 mu[2][64];
  float prof[2][64];
  int cand[OP_CAND];
};

}  // namespace op

// ---------------------------------------------------------------------------
// k_rd1p: one workgroup (8 waves, 2 per SIMD, 256 VGPRs per lane) = one range
// tile of one frame.  FULL: S == NR (no zero padding, no masking).
// ---------------------------------------------------------------------------
template <bool FULL>
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

  // ---- per-workgroup tables: window pairs, G'/H' (linearity constants) ----
  {
    const int n0 = 2 * lane + 128 * w;           // (j, l) = (w, lane)
    L.w[tid] = c2{n0 < S ? a.calw[n0].z : 0.f, n0 + 1 < S ? a.calw[n0 + 1].z : 0.f};
  }
  if (tid < 128) {                               // a = tid
    c2 g = c2{0.f, 0.f}, h = c2{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = tid + 128 * j;
      if (n < S) {
        const float4 cw = a.calw[n];
        const c2 c8 = tov(sload(a.tw_nr, (128 * j * t) & (NR - 1)));
        const c2 cc = c2{cw.x - a.cal_mean.x, cw.y - a.cal_mean.y} * cw.z;
        g = cmacv(g, cc, c8, c2{-c8.y, c8.x});
        h = __builtin_elementwise_fma(c2{cw.z, cw.z}, c8, h);
      }
    }
    const c2 ta = tov(a.tw_nr[(tid * t) & (NR - 1)]);
    L.g[tid] = cmv(g, ta);
    L.h[tid] = cmv(h, ta);
  }

  // per-lane / per-tile twiddles (all from the float64-rounded table)
  const c2 twa0 = tov(a.tw_nr[(2 * lane * t) & (NR - 1)]);
  const c2 twa1 = tov(a.tw_nr[((2 * lane + 1) * t) & (NR - 1)]);
  c2 w8[8], w8s[8];                              // W8^(j t): wave-uniform (SGPRs)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    w8[j] = tov(sload(a.tw_nr, (128 * j * t) & (NR - 1)));
    w8s[j] = c2{-w8[j].y, w8[j].x};
  }
  c2 twh[5];                                     // spans 32, 16, 8, 4, 2 (1 on clear lanes)
  float sg[6];                                   // spans 32 .. 1
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int hh = 32 >> i;
    sg[i] = (lane & hh) ? -1.f : 1.f;
    if (i < 5) twh[i] = (lane & hh) ? tov(a.tw_nr[((lane & (hh - 1)) * (512 / hh)) & (NR - 1)]) : c2{1.f, 0.f};
  }
  const int m0 = bitrev6(lane);
  const c2 w128 = tov(a.tw_nr[8 * m0]);
  const int r0 = t + 8 * m0, r1 = r0 + 512;      // this lane's two range bins
  __syncthreads();

  // ---------------- range phase: :203-205 for chirps w + 8 k2 --------------
  const f4v* __restrict__ fr = reinterpret_cast<const f4v*>(a.iq + f * (int64_t)C * S);
  const int S2 = S >> 1;                         // float4 (sample pairs) per chirp
  const float invS = 1.0f / (float)S;
  auto ld_chirp = [&](int k, f4v (&x)[8]) {
    const f4v* __restrict__ q = fr + (int64_t)k * S2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = lane + 64 * j;               // sample pair: samples 2p, 2p+1
      if constexpr (FULL) x[j] = (q + 64 * j)[lane];
      else x[j] = q[p < S2 ? p : 0];
    }
  };
  float2 tile0[CPW];                             // slot 1 goes to LDS (L.t1)
  f4v buf[3][8];                                 // chirp ring: 2 chirps in flight while one is consumed
  ld_chirp(w, buf[0]);
  ld_chirp(w + NW, buf[1]);
#pragma unroll
  for (int k2 = 0; k2 < CPW; ++k2) {
    const int k = w + NW * k2;
    if (k2 + 2 < CPW) ld_chirp(k + 2 * NW, buf[(k2 + 2) % 3]);
    const f4v (&x)[8] = buf[k2 % 3];
    c2 B0, B1, sx = c2{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {                // stage A straight from the loads
      f4v v = x[j];
      if constexpr (!FULL)
        if (!(lane + 64 * j < S2)) v = f4v{0.f, 0.f, 0.f, 0.f};
      const c2 wv = L.w[j * 64 + lane];
      const c2 z0 = v.xy * wv.x, z1 = v.zw * wv.y;    // x .* (IF_scale * 2 blackman)
      sx += v.xy + v.zw;
      if (j == 0) {
        B0 = z0;
        B1 = z1;
      } else {                                   // sum_b y[a + 128 b] W8^(b t)
        B0 = cmacv(B0, z0, w8[j], w8s[j]);
        B1 = cmacv(B1, z1, w8[j], w8s[j]);
      }
    }
    // :204 mean over the S samples, applied after stage A (linearity)
    const c2 mx = c2{wave_sum(sx.x), wave_sum(sx.y)} * invS;
    const c2 mxs = c2{-mx.y, mx.x};
    const f4v g = reinterpret_cast<const f4v*>(L.g)[lane];
    const f4v h = reinterpret_cast<const f4v*>(L.h)[lane];
    c2 A0 = cmv(B0, twa0) - cmacv(g.xy, h.xy, mx, mxs);   // * W1024^(a t), - G' - mean(x) H'
    c2 A1 = cmv(B1, twa1) - cmacv(g.zw, h.zw, mx, mxs);
    A0 = dif_stage<32>(A0, lane, twh[0], sg[0]); A1 = dif_stage<32>(A1, lane, twh[0], sg[0]);
    A0 = dif_stage<16>(A0, lane, twh[1], sg[1]); A1 = dif_stage<16>(A1, lane, twh[1], sg[1]);
    A0 = dif_stage<8>(A0, lane, twh[2], sg[2]);  A1 = dif_stage<8>(A1, lane, twh[2], sg[2]);
    A0 = dif_stage<4>(A0, lane, twh[3], sg[3]);  A1 = dif_stage<4>(A1, lane, twh[3], sg[3]);
    A0 = dif_stage<2>(A0, lane, twh[4], sg[4]);  A1 = dif_stage<2>(A1, lane, twh[4], sg[4]);
    A0 = dif_stage<1>(A0, lane, twh[4], sg[5]);  A1 = dif_stage<1>(A1, lane, twh[4], sg[5]);
    const c2 ow = cmv(A1, w128);
    const c2 X0 = A0 + ow, X1 = A0 - ow;         // bins r0, r1 of chirp k
    tile0[k2] = tof(X0);
    L.t1[k * 64 + lane] = X1;
    if (f == a.probe_frame && k == a.probe_chirp && a.probe_mag) {   // :410-411 |cube(:, col)|
      a.probe_mag[r0] = sqrtf(abs2v(X0));
      a.probe_mag[r1] = sqrtf(abs2v(X1));
    }
  }

  // ---------------- per-row reductions over the 8 waves --------------------
  __syncthreads();                               // slot 1 complete in LDS
  float2 tile1[CPW];
#pragma unroll
  for (int k2 = 0; k2 < CPW; ++k2) tile1[k2] = tof(L.t1[(w + NW * k2) * 64 + lane]);
  c2 s0 = c2{0.f, 0.f}, s1 = c2{0.f, 0.f};
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int k2 = 0; k2 < CPW; ++k2) {
    s0 += tov(tile0[k2]);
    s1 += tov(tile1[k2]);
    p0 = fmaxf(p0, cabs2(tile0[k2]));
    p1 = fmaxf(p1, cabs2(tile1[k2]));
  }
  __syncthreads();                               // L.t1 read out: reuse it as reduction scratch
  float* red = reinterpret_cast<float*>(L.t1);   // [slot][wave][lane][3]
  red[((0 * NW + w) * 64 + lane) * 3 + 0] = s0.x;
  red[((0 * NW + w) * 64 + lane) * 3 + 1] = s0.y;
  red[((0 * NW + w) * 64 + lane) * 3 + 2] = p0;
  red[((1 * NW + w) * 64 + lane) * 3 + 0] = s1.x;
  red[((1 * NW + w) * 64 + lane) * 3 + 1] = s1.y;
  red[((1 * NW + w) * 64 + lane) * 3 + 2] = p1;
  __syncthreads();
  if (tid < 128) {
    const int sl = tid >> 6;
    c2 sum = c2{0.f, 0.f};
    float pm = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const float* rr = red + ((sl * NW + i) * 64 + lane) * 3;
      sum += c2{rr[0], rr[1]};
      pm = fmaxf(pm, rr[2]);
    }
    const float pr = sqrtf(pm);                                    // :210 / :265 abs(max(X,[],2))
    L.mu[sl][lane] = sum * (1.0f / (float)C);                      // :217 mean over all chirps
    L.prof[sl][lane] = pr;
    a.profile[f * NR + (sl ? r1 : r0)] = pr;
  }
  __syncthreads();

  // ---------------- slow-time candidates (:257-259) -------------------------
  if (w == 0) {
    const double dpb = a.dist_per_bin, lo = a.min_d, hi = a.max_d;
    auto key = [&](int r, float p) {
      const double rng = (double)r * dpb;
      return (r >= 1 && r <= NR - 2 && rng >= lo && rng <= hi && p > a.range_thr) ? p : -1.f;
    };
    float v0 = key(r0, L.prof[0][lane]), v1 = key(r1, L.prof[1][lane]);
#pragma unroll
    for (int c = 0; c < OP_CAND; ++c) {
      float bv = v0;
      int bi = r0;
      if (v1 > bv) { bv = v1; bi = r1; }                           // r0 < r1: ties keep r0
      wave_argmax(bv, bi);
      const int sel = (bv < 0.f || a.force_fix) ? -1 : bi;
      if (lane == 0) {
        a.cand_idx[(f * OP_TILES + t) * OP_CAND + c] = sel;
        L.cand[c] = sel;
      }
      if (r0 == sel) v0 = -1.f;
      if (r1 == sel) v1 = -1.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < OP_CAND; ++c) {
    const int rc = L.cand[c];
    if (rc >= 0) {
      const int q = (rc - t) >> 3, sc = q >> 6, lc = bitrev6(q & 63);
      if (lane == lc) {
        float* row = a.cand_rows + ((f * OP_TILES + t) * OP_CAND + c) * (int64_t)C;
#pragma unroll
        for (int k2 = 0; k2 < CPW; ++k2) row[w + NW * k2] = sqrtf(cabs2(sc ? tile1[k2] : tile0[k2]));
      }
    }
  }

  // ---------------- Doppler: :217-219 on every row of the tile -------------
  // k = w + 8 k2, d = d2 + 32 d1: each lane's 32-point DFT over its own chirps
  // (W32^(k2 d2)), corner turn through LDS, twiddle W256^(w d2) by the reader,
  // 8-point DFT over the waves (W8^(w d1)).
  auto pre = [&](float2 (&x)[CPW], c2 mu) {
#pragma unroll
    for (int k2 = 0; k2 < CPW; ++k2) x[k2] = tof((tov(x[k2]) - mu) * sload(a.wd, w + NW * k2));   // :218 (X - mean) .* 2chebwin
    dft32(x);
  };
  c2* stg = L.t1;                                // [wave][row lane][d2 ^ (lane & 31)]: conflict-free both ways
  auto post = [&](const float2 (&z)[CPW], int sl) {
#pragma unroll
    for (int d2 = 0; d2 < CPW; ++d2) stg[(w * 64 + lane) * CPW + (d2 ^ (lane & 31))] = tov(z[d2]);
    __syncthreads();
    const int d2o = tid & 31;
    float2 tw[NW];                               // W256^(i d2o): the inter-stage twiddle, applied by the reader
#pragma unroll
    for (int i = 1; i < NW; ++i) tw[i] = a.tw_nd[(i * d2o) & (ND - 1)];
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {       // 16 rows per pass, 32 threads per row
      const int lb = (tid >> 5) + 16 * pass;
      float2 v[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) v[i] = tof(stg[(i * 64 + lb) * CPW + (d2o ^ (lb & 31))]);
#pragma unroll
      for (int i = 1; i < NW; ++i) v[i] = cmul(v[i], tw[i]);
      dft<NW>(v);
      const int r = t + 8 * bitrev6(lb) + 512 * sl;
      float2* __restrict__ out = a.rd ? a.rd + (f * NR + r) * (int64_t)ND : nullptr;
      float bv = -1.f;
      int bi = INT_MAX;
#pragma unroll
      for (int d1s = 0; d1s < NW; ++d1s) {                          // :219 fftshift(., 2)
        const float2 val = v[(d1s + NW / 2) & (NW - 1)];
        const int e = d2o + CPW * d1s;
        const float mag = sqrtf(cabs2(val));
        if (mag > bv) { bv = mag; bi = e; }
        if (out) out[e] = val;
      }
#pragma unroll
      for (int o = CPW / 2; o > 0; o >>= 1) {                       // :233 max(abs(.)) over the row
        const float ov = __shfl_xor(bv, o);
        const int oi = __shfl_xor(bi, o);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if (d2o == 0) a.rowpk[f * NR + r] = make_int2(__float_as_int(bv), bi);
    }
  };
  pre(tile0, L.mu[0][lane]);
  pre(tile1, L.mu[1][lane]);
  post(tile0, 0);
  __syncthreads();                               // slot-0 corner turn read out
  post(tile1, 1);
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
    const int row = sel[0], tt = row & (OP_TILES - 1);
    const int32_t* ci = a.cand_idx + (f * OP_TILES + tt) * OP_CAND;
    int c = -1;
#pragma unroll
    for (int i = OP_CAND - 1; i >= 0; --i)
      if (ci[i] == row) c = i;
    if (c >= 0) {
      const float* src = a.cand_rows + ((f * OP_TILES + tt) * OP_CAND + c) * (int64_t)C;
      for (int k = lane; k < C; k += 64) slow[k] = src[k];
    } else if (lane == 0) {
      a.fix_list[atomicAdd(a.fix_count, 1)] = (int32_t)f;
    }
  } else {
    for (int k = lane; k < C; k += 64) slow[k] = 0.f;
  }
  if (lane < M) {
    int ri = 0, di = 0;
    float rm = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j == lane && j < n) {
        const int2 pk = a.rowpk[f * NR + sel[j]];
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
      const float2* __restrict__ xc = a.iq + (f * C + k) * (int64_t)S;
      float2 s = make_float2(0.f, 0.f);
      for (int n = lane; n < S; n += 64) {
        const float4 c = a.calw[n];
        s = cadd(s, make_float2(xc[n].x - c.x, xc[n].y - c.y));
      }
      s = make_float2(op::wave_sum(s.x), op::wave_sum(s.y));
      const float2 mu = cscale(s, 1.0f / (float)S);
      float2 acc = make_float2(0.f, 0.f);
      for (int n = lane; n < nmax; n += 64) {
        const float4 c = a.calw[n];
        const float2 y = cscale(make_float2(xc[n].x - c.x - mu.x, xc[n].y - c.y - mu.y), c.z);
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
  if (a.S == op::NR)
    hipLaunchKernelGGL((k_rd1p<true>), dim3(blocks), dim3(64 * op::NW), 0, s, a);
  else
    hipLaunchKernelGGL((k_rd1p<false>), dim3(blocks), dim3(64 * op::NW), 0, s, a);
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

}  // namespace fmcw
