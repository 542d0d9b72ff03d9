// op_math.h -- register-level building blocks shared by the single-pass kernels
// (kernels_onepass.hip: k_rd1p, 8 range tiles per frame; kernels_xcd.hip: k_rdx,
// the chirp-split XCD-team schedule): packed complex MACs with op_sel modifiers,
// DPP / permlane lane exchanges, wave reductions and the packed small DFTs.
#pragma once
#include "frame_ops.h"

namespace fmcw {
namespace op {

constexpr int NR = 1024;

using c2 = f2v;                        // complex (re, im) in a packed-fp32 register pair
typedef _Float16 h4v __attribute__((ext_vector_type(4)));   // two fp16-storage samples (FMCW_C32H)

// Sample i of an IQ buffer holding c64 (h = 0) or c32h (h = 1) values.
__device__ __forceinline__ float2 ld_iq(const void* p, int64_t i, int h) {
  if (h) return __half22float2(static_cast<const __half2*>(p)[i]);
  return static_cast<const float2*>(p)[i];
}

// a * b in two packed ops: a.re * (b.re, b.im) + a.im * (-b.im, b.re)
__device__ __forceinline__ c2 cmv(c2 a, c2 b) { return __builtin_elementwise_fma(a.yy, c2{-b.y, b.x}, a.xx * b); }
// acc + a * b given bs = (-b.im, b.re)
__device__ __forceinline__ c2 cmacv(c2 acc, c2 a, c2 b, c2 bs) {
  return __builtin_elementwise_fma(a.yy, bs, __builtin_elementwise_fma(a.xx, b, acc));
}
// acc + a * b and a * b against a per-lane VGPR constant b: the rotation of b
// is done by operand modifiers (op_sel picks b.im for the low half, neg_lo
// negates it), so no rotated copy of b is kept.  Results must not feed a
// DPP / permlane op directly (the hazard recognizer does not see inline asm).
__device__ __forceinline__ c2 cmac_a(c2 acc, c2 a, c2 b) {
  c2 t, r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(a), "v"(b), "v"(acc));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ c2 cmul_a(c2 a, c2 b) {
  c2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
// 16-byte / 8-byte write-through store (global_store ... sc0 sc1): the line leaves the XCD's L2
#ifdef OP_RD_PLAIN
__device__ __forceinline__ void st_wt(f4v* p, f4v v) { *p = v; }
__device__ __forceinline__ void st_wt(h4v* p, h4v v) { *p = v; }
#else
// The s_nop covers the store-data hazard the compiler cannot see through inline asm: a
// VALU write to the data VGPRs of a > 8-byte VMEM store right after it needs wait states
// (without it the next lane-pair exchange overwrote the data before the store read it).
__device__ __forceinline__ void st_wt(f4v* p, f4v v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_wt(h4v* p, h4v v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}
#endif
__device__ __forceinline__ c2 tov(float2 v) { return c2{v.x, v.y}; }
__device__ __forceinline__ float2 tof(c2 v) { return make_float2(v.x, v.y); }
__device__ __forceinline__ float abs2v(c2 v) { return fmaf(v.x, v.x, v.y * v.y); }
__device__ __forceinline__ c2 mnegi(c2 a) { return c2{a.y, -a.x}; }   // a * (-i)
// a + (-i) b = (a.re + b.im, a.im - b.re) and a + i b = (a.re - b.im, a.im + b.re) as ONE
// v_pk_add_f32 (op_sel swaps b's halves, neg_* flips one of them): the compiler would
// build the rotated b with moves and sign flips first.  Not fed to DPP/permlane (the
// Doppler DFTs only): no hazard the compiler cannot see.
__device__ __forceinline__ c2 add_mi(c2 a, c2 b) {
  c2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ c2 add_pi(c2 a, c2 b) {
  c2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// DPP lane read; old = 0 with bound_ctrl lets the compiler fuse the move
// into the consuming VOP2 (v_add_f32_dpp, v_max_u32_dpp, ...).
template <int CTRL> __device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL> __device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

// Value of lane ^ H, H < 16, by DPP (FFT data: not uniform inside groups).
template <int H> __device__ __forceinline__ float xpart(float v) {
  if constexpr (H == 1) return dppf<0xB1>(v);            // quad_perm [1,0,3,2]
  if constexpr (H == 2) return dppf<0x4E>(v);            // quad_perm [2,3,0,1]
  if constexpr (H == 8) return dppf<0x128>(v);           // row_ror:8 == xor 8 inside a row
  return dppf<0x1B>(dppf<0x141>(v));                     // row_half_mirror (7-i), then quad_perm [3,2,1,0]: i ^ 4
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

// Wave-wide max / min of an int by DPP and the two half swaps (no LDS
// round trips): xor 1, xor 2, then the mirrors on group-uniform values, then
// the 16- and 32-lane swaps.  Every lane ends with the result.
template <bool MAX> __device__ __forceinline__ int wave_red_i(int v) {
  auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
  v = op(v, dppi<0xB1>(v));
  v = op(v, dppi<0x4E>(v));
  v = op(v, dppi<0x141>(v));
  v = op(v, dppi<0x140>(v));
  auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  v = op((int)r[0], (int)r[1]);
  r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return op((int)r[0], (int)r[1]);
}
// wave_argmax for keys that are either > 0 or -1 (frame_ops.h rule: largest
// value, ties -> lowest index): positive floats order as their int bits.
__device__ __forceinline__ void wave_argmax_dpp(float& v, int& i) {
  const int key = v < 0.f ? -1 : __float_as_int(v);
  const int m = wave_red_i<true>(key);
  i = wave_red_i<false>(key == m ? i : INT_MAX);
  v = m < 0 ? -1.f : __int_as_float(m);
}

// One radix-2 DIF stage of span H across lanes: bit-H-clear lane -> a + b,
// bit-H-set lane -> (a - b) * tw.  sg = -1 on set lanes, +1 on clear lanes.
template <int H>
__device__ __forceinline__ c2 dif_stage(c2 x, c2 tw, float sg) {
  c2 u;
  if constexpr (H >= 16) {
    float lr, hr, li, hi;
    xhalves<H>(x.x, lr, hr);
    xhalves<H>(x.y, li, hi);
    u = __builtin_elementwise_fma(c2{sg, sg}, c2{hr, hi}, c2{lr, li});
  } else {
    const c2 o = c2{xpart<H>(x.x), xpart<H>(x.y)};               // the partner's value
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

// Sub-bin m (r = t + 8 m) of lane l's slot-0 value after the range FFT below:
// 4 bitrev4(l mod 16) + l / 16 (the two pair stages leave the four 16-point
// sub-FFTs of each half-sequence in the four 16-lane rows).
__device__ __forceinline__ int lane_bin(int l) { return (int)(__brev((unsigned)(l & 15)) >> 26) + (l >> 4); }

// Pair butterfly of span H (32 or 16) on two registers: one half swap per
// component gives every lane both operands of one butterfly (no copies), and it
// keeps both outputs: R0 <- lo + hi, R1 <- (lo - hi) * tw.  Lane l < H-block
// handles R0's pair, the other block R1's pair (see lane_bin).
template <int H> __device__ __forceinline__ void pair_bfly(c2& R0, c2& R1, c2 tw) {
  const auto rx = H == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(R0.x), __float_as_uint(R1.x), false, false)
                          : __builtin_amdgcn_permlane16_swap(__float_as_uint(R0.x), __float_as_uint(R1.x), false, false);
  const auto ry = H == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(R0.y), __float_as_uint(R1.y), false, false)
                          : __builtin_amdgcn_permlane16_swap(__float_as_uint(R0.y), __float_as_uint(R1.y), false, false);
  const c2 lo = c2{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
  const c2 hi = c2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  R0 = lo + hi;
  R1 = cmv(lo - hi, tw);
}
// The final half swap without arithmetic: lane l then holds (E[m], O[m]) of
// one sub-bin m = lane_bin(l).
__device__ __forceinline__ void pair_swap32(c2& R0, c2& R1) {
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(R0.x), __float_as_uint(R1.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(R0.y), __float_as_uint(R1.y), false, false);
  R0 = c2{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
  R1 = c2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}

// Wave-wide complex sum, every lane gets it.  The 16-lane swap of re against im
// first puts re partials in rows 0, 2 and im partials in rows 1, 3 of ONE
// register, so the four DPP levels run once (symmetric pairings: identical bits
// in every lane of a row), then the 32-lane swap adds the row pairs and a last
// 16-lane swap spreads re and im to every lane.
__device__ __forceinline__ c2 wave_sum_c(c2 s) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s.x), __float_as_uint(s.y), false, false);
  float v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float u = __uint_as_float(q[0]) + __uint_as_float(q[1]);
  const auto z = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
  return c2{__uint_as_float(z[0]), __uint_as_float(z[1])};
}

// ---- packed small DFTs (natural order in and out) ------------------------
__device__ __forceinline__ void dft4p(c2& a0, c2& a1, c2& a2, c2& a3) {
  const c2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = add_mi(t1, d);                            // t1 + (-i) d
  a3 = add_pi(t1, d);                            // t1 - (-i) d
}
// the same with a2 entering as (-i) a2 (the W16^4 twiddle of dft16p folded in)
__device__ __forceinline__ void dft4p_m2(c2& a0, c2& a1, c2& a2, c2& a3) {
  const c2 t0 = add_mi(a0, a2), t1 = add_pi(a0, a2), t2 = a1 + a3, d = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = add_mi(t1, d);
  a3 = add_pi(t1, d);
}
constexpr float kH = 0.70710678118654752440f;
__device__ __forceinline__ void dft8p(c2 (&v)[8]) {
  c2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  c2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
  dft4p(e0, e1, e2, e3);
  dft4p(o0, o1, o2, o3);
  o1 = add_mi(o1, o1) * kH;                     // * W8^1 = h(1 - i): h (re + im, im - re)
  o3 = add_pi(o3, o3) * -kH;                     // * W8^3 = h(-1 - i): -h (re - im, im + re)
  v[0] = e0 + o0; v[4] = e0 - o0;
  v[1] = e1 + o1; v[5] = e1 - o1;
  v[2] = add_mi(e2, o2); v[6] = add_pi(e2, o2);  // * W8^2 = -i folded into the butterfly
  v[3] = e3 + o3; v[7] = e3 - o3;
}
// 16 points: X[k1 + 4 k2] = sum_n2 W4^(n2 k2) W16^(n2 k1) sum_n1 x[4 n1 + n2] W4^(n1 k1)
template <int STRIDE>
__device__ __forceinline__ void dft16p(c2* v) {
  c2 y[16];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    c2 a0 = v[STRIDE * n2], a1 = v[STRIDE * (4 + n2)], a2 = v[STRIDE * (8 + n2)], a3 = v[STRIDE * (12 + n2)];
    dft4p(a0, a1, a2, a3);
    y[4 * n2 + 0] = a0; y[4 * n2 + 1] = a1; y[4 * n2 + 2] = a2; y[4 * n2 + 3] = a3;
  }
  constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
  y[5] = cmv(y[5], c2{c1, -s1});
  y[6] = cmv(y[6], c2{kH, -kH});
  y[7] = cmv(y[7], c2{s1, -c1});
  y[9] = cmv(y[9], c2{kH, -kH});
  // y[10] * W16^4 = -i: folded into the k1 = 2 column's DFT4 (dft4p_m2)
  y[11] = cmv(y[11], c2{-kH, -kH});
  y[13] = cmv(y[13], c2{s1, -c1});
  y[14] = cmv(y[14], c2{-kH, -kH});
  y[15] = cmv(y[15], c2{-c1, s1});
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    c2 a0 = y[k1], a1 = y[4 + k1], a2 = y[8 + k1], a3 = y[12 + k1];
    if (k1 == 2) dft4p_m2(a0, a1, a2, a3);
    else dft4p(a0, a1, a2, a3);
    v[STRIDE * k1] = a0; v[STRIDE * (k1 + 4)] = a1; v[STRIDE * (k1 + 8)] = a2; v[STRIDE * (k1 + 12)] = a3;
  }
}
// 32 points, in place: radix-2 DIT over the even / odd dft16p (stride 2).
__device__ __forceinline__ void dft32p(c2 (&v)[32]) {
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
  dft16p<2>(v);                                  // evens: v[2k] = E[k]
  dft16p<2>(v + 1);                              // odds:  v[2k+1] = O[k]
  c2 r[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const c2 e = v[2 * k];
    if (k == 8) {                                // W32^8 O[8] = -i O[8]
      r[k] = add_mi(e, v[17]);
      r[k + 16] = add_pi(e, v[17]);
      continue;
    }
    const c2 ot = k == 0 ? v[1] : cmv(v[2 * k + 1], c2{kc[k], -ks[k]});   // W32^k O[k]
    r[k] = e + ot;
    r[k + 16] = e - ot;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = r[k];
}

}  // namespace op
}  // namespace fmcw
