// op_math.h -- register-level building blocks of the single-pass schedule
// (kernels_xcd.hip: k_rdx, the chirp-split XCD-team schedule; kernels_detect.hip):
// packed complex multiplies with op_sel modifiers, DPP / permlane lane exchanges,
// wave reductions and the packed small DFTs.
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
// a * b against a per-lane VGPR constant b: the rotation of b is done by operand
// modifiers (op_sel picks b.im for the low half, neg_lo negates it), so no rotated
// copy of b is kept.  Results must not feed a DPP / permlane op directly (the
// hazard recognizer does not see inline asm).
__device__ __forceinline__ c2 cmul_a(c2 a, c2 b) {
  c2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ c2 tov(float2 v) { return c2{v.x, v.y}; }
__device__ __forceinline__ float abs2v(c2 v) { return fmaf(v.x, v.x, v.y * v.y); }
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
}  // namespace op
}  // namespace fmcw
