// fft_team.h -- register/LDS FFT building block for gfx950 (wave64).
//
// An N-point forward FFT (N a power of two, 2..2048) is executed by a *team*
// of T = N/P threads, each holding P = min(N,16) complex values in VGPRs.
// The transform is a Stockham autosort sequence of radix-16 passes followed
// by one radix-2/4/8 pass (N = 16^a * R0), e.g. 1024 = 16*16*4, 256 = 16*16.
// Inside a pass every thread does its butterflies entirely in registers; the
// data exchange between passes goes through the team's LDS region, padded by
// one complex every 16 (32 for N >= 512) so the stride-16 write of pass 1 and
// the reads are bank-conflict free (FftPlan::PADSH).
//
// Data distribution (the property the kernels are built on):
//   on entry  thread t holds x[t + T*m], m = 0..P-1  ("cyclic")
//   on exit   thread t holds X[t + T*m], m = 0..P-1
// so global loads and stores of consecutive t are coalesced both ways.
//
// This replaces MATLAB's fft(...) calls at radar_processing.m:205 (range,
// along samples) and :219 (Doppler, along chirps).  Twiddles come from a
// per-size table tw[i] = exp(-2*pi*i*i/N) rounded once from float64.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

namespace fmcw {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)
__device__ __forceinline__ float cabs2(float2 a) { return fmaf(a.x, a.x, a.y * a.y); }

// ---- element I/O: complex float32 or complex float16 storage --------------
__device__ __forceinline__ float2 ld_c(const float2* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float2 ld_c(const __half2* p, int64_t i) { return __half22float2(p[i]); }
__device__ __forceinline__ void st_c(float2* p, int64_t i, float2 v) { p[i] = v; }
__device__ __forceinline__ void st_c(__half2* p, int64_t i, float2 v) { p[i] = __float22half2_rn(v); }

// Two adjacent complex elements in one 16-byte (c64) / 8-byte (c32h) access.
__device__ __forceinline__ void ld_c2(const float2* p, int64_t i, float2& a, float2& b) {
  const float4 v = *reinterpret_cast<const float4*>(p + i);
  a = make_float2(v.x, v.y);
  b = make_float2(v.z, v.w);
}
__device__ __forceinline__ void ld_c2(const __half2* p, int64_t i, float2& a, float2& b) {
  const uint2 v = *reinterpret_cast<const uint2*>(p + i);
  a = __half22float2(*reinterpret_cast<const __half2*>(&v.x));
  b = __half22float2(*reinterpret_cast<const __half2*>(&v.y));
}
__device__ __forceinline__ void st_c2(float2* p, int64_t i, float2 a, float2 b) {
  *reinterpret_cast<float4*>(p + i) = make_float4(a.x, a.y, b.x, b.y);
}
__device__ __forceinline__ void st_c2(__half2* p, int64_t i, float2 a, float2 b) {
  const __half2 ha = __float22half2_rn(a), hb = __float22half2_rn(b);
  uint2 v;
  v.x = *reinterpret_cast<const unsigned*>(&ha);
  v.y = *reinterpret_cast<const unsigned*>(&hb);
  *reinterpret_cast<uint2*>(p + i) = v;
}

// Lane pair exchange (hardware lanes 2i <-> 2i+1, one DPP quad_perm [1,0,3,2]
// per float, no LDS).  Each lane of a pair accessed two ADJACENT elements of
// its own block (even lane: block A, odd lane: block B); afterwards the even
// lane holds element 0 of blocks (A, B) and the odd lane element 1 of (A, B).
// The same call turns the cyclic FFT layout back into adjacent pairs for
// 16-byte stores.  Must be executed by both lanes of every pair.
__device__ __forceinline__ float lane_swap1(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ void pair_xchg(bool odd, float2& first, float2& second) {
  const float2 send = odd ? first : second;
  const float2 r = make_float2(lane_swap1(send.x), lane_swap1(send.y));
  if (odd) first = r; else second = r;
}

// ---- small forward DFTs in registers (natural order in and out) -----------
__device__ __forceinline__ void dft2(float2& a, float2& b) {
  const float2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_negi(csub(a1, a3));
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = cadd(t1, t3);
  a3 = csub(t1, t3);
}

template <int R> __device__ __forceinline__ void dft(float2* v);

template <> __device__ __forceinline__ void dft<1>(float2*) {}
template <> __device__ __forceinline__ void dft<2>(float2* v) { dft2(v[0], v[1]); }
template <> __device__ __forceinline__ void dft<4>(float2* v) { dft4(v[0], v[1], v[2], v[3]); }

template <> __device__ __forceinline__ void dft<8>(float2* v) {
  // radix-2 DIT over two 4-point DFTs of the even and odd samples
  float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
  dft4(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  const float h = 0.70710678118654752440f;
  o1 = make_float2(h * (o1.x + o1.y), h * (o1.y - o1.x));    // * W8^1 = h(1 - i)
  o2 = mul_negi(o2);                                         // * W8^2 = -i
  o3 = make_float2(h * (o3.y - o3.x), -h * (o3.x + o3.y));   // * W8^3 = h(-1 - i)
  v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
  v[1] = cadd(e1, o1); v[5] = csub(e1, o1);
  v[2] = cadd(e2, o2); v[6] = csub(e2, o2);
  v[3] = cadd(e3, o3); v[7] = csub(e3, o3);
}

template <> __device__ __forceinline__ void dft<16>(float2* v) {
  // X[k1 + 4 k2] = sum_n2 W4^(n2 k2) W16^(n2 k1) sum_n1 x[4 n1 + n2] W4^(n1 k1)
  float2 y[16];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    float2 a0 = v[n2], a1 = v[4 + n2], a2 = v[8 + n2], a3 = v[12 + n2];
    dft4(a0, a1, a2, a3);
    y[4 * n2 + 0] = a0; y[4 * n2 + 1] = a1; y[4 * n2 + 2] = a2; y[4 * n2 + 3] = a3;
  }
  // twiddles W16^m, m = n2*k1 in {1,2,3,2,4,6,3,6,9}
  const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, h = 0.70710678118654752440f;
  y[5] = cmul(y[5], make_float2(c1, -s1));    // n2=1,k1=1: W^1
  y[6] = cmul(y[6], make_float2(h, -h));      // n2=1,k1=2: W^2
  y[7] = cmul(y[7], make_float2(s1, -c1));    // n2=1,k1=3: W^3
  y[9] = cmul(y[9], make_float2(h, -h));      // n2=2,k1=1: W^2
  y[10] = mul_negi(y[10]);                    // n2=2,k1=2: W^4 = -i
  y[11] = cmul(y[11], make_float2(-h, -h));   // n2=2,k1=3: W^6
  y[13] = cmul(y[13], make_float2(s1, -c1));  // n2=3,k1=1: W^3
  y[14] = cmul(y[14], make_float2(-h, -h));   // n2=3,k1=2: W^6
  y[15] = cmul(y[15], make_float2(-c1, s1));  // n2=3,k1=3: W^9
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float2 a0 = y[k1], a1 = y[4 + k1], a2 = y[8 + k1], a3 = y[12 + k1];
    dft4(a0, a1, a2, a3);
    v[k1] = a0; v[k1 + 4] = a1; v[k1 + 8] = a2; v[k1 + 12] = a3;
  }
}

// ---- plan --------------------------------------------------------------------
template <int N> struct FftPlan {
  static_assert(N >= 2 && N <= 4096 && (N & (N - 1)) == 0, "FFT size must be a power of two");
  static constexpr int P = N < 16 ? N : 16;   // values per thread
  static constexpr int T = N / P;             // threads per team
  // LDS padding: one complex every 2^PADSH.  Teams of >= 32 threads (N >= 512) pad one in
  // 32, so every pass's loads (32 consecutive elements per 32-lane ds_read_b64 group, banks
  // (a/4) mod 64) are conflict-free (a 1-in-16 pad maps elements 0 and 31 of a load onto one
  // bank pair).  Their stores (ds_write_b64: 16-lane groups, banks (a/4) mod 32) are
  // conflict-free when the team index of a lane is team_index<T> (below), not the lane.
  // Smaller teams share 32-lane groups and keep the 1-in-16 pad with odd team strides.
  static constexpr int PADSH = T >= 32 ? 5 : 4;
  static constexpr int LDS = (N < 16) ? 0 : N + (N >> PADSH);  // complex elements of LDS per team
  // stride between the LDS regions of teams that share a wave: odd, so the same
  // element of 16 neighbouring teams lands on 16 different bank pairs
  static constexpr int STRIDE = (N < 16) ? 0 : (LDS | 1);
};

template <int N> __device__ __forceinline__ int lds_pad(int i) { return i + (i >> FftPlan<N>::PADSH); }

// Team index of lane l for teams of T >= 32 threads.  With the 1-in-32 pad, the first pass's
// store r of index t goes to bank pair (t/2 + r) mod 16 and the second pass's to
// (t + 8 (t/16 mod 2) + r/2) mod 16: consecutive t put t = 2i and 2i + 1 on one pair (2-way on
// every first-pass store).  Within each 32-lane block, lanes 0-15 take t = 0, 2, .., 14, 17, 19,
// .., 31 and lanes 16-31 the rest: one t of every pair {2i, 2i + 1} per 16-lane group, and the
// second pass's pairs distinct as well.  A permutation inside 32-lane blocks keeps every
// 32-lane load group on the same consecutive elements and the DPP team sums unchanged.
template <int T> __device__ __forceinline__ int team_index(int l) {
  if constexpr (T >= 32) {
    const int i = l & 31;
    return (l & ~31) | (2 * (i & 15)) | (((i >> 3) ^ (i >> 4)) & 1);
  } else {
    return l;
  }
}

constexpr int fft_num_r16(int n) { return n >= 16 ? 1 + fft_num_r16(n / 16) : 0; }
constexpr int fft_pow16(int k) { return k == 0 ? 1 : 16 * fft_pow16(k - 1); }
constexpr int tw_nb(int R) { return R >= 16 ? 4 : R >= 8 ? 3 : R >= 4 ? 2 : R >= 2 ? 1 : 0; }

// Pass structure of an N-point transform: radix-16 passes, then radix R0.
template <int N> struct FftPasses {
  static constexpr int NR16 = fft_num_r16(N);
  static constexpr int R0 = N / fft_pow16(NR16);
  static constexpr int NPASS = NR16 + (R0 > 1 ? 1 : 0);
  static constexpr int radix(int p) { return p < NR16 ? 16 : R0; }
  static constexpr int q(int p) { return FftPlan<N>::P / radix(p); }
  // offset of pass p's base twiddles in a preloaded block (pass 0 has none)
  static constexpr int off(int p) {
    int o = 0;
    for (int i = 1; i < p; ++i) o += q(i) * tw_nb(radix(i));
    return o;
  }
  static constexpr int NB = off(NPASS) > 0 ? off(NPASS) : 1;
};

// Twiddle sources for a pass.  TwTable reads w^1, w^2, w^4, w^8 from the
// table where the pass needs them; TwPre takes them from a block a kernel
// loaded up front (load_tw_bases), so a kernel that prefetches the next
// chirp never waits on a twiddle load queued behind it (vmcnt is in order).
// Both give bit-identical twiddles.
struct TwTable {
  const float2* __restrict__ tw;
  // b[0..nb-1] = w^1, w^2, w^4, w^8 with w = tw[k * N/(Ns*R)]
  template <int N, int PASS, int R, int Ns>
  __device__ __forceinline__ void get(float2* b, int q, int t) const {
    constexpr int T = FftPlan<N>::T, nb = tw_nb(R);
    const int k = (t + T * q) & (Ns - 1);
    const int base = k * (N / (Ns * R));
    b[0] = tw[base & (N - 1)];
    if constexpr (nb > 1) b[1] = tw[(2 * base) & (N - 1)];
    if constexpr (nb > 2) b[2] = tw[(4 * base) & (N - 1)];
    if constexpr (nb > 3) b[3] = tw[(8 * base) & (N - 1)];
  }
};

struct TwPre {
  const float2* tb;      // FftPasses<N>::NB values from load_tw_bases<N>
  template <int N, int PASS, int R, int Ns>
  __device__ __forceinline__ void get(float2* b, int q, int) const {
    constexpr int nb = tw_nb(R), o = FftPasses<N>::off(PASS);
#pragma unroll
    for (int i = 0; i < nb; ++i) b[i] = tb[o + q * nb + i];
  }
};

// v[r] *= w^r for r = 1..R-1, from the bases w^1, w^2, w^4, w^8: one complex
// product per set bit of r (<= 4 roundings, like a product-formed table, but
// only the four bases stay live -- the FFT passes are register-bound).
template <int R>
__device__ __forceinline__ void apply_twiddles(float2* v, const float2* b) {
#pragma unroll
  for (int r = 1; r < R; ++r) {
    float2 x = v[r];
    if (r & 1) x = cmul(x, b[0]);
    if (r & 2) x = cmul(x, b[1]);
    if (r & 4) x = cmul(x, b[2]);
    if (r & 8) x = cmul(x, b[3]);
    v[r] = x;
  }
}

template <int N, int PASS = 1>
__device__ __forceinline__ void load_tw_bases(float2* tb, int t, const float2* __restrict__ tw) {
  using F = FftPasses<N>;
  if constexpr (PASS < F::NPASS) {
    constexpr int R = F::radix(PASS), Q = F::q(PASS), nb = tw_nb(R), o = F::off(PASS);
    constexpr int T = FftPlan<N>::T;
    int Ns = 1;
#pragma unroll
    for (int i = 0; i < PASS; ++i) Ns *= F::radix(i);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int k = (t + T * q) & (Ns - 1);
      const int base = k * (N / (Ns * R));
      tb[o + q * nb] = tw[base & (N - 1)];
      if constexpr (nb > 1) tb[o + q * nb + 1] = tw[(2 * base) & (N - 1)];
      if constexpr (nb > 2) tb[o + q * nb + 2] = tw[(4 * base) & (N - 1)];
      if constexpr (nb > 3) tb[o + q * nb + 3] = tw[(8 * base) & (N - 1)];
    }
    load_tw_bases<N, PASS + 1>(tb, t, tw);
  }
}

// One Stockham pass of radix R with stride Ns on registers in butterfly layout
// v[q*R + r] = in[t + T*q + r*N/R].  Applies the inter-pass twiddles and the
// radix-R DFTs in place.
template <int N, int PASS, int R, int Ns, class TW>
__device__ __forceinline__ void stockham_pass_regs(float2* v, int t, const TW& src) {
  constexpr int P = FftPlan<N>::P, Q = P / R;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    if constexpr (Ns > 1) {
      float2 b[4];
      src.template get<N, PASS, R, Ns>(b, q, t);
      apply_twiddles<R>(v + q * R, b);
    }
    dft<R>(v + q * R);
  }
}

// Write the pass output to LDS: out[(j/Ns)*Ns*R + j%Ns + r*Ns] = v[q*R + r].
// One 8-byte store per element (ds_write_b64, 16-lane groups): the 1-in-16 pad
// makes the stride-16 first pass conflict-free for exactly that width, so the
// compiler must not merge a lane's adjacent elements into write2 / b128 forms
// (2-way conflicts: b32 halves in 32-lane groups, b128 spans of 4 banks) -- the
// empty asm between the stores keeps them separate.
template <int N, int R, int Ns>
__device__ __forceinline__ void stockham_store_lds(const float2* v, int t, float2* lds) {
  constexpr int P = FftPlan<N>::P, T = FftPlan<N>::T, Q = P / R;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int j = t + T * q;
    const int base = (j / Ns) * Ns * R + (j & (Ns - 1));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      *reinterpret_cast<double*>(&lds[lds_pad<N>(base + r * Ns)]) = __builtin_bit_cast(double, v[q * R + r]);
      asm volatile("" ::: "memory");
    }
  }
}

// Read the next pass's input from LDS: v[q*R + r] = in[t + T*q + r*N/R].
template <int N, int R>
__device__ __forceinline__ void stockham_load_lds(float2* v, int t, const float2* lds) {
  constexpr int P = FftPlan<N>::P, T = FftPlan<N>::T, Q = P / R;
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int r = 0; r < R; ++r) v[q * R + r] = lds[lds_pad<N>(t + T * q + r * (N / R))];
}

// Recursive pass driver.  `PASS` indexes the pass, Ns = product of radices so far.
template <int N, int PASS, int Ns, class Sync, class TW>
__device__ __forceinline__ void team_fft_passes(float2* v, float2* lds, int t, const TW& src, Sync sync) {
  using F = FftPasses<N>;
  constexpr int NR16 = F::NR16, R0 = F::R0, NPASS = F::NPASS;
  constexpr int R = (PASS < NR16) ? 16 : R0;
  constexpr int P = FftPlan<N>::P, Q = P / R;
  stockham_pass_regs<N, PASS, R, Ns>(v, t, src);
  if constexpr (PASS + 1 < NPASS) {
    constexpr int RN = (PASS + 1 < NR16) ? 16 : R0;
    sync();                      // previous readers of `lds` are done (WAR)
    stockham_store_lds<N, R, Ns>(v, t, lds);
    sync();                      // stores visible (RAW)
    stockham_load_lds<N, RN>(v, t, lds);
    team_fft_passes<N, PASS + 1, Ns * R, Sync>(v, lds, t, src, sync);
  } else {
    // last pass: the butterfly layout v[q*R + r] holds X[t + T*(q + r*Q)];
    // permute to the cyclic layout v[m] = X[t + T*m] (compile-time moves).
    if constexpr (Q > 1) {
      float2 w[P];
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int r = 0; r < R; ++r) w[q + r * Q] = v[q * R + r];
#pragma unroll
      for (int m = 0; m < P; ++m) v[m] = w[m];
    }
  }
}

// Forward FFT of N points by a team; see the header comment for layouts.
// `lds` is the team's private region of FftPlan<N>::LDS complex elements;
// `sync` must order LDS accesses of all threads of the team.
template <int N, class Sync>
__device__ __forceinline__ void team_fft(float2* v, float2* lds, int t, const float2* __restrict__ tw, Sync sync) {
  team_fft_passes<N, 0, 1, Sync>(v, lds, t, TwTable{tw}, sync);
}
// Same transform with the base twiddles preloaded by load_tw_bases<N>.
template <int N, class Sync>
__device__ __forceinline__ void team_fft_pre(float2* v, float2* lds, int t, const float2* tb, Sync sync) {
  team_fft_passes<N, 0, 1, Sync>(v, lds, t, TwPre{tb}, sync);
}

struct BlockSync {
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

// A team that lives inside one wave only needs the wave's LDS accesses
// ordered: LDS executes one wave's instructions in order, so a compiler
// barrier with wavefront-scope fences is enough (no s_barrier).
struct WaveSync {
  __device__ __forceinline__ void operator()() const {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

template <int T> struct TeamSync { using type = BlockSync; };
template <> struct TeamSync<1> { using type = WaveSync; };
template <> struct TeamSync<2> { using type = WaveSync; };
template <> struct TeamSync<4> { using type = WaveSync; };
template <> struct TeamSync<8> { using type = WaveSync; };
template <> struct TeamSync<16> { using type = WaveSync; };
template <> struct TeamSync<32> { using type = WaveSync; };
template <> struct TeamSync<64> { using type = WaveSync; };

}  // namespace fmcw
