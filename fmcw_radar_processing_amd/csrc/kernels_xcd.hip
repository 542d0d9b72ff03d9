// kernels_xcd.hip -- the XCD-team schedule of range + Doppler (k_rdx) for gfx950.
//
// A config-3 frame (256 chirps x 1024 samples, 2 MiB) and its range cube do not fit one CU
// (512 KiB of VGPRs + 160 KiB of LDS), so the 32 CUs of one XCD share a frame the way the
// reference computes it (radar_processing.m:199-219):
//
//   range   (:203-205): member k transforms chirps 8k .. 8k+7, one per wave,
//                       as a full 1024-point FFT, and writes its 1024 bins of
//                       each chirp into the XCD's hand-off slot as 32 groups
//                       of 32 bins;
//   Doppler (:210, :216-219): member k reads group k (32 range bins x 256
//                       chirps, 64 KiB) back, takes the row means / maxima,
//                       windows, runs 32 Doppler FFTs and writes its RD rows.
//
// So each input byte is read once from HBM and the cube (2 MiB per frame) makes one trip
// through the XCD's L2 (the retired 8-tile pass re-read the whole frame from L2 eight
// times: DESIGN.md 4.1).  One persistent 512-thread workgroup per CU; the 32 blocks that
// land on XCD x (HW_REG_XCC_ID; xcd_census checks the 32-per-XCD deal and the occupancy
// before the schedule is enabled) form its team, members k = 0..31 by ticket, and take
// frames x + 8 j.  Step j publishes R(j-1), runs R(j) and D(j-2) (the Doppler two steps
// behind, see the step loop); a ring of kNS = 2 slots of 2 MiB per XCD with one ready counter
// each: D(j-2) reads group k of frame j-2's slot once all 32 members published it.
//
// Hand-off protocol: producers store the slot with plain buffer stores (write-back in the
// XCD's L2: a line rewritten while resident never leaves it, tools/r04_probe.hip part C; the
// 2-slot ring competes with the input and RD lines, so about half its lines are written back
// and re-read through the fabric), `s_waitcnt vmcnt` in every wave, a
// workgroup barrier, then one agent-scope atomic add on the slot's ready counter.
// Consumers poll with scalar loads that miss the scalar cache (s_load glc), then read the
// slot with buffer_load sc1, which bypasses the CU's L1 and is served by the XCD's L2.
// Producer and consumer are on the same XCD, so no L2 write-back is needed for visibility.
// Every wait is bounded: a timeout sets xerr bit 0 and lets the grid drain.
//
// Reference chirp (static-target cancellation, :204 / :217-218).  Every chirp
// except chirp 0 is transformed as the difference x_k - x_0 from the frame's
// chirp 0 (loaded by every member into LDS): X'_k = FFT((d_k - mean d_k) w'),
// d_k = x_k - x_0, so X_k = X'_k + X_0 by linearity, and the slot holds X_0 for
// chirp 0 and X'_k for the others.  The Doppler stage forms the row mean from
// the X'_k (X'_0 = 0), so a static target -- a component identical in every
// chirp, removed by the :218 mean -- cancels in the time domain, before any
// rounding of its large FFT values; the profile and the slow-time rows use
// X_k = X'_k + X_0.  Without it the fp32 RD map of a static-target frame is off
// by ~2.5e-5 of the frame's (small, cancelled) norm; with it every frame meets
// the 1e-5 bar of SURVEY 8d.
// Range FFT of one chirp in one wave (n = a + 128 i, r = k1 + 8 (s1 + 16 s2),
// a = a0 + 8 a1):  lane l holds samples n = 2l + e + 128 i (8 16-byte loads);
//   stage 1: DFT8 over i of both a = 2l + e, twiddle W1024^(a k1);
//   LDS transpose; stage 2: lane 8 k1 + a0 runs DFT16 over a1, twiddle W128^(a0 s1);
//   LDS transpose; stage 3: lane 8 k1 + h runs DFT8 over a0 for s1 = 2h, 2h + 1;
// giving bins r = k1 + 16 h + 8 e + 128 s2: for a fixed register (e, s2) the 32
// lanes of each half-wave hold the 32 bins of one group (xcd_bin), so every
// slot store is a contiguous 256-byte row.
// Doppler of one group: 64 KiB staged through LDS, lane (pp, q) of wave w holds
// bin p = 4w + pp at chirps q + 16 i; DFT16 over i, twiddle W256^(q d0), LDS
// transpose, DFT16 over q: D[d0 + 16 d1] in lane (pp, d0); fftshift is the
// store index.
#include "op_math.h"

#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace fmcw {
namespace xk {
using namespace op;

#ifdef XK_NOREF
#define XK_REF 0
#else
#define XK_REF 1
#endif
#ifndef XK_RD_AUX
#define XK_RD_AUX 2                    // RD store cache policy: nt (A/B: 16 = sc1, 17 = sc0 sc1, 18 = sc1 nt, 3 = sc0 nt)
#endif
constexpr int kRdAux = XK_RD_AUX;
#ifndef XK_LAG
#define XK_LAG 1                       // A/B: the group polled and loaded in step j is frame j - XK_LAG
#endif
#ifndef XK_NS
#define XK_NS (2 * XK_LAG)
#endif
constexpr int kLag = XK_LAG;
#ifndef XK_POLLAT
#define XK_POLLAT 2                    // where wave 0 first polls ready(j - lag) in the step (see the step loop;
                                       // round 6: 2 -- after R1 and the next frame's loads -- is 3-5 % faster than 0)
#endif
#ifndef XK_SKEW_STEPS
#define XK_SKEW_STEPS 256
#endif
static_assert(kLag == 1 || kLag == 2, "poll lag 1 (shipped) or 2");
constexpr int kNS = XK_NS;            // hand-off slots in use per XCD (2..XCD_MAX_SLOTS; see the step loop)
static_assert(kNS >= 2 * kLag && kNS <= 4, "slot reuse: seeing ready(j - lag) proves frame j - 2 lag read");
constexpr int NK = 32;                 // team members (CUs) per XCD
constexpr int C = 256;                 // chirps = Doppler points
constexpr int NW = 8;                  // waves per workgroup = chirps per member
constexpr int GP = 32;                 // bins per group
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
static_assert(NK * NW == C && NK * GP == NR && NK == XCD_TILES, "team geometry");

struct LdsX {
  union {
    f4v stg[C * 17];                   // Doppler staging [chirp][34 c2]: 32 bins + 2 pad (conflict-free both ways)
    c2 rt[NW][1216];                   // per-wave transposes: range 8 x 136 and 64 x 18, Doppler 4 x 304
  } u;
  // per-lane constants packed so that every read is one ds_read_b128 (4 LDS cycles per wave;
  // a c2 table read by pairs became ds_read2_b64 at 8 cycles, the {cal w', w'} table ds_read_b96 at 8)
#ifndef XK_HALF
  f4v tw1[7][64];                      // {W1024^((2l) k1), W1024^((2l + 1) k1)}, k1 = 1..7
  f4v tw2[8][64];                      // {W128^(a0 s1), W128^(a0 (s1 + 1))}, s1 = 1, 3, .., 15 (a0 = l & 7)
#else
  c2 th1[7][64];                       // half-frame build: W512^(l k1), k1 = 1..7
  c2 th2[7][64];                       // W64^((l & 7) s1), s1 = 1..7
  c2 thc[8][64];                       // W1024^(l + 64 s2): the pair's radix-2 combine
#endif
  f4v twd[8][64];                      // {W256^(q d0), W256^(q (d0 + 1))}, d0 = 1, 3, .., 15 (q = l & 15)
  f4v wdl[4][64];                      // 2chebwin of chirps (l & 15) + 16 i, i = 4 g .. 4 g + 3
  f4v wq[4][64];                       // w' = IF_scale 2blackman of samples 2 l + e + 128 i, index v = 2 i + e = 4 g .. 4 g + 3
  c2 cwq[16][64];                      // cal w' of the same samples (read by the reference-chirp wave only)
  float key[GP];                       // candidate key per group position (profile or -1)
#ifndef XK_NOREF
#ifndef XK_HALF
  f4v x0[512];                         // the frame's reference chirp (chirp 0) as loaded, c64 pairs (fp16: widened)
#else
  f4v x0[2][512];                      // half-frame build: frames 2 j' and 2 j' + 1 (put one half-step ahead)
  c2 psum[8];                          // each wave's sum of its half of the chirp (the pair's mean)
#endif
#endif
};

// Poll of a hand-off counter: a scalar load that misses the scalar cache (glc: served by
// the L2, where the agent-scope adds land).  It counts on lgkmcnt, not vmcnt, so the
// polling wave's vector loads and stores stay in flight (a vector poll, or a call, would
// make it wait for all of them first).  The value is waited for inside the asm.
// (The address goes through readfirstlane, a no-op for a value already in SGPRs: a loop-invariant
// counter address may otherwise be kept in VGPRs, which the "s" constraint cannot take.)
__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  const unsigned long long u = reinterpret_cast<unsigned long long>(p);
  const unsigned long long su = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(u >> 32)) << 32) |
                                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)u);
  unsigned v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(reinterpret_cast<const unsigned*>(su)) : "memory");
  return v;
}
// Bounded wait for *p >= v (wave-uniform).  ~1 s before giving up; once any wait of
// the launch timed out (its abort word, zeroed per launch), the others return at
// once so the grid drains.  The timeout is also or-ed into the sticky error word
// that fmcw_synchronize reports; a later launch is not affected by it.  Inlined:
// no call (a call waits for every outstanding memory operation of the wave).
__device__ __forceinline__ void wait_ge(const unsigned* p, unsigned v, unsigned* abort, unsigned* err) {
  for (int it = 0; it < (1 << 20); ++it) {
    if (ld_flag(p) >= v) return;
    if ((it & 63) == 63 && ld_flag(abort)) return;
#ifndef XK_PSLEEP
#define XK_PSLEEP 2                    // A/B: s_sleep between two polls (x 64 cycles)
#endif
    __builtin_amdgcn_s_sleep(XK_PSLEEP);
  }
  if (threadIdx.x == 0) {   // global atomics (a flat atomic here tripped an LLVM aperture-check bug)
    typedef __attribute__((address_space(1))) unsigned gu32;
    __hip_atomic_fetch_or((gu32*)abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void cfence() { asm volatile("" ::: "memory"); }
// c32h bits -> complex fp32.  (Through memcpy: ROCm 7.2 clang folds __builtin_bit_cast(__half2,
// v.y) of an ext-vector element to the bits of v.x.)
__device__ __forceinline__ float2 h2f(unsigned b) {
  __half2 h;
  __builtin_memcpy(&h, &b, 4);
  return __half22float2(h);
}

// s_waitcnt vmcnt(N) for a compile-time N (the k_rdx publish counts; tools/check_vmcnt.py
// proves them on the built code)
template <int N> __device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


// row (16-lane group) reductions by DPP: symmetric pairings, every lane of the row gets the result
__device__ __forceinline__ float row_sum16(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  return v + dppf<0x140>(v);
}
__device__ __forceinline__ int row_max16(int v) {
  v = max(v, dppi<0xB1>(v));
  v = max(v, dppi<0x4E>(v));
  v = max(v, dppi<0x141>(v));
  return max(v, dppi<0x140>(v));
}
__device__ __forceinline__ int row_min16(int v) {
  v = min(v, dppi<0xB1>(v));
  v = min(v, dppi<0x4E>(v));
  v = min(v, dppi<0x141>(v));
  return min(v, dppi<0x140>(v));
}

// Lanes 2m, 2m + 1 hold columns p, p + 1 of two rows A and B (one value each): afterwards the
// even lane holds both columns of row A, the odd lane both columns of row B, ready for one
// double-width store at column p (even) / p - 1 (odd) of its row.  One DPP swap per dword.
__device__ __forceinline__ f4v pair_cols(c2 A, c2 B, bool odd) {
  const c2 snd = odd ? A : B;
  const c2 rcv = c2{dppf<0xB1>(snd.x), dppf<0xB1>(snd.y)};
  return odd ? f4v{rcv.x, rcv.y, B.x, B.y} : f4v{A.x, A.y, rcv.x, rcv.y};
}

}  // namespace xk

// H: fp16 storage (c32h IQ in, c32h RD out), fp32 arithmetic; RD: the RD map is written
// (else only the row peaks), a template flag so that every hand-off wait count is static
template <bool FULL, bool H, bool RD>
__global__ __launch_bounds__(512, 1) void k_rdx(OnePassArgs a) {
  using namespace xk;
  __shared__ __attribute__((aligned(16))) LdsX L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Team = the workgroups on one XCD (they share its L2).  The dispatcher deals
  // blocks round-robin over the 8 XCDs from wherever the previous launch
  // stopped, so the XCD is read from HW_REG_XCC_ID and the member index is a
  // ticket drawn on that XCD's counter: 256 blocks give every XCD exactly 32.
  __shared__ int team[2];
  __shared__ unsigned gflag;           // the last step whose ready(j - 1) wave 0 has seen
  if (tid == 0) {
    gflag = 0;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int xx = a.xcc_team[xcc & 15];   // the census's team index of this XCC
    int kk = NK;
    if (xx >= 0) kk = (int)__hip_atomic_fetch_add(a.xctr + XCD_TICKETS + xx * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kk >= NK) { atomicOr(a.xerr, 2u); atomicOr(a.xctr + XCD_ABORT, 1u); }
    team[0] = xx;
    team[1] = kk;
  }
  __syncthreads();
  // the other counter set, for the next launch (nothing reads it during this one; vector stores, visible to
  // the next launch at the kernel boundary like a memset's).  The idle words only ever receive + 0.
  if (a.xclr && blockIdx.x == 0)
    for (int i = tid; i < XCD_IDLE; i += 512) a.xclr[i] = 0u;
  const int x = __builtin_amdgcn_readfirstlane(team[0]), k = __builtin_amdgcn_readfirstlane(team[1]);
  if (k >= NK) return;                 // more than 32 blocks on one XCD: its team is short (waits time out)
  // the effective shader clock of the launch: team 0's member 0 stamps both clocks (vector stores)
  const bool stamper = a.clk != nullptr && x == 0 && k == 0 && tid == 0;
  if (stamper) {
    a.clk[0] = __builtin_amdgcn_s_memtime();
    a.clk[1] = __builtin_amdgcn_s_memrealtime();
  }
  const int T = a.nteams;              // teams (XCDs) of the device: frames x + T j for team x
  const int nj = a.F > x ? (int)((a.F - x + T - 1) / T) : 0;
  const int S = FULL ? NR : a.S, S2 = S >> 1, NS = a.slots;
  unsigned* ready = a.xctr + (x * 2 + 0) * 32 * XCD_MAX_SLOTS;
  // slot s's ready counter (round 6 A/B: 4, 8 or 32 replicas, every publish adding to all, a member polling
  // its own, ran 0-3 % slower: the counter's line is not a hot spot at one poller per CU,
  // profiles/r06_poll_ab.txt)
  auto rdy = [&](int s_) __attribute__((always_inline)) -> unsigned* { return &ready[s_ * 32]; };
#ifdef XK_DONE
  unsigned* done = ready + 32 * XCD_MAX_SLOTS;
#endif

  using TP = std::conditional_t<H, h4v, f4v>;
  const TP* __restrict__ iq = reinterpret_cast<const TP*>(a.iq);
  // hand-off slot element: c64; under fp16 storage the groups of the 128-bin blocks in
  // a.s16mask hold X / Nr as c32h (half the bytes).  Those blocks hold no bin that can become a
  // detection or slow-time candidate, so the slow-time rows (and the profile around a target)
  // still come from fp32 values: all-c32h slots put the slow rows at 4.5e-4 relative and the
  // 4096-frame spectrogram at 0.15 dB against the 0.05 dB bar of SURVEY 8d.  Every group keeps
  // the c64 stride in the slot (64 KiB; a c32h group uses its first half).
  constexpr int kES = 8;
  constexpr int64_t kSlotBytes = (int64_t)NK * C * GP * kES;
  const unsigned s16m = H ? a.s16mask : 0u;
  const bool g16 = (s16m >> (k >> 2)) & 1;            // this member's group k is c32h (fixed per member)
  constexpr float kXS = 1.0f / NR, kXU = (float)NR;
#ifndef XK_NOREF
  // the reference chirp (chirp 0) of the next frame: one sample pair per thread, loaded one
  // step ahead (before the chirp loads, so the step's vmcnt counts cover it) and put into LDS
  // before the barrier that opens the step
  TP x0n{};
  auto ld_ref = [&](int64_t f) __attribute__((always_inline)) {
    const TP* __restrict__ q = iq + f * C * (int64_t)S2;
    if constexpr (FULL) x0n = __builtin_nontemporal_load(q + tid);
    else x0n = __builtin_nontemporal_load(q + (tid < S2 ? tid : 0));
  };
  auto put_ref = [&](int b) __attribute__((always_inline)) {
    f4v t;
    if constexpr (H) t = __builtin_convertvector(x0n, f4v);
    else t = x0n;
    if constexpr (!FULL)
      if (tid >= S2) t = f4v{0.f, 0.f, 0.f, 0.f};
#ifndef XK_HALF
    (void)b;
    L.x0[tid] = t;
#else
    L.x0[b][tid] = t;
#endif
  };
  if (nj > 0) ld_ref(x);
#endif
#ifndef XK_HALF
  for (int i = tid; i < 44 * 64; i += 512) {
    const c2 v = tov(a.xtab[i]);
    const int l = i & 63;
    c2* d;
    if (i < XT_R2) { const int t = i >> 6; d = reinterpret_cast<c2*>(&L.tw1[t >> 1][l]) + (t & 1); }
    else if (i < XT_D1) { const int t = (i - XT_R2) >> 6; d = reinterpret_cast<c2*>(&L.tw2[t >> 1][l]) + (t & 1); }
    else { const int t = (i - XT_D1) >> 6; d = reinterpret_cast<c2*>(&L.twd[t >> 1][l]) + (t & 1); }
    *d = v;
  }
#else
  for (int i = XT_D1 + tid; i < XT_H1; i += 512) {
    const int t = (i - XT_D1) >> 6;
    reinterpret_cast<c2*>(&L.twd[t >> 1][i & 63])[t & 1] = tov(a.xtab[i]);
  }
  for (int i = tid; i < 22 * 64; i += 512) {
    const c2 v = tov(a.xtab[XT_H1 + i]);
    const int t = i >> 6, l = i & 63;
    if (t < 7) L.th1[t][l] = v;
    else if (t < 14) L.th2[t - 7][l] = v;
    else L.thc[t - 14][l] = v;
  }
#endif
  // the Doppler window carries the two power-of-two scales of fp16 storage (exact, so the outputs
  // keep their bits): the RD map's 1 / (Nr Nd) and, for a member whose group is handed over as
  // c32h, the Nr its staging no longer multiplies back in (VALU work taken out of every step)
  const float wd_scale = (H && RD ? a.rd_scale : 1.0f) * (g16 ? kXU : 1.0f);
  for (int i = tid; i < 16 * 64; i += 512)
    reinterpret_cast<float*>(&L.wdl[i >> 8][i & 63])[(i >> 6) & 3] = a.wd[(i & 15) + 16 * (i >> 6)] * wd_scale;
  // :203-205 per-lane constants of samples n = 2 lane + e + 128 i: w' = IF_scale 2blackman, cal w'
  for (int i = tid; i < 16 * 64; i += 512) {
    const int l = i & 63, v = i >> 6, n = 2 * l + (v & 1) + 128 * (v >> 1);
    const float4 cv = n < S ? a.calw[n] : make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float*>(&L.wq[v >> 2][l])[v & 3] = cv.z;
    L.cwq[v][l] = c2{cv.x * cv.z, cv.y * cv.z};
  }
  const c2 csum = c2{a.cal_sum.x, a.cal_sum.y};
  const float invS = 1.0f / (float)S;
#ifndef XK_NOREF
  if (nj > 0) put_ref(0);
#endif
  __syncthreads();
#ifdef XK_PRIO     // A/B: static priority for the second-dispatched half of the waves (MI355X_MICROARCH item 4)
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef XK_STAMPS   // diagnostic build: per-phase time of every block's steps, waves 0 and 4 (100 MHz clock)
  constexpr int NST = 10;
  unsigned long long st_acc[NST] = {}, st_t = __builtin_amdgcn_s_memrealtime();
  const unsigned long long st_c0 = __builtin_amdgcn_s_memtime(), st_r0 = st_t;   // shader clock vs 100 MHz
  auto stamp = [&](int i) {
    const unsigned long long n = __builtin_amdgcn_s_memrealtime();
    st_acc[i] += n - st_t;
    st_t = n;
  };
#else
  auto stamp = [](int) {};
#endif


  auto ld_chirp = [&](int64_t f, TP (&xin)[8]) __attribute__((always_inline)) {
    const TP* __restrict__ q = iq + (f * C + (k * NW + w)) * (int64_t)S2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = lane + 64 * i;
      if constexpr (FULL) xin[i] = __builtin_nontemporal_load(q + p);
      else xin[i] = __builtin_nontemporal_load(q + (p < S2 ? p : 0));
    }
  };

  c2* const rt = L.u.rt[w];                             // this wave's transpose region (range T1, T2; Doppler TD)
#ifndef XK_HALF
  // ---------------- R: one chirp per wave (:203-205), in pieces ----------------
#ifndef XK_NOREF
  const bool refw = k == 0 && w == 0;                   // chirp 0: the frame's reference, transformed as it is
  const float dsc = refw ? 0.f : 1.f;                   // other chirps: x - x_0 (cal cancels)
  const c2 csum_w = refw ? csum : c2{0.f, 0.f};
#endif
  // R1: conditioning, DFT8 over i of both a = 2 lane + e, twiddle W1024^(a k1)
  auto r_prep = [&](const TP (&xin)[8], c2 (&z0)[8], c2 (&z1)[8]) __attribute__((always_inline)) {
    c2 v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f4v t;
      if constexpr (H) t = __builtin_convertvector(xin[i], f4v);
      else t = xin[i];
#ifndef XK_NOREF
      // x - x_0 (exact for near-equal values).  (Round 6, fp16 storage: the widening folded into this as
      // v_fma_mix_f32 took 16 VALU instructions per wave-step out and no time: profiles/r06_fp16_bounds.txt)
      t = __builtin_elementwise_fma(f4v{-dsc, -dsc, -dsc, -dsc}, L.x0[lane + 64 * i], t);
#endif
      if constexpr (!FULL)
        if (!(lane + 64 * i < S2)) t = f4v{0.f, 0.f, 0.f, 0.f};
      v[2 * i] = t.xy;
      v[2 * i + 1] = t.zw;
    }
    c2 sm = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
    for (int n = 4; n < 16; n += 4) sm += (v[n] + v[n + 1]) + (v[n + 2] + v[n + 3]);
    float wv[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f4v t = L.wq[g][lane];
      wv[4 * g] = t.x; wv[4 * g + 1] = t.y; wv[4 * g + 2] = t.z; wv[4 * g + 3] = t.w;
    }
#ifndef XK_NOREF
    const c2 mu = (wave_sum_c(sm) - csum_w) * invS;     // :204 mean of (x - cal), or of x - x_0, over the chirp
    // (d - mu_d) w' for the chirps taken against the reference (cal cancels); the reference
    // chirp's wave (uniform branch) also subtracts cal w': (x - cal - mu) w'
    if (refw) {
#pragma unroll
      for (int n = 0; n < 16; ++n) v[n] = __builtin_elementwise_fma(v[n] - mu, c2{wv[n], wv[n]}, -L.cwq[n][lane]);
    } else {
#pragma unroll
      for (int n = 0; n < 16; ++n) v[n] = (v[n] - mu) * wv[n];
    }
#else
    const c2 mu = (wave_sum_c(sm) - csum) * invS;       // :204 mean of (x - cal) over the chirp
#pragma unroll
    for (int n = 0; n < 16; ++n) v[n] = __builtin_elementwise_fma(v[n] - mu, c2{wv[n], wv[n]}, -L.cwq[n][lane]);
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i) { z0[i] = v[2 * i]; z1[i] = v[2 * i + 1]; }
#ifndef XK_NORANGEFFT   // diagnostic A/B (wrong outputs): the range DFTs and twiddles removed, transposes and stores kept
    dft8p(z0);
    dft8p(z1);
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) {
      const f4v t = L.tw1[k1 - 1][lane];
      z0[k1] = cmul_a(z0[k1], t.xy);
      z1[k1] = cmul_a(z1[k1], t.zw);
    }
#endif
  };
  const int k1 = lane >> 3, a0 = lane & 7, hh = lane & 7;
  // R2: DFT16 over a1 (lane 8 k1 + a0), twiddle W128^(a0 s1)
  auto r_mid = [&](c2 (&u)[16]) __attribute__((always_inline)) {
#ifndef XK_NORANGEFFT
    dft16p<1>(u);
#pragma unroll
    for (int s1 = 1; s1 < 16; s1 += 2) {
      const f4v t = L.tw2[s1 >> 1][lane];
      u[s1] = cmul_a(u[s1], t.xy);
      if (s1 < 15) u[s1 + 1] = cmul_a(u[s1 + 1], t.zw);
    }
#endif
  };
  auto r_t2 = [&](const c2 (&u)[16], c2 (&q0)[8], c2 (&q1)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 8; ++h)
      *reinterpret_cast<f4v*>(&rt[lane * 18 + 2 * h]) = f4v{u[2 * h].x, u[2 * h].y, u[2 * h + 1].x, u[2 * h + 1].y};
    cfence();
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const f4v t = *reinterpret_cast<const f4v*>(&rt[(k1 * 8 + jj) * 18 + 2 * hh]);
      q0[jj] = t.xy;
      q1[jj] = t.zw;
    }
    cfence();
  };
  // R3: DFT8 over a0 and the slot stores
  auto r_end = [&](c2 (&q0)[8], c2 (&q1)[8], char* __restrict__ slot) __attribute__((always_inline)) {
#ifndef XK_NORANGEFFT
    dft8p(q0);
    dft8p(q1);
#endif
    // bins k1 + 16 hh + 8 e + 128 s2 -> group 4 s2 + 2 e + (k1 >> 2), position lane & 31
    const int c = k * NW + w;
    // slot stores are buffer stores without a cache-policy flag (the only such stores in k_rdx):
    // tools/check_vmcnt.py finds them by that to prove, on the built code, that every publish
    // waits for them
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slot, (short)0, kSlotBytes, 0x00020000);
    // 16-byte stores (cdna_hip_programming.md T21: a store tail is issue-bound per instruction;
    // 4.69 -> 4.63 ms per 4096 frames against 16 8-byte stores): lane pairs swap one value, the
    // even lane stores both columns of the e = 0 row, the odd lane both of the e = 1 row
    const bool odd = lane & 1;
    const int gl = (lane >> 5) + (odd ? 2 : 0), el = c * GP + (lane & 31) - (odd ? 1 : 0);   // group 4 s2 + gl, element el
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) {
      const f4v v = pair_cols(q0[s2], q1[s2], odd);
      const int gb = (4 * s2 + gl) * C * GP * 8;
      if (H && ((s16m >> s2) & 1)) {   // c32h block (wave-uniform): X / Nr, 8 bytes per lane
        const __half2 h0 = __floats2half2_rn(v.x * kXS, v.y * kXS), h1 = __floats2half2_rn(v.z * kXS, v.w * kXS);
        __builtin_amdgcn_raw_buffer_store_b64(u2v{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1)}, rs,
                                              gb + el * 4, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, gb + el * 8, 0, 0);
      }
    }
  };

#else
  // ---------------- R, half-frame build (-DXK_HALF): a wave pair per chirp (:203-205) ----------------
  // Half-step h holds half hf = h & 1 of frame h >> 1: member k's waves w and w + 4 share chirp
  // 128 hf + 4 k + (w & 3), wave w taking the samples of parity e = w >> 2 (n = 2 m + e, m = lane + 64 i).
  // Each wave runs a 512-point FFT of its samples (DFT8 over i, twiddle W512^(lane k1), LDS transpose,
  // DFT8 over l1, twiddle W64^(l0 s1), LDS transpose, DFT8 over l0: F[r'] in lane 8 s1 + k1, register s2,
  // r' = lane + 64 s2), and the pair combines them (radix 2 in time): X[r'] = E[r'] + W1024^r' O[r'] in
  // wave e = 0, X[r' + 512] = E[r'] - W1024^r' O[r'] in wave e = 1, through LDS after a barrier.  Group g
  // of the half slot then holds bins 32 g .. 32 g + 31 (xcd_bin of the half build).  Both waves read the
  // whole chirp (16-byte sample pairs) so that each forms the :204 mean over all 1024 samples itself.
#ifdef XK_NOREF
#error "the half-frame build keeps the reference chirp"
#endif
  const int eh = w >> 2;                                // this wave's sample parity (wave-uniform)
  const bool refw0 = k == 0 && (w & 3) == 0;            // chirp 0 (half 0) is the frame's reference
  // this wave's 512 samples of the chirp (8-byte loads; c32h: 4-byte)
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  using XH = std::conditional_t<H, h2v, c2>;
  auto ld_chirp_h = [&](int64_t f, int hf, XH (&xin)[8]) __attribute__((always_inline)) {
    const XH* __restrict__ q = reinterpret_cast<const XH*>(iq + (f * C + (128 * hf + 4 * k + (w & 3))) * (int64_t)S2) + eh;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = lane + 64 * i;
      if constexpr (FULL) xin[i] = __builtin_nontemporal_load(q + 2 * p);
      else xin[i] = __builtin_nontemporal_load(q + 2 * (p < S2 ? p : 0));
    }
  };
  // before B2: d = x - x_0 (x for the reference chirp) of this wave's samples, its sum to LDS for the
  // partner (the :204 mean is over all 1024 samples); x_0 of frame j' sits in buffer j' & 1 from half-step 2 j' - 1
  auto rh_sum = [&](const XH (&xin)[8], bool refw, int xb, c2 (&d)[8]) __attribute__((always_inline)) {
    const float dsc = refw ? 0.f : 1.f;
    const c2* x0p = reinterpret_cast<const c2*>(L.x0[xb]) + eh;
    c2 sm{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c2 t;
      if constexpr (H) t = __builtin_convertvector(xin[i], c2);
      else t = xin[i];
      t = __builtin_elementwise_fma(c2{-dsc, -dsc}, x0p[2 * (lane + 64 * i)], t);
      if constexpr (!FULL)
        if (!(lane + 64 * i < S2)) t = c2{0.f, 0.f};
      d[i] = t;
      sm += t;
    }
    sm = wave_sum_c(sm);
    if (lane == 0) L.psum[w] = sm;
  };
  // R1 (after B2): the mean, (d - mu) w' (the reference chirp: (x - cal - mu) w'), DFT8 over i, twiddle W512^(lane k1)
  auto rh_prep = [&](c2 (&z)[8], bool refw) __attribute__((always_inline)) {
    const c2 csum_w = refw ? csum : c2{0.f, 0.f};
    const c2 mu = (L.psum[w] + L.psum[w ^ 4] - csum_w) * invS;   // a + b == b + a: the pair's mu agree
    float wv[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f4v t = L.wq[g][lane];                      // w' of samples 2 lane + e + 128 i, v = 2 i + e = 4 g ..
      wv[2 * g] = eh ? t.y : t.x;
      wv[2 * g + 1] = eh ? t.w : t.z;
    }
    if (refw) {
#pragma unroll
      for (int i = 0; i < 8; ++i) z[i] = __builtin_elementwise_fma(z[i] - mu, c2{wv[i], wv[i]}, -L.cwq[2 * i + eh][lane]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) z[i] = (z[i] - mu) * wv[i];
    }
    dft8p(z);
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) z[k1] = cmul_a(z[k1], L.th1[k1 - 1][lane]);
  };
  // T1 (lane l, register k1 -> lane 8 k1 + l0, register l1; row stride 72: conflict-free both ways)
  auto rh_t1w = [&](const c2 (&z)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) rt[k1 * 72 + lane] = z[k1];
    cfence();
  };
  auto rh_t1r = [&](c2 (&u)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int l1 = 0; l1 < 8; ++l1) u[l1] = rt[(lane >> 3) * 72 + (lane & 7) + 8 * l1];
    cfence();
  };
  // R2: DFT8 over l1, twiddle W64^(l0 s1); T2 (lane 8 k1 + l0, register s1 -> lane 8 s1 + k1, register l0;
  // element s1 97 + 8 k1 + 4 (k1 >> 2) + l0: conflict-free both ways); R3: DFT8 over l0
  auto rh_mid = [&](c2 (&u)[8], c2 (&v)[8]) __attribute__((always_inline)) {
    dft8p(u);
#pragma unroll
    for (int s1 = 1; s1 < 8; ++s1) u[s1] = cmul_a(u[s1], L.th2[s1 - 1][lane]);
#pragma unroll
    for (int s1 = 0; s1 < 8; ++s1) rt[s1 * 97 + lane + 4 * (lane >> 5)] = u[s1];
    cfence();
    const int rb = (lane >> 3) * 97 + 8 * (lane & 7) + 4 * ((lane & 7) >> 2);
#pragma unroll
    for (int l0 = 0; l0 < 8; ++l0) v[l0] = rt[rb + l0];
    cfence();
    dft8p(v);
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) rt[s2 * 64 + lane] = v[s2];   // for the partner wave, read after B4
  };
  // after B4: the combine and the slot stores (bins 512 e + lane + 64 s2 -> group 16 e + 2 s2 + (lane >> 5),
  // position lane & 31; the 16-byte stores pair registers 2 t, 2 t + 1 as the frame build pairs e = 0, 1)
  auto rh_end = [&](c2 (&v)[8], char* __restrict__ slot) __attribute__((always_inline)) {
    const c2* pr = L.u.rt[w ^ 4];
    if (eh) {
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) v[s2] = pr[s2 * 64 + lane] - cmul_a(v[s2], L.thc[s2][lane]);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) v[s2] = v[s2] + cmul_a(pr[s2 * 64 + lane], L.thc[s2][lane]);
    }
    constexpr int64_t kHalfBytes = (int64_t)NK * (C / 2) * GP * kES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slot, (short)0, kHalfBytes, 0x00020000);
    const bool odd = lane & 1;
    const int ch = 4 * k + (w & 3);
    const int gl = (lane >> 5) + (odd ? 2 : 0), el = ch * GP + (lane & 31) - (odd ? 1 : 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f4v pv = pair_cols(v[2 * t], v[2 * t + 1], odd);
      const int gb = (16 * eh + 4 * t + gl) * (C / 2) * GP * 8;
      if (H && ((s16m >> (4 * eh + t)) & 1)) {   // c32h block (wave-uniform): X / Nr
        const __half2 h0 = __floats2half2_rn(pv.x * kXS, pv.y * kXS), h1 = __floats2half2_rn(pv.z * kXS, pv.w * kXS);
        __builtin_amdgcn_raw_buffer_store_b64(u2v{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1)}, rs,
                                              gb + el * 4, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(pv, rs, gb + el * 8, 0, 0);
      }
    }
  };
#endif

  // ---------------- D: the 32 bins of group k (:210, :216-219, :257-259), in pieces ----------------
  // buffer_load ... sc1: the CU's L1 is bypassed (no stale lines from the slot's
  // previous frame); compiler-visible, so its vmcnt bookkeeping covers the data
  // (XK_SLOT16: the group is 32 KiB of c32h, 4 loads per thread, widened and scaled back by Nr
  // into the same fp32 staging image)
  // G16 (compile time: the step loop is instantiated per member format): a c32h group is 32 KiB,
  // 4 loads per thread, widened and scaled back by Nr into the same fp32 staging image
  auto ld_group = [&](const char* __restrict__ grp, f4v (&t)[8], auto G16) __attribute__((always_inline)) {
    constexpr int NL = decltype(G16)::value ? 4 : 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(grp), (short)0, C * GP * kES, 0x00020000);
#pragma unroll
    for (int i = 0; i < NL; ++i) t[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 512 * i) * 16, 0, 16);
  };
  auto stage = [&](const f4v (&t)[8], auto G16) __attribute__((always_inline)) {
    if constexpr (decltype(G16)::value) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 512 * i;            // 16-byte piece: chirp e >> 3, positions 4 (e & 7) .. + 3
        const u4v u = __builtin_bit_cast(u4v, t[i]);
        f4v* d = &L.u.stg[(e >> 3) * 17 + (e & 7) * 2];
        // kept as X / Nr: the rows below scale their outputs, the Doppler window the rest
        // lanes 4-7 of each 8-lane store group write their upper half first: the group's 8 stores
        // then hit 8 different 16-byte bank groups (conflict-free ds_write_b128)
        const bool sw = (e >> 2) & 1;
#ifndef XK_ST16SEL
        // the swap applied to the packed halves before they are widened: 4 selects of 32-bit words
        // instead of 8 of floats (round 6)
        const float2 b0 = h2f(sw ? u.z : u.x), b1 = h2f(sw ? u.w : u.y), c0 = h2f(sw ? u.x : u.z), c1 = h2f(sw ? u.y : u.w);
        d[sw ? 1 : 0] = f4v{b0.x, b0.y, b1.x, b1.y};
        d[sw ? 0 : 1] = f4v{c0.x, c0.y, c1.x, c1.y};
#else
        const float2 a0 = h2f(u.x), a1 = h2f(u.y), a2 = h2f(u.z), a3 = h2f(u.w);
        const f4v lo = f4v{a0.x, a0.y, a1.x, a1.y}, hi = f4v{a2.x, a2.y, a3.x, a3.y};
        d[sw ? 1 : 0] = sw ? hi : lo;
        d[sw ? 0 : 1] = sw ? lo : hi;
#endif
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e4 = tid + 512 * i;
        L.u.stg[(e4 >> 4) * 17 + (e4 & 15)] = t[i];
      }
    }
  };
  const int pp = lane >> 4, q = lane & 15, p = 4 * w + pp;
  const int r = xcd_bin(k, p);
  // D1: the rows from the staged group, :217 row mean, :210 / :265 row max |X| -> profile, candidate keys
  // G16: the staged group holds X / Nr (c32h hand-off): the profile and the keys are scaled back here
  auto d_rows = [&](int64_t f, c2 (&xv)[16], c2& x0r, c2& mu, auto G16) __attribute__((always_inline)) {
    {
      const c2* stg = reinterpret_cast<const c2*>(L.u.stg);
#pragma unroll
      for (int i = 0; i < 16; ++i) xv[i] = stg[(q + 16 * i) * 34 + p];
    }
#ifndef XK_NOREF
    // the slot holds X_0 for chirp 0 and X'_k = X_k - X_0 for the others (reference chirp above)
    x0r = reinterpret_cast<const c2*>(L.u.stg)[p];       // X_0 of this row (chirp 0: q = 0, i = 0)
    if (q == 0) xv[0] = c2{0.f, 0.f};                     // X'_0 = 0
    // :210 / :265 row max |X| over the 256 chirps, X_k = X'_k + X_0
    float pm = fmaxf(fmaxf(abs2v(xv[0] + x0r), abs2v(xv[1] + x0r)), fmaxf(abs2v(xv[2] + x0r), abs2v(xv[3] + x0r)));
#pragma unroll
    for (int i = 4; i < 16; i += 4)
      pm = fmaxf(pm, fmaxf(fmaxf(abs2v(xv[i] + x0r), abs2v(xv[i + 1] + x0r)),
                           fmaxf(abs2v(xv[i + 2] + x0r), abs2v(xv[i + 3] + x0r))));
    // :217 row mean of the X'_k: X_k - mean(X) = X'_k - mean(X')
    c2 sm = (xv[0] + xv[1]) + (xv[2] + xv[3]);
#pragma unroll
    for (int i = 4; i < 16; i += 4) sm += (xv[i] + xv[i + 1]) + (xv[i + 2] + xv[i + 3]);
#else
    x0r = c2{0.f, 0.f};
    c2 sm = (xv[0] + xv[1]) + (xv[2] + xv[3]);
    float pm = fmaxf(fmaxf(abs2v(xv[0]), abs2v(xv[1])), fmaxf(abs2v(xv[2]), abs2v(xv[3])));
#pragma unroll
    for (int i = 4; i < 16; i += 4) {
      sm += (xv[i] + xv[i + 1]) + (xv[i + 2] + xv[i + 3]);
      pm = fmaxf(pm, fmaxf(fmaxf(abs2v(xv[i]), abs2v(xv[i + 1])), fmaxf(abs2v(xv[i + 2]), abs2v(xv[i + 3]))));
    }
#endif
    sm = c2{row_sum16(sm.x), row_sum16(sm.y)};
    pm = __int_as_float(row_max16(__float_as_int(pm)));
    mu = sm * (1.0f / (float)C);
    const float pr = decltype(G16)::value ? sqrtf(pm) * kXU : sqrtf(pm);
    a.profile[f * NR + r] = pr;        // all 16 lanes of the row (same value): a store on every path
    if (q == 0) {
      const double rng = (double)r * a.dist_per_bin;
      L.key[p] = (r >= 1 && r <= NR - 2 && rng >= a.min_d && rng <= a.max_d && pr > a.range_thr) ? pr : -1.f;
    }
  };
  // D2 (after the keys barrier): slow-time candidates (:257-259), the XCD_CAND strongest
  // in-window rows of the group
  auto d_cand = [&](int64_t f, const c2 (&xv)[16], c2 x0r, auto G16) __attribute__((always_inline)) {
    float kv = lane < GP ? L.key[lane] : -1.f;
    const int ki = xcd_bin(k, lane & (GP - 1));
#pragma unroll
    for (int c = 0; c < XCD_CAND; ++c) {
      float bv = kv;
      int bi = ki;
      wave_argmax_dpp(bv, bi);                               // same in every wave: ties -> lowest bin
      const int sel = (bv < 0.f || a.force_fix) ? -1 : bi;
      if (w == 0 && lane == 0) a.cand_idx[(f * XCD_TILES + k) * XCD_CAND + c] = sel;
      if (sel >= 0 && r == sel) {
        float* __restrict__ row = a.cand_rows + ((f * XCD_TILES + k) * XCD_CAND + c) * (int64_t)C;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = abs2v(xv[i] + x0r);
          row[q + 16 * i] = decltype(G16)::value ? v * (kXU * kXU) : v;
        }
      }
      if (ki == sel) kv = -1.f;
    }
  };
  // D3: :218 (X - mean) .* 2chebwin, :219 DFT16 over i, twiddle W256^(q d0)
  auto d_a = [&](c2 (&xv)[16], c2 mu) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f4v wv = L.wdl[g][lane];
      xv[4 * g + 0] = (xv[4 * g + 0] - mu) * wv.x;
      xv[4 * g + 1] = (xv[4 * g + 1] - mu) * wv.y;
      xv[4 * g + 2] = (xv[4 * g + 2] - mu) * wv.z;
      xv[4 * g + 3] = (xv[4 * g + 3] - mu) * wv.w;
    }
#ifndef XK_NODOPFFT   // diagnostic A/B (wrong outputs): the Doppler DFTs, twiddles and transpose removed
    dft16p<1>(xv);
#pragma unroll
    for (int d0 = 1; d0 < 16; d0 += 2) {
      const f4v t = L.twd[d0 >> 1][lane];
      xv[d0] = cmul_a(xv[d0], t.xy);
      if (d0 < 15) xv[d0 + 1] = cmul_a(xv[d0 + 1], t.zw);
    }
#endif
  };
  auto d_td = [&](c2 (&xv)[16]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 8; ++h)
      *reinterpret_cast<f4v*>(&rt[304 * pp + 18 * q + 2 * h]) = f4v{xv[2 * h].x, xv[2 * h].y, xv[2 * h + 1].x, xv[2 * h + 1].y};
    cfence();
#pragma unroll
    for (int m0 = 0; m0 < 16; ++m0) xv[m0] = rt[304 * pp + 18 * m0 + q];
    cfence();
  };
  // D4: the RD row stores (:219 fftshift(., 2): position q + 16 d1s holds D[q + 16 ((d1s + 8) mod 16)])
  // or, without an RD map, the row peak (:233)
  auto d_store = [&](int64_t f, const c2 (&xv)[16]) __attribute__((always_inline)) {
    if constexpr (RD) {
      // RD rows: buffer stores with the nt cache policy (with the 2-slot ring: 4.41 vs 4.49 ms per
      // 4096 frames for sc1, which was the faster one with round 2's 4-slot ring)
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          static_cast<char*>(a.rd) + f * NR * (int64_t)C * (H ? 4 : 8), (short)0, NR * C * (H ? 4 : 8), 0x00020000);
#pragma unroll
      for (int d1s = 0; d1s < 16; ++d1s) {
        const int off = r * C + q + 16 * d1s;
        if constexpr (H) {
          const c2 o = xv[(d1s + 8) & 15];                 // rd_scale is in the window
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, __floats2half2_rn(o.x, o.y)), rr, off * 4, 0,
                                                kRdAux);
        } else {
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xv[(d1s + 8) & 15]), rr, off * 8, 0, kRdAux);
        }
      }
    } else {   // :233 [val, di] = max(abs(.)) of the row: exact max of |D|^2, then its first position
      float m = abs2v(xv[8]);
#pragma unroll
      for (int d1s = 1; d1s < 16; ++d1s) m = fmaxf(m, abs2v(xv[(d1s + 8) & 15]));
      const float rm = __int_as_float(row_max16(__float_as_int(m)));
      int e = INT_MAX;
#pragma unroll
      for (int d1s = 15; d1s >= 0; --d1s)
        if (abs2v(xv[(d1s + 8) & 15]) == rm) e = q + 16 * d1s;
      e = row_min16(e);
      a.rowpk[f * NR + r] = make_int2(__float_as_int(sqrtf(rm)), e);   // all lanes of the row: same value
    }
  };

  char* __restrict__ slots0 = reinterpret_cast<char*>(a.xcube) + (int64_t)x * NS * kSlotBytes;
#ifdef XK_DONE       // A/B: one slot per XCD, its reuse proven by a done counter (tools/r04_probe.hip part J)
  auto slot = [&](int) __attribute__((always_inline)) { return slots0; };
#else
  auto slot = [&](int j) __attribute__((always_inline)) { return slots0 + (int64_t)(j % kNS) * kSlotBytes; };
#endif
  auto frame = [&](int j) __attribute__((always_inline)) { return x + (int64_t)T * j; };
#ifndef XK_HALF
  TP xin[8];
#else
  XH xin[8];
#endif
  f4v grp[8];
#ifndef XK_HALF
  if (nj > 0) ld_chirp(frame(0), xin);
#else
  if (nj > 0) ld_chirp_h(frame(0), 0, xin);
#endif
#ifndef XK_HALF
  // Step j runs R(j) and D(j - 2) side by side in every wave, so that the range FFT's and the
  // Doppler FFT's dependency chains (DPP sums, LDS transposes) cover each other:
  //   B1 (frame j's reference chirp into LDS) -> staging of group j - 2 (loaded into registers
  //   during step j - 1) -> B2 (R(j - 1)'s slot stores waited for) -> publish R(j - 1) -> rows,
  //   profile, keys -> B3 -> candidates -> R1 | D3 -> the next frame's chirp loads (R1 freed the registers)
  //   -> wave 0 polls ready(j - 1), every wave loads group k of frame j - 1 -> TD -> T1 | D DFT16
  //   -> R2 -> T2 -> R3 + slot stores -> RD stores.
  // The group of frame j - 1 is read about one step after its slot was written, while the
  // slot's lines are still in the XCD's L2 (a ring of kNS slots: 4 MiB at kNS = 2).
  // Slot reuse needs no done counters: R(j) writes its slot after this member saw ready(j - 1),
  // i.e. after every member published R(j - 1); a member publishes R(j - 1) only after its slot
  // stores of R(j - 1) returned, and its group loads of frame j - 2 were issued before them
  // (vmcnt retires in order), so every read of frames <= j - 2 is done: kNS >= 2 suffices.
  // The publish wait counts what every path issues after the slot stores: D(j - 3)'s RD stores
  // (or row peaks); tools/check_vmcnt.py proves it on the built code.  Steps 0-2 and the last two are peeled, every flag a compile-time constant.
  constexpr int kRDs = RD ? 16 : 1;                             // D's stores after the slot stores (RD rows / row peak)
  // flags: std::integral_constant (folded: straight-line copies) or bool (the short-launch copy)
  auto body = [&](int j, auto DJ, auto RJ, auto PUB, auto CNT, auto GJ, auto NEXT, auto G16) __attribute__((always_inline)) {
    const bool dj = DJ, rj = RJ, pub = PUB, gj = GJ, next = NEXT;
    const int64_t fd = frame(j - 1 - kLag);
    if (j >= 1) __syncthreads();       // B1: step j - 1 done in every wave (transpose regions, keys, x0)
    stamp(0);
#ifndef XK_NOREF
    if (rj)
      if (j >= 1) put_ref(0);          // frame j's reference chirp (read by R1 after B3)
#endif
    if (dj) stage(grp, G16);
    stamp(1);
    // the publish of R(j - 1) at B2: its slot stores (issued at the end of step j - 1, before D(j - 3)'s
    // RD stores) have had the staging to drain; earlier (at B1) the wait exposes their latency, later
    // (after the rows, at B3) the other members' polls wait on it (4.31-4.36 vs 4.46 / 4.40 ms)
    // (the short-launch copy waits on every path: a wait behind its own `if (pub)` leaves the
    // path-insensitive proof a path that skips it and still reaches the publish)
    if constexpr (std::is_same_v<decltype(PUB), bool>) vm_wait<0>();
    else if (pub) vm_wait<decltype(CNT)::value>();
    __syncthreads();                   // B2: staged; x0 of frame j in; every wave's R(j - 1) slot stores done
    // wave 0 adds 1 to the slot's ready counter; every other wave adds 0 to a word of its own, so that
    // every wave issues the same vector-memory operations and the compiler's vmcnt waits behind them
    // never wait for an atomic
    if (pub)
      if (lane == 0)
        __hip_atomic_fetch_add(w == 0 ? rdy((j - 1) % kNS) : a.xctr + XCD_IDLE + (x * NK + k) * 32 + w,
                               w == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef XK_SKEW     // diagnostic build: when each member published R(j - 1) and when its poll of it returned
    if (pub && w == 0 && lane == 0 && j < XK_SKEW_STEPS)
      a.dbg[(int64_t)(x * NK + k) * (2 * XK_SKEW_STEPS) + 2 * j] = __builtin_amdgcn_s_memrealtime();
#endif
    stamp(2);
    c2 z0[8], z1[8], u[16];
    c2 xv[16], x0r{0.f, 0.f}, dmu{0.f, 0.f};
    if (dj) d_rows(fd, xv, x0r, dmu, G16);
    stamp(3);
    if (dj) __syncthreads();           // B3: keys in, staging read out
    stamp(4);
    if (dj) d_cand(fd, xv, x0r, G16);
    stamp(5);
    // wave 0's poll of ready(j - lag): XK_POLLAT 2 (shipped, round 6) right after R1 and the next frame's
    // loads, before D3; A/B 0 after D3 (rounds 3-5), 1 after the candidates.  The other waves still wait for
    // the flag and issue their group loads after D3, and wave 0 polls once more there (one load: the
    // counter is already there).  Measured (tools/onepass_perf.py, 4096 frames, same box): 0 4.50-4.60 ms,
    // 1 4.41-4.55, 2 4.29-4.44.  Not kept (profiles/r06_poll_ab.txt): the second poll skipped once the flag
    // is set (4.51), non-blocking looks before a blocking poll after D3 (4.55-4.65), a vector sc1 load of the
    // counter issued before the chirp loads (5.99-6.33), waves 0-1 / 0-3 each polling (5.93 / 9.2), waves
    // 1-3 sleeping or waves 4-7 prioritised at this point (+1-3 %), 4-32 replicas of the counter (0 to +3 %).
    // The stamps show the mechanism: wave 0 waits for the team in its early poll while wave 4, on the same
    // SIMD, runs its R1 and D3 alone (2.58 -> 1.84 us).
    // (a macro: the same statements in a lambda trip an LLVM aperture-check bug on the gflag store)
#define XK_POLL()                                                                                                   \
  do {                                                                                                              \
    wait_ge(rdy((j - kLag) % kNS), (unsigned)(NK * ((j - kLag) / kNS + 1)), a.xctr + XCD_ABORT, a.xerr);   \
    if (lane == 0) __hip_atomic_store(&gflag, (unsigned)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);         \
  } while (0)
    if (XK_POLLAT == 1 && gj && w == 0) XK_POLL();
    if (rj) r_prep(xin, z0, z1);
    if (next) {                        // R1 freed the chirp registers: the next frame's loads go out
      const int jn = j + 1 < nj ? j + 1 : nj - 1;
#ifndef XK_NOREF
      ld_ref(frame(jn));
#endif
      ld_chirp(frame(jn), xin);
    }
    if (XK_POLLAT == 2 && gj && w == 0) XK_POLL();
#ifdef XK_SKEW
    if (gj && w == 0 && lane == 0 && j < XK_SKEW_STEPS)
      a.dbg[(int64_t)(x * NK + k) * (2 * XK_SKEW_STEPS) + 2 * j + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (dj) d_a(xv, dmu);
    stamp(6);
    if (gj) {   // wave 0 polls ready(j - 1) (scalar: its vector memory operations stay in flight) and
                // tells the other waves through LDS; then every wave loads its share of group k
      if (w == 0) {
        XK_POLL();                       // (after the early poll it returns at its first load; without a
                                         // call here LLVM 20 emits an illegal aperture compare)
      } else {
        while (*reinterpret_cast<volatile unsigned*>(&gflag) < (unsigned)j) __builtin_amdgcn_s_sleep(1);
      }
      ld_group(slot(j - kLag) + (int64_t)k * C * GP * kES, grp, G16);
    }
    stamp(7);
#ifndef XK_NODOPFFT
    if (dj) d_td(xv);
#endif
    if (rj) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        *reinterpret_cast<f4v*>(&rt[kk * 136 + 2 * lane]) = f4v{z0[kk].x, z0[kk].y, z1[kk].x, z1[kk].y};
      cfence();
    }
#ifndef XK_NODOPFFT
    if (dj) dft16p<1>(xv);             // lane (pp, d0 = q): D[q + 16 d1] = xv[d1]
#endif
    if (rj) {
#pragma unroll
      for (int a1 = 0; a1 < 16; ++a1) u[a1] = rt[k1 * 136 + a0 + 8 * a1];
      cfence();
    }
    if (rj) {
      c2 q0[8], q1[8];
      r_mid(u);
      r_t2(u, q0, q1);
#ifdef XK_DONE
      static_assert(kLag == 1, "the done-counter A/B is written for lag 1");
      // one slot: every member's group loads of frame j - 1 (issued above) must have returned
      // before R(j) rewrites it.  Count them out (done), then wait for the whole team.
      if (gj) {
        vm_wait<0>();
        __syncthreads();
        if (w == 0) {
          if (lane == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          wait_ge(done, (unsigned)(NK * j), a.xctr + XCD_ABORT, a.xerr);
        }
        __syncthreads();
      }
#endif
      r_end(q0, q1, slot(j));
    }
    stamp(8);
    if (dj) d_store(fd, xv);           // after R(j)'s slot stores (RD stores before them: 4.64 vs 4.36 ms)
    stamp(9);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using C0 = std::integral_constant<int, 0>;
  // the publish wait counts D(j - 3)'s RD stores (row peaks), issued after R(j - 1)'s slot stores
  using C1 = std::integral_constant<int, 0>;
  using CF = std::integral_constant<int, kRDs>;
  auto run = [&](auto G16) __attribute__((always_inline)) {
#if XK_LAG == 2
    // lag 2: the Doppler runs three steps behind; 4 slots
    if (nj >= 5) {
      //   j       DJ   RJ   PUB  CNT                              GJ   NEXT
      body(0,      F_{}, T_{}, F_{}, C0{},                          F_{}, T_{}, G16);
      body(1,      F_{}, T_{}, T_{}, C0{},                          F_{}, T_{}, G16);
      body(2,      F_{}, T_{}, T_{}, C0{},                          T_{}, T_{}, G16);
      body(3,      T_{}, T_{}, T_{}, C0{},                          T_{}, T_{}, G16);
      for (int j = 4; j < nj; ++j) body(j, T_{}, T_{}, T_{}, CF{}, T_{}, T_{}, G16);
      body(nj,     T_{}, F_{}, T_{}, CF{},                          T_{}, F_{}, G16);
      body(nj + 1, T_{}, F_{}, F_{}, C0{},                          T_{}, F_{}, G16);
      body(nj + 2, T_{}, F_{}, F_{}, C0{},                          F_{}, F_{}, G16);
    } else {
      for (int j = 0; j < nj + 3; ++j)
        body(j, j >= 3, j < nj, j >= 1 && j - 1 < nj, C0{}, j >= 2 && j - 2 < nj, j + 1 < nj, G16);
    }
    return;
#endif
    if (nj >= 3) {
      //   j       DJ   RJ   PUB  CNT                              GJ   NEXT
      body(0,      F_{}, T_{}, F_{}, C0{},                          F_{}, T_{}, G16);
      body(1,      F_{}, T_{}, T_{}, C1{},                          T_{}, T_{}, G16);
      body(2,      T_{}, T_{}, T_{}, C1{},                          T_{}, T_{}, G16);
      for (int j = 3; j < nj; ++j) body(j, T_{}, T_{}, T_{}, CF{}, T_{}, T_{}, G16);
      body(nj,     T_{}, F_{}, T_{}, CF{},                          T_{}, F_{}, G16);
      body(nj + 1, T_{}, F_{}, F_{}, C0{},                          F_{}, F_{}, G16);
    } else {
      // 1-2 frames on this XCD (launches of < 24 frames): one copy with run-time flags, every
      // publish waiting for everything
      for (int j = 0; j < nj + 2; ++j)
        body(j, j >= 2, j < nj, j >= 1 && j - 1 < nj, C0{}, j >= 1 && j - 1 < nj, j + 1 < nj, G16);
    }
  };
  if constexpr (H) {
    if (g16) run(T_{});
    else run(F_{});
  } else {
    run(F_{});
  }
#else
  // Half-frame build (-DXK_HALF): the hand-off unit is half a frame (128 chirps, a 1 MiB half slot), so the
  // team runs two half-steps per frame.  Half-step h: B1 -> (h even) frame h / 2's reference chirp into LDS
  // -> (D1) staging of group k of frame jd (its two halves loaded in the two half-steps before) -> B2 ->
  // publish R(h - 1) -> (D1) rows, profile, keys -> B3 -> candidates -> R1 -> the next half-step's chirp
  // loads -> wave 0's early poll of ready(h - lag) -> (D1) D3 -> every wave loads its half of group k of
  // R(h - lag) -> (D2) TD -> T1 | (D2) DFT16 -> R2, T2, R3 -> B4 (the pair's halves in LDS) -> combine,
  // slot stores -> (D2) RD stores.  D1 of frame jd runs in half-step 2 jd + 2 + lag, D2 in the next one,
  // so the Doppler ends two frames behind the range FFT, as in the frame build.  Slot reuse: R(h) rewrites
  // half slot h mod kNS after this member saw ready(h - lag); the members' loads of R(h - 2 lag) were issued
  // before their slot stores of R(h - lag), so kNS = 2 lag half slots suffice (the frame build's argument).
  (void)ld_chirp;                                              // the frame build's pieces, unused here
  (void)ld_group;
  (void)slot;
  (void)stamp;
  constexpr int64_t kHalfSlot = (int64_t)NK * (C / 2) * GP * kES;
  auto hslot = [&](int h) __attribute__((always_inline)) { return slots0 + (int64_t)(h % kNS) * kHalfSlot; };
  constexpr int kRDs = RD ? 16 : 1;
  const int nh = 2 * nj;                                        // half-steps with range work
  c2 xvd[16];                                                   // D(jd)'s rows, from D1 to D2
  // load this member's half of group k of R(hh) into grp[hf * NL ..] (NL = 4 c64 / 2 c32h pieces per thread)
  auto ld_group_h = [&](int hh, auto HFL, auto G16) __attribute__((always_inline)) {
    constexpr int NL = decltype(G16)::value ? 2 : 4;
    const char* grb = hslot(hh) + (int64_t)k * (C / 2) * GP * kES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(grb), (short)0, (C / 2) * GP * kES, 0x00020000);
    if constexpr (std::is_same_v<decltype(HFL), bool>) {
      // value selects, not two stores: a store through a selected address would keep grp in scratch
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const f4v t = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 512 * i) * 16, 0, 16);
        grp[i] = HFL ? grp[i] : t;
        grp[NL + i] = HFL ? t : grp[NL + i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NL; ++i)
        grp[decltype(HFL)::value * NL + i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + 512 * i) * 16, 0, 16);
    }
  };
  // gflag through an LDS pointer: the flat accesses of the frame build trip LLVM 20's aperture-compare
  // bug in the half-step copies
  typedef __attribute__((address_space(3))) unsigned lu32;
  lu32* const gfl = (lu32*)&gflag;
#define XK_HPOLL()                                                                                                  \
  do {                                                                                                              \
    wait_ge(rdy((h - kLag) % kNS), (unsigned)(NK * ((h - kLag) / kNS + 1)), a.xctr + XCD_ABORT, a.xerr);   \
    if (lane == 0) __hip_atomic_store(gfl, (unsigned)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);             \
  } while (0)
  // flags: std::integral_constant in the steady pairs (every wait count static), bool elsewhere
  auto hbody = [&](int h, auto D1, auto D2, auto RJ, auto PUB, auto CNT, auto GJ, auto NEXT, auto HF, auto GHF,
                   auto G16) __attribute__((always_inline)) {
    const bool d1 = D1, d2 = D2, rj = RJ, pub = PUB, gj = GJ, next = NEXT;
    const bool hf = HF;
    const int64_t fd1 = frame((h - 2 - kLag) >> 1), fd2 = frame((h - 3 - kLag) >> 1);
    if (h >= 1) __syncthreads();       // B1
    if (hf && h + 1 < nh) put_ref(((h + 1) >> 1) & 1);   // frame (h + 1) / 2's reference chirp, read from half-step h + 1
    if (d1) stage(grp, G16);
    c2 z[8], u[8];
    if (rj) rh_sum(xin, refw0 && !hf, (h >> 1) & 1, z);
    if constexpr (std::is_same_v<decltype(PUB), bool>) vm_wait<0>();
    else if (pub) vm_wait<decltype(CNT)::value>();
    __syncthreads();                   // B2
    if (pub)
      if (lane == 0)
        __hip_atomic_fetch_add(w == 0 ? rdy((h - 1) % kNS) : a.xctr + XCD_IDLE + (x * NK + k) * 32 + w,
                               w == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c2 x0r{0.f, 0.f}, dmu{0.f, 0.f};
    if (d1) d_rows(fd1, xvd, x0r, dmu, G16);
    if (d1) __syncthreads();           // B3
    if (d1) d_cand(fd1, xvd, x0r, G16);
    if (rj) rh_prep(z, refw0 && !hf);
    if (next) {
      const int hn = h + 1;
      if (!hf && h + 2 < nh) ld_ref(frame((h >> 1) + 1));   // put at B1 of half-step h + 1
      ld_chirp_h(frame(hn >> 1), hn & 1, xin);
    }
    if (XK_POLLAT == 2 && gj && w == 0) XK_HPOLL();
    if (d1) d_a(xvd, dmu);
    if (gj) {
      if (w == 0) {
        XK_HPOLL();
      } else {
        while (__hip_atomic_load(gfl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)h) __builtin_amdgcn_s_sleep(1);
      }
      ld_group_h(h - kLag, GHF, G16);
    }
    if (d2) d_td(xvd);
    if (rj) rh_t1w(z);
    if (d2) dft16p<1>(xvd);
    if (rj) {
      rh_t1r(u);
      rh_mid(u, z);
    }
    __syncthreads();                   // B4: both halves of every pair's chirp in LDS
    if (rj) rh_end(z, hslot(h));
    if (d2) d_store(fd2, xvd);
  };
#undef XK_HPOLL
  using T_ = std::true_type;
  using F_ = std::false_type;
  using C0 = std::integral_constant<int, 0>;
  // Peeled: the first P0 half-steps and the last 4 + lag, every flag and wait count a compile-time constant
  // (tools/check_vmcnt.py's proof is path-insensitive); the steady pairs in between; a short launch runs
  // one copy with run-time flags, every publish waiting for everything.
  constexpr int P0 = kLag == 1 ? 4 : 6;
  const int nhs = nh + 2 + kLag;                               // half-steps in all
  auto pro = [&](auto HC, auto G16) __attribute__((always_inline)) {
    constexpr int h = decltype(HC)::value;
    hbody(h, std::bool_constant<(h >= 2 + kLag && ((h - 2 - kLag) & 1) == 0)>{},
          std::bool_constant<(h >= 3 + kLag && ((h - 3 - kLag) & 1) == 0)>{}, T_{}, std::bool_constant<(h >= 1)>{},
          std::integral_constant<int, (h - 1 >= 3 + kLag && ((h - 4 - kLag) & 1) == 0) ? kRDs : 0>{},
          std::bool_constant<(h >= kLag)>{}, T_{}, std::bool_constant<(h & 1) != 0>{},
          std::bool_constant<(((h - kLag) & 1) != 0)>{}, G16);
  };
  auto mid = [&](int h, auto G16) __attribute__((always_inline)) {   // h even, both half-steps steady
    constexpr bool d1o = kLag & 1;                              // D1 on odd half-steps at lag 1, even ones at lag 2
    hbody(h, std::bool_constant<!d1o>{}, std::bool_constant<d1o>{}, T_{}, T_{},
          std::integral_constant<int, d1o ? 0 : kRDs>{}, T_{}, T_{}, F_{}, std::bool_constant<(kLag & 1) != 0>{}, G16);
    hbody(h + 1, std::bool_constant<d1o>{}, std::bool_constant<!d1o>{}, T_{}, T_{},
          std::integral_constant<int, d1o ? kRDs : 0>{}, T_{}, T_{}, T_{}, std::bool_constant<(kLag & 1) == 0>{}, G16);
  };
  auto epi = [&](auto IC, auto G16) __attribute__((always_inline)) {   // half-step nh - 2 + i (nh even)
    constexpr int i = decltype(IC)::value;
    hbody(nh - 2 + i, std::bool_constant<((kLag + i) & 1) == 0 && i < 4 + kLag>{},
          std::bool_constant<((kLag + i + 1) & 1) == 0 && i < 5 + kLag>{}, std::bool_constant<(i < 2)>{},
          std::bool_constant<(i < 3)>{}, std::integral_constant<int, ((kLag + i) & 1) == 0 ? kRDs : 0>{},
          std::bool_constant<(i < 2 + kLag)>{}, std::bool_constant<(i == 0)>{}, std::bool_constant<(i & 1) != 0>{},
          std::bool_constant<((i + kLag) & 1) != 0>{}, G16);
  };
  auto hrun = [&](auto G16) __attribute__((always_inline)) {
    if (nh - 2 > P0) {
      using std::integral_constant;
      pro(integral_constant<int, 0>{}, G16);
      pro(integral_constant<int, 1>{}, G16);
      pro(integral_constant<int, 2>{}, G16);
      pro(integral_constant<int, 3>{}, G16);
      if constexpr (P0 > 4) {
        pro(integral_constant<int, 4>{}, G16);
        pro(integral_constant<int, 5>{}, G16);
      }
      for (int h = P0; h < nh - 2; h += 2) mid(h, G16);
      epi(integral_constant<int, 0>{}, G16);
      epi(integral_constant<int, 1>{}, G16);
      epi(integral_constant<int, 2>{}, G16);
      epi(integral_constant<int, 3>{}, G16);
      epi(integral_constant<int, 4>{}, G16);
      if constexpr (kLag == 2) epi(integral_constant<int, 5>{}, G16);
    } else {
      for (int h = 0; h < nhs; ++h) {
        const int h1 = h - 2 - kLag, h2 = h - 3 - kLag;
        hbody(h, h1 >= 0 && !(h1 & 1) && (h1 >> 1) < nj, h2 >= 0 && !(h2 & 1) && (h2 >> 1) < nj, h < nh,
              h >= 1 && h - 1 < nh, C0{}, h >= kLag && h - kLag < nh, h + 1 < nh, (h & 1) != 0, ((h - kLag) & 1) != 0, G16);
      }
    }
  };
  if constexpr (H) {
    if (g16) hrun(T_{});
    else hrun(F_{});
  } else {
    hrun(F_{});
  }
#endif
  if (stamper) {
    a.clk[2] = __builtin_amdgcn_s_memtime();
    a.clk[3] = __builtin_amdgcn_s_memrealtime();
  }
#ifdef XK_STAMPS
  if (lane == 0 && (w == 0 || w == 4)) {
    unsigned long long* d = a.dbg + ((int64_t)blockIdx.x * 2 + (w >> 2)) * 16;
    for (int i = 0; i < NST; ++i) d[i] = st_acc[i];
    d[13] = __builtin_amdgcn_s_memtime() - st_c0;
    d[14] = __builtin_amdgcn_s_memrealtime() - st_r0;
    d[15] = (unsigned long long)nj;
  }
#endif
}

// A grid of one block per CU shaped like k_rdx (512 threads, the same LDS): block b
// records the XCD it runs on; k_rdx needs 32 blocks on each of the device's XCDs.
// (dynamic LDS of sizeof(LdsX): one workgroup per CU, as k_rdx)
__global__ __launch_bounds__(512, 1) void k_xcd_census(int* out) {
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x] = (int)(xcc & 15);
  }
}

// k_rdx needs all 256 of its workgroups resident together (team members wait for
// each other), so two of its launches must never share a device at the same time:
// launches from different streams (several contexts over one device, host threads)
// are chained on the device through one event per device.  Only k_rdx launches are
// chained: other kernels (RCCL's, another process's) run beside it; they finish on
// their own, and while they hold CUs the bounded waits report FMCW_E_HIP (outputs
// invalid) instead of hanging.
namespace {
std::mutex xcd_chain_mu;
hipEvent_t xcd_chain_ev[64] = {};
}  // namespace

hipError_t launch_xcd(const OnePassArgs& a, hipStream_t s) {
  if (a.F <= 0) return hipSuccess;
  if (!onepass_supported(a.S, a.C, op::NR, a.C) || a.slots < 4 || a.slots > XCD_MAX_SLOTS) return hipErrorInvalidValue;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(xcd_chain_mu);
  if (!xcd_chain_ev[dev]) {
    if ((e = hipEventCreateWithFlags(&xcd_chain_ev[dev], hipEventDisableTiming | kEvDevice)) != hipSuccess) return e;
  } else if (hipStreamWaitEvent(s, xcd_chain_ev[dev], 0) != hipSuccess) {
    // a stale handle (the runtime tore the device's state down, e.g. hipDeviceReset): no
    // earlier launch can still run, so a fresh event restarts the chain
    (void)hipGetLastError();
    if ((e = hipEventCreateWithFlags(&xcd_chain_ev[dev], hipEventDisableTiming | kEvDevice)) != hipSuccess) return e;
  }
  // the counters start at zero: zeroed by the previous launch's block 0 (a.xclr of that launch), or here
  if (!a.xclr)
    if ((e = hipMemsetAsync(a.xctr, 0, sizeof(unsigned) * XCD_CTR_WORDS, s)) != hipSuccess) return e;
  if (a.nteams < 1 || a.nteams > 8) return hipErrorInvalidValue;
  const dim3 g(xk::NK * a.nteams), bl(64 * xk::NW);
  // Residency.  The grid (one 512-thread block per CU) is checked against the occupancy query
  // once per context (xcd_census: every k_rdx instantiation must fit one block per CU, else
  // AUTO takes the streams schedule); kernels of other streams or processes that hold CUs are
  // covered by the bounded waits (FMCW_E_HIP, tests/test_gpu_coresidency.py).  A cooperative
  // launch makes the same check per launch, but on MI355X / ROCm 7.2 it measured 4.69-4.70 ms
  // per 4096 frames against 4.32 for the plain launch, and the detection, compaction and STFT
  // kernels behind it on the stream 3-8x slower (profiles/r04c_coop_ab.txt), so it is opt-in:
  // FMCW_XCD_COOP=1.
  const char* coop_env = std::getenv("FMCW_XCD_COOP");   // read per launch (tests switch it)
  const bool coop = coop_env && coop_env[0] == '1';
  auto go = [&](auto kern) {
    if (!coop) {
      hipLaunchKernelGGL(kern, g, bl, 0, s, a);
      return hipGetLastError();
    }
    void* args[] = {const_cast<OnePassArgs*>(&a)};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kern), g, bl, args, 0, s);
  };
  const bool rd = a.rd != nullptr;
  if (a.S == op::NR) {
    if (a.h) e = rd ? go(k_rdx<true, true, true>) : go(k_rdx<true, true, false>);
    else e = rd ? go(k_rdx<true, false, true>) : go(k_rdx<true, false, false>);
  } else {
    if (a.h) e = rd ? go(k_rdx<false, true, true>) : go(k_rdx<false, true, false>);
    else e = rd ? go(k_rdx<false, false, true>) : go(k_rdx<false, false, false>);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return e;
  }
  return hipEventRecord(xcd_chain_ev[dev], s);
}

hipError_t xcd_census(int* nteams, int8_t* xcc_team) {
  *nteams = 0;
  for (int i = 0; i < 16; ++i) xcc_team[i] = -1;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const bool dbg = [] { const char* v = std::getenv("FMCW_XCD_DEBUG"); return v && v[0] == '1'; }();
  // 32 CUs per XCD: 256 in SPX mode, 128 / 64 / 32 per device in the DPX / QPX / CPX partition modes
  if (cus < xk::NK || cus > XCD_GRID || cus % xk::NK) {
    if (dbg) std::fprintf(stderr, "xcd_census: %d CUs\n", cus);
    return hipSuccess;
  }
  // every k_rdx instantiation must be resident at one 512-thread block per CU (what a
  // cooperative launch would check per launch)
  {
    const void* ks[] = {reinterpret_cast<const void*>(k_rdx<true, false, true>), reinterpret_cast<const void*>(k_rdx<true, false, false>),
                        reinterpret_cast<const void*>(k_rdx<true, true, true>), reinterpret_cast<const void*>(k_rdx<true, true, false>),
                        reinterpret_cast<const void*>(k_rdx<false, false, true>), reinterpret_cast<const void*>(k_rdx<false, false, false>),
                        reinterpret_cast<const void*>(k_rdx<false, true, true>), reinterpret_cast<const void*>(k_rdx<false, true, false>)};
    for (const void* kf : ks) {
      int nb = 0;
      if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 64 * xk::NW, 0)) != hipSuccess) return e;
      if (nb < 1) {
        if (dbg) std::fprintf(stderr, "xcd_census: k_rdx not resident at one block per CU\n");
        return hipSuccess;
      }
    }
  }
  int* d = nullptr;
  if ((e = hipMalloc(&d, XCD_GRID * sizeof(int))) != hipSuccess) return e;
  int h[XCD_GRID];
  hipLaunchKernelGGL(k_xcd_census, dim3(cus), dim3(512), sizeof(xk::LdsX), 0, d);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(int) * cus, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return e;
  int n[16] = {};
  bool good = true;
  for (int b = 0; b < cus; ++b) {
    if (h[b] < 0 || h[b] > 15) good = false;
    else ++n[h[b]];
  }
  int t = 0;
  for (int i = 0; i < 16 && good; ++i) {
    if (n[i] == 0) continue;
    if (n[i] != xk::NK) good = false;     // every XCD of the device must hold exactly one team
    else xcc_team[i] = (int8_t)t++;
  }
  good = good && t * xk::NK == cus;
  if (good) *nteams = t;
  else
    for (int i = 0; i < 16; ++i) xcc_team[i] = -1;
  if (dbg) {
    std::fprintf(stderr, "xcd_census: cus %d teams %d, XCC of blocks 0..15:", cus, *nteams);
    for (int b = 0; b < 16 && b < cus; ++b) std::fprintf(stderr, " %d", h[b]);
    std::fprintf(stderr, "\n");
  }
  return hipSuccess;
}

}  // namespace fmcw
