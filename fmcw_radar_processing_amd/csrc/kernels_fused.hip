// kernels_fused.hip -- persistent, XCD-local range+Doppler+detect pipeline.
//
// Why: a config-3 frame's range cube (the corner-turn intermediate between the
// range FFT along samples, radar_processing.m:205, and the Doppler FFT along
// chirps, :219) is 2 MiB -- larger than any on-chip store of one CU -- and its
// HBM round trip doubles the path's memory traffic (8.4 vs 4.2 MB/frame).
// MI355X's 8 XCDs each own a 4 MiB L2, so the corner turn of one frame fits
// in the L2 of the XCD that runs it.
//
// How: one persistent grid; every workgroup reads its XCD id (HW_REG_XCC_ID)
// and pulls tickets from that XCD's queue.  XCD x owns frames f = x, x+8, ...
// A frame is n1 range items (4 chirps each at Nr 1024: k_range's body) and n2
// Doppler items (16 rows each: k_doppler's body).  Queue order per XCD:
//   R(0) .. R(NSLOT-2), then D(i), R(i+NSLOT-1) for i = 0, 1, ...
// Range items write the frame's cube slot with plain stores (they stay in the
// XCD's L2); after every storing wave's vmcnt(0) and a barrier, one lane bumps
// k1done[f].  A Doppler item polls k1done[f] == n1 and reads the slot with
// L1-bypassing `nt` loads, i.e. from the shared L2 of the SAME XCD (it runs
// there by construction); the last Doppler item of a frame (k2done ticket)
// runs the detection and releases the slot (done[f]).  Every wait is on an
// item with a smaller ticket of the same queue, and a ticket is only drawn by
// a running workgroup, so the schedule cannot deadlock; every spin is still
// bounded and sets an error word instead of hanging the GPU.
#include "frame_ops.h"
#include "../../include/fmcw.h"

namespace fmcw {

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x & 7u;
}

__device__ __forceinline__ unsigned ld_acq(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_load sc1 (L2)
}

// Spin until *p >= target (one lane).  False on timeout or when another
// workgroup already reported one (then the whole launch drains quickly).
__device__ __forceinline__ bool wait_geq(const unsigned* p, unsigned target, unsigned* err, unsigned* sticky,
                                         unsigned limit) {
  for (unsigned it = 0;; ++it) {
    if (ld_acq(p) >= target) return true;
    if (ld_acq(err) != 0u) return false;
    if (it >= limit) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sticky, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// STRICT: the placement-independent hand-off of MI355X_MICROARCH.md's
// visibility section (producer agent release = buffer_wbl2, consumer agent
// acquire = buffer_inv) on top of the XCD-local one.  It costs an L2
// write-back of every slot and ~2-7 us of fence latency per item.
__device__ __forceinline__ void publish_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void consume_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int NR, int ND, typename TIn, typename TRd, bool STRICT>
__global__ __launch_bounds__(256, 3) void k_rd_fused(FusedArgs a) {
  using P1 = FftPlan<NR>;
  constexpr int T1 = P1::T, TEAMS1 = T1 >= 256 ? 1 : 256 / T1;
  constexpr int L1N = P1::STRIDE > 0 ? P1::STRIDE : 1, R1N = T1 > 64 ? T1 / 64 : 1;
  constexpr int K1LDS = TEAMS1 * L1N + TEAMS1 * R1N;
  using L2 = DopplerLds<ND, false>;
  constexpr int RB = L2::RB;
  constexpr int K2LDS = L2::N + 256 + 128;                   // + red_s (256 float2) + red_m (256 float)
  constexpr int SMEM = K1LDS > K2LDS ? K1LDS : K2LDS;
  __shared__ __attribute__((aligned(16))) float2 smem[SMEM];
  __shared__ unsigned s_ticket, s_flag;

  const unsigned x = xcc_id();
  const int C = a.C, tid = threadIdx.x;
  const int64_t nf = a.F > (int64_t)x ? (a.F - 1 - x) / 8 + 1 : 0;   // frames of this XCD
  const int n1 = (C + TEAMS1 - 1) / TEAMS1, n2 = (NR + RB - 1) / RB;
  const int ns = a.nslot;
  unsigned* head = a.ctrl + 32 * x;
  unsigned* k1done = a.ctrl + 256;
  unsigned* k2done = k1done + a.F;
  unsigned* done = k2done + a.F;
  unsigned* err = done + a.F;
  float2* xslots = a.slots + (int64_t)x * ns * C * NR;
  const TIn* __restrict__ iq = static_cast<const TIn*>(a.iq);
  TRd* __restrict__ rd = static_cast<TRd*>(a.rd);
  TRd* rd_xslots = a.rd_slots ? static_cast<TRd*>(a.rd_slots) + (int64_t)x * ns * NR * ND : nullptr;

  for (;;) {
    if (tid == 0) s_ticket = atomicAdd(head, 1u);
    __syncthreads();
    const int64_t t = s_ticket;
    __syncthreads();
    // decode the ticket: R(0..ns-2) first, then blocks [D(b) x n2, R(b+ns-1) x n1].
    // R(b+ns-1) reuses the slot of frame b-1 (released in the previous block),
    // so a block's range items overlap its Doppler items instead of waiting.
    bool is_range;
    int64_t i;
    int j;
    const int64_t pre = (int64_t)(ns - 1) * n1;
    if (t < pre) {
      is_range = true;
      i = t / n1;
      j = (int)(t - i * n1);
    } else {
      const int64_t b = (t - pre) / (n1 + n2);
      const int r = (int)((t - pre) - b * (n1 + n2));
      if (b >= nf) break;                                      // queue exhausted
      if (r < n2) { is_range = false; i = b; j = r; }
      else { is_range = true; i = b + ns - 1; j = r - n2; }
    }
    if (i >= nf) continue;                                     // range item past this XCD's frames
    const int64_t f = (int64_t)x + 8 * i;
    float2* slot = xslots + (i % ns) * (int64_t)C * NR;
    TRd* rd_f = rd ? rd + f * NR * (int64_t)ND : rd_xslots + (i % ns) * (int64_t)NR * ND;

    if (is_range) {
      // ---- range item: chirps [j*TEAMS1, (j+1)*TEAMS1) of frame f ----------
      if (i >= ns) {                                           // WAR: the slot's previous frame is done
        if (tid == 0) s_flag = wait_geq(done + (f - 8 * ns), 1u, err, a.sticky, a.spin_limit);
        __syncthreads();
        if (!s_flag) break;
      }
      const int team = tid / T1;
      int tt = tid % T1;
      asm volatile("" : "+v"(tt));
      const int chirp = j * TEAMS1 + team;
      const bool valid = chirp < C;
      float2 v[P1::P];
      range_team<NR, false>(iq + (f * C + (valid ? chirp : 0)) * (int64_t)a.S, valid,
                            slot + (int64_t)(valid ? chirp : 0) * NR, a.S, a.calw, a.cal_sum, a.if_scale, 1.0f,
                            a.tw_nr, smem + team * L1N, smem + TEAMS1 * L1N + team * R1N, tt, v);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every storing wave: stores at L2
      __syncthreads();
      if (tid == 0) {
        if constexpr (STRICT) publish_release();
        __hip_atomic_fetch_add(k1done + f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      // ---- Doppler item: rows [j*RB, (j+1)*RB) of frame f -------------------
      if (tid == 0) {
        s_flag = wait_geq(k1done + f, (unsigned)n1, err, a.sticky, a.spin_limit);
        if constexpr (STRICT) consume_acquire();
      }
      __syncthreads();
      if (!s_flag) break;
      float2* red_s = smem + L2::N;
      float* red_m = reinterpret_cast<float*>(smem + L2::N + 256);
      int td = tid;
      asm volatile("" : "+v"(td));                             // no hoisting of per-thread setup out of the loop
      doppler_tile<ND, false, true>(slot, C, NR, j * RB, 1.0f, a.wd, a.tw_nd, rd_f,
                                    a.rd_scale, a.profile + f * NR, smem, red_s, red_m, td);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if constexpr (STRICT) publish_release();
        const unsigned old = __hip_atomic_fetch_add(k2done + f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_flag = old == (unsigned)(n2 - 1);
        if constexpr (STRICT) {
          if (s_flag) consume_acquire();
        }
      }
      __syncthreads();
      if (s_flag && tid < 64) {
        int lane = tid;
        asm volatile("" : "+v"(lane));
        // last Doppler item of the frame: detection (:211, :227-239, :257-259)
        const int M = a.det.M;
        detect_frame<NR, true>(a.det, lane, a.profile + f * NR, rd_f, slot, a.count + f,
                               a.ridx + f * M, a.rmag + f * M, a.didx + f * M, a.slow_mag + f * C,
                               f == a.probe_frame, a.probe_chirp, a.probe_mag);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) __hip_atomic_store(done + f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int NR, int ND, typename TIn, typename TRd, bool STRICT>
static hipError_t go_fused2(const FusedArgs& a, hipStream_t s) {
  // No co-residency is needed (a ticket is only drawn by a running
  // workgroup), so the occupancy query only sizes the grid for speed.
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_rd_fused<NR, ND, TIn, TRd, STRICT>, 256, 0);
  if (e != hipSuccess) return e;
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const unsigned grid = (unsigned)(per_cu * (cus > 0 ? cus : 256));
  hipLaunchKernelGGL((k_rd_fused<NR, ND, TIn, TRd, STRICT>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int NR, int ND, typename TIn, typename TRd>
static hipError_t go_fused(const FusedArgs& a, hipStream_t s) {
  if (a.strict) return go_fused2<NR, ND, TIn, TRd, true>(a, s);
  return go_fused2<NR, ND, TIn, TRd, false>(a, s);
}

bool fused_supported(int nr, int nd) { return nr == 1024 && (nd == 256 || nd == 16); }

hipError_t launch_fused(const FusedArgs& a, hipStream_t s) {
  if (a.F <= 0) return hipSuccess;
  const bool h_in = a.in_dtype == FMCW_C32H, h_rd = a.rd_dtype == FMCW_C32H;
#define FMCW_FUSED_CASE(NR_, ND_)                                                          \
  if (a.NR == NR_ && a.ND == ND_) {                                                        \
    if (!h_in && !h_rd) return go_fused<NR_, ND_, float2, float2>(a, s);                   \
    if (h_in && h_rd) return go_fused<NR_, ND_, __half2, __half2>(a, s);                   \
    if (!h_in && h_rd) return go_fused<NR_, ND_, float2, __half2>(a, s);                   \
    return go_fused<NR_, ND_, __half2, float2>(a, s);                                      \
  }
  FMCW_FUSED_CASE(1024, 256)
  FMCW_FUSED_CASE(1024, 16)
#undef FMCW_FUSED_CASE
  return hipErrorInvalidValue;
}

}  // namespace fmcw
