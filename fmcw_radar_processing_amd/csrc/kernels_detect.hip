// kernels_detect.hip -- detection and the slow-time row of the single-pass
// (XCD-team) schedule, and the fft_data probe, for gfx950.
//
// k_rdx (kernels_xcd.hip) writes the profile, the RD map (or each row's Doppler
// peak) and, per range-bin group, the |X|^2 rows of its XCD_CAND strongest
// in-window bins -- but not the range cube.  Here, per frame:
//   k_detect_1p  :211 f_search_peak (the rule of SURVEY 8a a9) on the profile,
//                :227-239 the target row's Doppler peak (read back from RD) with
//                threshold and fallback, :257-259 the slow-time row |X[ridx, :]|
//                taken from the group's candidate rows;
//                (the rare target row that was not a candidate: recomputed by the
//                frame's wave, a direct DFT of its chirps at that bin), and, when
//                asked, the compaction of :257-260 in its last workgroup;
//   k_probe      the fft_data column of :410-411 (one chirp), a direct DFT.
// (ABI 2's 8-tile single pass k_rd1p, which shared these kernels, is retired:
// the XCD-team schedule reads every frame once instead of 8 times from L2.)
#include "frame_ops.h"
#include "../../include/fmcw.h"

#include "op_math.h"

namespace fmcw {

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
// The slow-time row |X[r, k]|, k = 0..C-1, of frame f by a direct DFT at bin r (:203-205 at one
// bin), one wave: for a target row that was not among its group's candidates (rare: needs a
// larger non-peak bin of the same group inside the window).
// ---------------------------------------------------------------------------
__device__ void slow_row_direct(const Detect1pArgs& a, int64_t f, int r, int lane, float* __restrict__ slow) {
  const int S = a.S, NR = a.NR, C = a.C;
  const int nmax = S < NR ? S : NR;
  for (int k = 0; k < C; ++k) {
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
    if (lane == 0) slow[k] = sqrtf(cabs2(acc));
  }
}

// ---------------------------------------------------------------------------
// k_detect_1p: one wave per frame.  Peak rule on the profile (:211), Doppler
// index from the row peaks (:227-239), slow-time row from the candidates (or,
// rarely, by slow_row_direct).  With a.list set, the last workgroup to finish
// also runs the compaction of :257-260 (what k_compact does) over every frame
// of the call, so the slow-time leg needs no launch of its own before the STFT.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_detect_1p(Detect1pArgs a) {
  constexpr int NR = op::NR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f = (int64_t)blockIdx.x * 4 + w;
  const bool fused = a.list != nullptr;
  if (f < a.nframes) {
    const DetectParams& q = a.det;
    const int C = a.C, M = a.M;
    int sel[8];
    float selv[8];
    const int n = select_peaks<NR, false>(q, lane, a.profile + f * NR, sel, selv);
    float* slow = a.slow_mag + f * C;
    if (n > 0) {
      const int row = sel[0], tt = xcd_group(row);
      const int32_t* ci = a.cand_idx + (f * a.tiles + tt) * a.ncand;
      int c = -1;
      for (int i = a.ncand - 1; i >= 0; --i)
        if (ci[i] == row) c = i;
      if (c >= 0) {
        const float* src = a.cand_rows + ((f * a.tiles + tt) * a.ncand + c) * (int64_t)C;
        for (int k = lane; k < C; k += 64) slow[k] = sqrtf(src[k]);     // candidates hold |X|^2
      } else {
        slow_row_direct(a, f, row, lane, slow);                         // wave-uniform branch
      }
    } else {
      for (int k = lane; k < C; k += 64) slow[k] = 0.f;
    }
    // :233 [val, di] = max(abs(D)) of each target row: from the RD map when it
    // was written, else from rowpk
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
    if (lane == 0) {
      if (fused) __hip_atomic_store(a.count + f, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // write-through (sc1)
      else a.count[f] = n;
    }
  }
  if (!fused) return;
  // Hand-off of the counts to the last workgroup (MI355X_MICROARCH.md, inter-workgroup visibility,
  // the "one lane of each storing workgroup adds to ONE counter" row): sc1 stores, every storing
  // wave's vmcnt(0), a workgroup barrier, one agent-scope add; the last adder acquires and reads
  // the counts with sc1 loads.
  // The arrivals are sharded (MI355X_MICROARCH.md fanin: ~12 ns per atomic on ONE word, ~12 us for
  // the 1,024 workgroups of a 4096-frame launch): workgroup b adds to shard b % 8 (its own 128-byte
  // line), the shard's last arriver adds to the top counter, and the top's last arriver scans.
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int G = (int)gridDim.x, sh = (int)(blockIdx.x & 7u);
    const int in_shard = (G - sh + 7) / 8, shards = G < 8 ? G : 8;
    int l = 0;
    if (__hip_atomic_fetch_add(a.done + 32 * sh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_shard - 1)
      l = __hip_atomic_fetch_add(a.done + 32 * 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shards - 1;
    last = l;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // exclusive scan of (count > 0) over F_all frames, 16 consecutive frames per thread per pass
  __shared__ int wsum[4];
  int64_t carry = 0;
  for (int64_t base = 0; base < a.F_all; base += 256 * 16) {
    const int64_t f0 = base + (int64_t)threadIdx.x * 16;
    // 16 counts per thread as four 16-byte sc1 buffer loads (all in flight at once)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int32_t*>(a.count_all), (short)0, (int)(a.F_all * 4 < 0x7fffffff ? a.F_all * 4 : 0x7fffffff), 0x00020000);
    int4 c4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t fi = f0 + 4 * i;
      if (fi + 4 <= a.F_all && fi * 4 + 16 <= 0x7fffffffLL) {
        c4[i] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(fi * 4), 0, 16));
      } else {                                          // the last, partial vector: element by element
        int e[4];
        for (int j = 0; j < 4; ++j)
          e[j] = fi + j < a.F_all ? __hip_atomic_load(a.count_all + fi + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        c4[i] = make_int4(e[0], e[1], e[2], e[3]);
      }
    }
    unsigned bits = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bits |= (c4[i].x > 0 ? 1u : 0u) << (4 * i);
      bits |= (c4[i].y > 0 ? 1u : 0u) << (4 * i + 1);
      bits |= (c4[i].z > 0 ? 1u : 0u) << (4 * i + 2);
      bits |= (c4[i].w > 0 ? 1u : 0u) << (4 * i + 3);
    }
    const int mine = __popc(bits);
    int incl = mine;                                    // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int pre = incl - mine;
    int tot = 0;
    for (int i = 0; i < 4; ++i) {
      if (i < w) pre += wsum[i];
      tot += wsum[i];
    }
    int pos = (int)carry + pre;
    for (int i = 0; i < 16; ++i)
      if ((bits >> i) & 1u) a.list[pos++] = (int32_t)(f0 + i);
    carry += tot;
    __syncthreads();                                    // wsum reused by the next pass
  }
  if (threadIdx.x == 0) {
    *a.len = carry * a.pn;
    if (a.pmax_reset) *a.pmax_reset = 0.f;
  }
  if (threadIdx.x < 9) __hip_atomic_store(a.done + 32 * threadIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
bool onepass_supported(int nts, int pn, int nr, int nd) {
  return nr == op::NR && pn == nd && nd == 256 && nts >= 2 && nts <= nr && (nts % 2) == 0;
}

hipError_t launch_detect_1p(const Detect1pArgs& a, hipStream_t s) {
  if (a.nframes <= 0) return hipSuccess;
  if (a.NR != op::NR) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_detect_1p, dim3((unsigned)((a.nframes + 3) / 4)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_probe(const ProbeArgs& a, hipStream_t s) {
  if (a.S > a.NR || a.NR != op::NR) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

}  // namespace fmcw
