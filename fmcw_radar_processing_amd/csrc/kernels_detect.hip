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
//   k_slow_fix   the rare target row that was not a candidate, recomputed by a
//                direct DFT of the frame's chirps at that bin;
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
    const int row = sel[0], tt = xcd_group(row);
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
