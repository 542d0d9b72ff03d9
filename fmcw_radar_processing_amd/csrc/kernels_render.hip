// kernels_render.hip -- spectrogram.png of radar_processing.m:331-348 on the GPU.
//
//   surf(T, F, psd, 'EdgeColor','none'); view(0,90); axis tight;
//   ylim([0 150]); clim([-40 0]); axis off; colormap(jet);
//   exportgraphics(fig, 'spectrogram.png', 'Resolution', 600)
//
// with F = fftshift(F), psd = 20*log10(P/max(P(:))) and P = fftshift(P, 1)
// (:277-283).  F is the ONE-sided axis (nb = nfft/2 + 1 bins), so fftshift
// rotates it: the rows run bins [nb-h .. nb-1, 0 .. nb-h-1], h = floor(nb/2).
// surf joins consecutive rows, so the surface has
//   - a face between bins m and m+1 for every m except m = nb-h-1 (the seam),
//   - one "fold" face from bin nb-1 (y = fs/2) straight back to bin 0 (y = 0)
//     over the whole frequency range.
// Seen from +z (view(0, 90)) the fold and the ordinary face at (t, y) overlap;
// the depth test shows the higher one (z = psd, bilinear over each face).
// Faces are flat-shaded with the colour of their first vertex (row of the
// lower rotated index, column s), mapped through jet(256) on clim [-40 0]
// (MATLAB scaled CData mapping: index = fix((c - cmin)/(cmax - cmin) * 256),
// clamped to [0, 255]).  Each pixel samples its centre; x spans [T(1), T(end)]
// (axis tight), y spans [0, fmax] (ylim), top row at fmax.
//
// Output: palette indices [H][1 + W] with the PNG row filter byte (0) in
// column 0, so the host deflates the buffer as is.  Arithmetic in double with
// FMA contraction off: tests/test_gpu_render.py restates the same rules in
// numpy and requires identical indices.
#include "fmcw_internal.h"

namespace fmcw {

#pragma clang fp contract(off)

__device__ __forceinline__ double zval(const RenderArgs& a, double inv_pmax, int64_t s, int col) {
  // psd (:283) of stored column `col` (bins 0 .. nq-1, Nyquist at nq) at segment s,
  // floored so that bilinear weights of 0 never meet -inf (P = 0)
  const double p = (double)a.Q[s * (a.nq + 1) + col];
  const double v = p > 0.0 ? 20.0 * log10(p * inv_pmax) : -1.0e30;
  return v < -1.0e30 ? -1.0e30 : v;
}

__device__ __forceinline__ double bilin(double z00, double z10, double z01, double z11, double fy, double fx) {
  const double a = z00 + (z10 - z00) * fy, b = z01 + (z11 - z01) * fy;
  return a + (b - a) * fx;
}

__global__ __launch_bounds__(256) void k_render(RenderArgs a) {
  const int px = blockIdx.x * 256 + threadIdx.x, py = blockIdx.y;
  if (px >= a.W) return;
  uint8_t* row = a.img + (int64_t)py * (a.W + 1);
  if (px == 0) row[0] = 0;                                   // PNG filter type None
  const int64_t nseg = *a.nseg;
  const float pm = *a.pmax;
  const double inv = pm > 0.f ? 1.0 / (double)pm : 0.0;
  uint8_t idx = 0;
  if (nseg >= 2) {
    const double t0 = a.t0, t1 = a.t0 + (double)(nseg - 1) * a.dt;
    const double t = t0 + ((double)px + 0.5) * (t1 - t0) / (double)a.W;
    const double y = a.fmax * (1.0 - ((double)py + 0.5) / (double)a.H);
    const double u = (t - t0) / a.dt;
    int64_t s = (int64_t)floor(u);
    if (s < 0) s = 0;
    if (s > nseg - 2) s = nseg - 2;
    const double fx = u - (double)s;
    const double df = a.fs / (double)a.nfft, nyq_f = a.fs * 0.5;
    const int nyq = a.nq;                                    // stored column of bin nb-1
    // the fold face: bin 0 (y = 0) .. bin nb-1 (y = fs/2)
    const double zf = bilin(zval(a, inv, s, 0), zval(a, inv, s, nyq), zval(a, inv, s + 1, 0), zval(a, inv, s + 1, nyq), y / nyq_f, fx);
    double zc = zval(a, inv, s, nyq);                            // fold face colour: first vertex = bin nb-1
    const double my = y / df;
    const int64_t m = (int64_t)floor(my);
    // stored column of bin b: bins 0 .. nq-1 directly, bin nb-1 at column nq
    auto col = [&](int64_t b) { return b < a.nq ? (int)b : (b == a.nb - 1 ? nyq : -1); };
    // the ordinary face between bins m and m+1 (absent at the seam m = nb-h-1)
    if (m >= 0 && m + 1 <= a.nb - 1 && m != a.seam && col(m) >= 0 && col(m + 1) >= 0) {
      const int c0 = col(m), c1 = col(m + 1);
      const double zn = bilin(zval(a, inv, s, c0), zval(a, inv, s, c1), zval(a, inv, s + 1, c0),
                              zval(a, inv, s + 1, c1), my - (double)m, fx);
      if (zn >= zf) zc = zval(a, inv, s, c0);
    }
    const double q = (zc - a.cmin) / (a.cmax - a.cmin) * 256.0;
    const double qf = q < 0.0 ? 0.0 : (q > 255.0 ? 255.0 : floor(q));
    idx = (uint8_t)qf;
  }
  row[1 + px] = idx;
}

#pragma clang fp contract(on)

hipError_t launch_render(const RenderArgs& a, hipStream_t s) {
  if (a.W <= 0 || a.H <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_render, dim3((unsigned)((a.W + 255) / 256), (unsigned)a.H), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace fmcw
