/*
 * fmcw_oracle.c -- float64 C restatement of the FMCW hot path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for libfmcw (HIP) and the timed CPU
 * baseline of bench.py ("kind": "port").  Nothing in fmcw_radar_processing_amd
 * links or loads this file.  Built by oracle/Makefile into oracle/build/.
 *
 * It follows radar-etl-pipeline/radar_processing.m of alepnabil/fmcw_radar_processing
 * (the same steps, in the same order, as oracle/oracle.py):
 *   :203  y = (x - calib_rx1) * IF_scale
 *   :204  y -= mean(y)                      (per chirp, over samples)
 *   :205  X = fft(y .* 2*blackman, Nr)      (zero-pad / truncate)
 *   :210  prof = abs(max(X, [], 2))         (max |.| over chirps)
 *   :211  f_search_peak -- absent from the reference; rule of SURVEY.md 8a a9
 *   :217-219 Doppler: mean over ALL chirps removed, .* 2*chebwin, fft(., Nd, 2)
 *            (truncating when Nd < PN), fftshift; here for every range row
 *   :233-238 [val, idx] = max(abs(row)); idx unless val < thr or idx == fallback
 *   :259  slow-time row |X(ridx(1), :)|
 *   :270-299 spectrogram (one-sided PSD), 20*log10(P/max), logspace + interp1
 * PARITY STATUS: parity unpinned against MATLAB (no MATLAB runtime, no reference
 * fixtures); cross-checked against oracle/oracle.py and the known-answer tests.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { double re, im; } cd;

typedef struct {
  int n;
  cd* w;      /* w[k] = exp(-2 pi i k / n), k < n/2, computed once in float64 */
} plan_t;

static plan_t plan_make(int n) {
  plan_t p = {n, (cd*)malloc(sizeof(cd) * (size_t)(n / 2 > 0 ? n / 2 : 1))};
  for (int k = 0; k < n / 2; ++k) { p.w[k].re = cos(-2.0 * M_PI * k / n); p.w[k].im = sin(-2.0 * M_PI * k / n); }
  return p;
}

static void plan_free(plan_t* p) { free(p->w); p->w = NULL; }

static void fft_inplace(cd* a, const plan_t* p) {  /* iterative radix-2 DIT, forward, n power of two */
  const int n = p->n;
  for (int i = 1, j = 0; i < n; ++i) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { cd t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (int len = 2; len <= n; len <<= 1) {
    const int step = n / len;
    for (int i = 0; i < n; i += len) {
      for (int k = 0; k < len / 2; ++k) {
        const cd tw = p->w[k * step];
        cd u = a[i + k], v = a[i + k + len / 2];
        cd w = {v.re * tw.re - v.im * tw.im, v.re * tw.im + v.im * tw.re};
        a[i + k].re = u.re + w.re; a[i + k].im = u.im + w.im;
        a[i + k + len / 2].re = u.re - w.re; a[i + k + len / 2].im = u.im - w.im;
      }
    }
  }
}

static double cabs_(cd a) { return sqrt(a.re * a.re + a.im * a.im); }

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* One frame; X is scratch [C][Nr] (chirp-major, the C layout of MATLAB's Nr x PN). */
static void one_frame(int S, int C, int Nr, int Nd, int M, int fallback, double if_scale, double thr_r,
                      double thr_d, double min_d, double max_d, double dpb, const double* wr, const double* wd,
                      const double* cal, const float* iq, double* prof, int32_t* count, int32_t* ridx,
                      double* rmag, int32_t* didx, double* slow, double* cube, double* rd, double* pre, cd* X,
                      cd* row, const plan_t* pr, const plan_t* pd) {
  const int nmax = S < Nr ? S : Nr;
  for (int k = 0; k < C; ++k) {                       /* :203-205 */
    const float* x = iq + (size_t)k * S * 2;
    double mr = 0, mi = 0;
    for (int n = 0; n < S; ++n) {
      mr += (x[2 * n] - cal[2 * n]) * if_scale;
      mi += (x[2 * n + 1] - cal[2 * n + 1]) * if_scale;
    }
    mr /= S; mi /= S;
    cd* Xk = X + (size_t)k * Nr;
    for (int n = 0; n < Nr; ++n) {
      if (n < nmax) {
        Xk[n].re = ((x[2 * n] - cal[2 * n]) * if_scale - mr) * wr[n];
        Xk[n].im = ((x[2 * n + 1] - cal[2 * n + 1]) * if_scale - mi) * wr[n];
      } else {
        Xk[n].re = Xk[n].im = 0;
      }
    }
    fft_inplace(Xk, pr);
  }
  if (cube) memcpy(cube, X, sizeof(cd) * (size_t)C * Nr);
  if (pre) {   /* energy entering the Doppler FFT before the :218 mean removal, Nd * sum |X w|^2 */
    const int kq = C < Nd ? C : Nd;
    double e = 0;
    for (int k = 0; k < kq; ++k)
      for (int r = 0; r < Nr; ++r) {
        const cd v = X[(size_t)k * Nr + r];
        e += (v.re * v.re + v.im * v.im) * wd[k] * wd[k];
      }
    *pre = Nd * e;
  }
  /* rows are gathered RB at a time (RB*16 B contiguous per chirp) */
  enum { RB = 8 };
  cd* rows = row;   /* scratch [RB][max(C, Nd)] */
  const int rl = C > Nd ? C : Nd;
  for (int r0 = 0; r0 < Nr; r0 += RB) {            /* :210 profile over the gathered rows */
    const int nb = Nr - r0 < RB ? Nr - r0 : RB;
    for (int k = 0; k < C; ++k)
      for (int q = 0; q < nb; ++q) rows[q * rl + k] = X[(size_t)k * Nr + r0 + q];
    for (int q = 0; q < nb; ++q) {
      double m = 0;
      for (int k = 0; k < C; ++k) { double v = cabs_(rows[q * rl + k]); if (v > m) m = v; }
      prof[r0 + q] = m;
    }
  }
  /* :211 f_search_peak */
  int sel[8], n = 0;
  double selv[8];
  for (int j = 0; j < M; ++j) {
    double bv = -1; int bi = -1;
    for (int i = 1; i <= Nr - 2; ++i) {
      const double rg = i * dpb;
      if (rg < min_d || rg > max_d) continue;
      const double v = prof[i];
      if (!(v > thr_r && v >= prof[i - 1] && v > prof[i + 1])) continue;
      int taken = 0;
      for (int q = 0; q < n; ++q) taken |= sel[q] == i;
      if (taken) continue;
      if (v > bv) { bv = v; bi = i; }
    }
    if (bi < 0) break;
    sel[n] = bi; selv[n] = bv; ++n;
  }
  /* :216-219 every row (rd != NULL) or the target rows only; :233-238 */
  const int kf = C < Nd ? C : Nd;
  for (int r0 = 0; r0 < Nr; r0 += RB) {
    const int nb = Nr - r0 < RB ? Nr - r0 : RB;
    int any = rd != NULL;
    for (int j = 0; j < n; ++j) any |= (sel[j] >= r0 && sel[j] < r0 + nb);
    if (!any) continue;
    for (int k = 0; k < C; ++k)
      for (int q = 0; q < nb; ++q) rows[q * rl + k] = X[(size_t)k * Nr + r0 + q];
    for (int q = 0; q < nb; ++q) {
      const int r = r0 + q;
      int tj = -1;
      for (int j = 0; j < n; ++j) if (sel[j] == r) tj = j;
      if (!rd && tj < 0) continue;
      cd* rw = rows + q * rl;
      double mr = 0, mi = 0;
      for (int k = 0; k < C; ++k) { mr += rw[k].re; mi += rw[k].im; }
      mr /= C; mi /= C;
      for (int k = 0; k < Nd; ++k) {
        if (k < kf) { rw[k].re = (rw[k].re - mr) * wd[k]; rw[k].im = (rw[k].im - mi) * wd[k]; }
        else { rw[k].re = rw[k].im = 0; }
      }
      fft_inplace(rw, pd);
      double bv = -1; int bi = 0;
      for (int d = 0; d < Nd; ++d) {
        const cd v = rw[(d + Nd / 2) % Nd];          /* fftshift(., 2) for even Nd */
        if (rd) { rd[((size_t)r * Nd + d) * 2] = v.re; rd[((size_t)r * Nd + d) * 2 + 1] = v.im; }
        const double a = cabs_(v);
        if (a > bv) { bv = a; bi = d; }
      }
      if (tj >= 0) {
        int di = bi + 1;
        if (!(bv >= thr_d && di != fallback)) di = fallback;
        didx[tj] = di;
      }
    }
  }
  count[0] = n;
  for (int j = 0; j < M; ++j) {
    ridx[j] = j < n ? sel[j] + 1 : 0;
    rmag[j] = j < n ? selv[j] : 0;
    if (j >= n) didx[j] = 0;
  }
  for (int k = 0; k < C; ++k) slow[k] = n > 0 ? cabs_(X[(size_t)k * Nr + sel[0]]) : 0.0;   /* :259 */
}

/* iq: [F][C][S] complex float32 interleaved.  Outputs [F]-major like libfmcw.
 * pre (optional, [F]): Nd * sum |X w_d|^2 per frame, the normalisation floor of
 * the relaxed RD error (tests/helpers.py rd_rel_err). */
int oracle_process2(int S, int C, int Nr, int Nd, int M, int fallback, double if_scale, double thr_r,
                    double thr_d, double min_d, double max_d, double dpb, const double* wr, const double* wd,
                    const double* cal, const float* iq, int64_t F, double* prof, int32_t* count, int32_t* ridx,
                    double* rmag, int32_t* didx, double* slow, double* cube, double* rd, double* pre, int nthreads) {
  if (M < 1 || M > 8) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    cd* X = (cd*)malloc(sizeof(cd) * (size_t)C * Nr);
    cd* row = (cd*)malloc(sizeof(cd) * (size_t)8 * (C > Nd ? C : Nd));
    plan_t pr = plan_make(Nr), pd = plan_make(Nd);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int64_t f = 0; f < F; ++f) {
      one_frame(S, C, Nr, Nd, M, fallback, if_scale, thr_r, thr_d, min_d, max_d, dpb, wr, wd, cal,
                iq + (size_t)f * C * S * 2, prof + (size_t)f * Nr, count + f, ridx + (size_t)f * M,
                rmag + (size_t)f * M, didx + (size_t)f * M, slow + (size_t)f * C,
                cube ? cube + (size_t)f * C * Nr * 2 : NULL, rd ? rd + (size_t)f * Nr * Nd * 2 : NULL,
                pre ? pre + f : NULL, X, row, &pr, &pd);
    }
    free(X);
    free(row);
    plan_free(&pr);
    plan_free(&pd);
  }
  return 0;
}

int oracle_process(int S, int C, int Nr, int Nd, int M, int fallback, double if_scale, double thr_r,
                   double thr_d, double min_d, double max_d, double dpb, const double* wr, const double* wd,
                   const double* cal, const float* iq, int64_t F, double* prof, int32_t* count, int32_t* ridx,
                   double* rmag, int32_t* didx, double* slow, double* cube, double* rd, int nthreads) {
  return oracle_process2(S, C, Nr, Nd, M, fallback, if_scale, thr_r, thr_d, min_d, max_d, dpb, wr, wd, cal, iq, F,
                         prof, count, ridx, rmag, didx, slow, cube, rd, NULL, nthreads);
}

/* Per-frame squared error of a device result against the float64 oracle:
 * num2[f] = sum |got * unscale - ref|^2, den2[f] = sum |ref|^2 over the n complex
 * values of frame f (got: complex float32 interleaved).  The bench's full-size
 * check (bench.py) uses it on every frame it times. */
void oracle_err2(const double* ref, const float* got, double unscale, int64_t F, int64_t n, double* num2,
                 double* den2, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
  for (int64_t f = 0; f < F; ++f) {
    const double* r = ref + (size_t)f * n * 2;
    const float* g = got + (size_t)f * n * 2;
    double a = 0, b = 0;
    for (int64_t i = 0; i < 2 * n; ++i) {
      const double d = (double)g[i] * unscale - r[i];
      a += d * d;
      b += r[i] * r[i];
    }
    num2[f] = a;
    den2[f] = b;
  }
}

/* :270-299.  x real [L]; nfft power of two >= wlen; nlog = 0 -> dB on the native
 * nfft/2+1 bins (intensity [nseg][nb]); else interp1 onto logspace bins
 * (intensity [nseg][nlog]).  Returns nseg (or -1). */
int64_t oracle_stft(const double* x, int64_t L, const double* win, int wlen, int noverlap, int nfft, double fs,
                    int nlog, double* T, double* freq, double* intensity, int nthreads) {
  const int hop = wlen - noverlap, nb = nfft / 2 + 1;
  const int64_t nseg = (L - noverlap) >= 0 ? (L - noverlap) / hop : 0;
  if (nseg < 1 || nfft < wlen || (nfft & (nfft - 1))) return -1;
  double u = 0;
  for (int m = 0; m < wlen; ++m) u += win[m] * win[m];
  const double scale = 1.0 / (fs * u);
  double* P = (double*)malloc(sizeof(double) * (size_t)nseg * nb);
  double gmax = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(max : gmax)
#endif
  {
    cd* buf = (cd*)malloc(sizeof(cd) * (size_t)nfft);
    plan_t pn = plan_make(nfft);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int64_t s = 0; s < nseg; ++s) {
      for (int m = 0; m < nfft; ++m) {
        buf[m].re = m < wlen ? x[s * hop + m] * win[m] : 0.0;
        buf[m].im = 0;
      }
      fft_inplace(buf, &pn);
      for (int b = 0; b < nb; ++b) {
        const double k = (b == 0 || 2 * b == nfft) ? 1.0 : 2.0;
        const double p = (buf[b].re * buf[b].re + buf[b].im * buf[b].im) * scale * k;
        P[(size_t)s * nb + b] = p;
        if (p > gmax) gmax = p;
      }
    }
    free(buf);
    plan_free(&pn);
  }
  for (int64_t s = 0; s < nseg; ++s) T[s] = ((double)s * hop + wlen / 2.0) / fs;
  const double df = fs / nfft;
  if (nlog == 0) {
    for (int b = 0; b < nb; ++b) freq[b] = b * df;
    for (int64_t i = 0; i < nseg * nb; ++i) intensity[i] = 20.0 * log10(P[i] / gmax);
  } else {
    const double a = log10(df), e = log10((nb - 1) * df);
    for (int j = 0; j < nlog; ++j) {
      const double ex = (j == nlog - 1) ? e : a + j * (e - a) / (nlog - 1);
      freq[j] = pow(10.0, ex);
    }
    for (int64_t s = 0; s < nseg; ++s) {
      const double* row = P + (size_t)s * nb;
      for (int j = 0; j < nlog; ++j) {
        int i0 = (int)floor(freq[j] / df);
        if (i0 < 0) i0 = 0;
        if (i0 > nb - 2) i0 = nb - 2;
        const double w = (freq[j] - i0 * df) / df;
        const double d0 = 20.0 * log10(row[i0] / gmax), d1 = 20.0 * log10(row[i0 + 1] / gmax);
        intensity[(size_t)s * nlog + j] = d0 + w * (d1 - d0);
      }
    }
  }
  free(P);
  return nseg;
}
