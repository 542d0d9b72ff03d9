/*
 * fmcw_mex.c -- MATLAB MEX gateway onto libfmcw (include/fmcw.h).
 *
 * Binds the C-ABI for matlab/radar_processing.m, which keeps the signature
 * radar_processing(process_animal_activity) of the reference
 * (radar-etl-pipeline/radar_processing.m:56) and calls:
 *
 *   fmcw_mex('init' [, device_ids])                              -> fmcw_ctx_create (once; mexLock);
 *                                        device_ids: vector; without it fmcw_default_devices (the env
 *                                        var FMCW_DEVICES, else every visible GPU); several ids = one
 *                                        context over several GPUs (frames and STFT segments sharded,
 *                                        RCCL max)
 *   ids = fmcw_mex('devices')                                    -> fmcw_ctx_devices (the ids in use)
 *   fmcw_mex('taps', P, range_win, doppler_win, calib_rx1)       -> fmcw_set_taps       (:138-139, :174)
 *   [prof, cnt, ridx, rmag, didx, slow, probe] =
 *       fmcw_mex('process', P, iq, probe_column)                  -> fmcw_process        (:197-261, :265, :410)
 *   [T, freq, intensity] =
 *       fmcw_mex('stft', x, win, noverlap, nfft, fs, n_log_bins)  -> fmcw_stft           (:270-299)
 *   [T, freq, intensity] =
 *       fmcw_mex('stft_png', x, win, noverlap, nfft, fs, n_log_bins, png_path)
 *                                                                 -> fmcw_stft_png  (:270-299 + :331-348)
 *   bytes = fmcw_mex('json', path, s)                             -> fmcw_json_write (:313-321 and the other
 *                                        jsonencode(s, 'PrettyPrint', true) + fprintf writes); s: a scalar
 *                                        struct of char rows and double / single / int32 arrays
 *   fmcw_mex('close')                                             -> fmcw_ctx_destroy
 *
 * P is a struct with the fields of fmcw_params (nts, pn, nr, nd, max_targets,
 * doppler_fallback_idx, if_scale, range_thr, doppler_thr, min_d, max_d,
 * dist_per_bin).  iq is a single complex NTS x PN x F array (interleaved
 * complex API: build with `mex -R2018a`), which is the C array [F][PN][NTS]
 * of the ABI -- no copy.  Outputs come back in MATLAB layout: prof Nr x F
 * (= range_tx1rx1_max_abs), ridx/rmag/didx M x F, slow PN x F, probe Nr x 1,
 * intensity nbins x nseg.
 *
 * Errors: a non-zero fmcw status becomes mexErrMsgIdAndTxt("fmcw:<status>",
 * fmcw_last_error()), i.e. a MATLAB exception that the unchanged try/catch of
 * radar_processing_with_azure.m:48-66 records in its steps struct.
 *
 * Build (MATLAB R2018a+):  mex -R2018a -I../include fmcw_mex.c -L../fmcw_radar_processing_amd -lfmcw
 * This file is compile-checked only where mex.h exists (not in this container).
 */
#include "mex.h"

#include <stdio.h>
#include <string.h>

#include "fmcw.h"

static fmcw_ctx* g_ctx = NULL;

static void at_exit(void) {
  if (g_ctx) fmcw_ctx_destroy(g_ctx);
  g_ctx = NULL;
}

static void check(int st) {
  if (st != FMCW_OK) {
    char id[32];
    const char* name = st == FMCW_E_ARG ? "arg" : st == FMCW_E_HIP ? "hip" : st == FMCW_E_OOM ? "oom"
                     : st == FMCW_E_STATE ? "state" : st == FMCW_E_DATA ? "data" : "error";
    snprintf(id, sizeof id, "fmcw:%s", name);
    mexErrMsgIdAndTxt(id, "%s", fmcw_last_error());
  }
}

static double field(const mxArray* s, const char* name) {
  const mxArray* f = mxGetField(s, 0, name);
  if (!f || !mxIsNumeric(f) || mxGetNumberOfElements(f) != 1) mexErrMsgIdAndTxt("fmcw:arg", "P.%s missing", name);
  return mxGetScalar(f);
}

static fmcw_params params_of(const mxArray* s) {
  fmcw_params p;
  if (!mxIsStruct(s)) mexErrMsgIdAndTxt("fmcw:arg", "P must be a struct");
  p.nts = (int32_t)field(s, "nts");
  p.pn = (int32_t)field(s, "pn");
  p.nr = (int32_t)field(s, "nr");
  p.nd = (int32_t)field(s, "nd");
  p.max_targets = (int32_t)field(s, "max_targets");
  p.doppler_fallback_idx = (int32_t)field(s, "doppler_fallback_idx");
  p.if_scale = (float)field(s, "if_scale");
  p.range_thr = (float)field(s, "range_thr");
  p.doppler_thr = (float)field(s, "doppler_thr");
  p.min_d = (float)field(s, "min_d");
  p.max_d = (float)field(s, "max_d");
  p.dist_per_bin = (float)field(s, "dist_per_bin");
  return p;
}

static float* single_real(const mxArray* a, mwSize n, const char* what) {
  if (!mxIsSingle(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != n)
    mexErrMsgIdAndTxt("fmcw:arg", "%s must be a real single array of %d elements", what, (int)n);
  return mxGetSingles(a);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  char cmd[16];
  if (nrhs < 1 || mxGetString(prhs[0], cmd, sizeof cmd)) mexErrMsgIdAndTxt("fmcw:arg", "first argument: command");

  if (!strcmp(cmd, "init")) {
    if (!g_ctx) {
      int32_t ids[64] = {0};
      int32_t n = 1;
      if (nrhs < 2) {
        check(fmcw_default_devices(64, ids, &n));
      } else {
        const mxArray* a = prhs[1];
        if (!mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) < 1 || mxGetNumberOfElements(a) > 64)
          mexErrMsgIdAndTxt("fmcw:arg", "init: device_ids must be a real double vector of 1..64 ids");
        n = (int32_t)mxGetNumberOfElements(a);
        for (int32_t i = 0; i < n; ++i) ids[i] = (int32_t)mxGetDoubles(a)[i];
      }
      check(fmcw_ctx_create(n, ids, &g_ctx));
      mexLock();
      mexAtExit(at_exit);
    }
    return;
  }
  if (!strcmp(cmd, "devices")) {            /* ids = fmcw_mex('devices'): the context's device ids */
    if (!g_ctx) mexErrMsgIdAndTxt("fmcw:state", "call fmcw_mex('init') first");
    int32_t ids[64], n = 0, rc = 0;
    check(fmcw_ctx_devices(g_ctx, &n, ids, &rc));
    plhs[0] = mxCreateDoubleMatrix(1, n, mxREAL);
    for (int32_t i = 0; i < n; ++i) mxGetDoubles(plhs[0])[i] = ids[i];
    return;
  }
  if (!strcmp(cmd, "close")) {
    if (g_ctx) { fmcw_ctx_destroy(g_ctx); g_ctx = NULL; mexUnlock(); }
    return;
  }
  if (!strcmp(cmd, "json")) {               /* bytes = fmcw_mex('json', path, s): needs no context */
    if (nrhs != 3 || !mxIsChar(prhs[1]) || !mxIsStruct(prhs[2]) || mxGetNumberOfElements(prhs[2]) != 1)
      mexErrMsgIdAndTxt("fmcw:arg", "json: path, scalar struct");
    char path[4096];
    if (mxGetString(prhs[1], path, sizeof path)) mexErrMsgIdAndTxt("fmcw:arg", "json: path too long");
    const int nf = mxGetNumberOfFields(prhs[2]);
    fmcw_json_field* fl = (fmcw_json_field*)mxCalloc(nf > 0 ? nf : 1, sizeof(fmcw_json_field));
    for (int k = 0; k < nf; ++k) {
      const mxArray* v = mxGetFieldByNumber(prhs[2], 0, k);
      fl[k].name = mxGetFieldNameByNumber(prhs[2], k);
      if (!v) mexErrMsgIdAndTxt("fmcw:arg", "json: field %s is empty", fl[k].name);
      if (mxIsChar(v)) {
        fl[k].kind = FMCW_JSON_STRING;
        fl[k].data = mxArrayToUTF8String(v);          /* freed with the MEX call's memory */
        continue;
      }
      if (mxIsComplex(v) || mxGetNumberOfDimensions(v) > 2)
        mexErrMsgIdAndTxt("fmcw:arg", "json: field %s must be a real vector or matrix", fl[k].name);
      fl[k].kind = mxIsDouble(v) ? FMCW_JSON_F64 : mxIsSingle(v) ? FMCW_JSON_F32 : mxIsInt32(v) ? FMCW_JSON_I32 : -1;
      if (fl[k].kind < 0) mexErrMsgIdAndTxt("fmcw:arg", "json: field %s: double, single, int32 or char", fl[k].name);
      fl[k].data = mxGetData(v);
      fl[k].rows = (int64_t)mxGetM(v);
      fl[k].cols = (int64_t)mxGetN(v);
      fl[k].row_stride = 1;                          /* MATLAB column-major */
      fl[k].col_stride = (int64_t)mxGetM(v);
    }
    int64_t bytes = 0;
    check(fmcw_json_write(path, fl, nf, 1, 0, &bytes));
    if (nlhs > 0) plhs[0] = mxCreateDoubleScalar((double)bytes);
    return;
  }
  if (!g_ctx) mexErrMsgIdAndTxt("fmcw:state", "call fmcw_mex('init') first");

  if (!strcmp(cmd, "taps")) {               /* fmcw_mex('taps', P, range_win, doppler_win, calib_rx1) */
    if (nrhs != 5) mexErrMsgIdAndTxt("fmcw:arg", "taps: P, range_win, doppler_win, calib");
    fmcw_params p = params_of(prhs[1]);
    const float* wr = single_real(prhs[2], p.nts, "range_win");
    const float* wd = single_real(prhs[3], p.pn, "doppler_win");
    if (!mxIsSingle(prhs[4]) || !mxIsComplex(prhs[4]) || mxGetNumberOfElements(prhs[4]) != (mwSize)p.nts)
      mexErrMsgIdAndTxt("fmcw:arg", "calib must be single complex, NTS elements");
    check(fmcw_set_taps(g_ctx, &p, wr, wd, (const float*)mxGetComplexSingles(prhs[4])));
    return;
  }

  if (!strcmp(cmd, "process")) {            /* fmcw_mex('process', P, iq, probe_column) */
    if (nrhs != 4) mexErrMsgIdAndTxt("fmcw:arg", "process: P, iq, probe_column");
    fmcw_params p = params_of(prhs[1]);
    const mxArray* iq = prhs[2];
    if (!mxIsSingle(iq) || !mxIsComplex(iq)) mexErrMsgIdAndTxt("fmcw:arg", "iq must be single complex NTS x PN x F");
    const mwSize nd = mxGetNumberOfDimensions(iq);
    const mwSize* dims = mxGetDimensions(iq);
    if (dims[0] != (mwSize)p.nts || dims[1] != (mwSize)p.pn) mexErrMsgIdAndTxt("fmcw:arg", "iq must be NTS x PN x F");
    const int64_t F = nd >= 3 ? (int64_t)dims[2] : 1;
    const int64_t probe = (int64_t)mxGetScalar(prhs[3]);
    const mwSize M = (mwSize)p.max_targets;
    plhs[0] = mxCreateNumericMatrix(p.nr, F, mxSINGLE_CLASS, mxREAL);   /* range_tx1rx1_max_abs */
    plhs[1] = mxCreateNumericMatrix(1, F, mxINT32_CLASS, mxREAL);
    plhs[2] = mxCreateNumericMatrix(M, F, mxINT32_CLASS, mxREAL);
    plhs[3] = mxCreateNumericMatrix(M, F, mxSINGLE_CLASS, mxREAL);
    plhs[4] = mxCreateNumericMatrix(M, F, mxINT32_CLASS, mxREAL);
    plhs[5] = mxCreateNumericMatrix(p.pn, F, mxSINGLE_CLASS, mxREAL);
    plhs[6] = mxCreateNumericMatrix(p.nr, 1, mxSINGLE_CLASS, mxREAL);
    check(fmcw_process(g_ctx, &p, mxGetComplexSingles(iq), FMCW_C64, F, mxGetSingles(plhs[0]),
                       mxGetInt32s(plhs[1]), mxGetInt32s(plhs[2]), mxGetSingles(plhs[3]), mxGetInt32s(plhs[4]),
                       mxGetSingles(plhs[5]), NULL, NULL, probe, probe > 0 ? mxGetSingles(plhs[6]) : NULL));
    return;
  }

  if (!strcmp(cmd, "stft") || !strcmp(cmd, "stft_png")) {
    /* fmcw_mex('stft', x, win, noverlap, nfft, fs, n_log_bins [, png_path]) */
    const int png = !strcmp(cmd, "stft_png");
    if (nrhs != 7 + png) mexErrMsgIdAndTxt("fmcw:arg", "stft: x, win, noverlap, nfft, fs, n_log_bins[, png_path]");
    char png_path[4096] = {0};
    if (png && (!mxIsChar(prhs[7]) || mxGetString(prhs[7], png_path, sizeof png_path)))
      mexErrMsgIdAndTxt("fmcw:arg", "stft_png: png_path must be a char row");
    const int64_t L = (int64_t)mxGetNumberOfElements(prhs[1]);
    const float* x = single_real(prhs[1], (mwSize)L, "x");
    const int32_t wlen = (int32_t)mxGetNumberOfElements(prhs[2]);
    const float* w = single_real(prhs[2], (mwSize)wlen, "win");
    const int32_t nov = (int32_t)mxGetScalar(prhs[3]), nfft = (int32_t)mxGetScalar(prhs[4]);
    const double fs = mxGetScalar(prhs[5]);
    const int32_t nlog = (int32_t)mxGetScalar(prhs[6]);
    int64_t nseg = 0;
    int32_t nf = 0, nb = 0;
    check(fmcw_stft_sizes(L, wlen, nov, nfft, nlog, &nseg, &nf, &nb));
    plhs[0] = mxCreateNumericMatrix(1, nseg, mxSINGLE_CLASS, mxREAL);   /* T */
    plhs[1] = mxCreateNumericMatrix(1, nb, mxSINGLE_CLASS, mxREAL);     /* log_freq_bins / F */
    plhs[2] = mxCreateNumericMatrix(nb, nseg, mxSINGLE_CLASS, mxREAL);  /* interp_intensity */
    if (png)
      check(fmcw_stft_png(g_ctx, x, L, w, wlen, nov, nfft, fs, nlog, mxGetSingles(plhs[0]), mxGetSingles(plhs[1]),
                          mxGetSingles(plhs[2]), png_path, 0, 0, NULL));
    else
      check(fmcw_stft(g_ctx, x, L, w, wlen, nov, nfft, fs, nlog, mxGetSingles(plhs[0]), mxGetSingles(plhs[1]),
                      mxGetSingles(plhs[2])));
    return;
  }
  mexErrMsgIdAndTxt("fmcw:arg", "unknown command '%s'", cmd);
}
