/*
 * fmcw.h -- C-ABI of libfmcw, the MI355X (gfx950) FMCW radar DSP path.
 *
 * Drop-in boundary for the per-frame fast-time / slow-time / STFT loop of
 * alepnabil/fmcw_radar_processing, radar-etl-pipeline/radar_processing.m
 * (function radar_processing(process_animal_activity), :56).  The reference
 * has no FFI layer of its own: every step is a MATLAB built-in call inside
 * one serial loop.  The entry points below replace exactly these lines, and
 * are what a MEX gateway (mex/fmcw_mex.c) binds; INTEGRATION.md shows the
 * MATLAB-side call sequence and a ctypes binding.
 *
 *   fmcw_set_taps      <- :121/:136 IF_scale, :138-139 window taps, :166-174 calib_rx1
 *   fmcw_process       <- :197-261 per-frame loop ('no' branch) + :265 range_tx1rx1_max_abs
 *                         (:457-498 per-frame part of the 'yes' branch is the same math)
 *   fmcw_range_fft     <- :203-205 + :207 + :210 only (range cube + profile; config 2)
 *   fmcw_stft          <- :270-299 (|slow|, nextpow2, spectrogram, fftshift, 20log10,
 *                         logspace + interp1)
 *
 * Conventions
 *   - Plain C types only.  Complex data is interleaved (re, im) float32, which
 *     is MATLAB's interleaved-complex `single` layout (-R2018a API).
 *   - Array shapes are written C-style, last index fastest.  Every one of them
 *     is also the memory layout of the MATLAB array named next to it, so a MEX
 *     gateway hands MATLAB buffers through without copies or transposes.
 *   - Return value: FMCW_OK (0) or a negative fmcw_status; the message of the
 *     last failure on the calling thread is in fmcw_last_error().
 *   - A context is NOT thread-safe: one per host thread (MEX keeps one static).
 *   - The caller owns every I/O buffer; the library never returns memory.
 *   - There is no CPU fallback: on a host without a usable gfx950 device
 *     fmcw_ctx_create fails with FMCW_E_HIP.
 */
#ifndef FMCW_H_
#define FMCW_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: FMCW_PIPE_ONEPASS names the XCD-team schedule (E_ARG where the XCD census fails),
 *    fmcw_default_devices, FMCW_JSON_BOOL */
#define FMCW_ABI_VERSION 4

typedef enum fmcw_status {
  FMCW_OK = 0,
  FMCW_E_ARG = -1,          /* bad argument / unsupported size                */
  FMCW_E_HIP = -2,          /* HIP runtime failure (no device, launch, copy)   */
  FMCW_E_OOM = -3,          /* device allocation failed                        */
  FMCW_E_STATE = -4,        /* call order (e.g. fmcw_set_taps not called)      */
  FMCW_E_DATA = -5          /* data-dependent failure MATLAB would raise, e.g.
                               spectrogram of a signal shorter than the window */
} fmcw_status;

/* Element type of IQ input and of complex outputs. */
typedef enum fmcw_dtype {
  FMCW_C64 = 0,             /* complex float32, 8 B per sample                 */
  FMCW_C32H = 1             /* complex float16, 4 B per sample (storage only;
                               all arithmetic is float32).  fp16 OUTPUTS hold
                               MATLAB's values divided by the FFT sizes applied
                               so far (exact powers of two, to stay inside the
                               fp16 range): range cube X/nr, RD map D/(nr*nd) */
} fmcw_dtype;

/* Algorithm parameters: radar_processing.m:117-154 (a1 in SURVEY.md 8a). */
typedef struct fmcw_params {
  int32_t nts;                  /* NTS, ADC samples per chirp            :109 */
  int32_t pn;                   /* PN, chirps per frame                  :112 */
  int32_t nr;                   /* range_fft_size (power of 2, 16..2048) :118 */
  int32_t nd;                   /* Doppler_fft_size (power of 2, 2..1024):119 */
  int32_t max_targets;          /* max_num_targets (1..8)                :129 */
  int32_t doppler_fallback_idx; /* 1-based; the literal 9 of :234 in parity
                                   mode, nd/2+1 in throughput mode            */
  float if_scale;               /* IF_scale                          :121/136 */
  float range_thr;              /* range_threshold                       :123 */
  float doppler_thr;            /* Doppler_threshold                     :124 */
  float min_d;                  /* min_distance [m]                      :126 */
  float max_d;                  /* max_distance [m]                      :127 */
  float dist_per_bin;           /* dist_per_bin [m]                      :147 */
} fmcw_params;

typedef struct fmcw_ctx fmcw_ctx;

int32_t     fmcw_abi_version(void);
const char* fmcw_last_error(void);
int         fmcw_device_count(int32_t* n);
/* The devices a caller that names none should use ("device choice
 * comes from an env var or an explicit id"): the comma-separated ids of the
 * environment variable FMCW_DEVICES (e.g. "0,1,2,3"), or every visible device
 * when it is unset, empty or "all".  Writes up to cap ids to ids[], their count
 * to *n.  FMCW_E_ARG for a malformed list or an id that is not present.  The
 * MEX gateway's fmcw_mex('init') (no ids) and matlab/radar_processing.m use it,
 * so one MATLAB call drives every GPU of the node (radar_processing_with_azure.m:50
 * -> radar_processing.m:197). */
int         fmcw_default_devices(int32_t cap, int32_t* ids, int32_t* n);

/* Bind a context to n_devices HIP devices (device_ids[n_devices], or NULL for
 * 0 .. n_devices-1), each with its own streams, scratch and tables, all in the
 * calling process.  With several distinct devices the context also holds one
 * RCCL communicator per device (ncclCommInitAll; RCCL is loaded
 * at run time).  The host-pointer calls (fmcw_process, fmcw_range_fft,
 * fmcw_stft) then split their work over the devices -- contiguous frame
 * shards, each written back in place (the range_speed concatenation of
 * :386-389 is the frame order), and contiguous spectrogram segment shards with
 * the global max(P) of :282-283 taken by an RCCL all_reduce(max) -- so one MEX
 * call from the serial loop's caller (radar_processing_with_azure.m:50 ->
 * radar_processing.m:197) drives every GPU.  The device-pointer calls act on
 * the first device (one process per GPU for torch.distributed drivers).
 * Results do not depend on the number of devices (bit-identical shards). */
int fmcw_ctx_create(int32_t n_devices, const int32_t* device_ids, fmcw_ctx** out);
int fmcw_ctx_destroy(fmcw_ctx* ctx);
/* n_devices, device_ids[n_devices] (may be NULL), rccl_comms: 1 if RCCL communicators exist. */
int fmcw_ctx_devices(fmcw_ctx* ctx, int32_t* n_devices, int32_t* device_ids, int32_t* rccl_comms);

/* Window taps and calibration (radar_processing.m:138, :139, :174):
 *   range_win   [nts]        = 2*blackman(NTS)
 *   doppler_win [pn]         = 2*chebwin(PN)
 *   calib       [nts] c64    = calib_rx1
 * Also builds the twiddle tables for nr and nd.  Must precede processing and
 * be repeated whenever nts/pn/nr/nd change.  Synchronous with the device: work
 * queued before it (on any stream) finishes with the old taps, and calls after it
 * (on any stream) see the new ones. */
int fmcw_set_taps(fmcw_ctx* ctx, const fmcw_params* p, const float* range_win,
                  const float* doppler_win, const float* calib);

/* ---------------------------------------------------------------------------
 * Host-pointer API (MEX / ctypes).  Data are staged through device memory
 * owned by the context; the call returns when the outputs are on the host.
 * ------------------------------------------------------------------------- */

/* Per-frame stages a5-a11 + a13 of SURVEY 8a over F frames
 * (radar_processing.m:199-239, :257-259, :265).
 *   iq              [F][pn][nts]  in_dtype   cat(3, frame.Chirp(:,:,1))
 *   range_profile   [F][nr]  f32   range_tx1rx1_max_abs (:265, Nr x F)
 *   tgt_count       [F]      i32   num_of_targets (:213)
 *   tgt_range_idx   [F][M]   i32   tgt_range_idx, 1-based, 0 where j >= count
 *   tgt_range_mag   [F][M]   f32   tgt_range_mag
 *   tgt_doppler_idx [F][M]   i32   tgt_doppler_idx (:227-239), 1-based
 *   slow_mag        [F][pn]  f32   abs(range_tx1rx1_complete(ridx(1),:,fr)),
 *                                  the slow-time samples appended at :259 and
 *                                  made real at :270; zero where count == 0
 *   range_cube      [F][pn][nr] c64 or NULL   range_tx1rx1_complete (:207)
 *   rd_map          [F][nr][nd] c64 or NULL   range_Doppler_tx1rx1 (:219) for
 *                                  EVERY range row (the reference fills only the
 *                                  target rows; each row is the same row op).
 *                                  Note the per-frame transpose vs MATLAB's Nr x Nd.
 *   probe_column    1-based linear column of the Nr x (pn*F) view of the cube
 *                   (:410-411 uses 100), 0 = none
 *   probe_mag       [nr] f32 or NULL  abs(range_tx1rx1_complete(:, probe_column))
 */
int fmcw_process(fmcw_ctx* ctx, const fmcw_params* p, const void* iq, int32_t in_dtype,
                 int64_t F, float* range_profile, int32_t* tgt_count, int32_t* tgt_range_idx,
                 float* tgt_range_mag, int32_t* tgt_doppler_idx, float* slow_mag,
                 float* range_cube, float* rd_map, int64_t probe_column, float* probe_mag);

/* Range stage only (config 2): :203-205, :207, :210 -> cube + profile. */
int fmcw_range_fft(fmcw_ctx* ctx, const fmcw_params* p, const void* iq, int32_t in_dtype,
                   int64_t F, float* range_cube, float* range_profile);

/* STFT + dB + optional log-frequency resampling (:270-299).
 *   x [L] f32        iq_data = abs(slow_time_signal_all_frames)
 *   win [wlen]       kaiser(20,3) (:276) in parity mode
 *   noverlap         19 (:179); hop = wlen - noverlap
 *   nfft             0 = the reference rule 2^nextpow2(L) (:273)
 *   fs               1/PRT
 *   n_log_bins       1024 (:293) -> intensity is interp1 onto logspace bins;
 *                    0 -> intensity is 20log10(P/max P) on the nfft/2+1 bins
 *   out: T [nseg], freq [n_log_bins or nfft/2+1], intensity [nseg][nbins_out]
 *        (MATLAB's nbins_out x nseg matrix), nseg = fix((L-noverlap)/hop)
 *   Query sizes first with fmcw_stft_sizes.  Fails with FMCW_E_DATA when
 *   nseg < 1 (MATLAB's spectrogram raises on such input). */
int fmcw_stft_sizes(int64_t L, int32_t wlen, int32_t noverlap, int32_t nfft,
                    int32_t n_log_bins, int64_t* nseg, int32_t* nfft_used, int32_t* nbins_out);
int fmcw_stft(fmcw_ctx* ctx, const float* x, int64_t L, const float* win, int32_t wlen,
              int32_t noverlap, int32_t nfft, double fs, int32_t n_log_bins, float* T,
              float* freq, float* intensity);

/* ---------------------------------------------------------------------------
 * Device-pointer API (benches, multi-GPU driver).  All pointers are device
 * pointers on the context's device; `stream` is a hipStream_t (NULL = the
 * context's own stream).  Calls are asynchronous on that stream.
 * ------------------------------------------------------------------------- */
int fmcw_process_device(fmcw_ctx* ctx, const fmcw_params* p, const void* d_iq, int32_t in_dtype,
                        int64_t F, float* d_range_profile, int32_t* d_tgt_count,
                        int32_t* d_tgt_range_idx, float* d_tgt_range_mag,
                        int32_t* d_tgt_doppler_idx, float* d_slow_mag, void* d_range_cube,
                        void* d_rd_map, int32_t out_dtype, int64_t probe_column,
                        float* d_probe_mag, void* stream);

/* Placement (a performance note, not a requirement): the range kernel reads d_iq and writes
 * d_range_cube at the same time, and on MI355X its time depends on where the two streams sit
 * relative to each other in HBM -- 748-860 us per 4096 frames of 128 x 512 for 18 byte gaps between
 * the end of d_iq and the start of d_range_cube (profiles/r06_k1_place.txt).  Carving both from one
 * allocation with the cube 64 KiB (or 4-16 MiB) past the input's end measured at the fast end. */
int fmcw_range_fft_device(fmcw_ctx* ctx, const fmcw_params* p, const void* d_iq, int32_t in_dtype,
                          int64_t F, void* d_range_cube, int32_t out_dtype, float* d_range_profile,
                          void* stream);

/* fmcw_process_device (no range cube, no probe column) followed by the start of the slow-time
 * leg, in one call (ABI 4): the compaction of :257-260 -- d_frame_list / *d_len exactly as
 * fmcw_compact_device(d_tgt_count, F, pn, ...) -- and *d_pmax = 0 (when d_pmax != NULL) for the
 * STFT passes that follow (fmcw_stft_power_device's running max(P), :276 / :282).  On the
 * single-pass schedule both run inside the detection kernel (its last workgroup), so the leg
 * costs no launches of its own (the reference's :257-260 append and the spectrogram call
 * `radar_processing.m:259`, `:276`). */
int fmcw_process_slow_device(fmcw_ctx* ctx, const fmcw_params* p, const void* d_iq, int32_t in_dtype,
                             int64_t F, float* d_range_profile, int32_t* d_tgt_count,
                             int32_t* d_tgt_range_idx, float* d_tgt_range_mag,
                             int32_t* d_tgt_doppler_idx, float* d_slow_mag, void* d_rd_map,
                             int32_t out_dtype, int32_t* d_frame_list, int64_t* d_len, float* d_pmax,
                             void* stream);

/* Slow-time compaction (:257-260): exclusive scan of (tgt_count>0) over F
 * frames.  Writes d_frame_list[i] = i-th frame with a target, *d_len = L
 * (= pn * #frames with a target, int64, device). */
int fmcw_compact_device(fmcw_ctx* ctx, const int32_t* d_tgt_count, int64_t F, int32_t pn,
                        int32_t* d_frame_list, int64_t* d_len, void* stream);

/* Power spectrogram of the compacted |slow| signal, segments [0, nseg) with
 * nseg = fix((L + H - noverlap)/hop) clipped to max_seg (all on device):
 * sample q < L is slow_mag[frame_list[q/pn]][q%pn], q >= L is d_halo[q-L].
 * H = *d_halo_len when d_halo_len != NULL (device int64, <= n_halo), else
 * n_halo.  The halo carries the first samples of the following shards in the
 * multi-GPU split of the concatenated slow-time signal (:259).
 *   d_P [max_seg][nfft/2+1]  MATLAB P (psd scaling, one-sided); NULL: only max(P) is formed
 *   d_pmax                   running max of P (float, atomically raised;
 *                            initialise to 0 before the first call)
 *   d_nseg                   int64 device: segments actually written */
int fmcw_stft_power_device(fmcw_ctx* ctx, const float* d_slow_mag, const int32_t* d_frame_list,
                           const int64_t* d_len, int32_t pn, const float* d_halo, int32_t n_halo,
                           const int64_t* d_halo_len, const float* d_win, int32_t wlen, int32_t noverlap, int32_t nfft,
                           double fs, int64_t max_seg, float* d_P, float* d_pmax,
                           int64_t* d_nseg, void* stream);

/* psd = 20*log10(P / pmax) (:282-283), optionally resampled onto n_log_bins
 * logspace bins (:293-299).  d_out [max_seg][n_log_bins or nfft/2+1]; may
 * alias d_P when n_log_bins == 0. */
int fmcw_stft_db_device(fmcw_ctx* ctx, const float* d_P, const int64_t* d_nseg, int64_t max_seg,
                        int32_t nfft, double fs, const float* d_pmax, int32_t n_log_bins,
                        float* d_out, void* stream);

/* Second pass of the two-pass STFT without a stored P (20-tap window, hop <= 4,
 * linear bins only): recomputes P of every segment and writes
 * psd = 20*log10(P / max) (:283) to d_out [max_seg][nfft/2+1].  With
 * fmcw_stft_power_device(..., d_P = NULL, ...) as the first pass (max(P) only)
 * the P map is never written to or read back from HBM.  Same inputs as the power
 * call; d_pmax is the (all-reduced) max. */
int fmcw_stft_db_direct_device(fmcw_ctx* ctx, const float* d_slow, const int32_t* d_list, const int64_t* d_len,
                               int32_t pn, const float* d_halo, int32_t n_halo, const int64_t* d_halo_len,
                               const float* d_win, int32_t wlen, int32_t noverlap, int32_t nfft, double fs,
                               int64_t max_seg, const float* d_pmax, float* d_out, void* stream);

/* Synthetic IQ frames of SURVEY 8d (seed 0xF3C0 ^ global frame index),
 * generated in place in HBM: d_iq [F][pn][nts] of dtype.  Bench input only. */
int fmcw_synth_device(fmcw_ctx* ctx, const fmcw_params* p, int64_t frame0, int64_t F,
                      void* d_iq, int32_t dtype, void* stream);

/* Per-stage device timing with HIP events on the launching streams.
 * enable: 0 off; 1 = the range+Doppler span of each fmcw_process_device call
 * (stage 7: event before the first range launch .. event after the last
 * Doppler launch; the chunks run as a 3-stream software pipeline) and one pair
 * per STFT-side launch (stages 3-6); 2 = additionally one pair per K1/K2/K3; 3 = only the
 * dominant kernel's launches (stage 8 k_rdx, stage 6 range-only K1), the cheapest form for a
 * timed run (each event pair costs the stream a few microseconds).
 * stage: 0 range, 1 doppler, 2 detect, 3 compact, 4 stft_power, 5 stft_db,
 *        6 range_only, 7 range+Doppler span, 8 k_rdx (single-pass schedule,
 *        level 2), 9 render (spectrogram.png).  fmcw_timing_read synchronises. */
int fmcw_timing_enable(fmcw_ctx* ctx, int32_t enable);
int fmcw_timing_read(fmcw_ctx* ctx, int32_t stage, double* total_ms, int64_t* launches);
int fmcw_timing_reset(fmcw_ctx* ctx);

/* Frames per range/Doppler chunk of the 3-stream pipeline (the range cube of
 * one chunk is its only intermediate; default 256 MiB of cube per chunk).
 * 0 restores the default. */
int fmcw_set_chunk_frames(fmcw_ctx* ctx, int64_t frames);

/* Schedule of fmcw_process_device / fmcw_process (the two agree to fp32 rounding):
 *  FMCW_PIPE_AUTO    the single-pass XCD-team schedule where it applies (geometry
 *                    and device below, no range cube requested), else the streams
 *                    schedule;
 *  FMCW_PIPE_STREAMS K1 | K2 | K3 kernels as a 3-stream chunk pipeline, the
 *                    range cube of each chunk round-trips through HBM;
 *  FMCW_PIPE_XCD     the XCD-team single pass (kernels_xcd.hip): the 32 CUs of each
 *                    XCD share a frame (range FFT split by chirps, Doppler FFT by
 *                    range-bin groups, the cube handed over in the XCD's L2), so
 *                    every input byte is read once and the range cube never goes
 *                    to HBM.  Needs nr 1024, pn == nd == 256, even nts <= nr, the RD
 *                    map (if any) in the IQ dtype (complex64 or fp16 storage), no
 *                    range cube (else E_ARG).  One persistent workgroup per CU: needs
 *                    32 CUs per XCD and a grid of one workgroup per CU dealt 32 per
 *                    XCD -- any XCD count, so the SPX mode (8 XCDs) and the DPX /
 *                    QPX / CPX partition modes (4 / 2 / 1 XCDs per device) alike;
 *                    checked once per context by a census, else E_ARG.  A hand-off
 *                    that does not complete within ~1 s is reported by
 *                    fmcw_synchronize (and the host-pointer calls) as FMCW_E_HIP.
 *  FMCW_PIPE_ONEPASS the same as FMCW_PIPE_XCD (ABI 2's 8-tile single pass, which
 *                    re-read every frame from L2 8 times, is retired).
 * (Value 2 is retired: the persistent "fused" schedule of ABI 1, slower than both.) */
enum { FMCW_PIPE_AUTO = 0, FMCW_PIPE_STREAMS = 1, FMCW_PIPE_ONEPASS = 3, FMCW_PIPE_XCD = 4 };
int fmcw_set_pipeline(fmcw_ctx* ctx, int32_t mode);

int fmcw_synchronize(fmcw_ctx* ctx);

/* Measurement helpers of the bench line (ABI 4; no part of the reference's path).
 * fmcw_rdx_clock: the effective shader clock (MHz) of the context's last k_rdx launch, from the
 *   shader-clock and 100 MHz stamps one member takes at its start and its end (*us: that span);
 *   0 when no launch ran.  Synchronises the device.
 * fmcw_copy_device: a 16-byte nontemporal copy of `bytes` (a multiple of 16, 16-byte aligned
 *   pointers), asynchronous on `stream`: the HBM copy ceiling of k_rdx's bytes (bench.py). */
int fmcw_rdx_clock(fmcw_ctx* ctx, double* mhz, double* us);
int fmcw_copy_device(fmcw_ctx* ctx, const void* d_src, void* d_dst, int64_t bytes, void* stream);

/* ---------------------------------------------------------------------------
 * spectrogram.png, replacing radar_processing.m:331-348:
 *   surf(T, fftshift(F), fftshift(psd,1), 'EdgeColor','none'); view(0,90);
 *   axis tight; ylim([0 150]); clim([-40 0]); axis off; colormap(jet);
 *   exportgraphics(fig, 'spectrogram.png', 'Resolution', 600)
 * rendered on the GPU (kernels_render.hip states the rules: the fftshift-ed
 * one-sided axis folds the surface; the depth test of the top view; flat
 * faces coloured by their first vertex through jet(256) on [-40 0] dB) and
 * written as an 8-bit palette PNG.  Default size 2906 x 2038: the default
 * axes box of a 600 x 400 figure (0.775 x 0.815 of it) at 600/96 px per
 * screen pixel, which is what exportgraphics crops to with the axis off.
 * MATLAB graphics cannot run here: the pixels are unpinned against it.
 * ------------------------------------------------------------------------- */
#define FMCW_PNG_FMAX_HZ 150.0
#define FMCW_PNG_CMIN_DB (-40.0)
#define FMCW_PNG_CMAX_DB 0.0
#define FMCW_PNG_DEFAULT_W 2906
#define FMCW_PNG_DEFAULT_H 2038

/* fmcw_stft (:270-299) plus the PNG of :331-348 written to png_path
 * (width/height 0: the defaults above); png_bytes may be NULL. */
int fmcw_stft_png(fmcw_ctx* ctx, const float* x, int64_t L, const float* win, int32_t wlen, int32_t noverlap,
                  int32_t nfft, double fs, int32_t n_log_bins, float* T, float* freq, float* intensity,
                  const char* png_path, int32_t width, int32_t height, int64_t* png_bytes);

/* Device call: palette indices img[height][1 + width] (PNG filter byte 0 first)
 * from Q[nseg][nq + 1] = the one-sided P (:276) of bins 0 .. nq-1 followed by
 * bin nfft/2 (for a full P row of nfft/2 + 1 bins: nq = nfft/2, Q = P), the
 * global max(P) (:282), T(1) = t0, T(2) - T(1) = dt. */
int fmcw_render_spectrogram_device(fmcw_ctx* ctx, const float* d_Q, int32_t nq, const int64_t* d_nseg,
                                   const float* d_pmax, int32_t nfft, double fs, double t0, double dt, int32_t width,
                                   int32_t height, uint8_t* d_img, void* stream);

/* ---------------------------------------------------------------------------
 * Output files: native jsonencode(struct, 'PrettyPrint', true).
 * Replaces the jsonencode + fprintf of radar_processing.m:313-321
 * (spectrogram_data.json), :362-369 (<file>_range_fft_data.json), :390-398
 * (<file>_range_speed_data.json), :424-431 (<file>_fft_data.json) and :590-593
 * (the 'yes' branch's batch JSONs).  One field per struct member, in order:
 *   FMCW_JSON_STRING  data = NUL-terminated char*, rows/cols ignored
 *   FMCW_JSON_F32/F64/I32  a rows x cols MATLAB array; element (i, j) at
 *     data[i * row_stride + j * col_stride] (so a [nseg][nbins] device-layout
 *     intensity is written as MATLAB's nbins x nseg without a transpose).
 *   FMCW_JSON_BOOL    the same with uint8 elements (0 / non-0): a MATLAB logical
 *     array, written as true / false.
 * jsonencode's shape rules: 1x1 -> number, 1xN / Nx1 -> flat array, MxN ->
 * array of M rows, empty -> []; NaN/Inf -> null; numbers as "%.15g" (integers
 * without a fraction).  threads <= 0: up to 16 host threads format in parallel.
 * No device work; no context needed.
 * ------------------------------------------------------------------------- */
enum { FMCW_JSON_STRING = 0, FMCW_JSON_F32 = 1, FMCW_JSON_F64 = 2, FMCW_JSON_I32 = 3, FMCW_JSON_BOOL = 4 };
typedef struct {
  const char* name;
  int32_t kind;
  const void* data;
  int64_t rows, cols, row_stride, col_stride;
} fmcw_json_field;
int fmcw_json_write(const char* path, const fmcw_json_field* fields, int32_t n_fields, int32_t pretty,
                    int32_t threads, int64_t* bytes_written);

#ifdef __cplusplus
}
#endif
#endif /* FMCW_H_ */
