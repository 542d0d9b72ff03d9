// fmcw_internal.h -- launch wrappers shared by kernels_*.hip and fmcw_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmcw {

// Flags of the events that only order work on one device (stream joins, per-stream scratch
// reuse, k_rdx's launch chain, the timing pairs read after a device synchronise): no system-scope
// release when they are recorded.  A default event's release makes the queue write the L2s back
// before the next packet runs; behind k_rdx (whose hand-off slots leave dirty lines in every XCD's
// L2) that showed as 6-19 us of idle GPU after every recorded event (profiles/r06_gaps.txt).
// The host-pointer path's copy events keep the default (the host reads what they guard).
// -DFMCW_EV_SYSFENCE restores the default flags (A/B).
#ifndef FMCW_EV_SYSFENCE
constexpr unsigned kEvDevice = hipEventDisableSystemFence;
#else
constexpr unsigned kEvDevice = 0;
#endif

struct RangeArgs {
  const void* iq;          // [nchirps][S] complex, dtype in_dtype
  int in_dtype;            // FMCW_C64 / FMCW_C32H
  int64_t nchirps;         // chirps in this launch (= frames * C)
  int C, S, NR;
  const float4* calw;      // [S] {cal.re, cal.im, if_scale*w, w}  (w = 2*blackman)
  float2 cal_sum;          // sum_n cal[n] over all S samples
  float if_scale;
  const float2* tw;        // [NR]
  void* cube;              // [nchirps][NR], dtype cube_dtype
  int cube_dtype;
  float cube_scale;        // stored value = X * cube_scale (1, or 1/NR for fp16)
  float* profile;          // [frames][NR] (max over chirps) or nullptr
  int cpt;                 // chirps per team (divides C when profile != nullptr)
  float* prof_part;        // [frames][parts][NR] per-workgroup maxima when a workgroup holds 1/parts of
  int parts;               // a frame (parts > 1), reduced by launch_profile_reduce; else nullptr / 0
};

struct DopplerArgs {
  const void* cube;        // [frames][C][NR]
  int cube_dtype;
  float cube_unscale;      // 1/cube_scale
  float rd_scale;          // stored value = D * rd_scale (1, or 1/(NR*ND) for fp16)
  int nframes, C, NR, ND;
  const float* wd;         // [C]
  const float2* tw;        // [ND]
  void* rd;                // [frames][NR][ND]
  int rd_dtype;
  float* profile;          // [frames][NR]
};

struct DetectArgs {
  const float* profile;    // [frames][NR]
  const void* rd;          // [frames][NR][ND]
  int rd_dtype;
  const void* cube;        // [frames][C][NR]
  int cube_dtype;
  float cube_unscale, rd_unscale;
  int nframes, NR, ND, C, M;
  float range_thr, doppler_thr, min_d, max_d, dist_per_bin;
  int fallback;
  int32_t* count;          // [frames]
  int32_t* ridx;           // [frames][M]
  float* rmag;             // [frames][M]
  int32_t* didx;           // [frames][M]
  float* slow_mag;         // [frames][C]
  int64_t probe_frame;     // frame within this launch, -1 = none
  int probe_chirp;
  float* probe_mag;        // [NR]
};

// detection constants shared by k_detect and k_detect_1p (frame_ops.h)
struct DetectParams {
  int ND, C, M;
  float range_thr, doppler_thr, min_d, max_d, dist_per_bin;
  int fallback;
  float cube_unscale, rd_unscale;
};

// Single-pass range+Doppler (kernels_xcd.hip, k_rdx): the range cube never
// reaches HBM; k_detect_1p / k_probe (kernels_detect.hip) finish
// the per-frame outputs.
struct OnePassArgs {
  const void* iq;          // [F][C][S] c64, or c32h when h
  int h;                   // fp16 storage (FMCW_C32H): c32h IQ in, c32h RD out holding D / (NR ND)
  float rd_scale;          // 1 / (NR ND) when h, else 1
  int64_t F;
  int C, S;                // NR = 1024, ND = C (kernel template)
  const float4* calw;      // [S] {cal.re, cal.im, IF_scale*w, w}
  const float2* tw_nr;     // [NR]
  const float2* tw_nd;     // [ND]
  const float* wd;         // [C]
  void* rd;                // [F][NR][ND] c64 (c32h when h), or nullptr (then only the row peaks are kept)
  float* profile;          // [F][NR]
  int2* rowpk;             // [F][NR] {float bits of max_d |D[r,d]|, first argmax d (fftshift-ed, 0-based)}; only when rd is nullptr
  int32_t* cand_idx;       // [F][XCD_TILES][XCD_CAND] 0-based bin or -1
  float* cand_rows;        // [F][XCD_TILES][XCD_CAND][C] |X[bin, k]|^2
  float range_thr, min_d, max_d, dist_per_bin;
  int force_fix;           // test knob (FMCW_ONEPASS_FORCE_FIX=1): keep no candidates, so every
                           // slow-time row goes through k_slow_fix
  unsigned long long* dbg; // diagnostic builds only (-DXK_STAMPS): [blocks][8] s_memrealtime stamps
  unsigned long long* clk; // or nullptr: {shader clock, 100 MHz clock} at the start and the end of team 0's
                           // member 0 (k_rdx's effective clock, fmcw_rdx_clock)
  // XCD-team schedule (k_rdx) only:
  float2* xcube;           // [8 XCDs][slots][XCD_TILES groups][C][32] range-cube hand-off slots
  unsigned* xctr;          // [8 XCDs][2: ready, (unused)][XCD_MAX_SLOTS][32] + [8][32] tickets + the abort word:
                           // one 128-byte line per counter, XCD_CTR_WORDS in all (zero when a launch starts)
  unsigned* xclr;          // the context's other counter set (launches alternate between two): k_rdx's block 0
                           // zeroes its first XCD_IDLE words for the next launch, which saves a memset packet per
                           // launch; nullptr: launch_xcd zeroes xctr before the launch (FMCW_XCD_MEMSET=1)
  unsigned* xerr;          // sticky, reported by fmcw_synchronize: bit 0 a hand-off wait timed out, bit 1 an XCD
                           // got more than 32 blocks (the launch's own abort word lets its grid drain; a later
                           // launch starts with a clear one)
  int slots;               // hand-off slots allocated per XCD (XCD_MAX_SLOTS; k_rdx uses 2 of them)
  unsigned s16mask;        // fp16 storage only: bit b set = range bins 128 b .. 128 b + 127 (groups 4 b .. 4 b + 3)
                           // are handed over as c32h (X / NR): no bin of the block can become a detection or
                           // slow-time candidate (host_s16mask in fmcw_api.cpp); 0 = every group c64
  int nteams;              // XCDs of the device (teams of 32 CUs): 8 in SPX mode, 1-4 in the partition modes
  int8_t xcc_team[16];     // HW_REG_XCC_ID -> team index 0..nteams-1, -1 for an XCC not in the device
  const float2* xtab;      // XT_* sections (host, float64, lane order)
  float2 cal_sum;          // sum_{n < S} cal[n]
};

// XCD-team schedule (kernels_xcd.hip): the 32 CUs of an XCD share each of its
// frames, split by chirps for the range FFT and by range-bin groups for the
// Doppler FFT; the range cube moves between them through the XCD's L2.
constexpr int XCD_TILES = 32;        // range-bin groups per frame (one per team member)
constexpr int XCD_CAND = 2;          // slow-time candidate rows kept per group
constexpr int XCD_MAX_SLOTS = 4;
constexpr int XCD_GRID = 256;        // at most 8 XCDs x 32 CUs, one persistent workgroup per CU
constexpr int XCD_TICKETS = 8 * 2 * 32 * XCD_MAX_SLOTS;   // xctr offset of the 8 per-XCD member tickets (128-byte lines)
constexpr int XCD_ABORT = XCD_TICKETS + 8 * 32;           // xctr offset of the launch's abort word (own line)
constexpr int XCD_IDLE = XCD_ABORT + 32;                  // xctr offset of [256 CUs][32] words the non-publishing
                                                          // waves add 0 to (kernels_xcd.hip, publish)
constexpr int XCD_CTR_WORDS = XCD_IDLE + 256 * 32;
// table sections (float2, [..][64 lanes])
constexpr int XT_R1 = 0;             // [14]: W1024^((2l + e) k1), index 2 (k1 - 1) + e
constexpr int XT_R2 = 14 * 64;       // [15]: W128^((l & 7) s1), s1 = 1..15
constexpr int XT_D1 = 29 * 64;       // [15]: W256^((l & 15) d0), d0 = 1..15
// the half-frame hand-off build (-DXK_HALF, kernels_xcd.hip): a wave pair per chirp, each wave a
// 512-point FFT of the even (odd) samples, combined across the pair
constexpr int XT_H1 = 44 * 64;       // [7]: W512^(l k1), k1 = 1..7
constexpr int XT_H2 = 51 * 64;       // [7]: W64^((l & 7) s1), s1 = 1..7
constexpr int XT_HC = 58 * 64;       // [8]: W1024^(l + 64 s2), s2 = 0..7
constexpr int XT_SIZE = 66 * 64;
#ifndef XK_HALF
// group g, position p (0..31) <-> range bin: r = k1 + 16 h + 8 e + 128 s2 with
// k1 = (p >> 3) + 4 (g & 1), h = p & 7, e = (g >> 1) & 1, s2 = g >> 2
__host__ __device__ inline int xcd_bin(int g, int p) {
  return (p >> 3) + 4 * (g & 1) + 8 * ((g >> 1) & 1) + 16 * (p & 7) + 128 * (g >> 2);
}
__host__ __device__ inline int xcd_group(int r) { return ((r >> 2) & 1) | (((r >> 3) & 1) << 1) | ((r >> 7) << 2); }
__host__ __device__ inline int xcd_pos(int r) { return ((r & 3) << 3) | ((r >> 4) & 7); }
#else
// half-frame build: group g holds bins 32 g .. 32 g + 31 in order
__host__ __device__ inline int xcd_bin(int g, int p) { return 32 * g + p; }
__host__ __device__ inline int xcd_group(int r) { return r >> 5; }
__host__ __device__ inline int xcd_pos(int r) { return r & 31; }
#endif

struct Detect1pArgs {
  const float* profile;    // [F][NR]
  const int2* rowpk;       // [F][NR] (used when rd is nullptr)
  const void* rd;          // [F][NR][ND] c64 (c32h when rd_h, holding D * det.rd_unscale^-1) or nullptr
  int ND, rd_h;
  const int32_t* cand_idx; // [F][tiles][ncand]
  const float* cand_rows;  // [F][tiles][ncand][C] |X|^2
  int tiles, ncand;        // XCD_TILES (tile = xcd_group) / XCD_CAND
  int nframes, NR, C, M;
  DetectParams det;
  int32_t* count;
  int32_t* ridx;
  float* rmag;
  int32_t* didx;
  float* slow_mag;         // [F][C]
  // the rare target row that was not a group candidate: its slow-time row (:257-259) recomputed
  // by the frame's own wave, a direct DFT of every chirp at that bin (was the k_slow_fix launch)
  const void* iq;          // [F][C][S] c64, or c32h when h
  int h, S;
  const float4* calw;
  const float2* tw_nr;
  // fused compaction (:257-260, as k_compact), when list != nullptr: every workgroup stores its
  // counts write-through and adds 1 to *done; the last one scans count_all[0..F_all) (the call's
  // earlier chunks included), writes list / *len, zeroes *pmax_reset (if set: the running max(P)
  // of the STFT passes that follow, :276 / :282) and resets *done for the next launch
  int32_t* done;           // device counters, 0 before the first launch: 8 shards + the top, 32 words apart
  const int32_t* count_all;
  int64_t F_all;
  int pn;
  int32_t* list;
  int64_t* len;
  float* pmax_reset;
};

hipError_t launch_detect_1p(const Detect1pArgs& a, hipStream_t s);
hipError_t launch_xcd(const OnePassArgs& a, hipStream_t s);
// The device's XCD teams: *nteams = its XCDs (0 when the XCD-team schedule cannot run: a CU count
// that is not 32 per XCD, or a grid of one workgroup per CU not dealt 32 per XCD), xcc_team[16]
// the team index of each HW_REG_XCC_ID.
hipError_t xcd_census(int* nteams, int8_t* xcc_team);

struct ProbeArgs {          // fft_data column (:410-411) for the single-pass schedule
  const void* iq;          // [F][C][S] of the launch, c64 or c32h (h)
  int h;
  int64_t frame;
  int chirp, C, S, NR;
  const float4* calw;
  const float2* tw_nr;
  float* probe_mag;        // [NR]
};
hipError_t launch_probe(const ProbeArgs& a, hipStream_t s);
bool onepass_supported(int nts, int pn, int nr, int nd);

struct StftArgs {
  const float* slow_mag;   // [*][pn]
  const int32_t* frame_list;
  const int64_t* len;      // device scalar L
  int pn;
  const float* halo;
  int n_halo;
  const int64_t* halo_len;  // device, or nullptr -> n_halo
  const float* win;        // device [wlen]
  int wlen, hop, nfft;
  float inv_fs;            // 1/fs; the 'psd' scale 1/(fs*sum(win^2)) is formed in-kernel
  int64_t max_seg;
  float* P;                // [max_seg][nfft/2+1]
  float* pmax;
  int64_t* nseg_out;
  const int32_t* bins;     // k_stft20 mode 3 / 4: the ascending bin list of the columns (device), else nullptr
  int ncol;                // k_stft20 mode 3 / 4: columns in `bins`
  const int32_t* tiles;    // k_stft_mfma mode 1: the 256-segment tiles to cover (device), nullptr = all
  int ntiles;
  int table_form;          // 1: the table-based k_stft_mfma / k_stft20 even at nfft 64 (the host call's
                           // max(P) pass, so that it forms P exactly as its listed-bins pass does)
};

// 20-tap fast path (kernels_stft.hip k_stft20): W table [nfft/2+1][20] from the window,
// then mode 0 P + max, 1 max only, 2 dB written to dst (given max), 3 P of the bins
// a.bins[0..a.ncol) only, written to dst as [seg][ncol], 4 each segment's max of P over the bins
// a.bins written to dst[seg] (matrix-core form only)
bool stft_fast_path(int wlen, int hop);
// the nfft-64 matrix-core kernel (k_stft64m) serves this nfft (not disabled by FMCW_STFT_MFMA=0);
// it verifies a cached W table against the call's window
bool stft64_form(int nfft);
hipError_t launch_stft_table(const float* win, int nfft, float2* tab, hipStream_t s);
// dst_cap: floats available at dst (mode 0: at a.P), tab_cap: float2 entries of tab; a launch
// whose writes would not fit returns hipErrorInvalidValue before anything is enqueued
hipError_t launch_stft20(const StftArgs& a, const float2* tab, int mode, float* dst, hipStream_t s, int64_t dst_cap,
                         int64_t tab_cap);


struct StftDbArgs {
  const float* P;
  const int64_t* nseg;
  int64_t max_seg;
  int nbins_in;            // nfft/2+1
  const float* pmax;
  int nlog;                // 0 = no resampling
  const int32_t* lidx;     // [nlog]
  const float* lw;         // [nlog]
  float* out;
};

struct SynthArgs {
  void* iq;
  int dtype;
  int64_t frame0, nframes;
  int C, S, NR, ND;
  float dist_per_bin;
  const float2* cal;
};

hipError_t launch_range(const RangeArgs& a, hipStream_t s);
// profile[f][b] = max over parts of prof_part[f][part][b] (K1's per-workgroup maxima)
hipError_t launch_profile_reduce(const float* part, int parts, int64_t frames, int nr, float* profile, hipStream_t s);
hipError_t launch_doppler(const DopplerArgs& a, hipStream_t s);
hipError_t launch_detect(const DetectArgs& a, hipStream_t s);
hipError_t launch_compact(const int32_t* count, int64_t F, int pn, int32_t* frame_list, int64_t* len,
                          hipStream_t s);
hipError_t launch_stft_power(const StftArgs& a, hipStream_t s);
hipError_t launch_stft_db(const StftDbArgs& a, hipStream_t s);
hipError_t launch_synth(const SynthArgs& a, hipStream_t s);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, int64_t n, hipStream_t s);
// kernels_util.hip: the bench's HBM copy ceiling (16-byte nontemporal loads and stores)
hipError_t launch_copy16(const void* src, void* dst, int64_t bytes, hipStream_t s);


bool range_size_supported(int nr);
bool doppler_size_supported(int nd);

// spectrogram.png of :331-348 (kernels_render.hip)
struct RenderArgs {
  const float* Q;          // [nseg][nq + 1]: P of bins 0 .. nq-1, then the Nyquist bin nb-1
  int nq;
  const int64_t* nseg;     // device scalar
  const float* pmax;       // device scalar: max(P(:)) (:282-283)
  int nb, nfft, seam;      // one-sided bins, FFT size, the bin m whose face (m, m+1) fftshift drops
  double fs, t0, dt;       // sample rate, T(1), T(2) - T(1)
  double fmax, cmin, cmax; // ylim([0 fmax]), clim([cmin cmax])
  int W, H;                // pixels
  uint8_t* img;            // [H][1 + W] palette indices, PNG filter byte first
};
hipError_t launch_render(const RenderArgs& a, hipStream_t s);

}  // namespace fmcw

#include "host_io.h"   // png_write_indexed, jet_palette, set_error
