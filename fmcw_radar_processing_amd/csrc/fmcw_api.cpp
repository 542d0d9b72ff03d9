// fmcw_api.cpp -- libfmcw C-ABI (include/fmcw.h) on top of the gfx950 kernels.
//
// Host responsibilities kept here, mirroring what radar_processing.m does
// around the loop: argument validation (MATLAB would raise), twiddle tables,
// scratch management for the per-chunk range cube, the chunked launch
// sequence K1 -> K2 -> K3, the STFT size rules of :273/:276 and the
// logspace/interp1 bin table of :293-299.
#include "../../include/fmcw.h"
#include "fmcw_internal.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(FMCW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define CHK(expr)            \
  do {                       \
    int r_ = (expr);         \
    if (r_ != FMCW_OK) return r_; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  int ensure(size_t bytes) {
    if (bytes <= n && p) return FMCW_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      return fail(FMCW_E_OOM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
    }
    n = bytes;
    return FMCW_OK;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
};

// Offsets of several arrays packed into one buffer (256-byte aligned).
struct Arena {
  size_t off = 0;
  size_t add(size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  }
};

// Page-locked host staging buffer (DMA source / target of the host-pointer calls).
struct PinBuf {
  void* p = nullptr;
  size_t n = 0;
  int ensure(size_t bytes) {
    if (bytes <= n && p) return FMCW_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    if (bytes == 0) bytes = 16;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return fail(FMCW_E_OOM, "hipHostMalloc of " + std::to_string(bytes) + " bytes failed");
    }
    n = bytes;
    return FMCW_OK;
  }
  char* at(size_t off) const { return static_cast<char*>(p) + off; }
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// Host memcpy between the caller's (pageable) arrays and the pinned slots,
// split over a few threads: one core copies ~10 GB/s, PCIe Gen5 x16 takes ~50.
void par_memcpy(void* dst, const void* src, size_t n) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned T = n >= (8u << 20) ? std::min(8u, hw) : 1u;
  if (T == 1) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t per = ((n + T - 1) / T + 4095) & ~(size_t)4095;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t) {
    const size_t o = (size_t)t * per;
    if (o >= n) break;
    th.emplace_back([=] { std::memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, std::min(per, n - o)); });
  }
  for (auto& x : th) x.join();
}

size_t esize(int dtype) { return dtype == FMCW_C32H ? 4 : 8; }

// RCCL, resolved at run time: a single-device context never needs it, and a
// process that already holds an RCCL (torch's) shares that copy.
struct Rccl {
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (h) break;
    }
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.comm_init_all = reinterpret_cast<decltype(x.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(h, "ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(h, "ncclGroupEnd"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.comm_init_all && x.comm_destroy && x.all_reduce && x.group_start && x.group_end && x.error_string;
    return x;
  }();
  return r;
}

#define NCCLCHK(expr)                                                                     \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess) return fail(FMCW_E_HIP, std::string(#expr) + ": " + rccl().error_string(r_)); \
  } while (0)

// contiguous shard [f0, f0 + n) of `total` items for member g of `world` (dist.py shard_range)
void shard(int64_t total, int g, int world, int64_t& f0, int64_t& n) {
  const int64_t base = total / world, rem = total % world;
  f0 = g * base + std::min<int64_t>(g, rem);
  n = base + (g < rem ? 1 : 0);
}

constexpr int kStages = 10;  // 0..6 per kernel (see fmcw.h), 7 range+Doppler span per call, 8 k_rdx, 9 render

}  // namespace

namespace fmcw {
int set_error(int code, const char* msg) { return fail(code, msg); }
}  // namespace fmcw

struct fmcw_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // software pipeline over chunks: K1 (range) on the caller's stream, K2
  // (Doppler) on sd, K3 (detect) on sx; chunk i's K2 overlaps chunk i+1's K1
  static constexpr int kSlots = 3;
  hipStream_t sd = nullptr, sx = nullptr;
  hipEvent_t ev_k1[kSlots] = {}, ev_k2[kSlots] = {}, ev_k3[kSlots] = {};
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool taps = false;
  fmcw_params p{};
  DevBuf cal, calw, wd, tw_nr, tw_nd;
  std::vector<float> h_wr, h_cal;   // host copies to rebuild calw when IF_scale changes
  float calw_scale = 0.f;
  float2 cal_sum{0.f, 0.f};
  DevBuf scratch_cube, scratch_rd;
  // host-pointer API staging: device slots and page-locked host slots, two of
  // each, so chunk i+1's H2D copy (stream cin) and chunk i-1's D2H copy (cout)
  // run under chunk i's kernels (the caller's data is copied into the pinned
  // slots by host threads meanwhile)
  DevBuf h_iq, h_prof, h_rd;
  PinBuf pin_in, pin_out;
  // small per-call arrays of the host-pointer calls, packed so that they cross PCIe as ONE copy
  // (each pageable copy costs ~20-30 us of latency: six of them were half of a deployed call)
  DevBuf h_small, s_in;
  PinBuf pin_small, pin_sin;
  hipStream_t cin = nullptr, cout = nullptr;
  hipEvent_t ev_h2d[2] = {}, ev_comp[2] = {}, ev_d2h[2] = {};
  DevBuf s_P, s_pmax, s_nseg, s_lidx, s_lw, s_out;
  DevBuf s_cbins, s_segmax, s_tiles;   // fmcw_stft's coarse-to-fine max(P) (stft_coarse_max)
  DevBuf r_q, r_nseg, r_img;                   // spectrogram.png render (device 0)
  // Device scratch kept per stream: device calls on different streams (with different windows,
  // nfft or frame counts) never share one.  At most kPerStream streams per kind (a caller that
  // passes a fresh stream per call does not grow device memory): the least recently used entry is
  // taken over, and the new stream first waits for the event recorded behind the old owner's last
  // readers (done()), so its rewrite cannot overtake them -- the event outlives a destroyed stream.
  struct PerStream {
    struct Entry {
      hipStream_t s = nullptr;
      DevBuf t;
      hipEvent_t done = nullptr;
      uint64_t tick = 0;
      const void* key = nullptr;   // what the contents were built from (STFT tables: the window pointer)
      int64_t key_n = 0;           // and its size (the nfft)
      ~Entry() {
        if (done) (void)hipEventDestroy(done);
      }
    };
    static constexpr size_t kPerStream = 8;
    std::vector<std::unique_ptr<Entry>> es;
    uint64_t tick = 0;
    void* get(hipStream_t st, size_t bytes, int* status, bool* fresh = nullptr) {
      Entry* e = nullptr;
      for (auto& x : es)
        if (x->s == st) e = x.get();
      if (!e && es.size() < kPerStream) {
        es.push_back(std::make_unique<Entry>());
        e = es.back().get();
        e->s = st;
      } else if (!e) {
        e = es[0].get();
        for (auto& x : es)
          if (x->tick < e->tick) e = x.get();
        if (e->done && hipStreamWaitEvent(st, e->done, 0) != hipSuccess) {
          (void)hipGetLastError();
          *status = fail(FMCW_E_HIP, "per-stream scratch: hipStreamWaitEvent failed");
          return nullptr;
        }
        e->s = st;
        e->key = nullptr;
        e->key_n = 0;
      }
      e->tick = ++tick;
      void* before = e->t.p;
      *status = e->t.ensure(bytes);
      if (e->t.p != before) {                  // newly allocated: its contents are undefined
        e->key = nullptr;
        e->key_n = 0;
      }
      if (fresh) *fresh = e->t.p != before;
      last = e;
      return e->t.p;
    }
    Entry* last = nullptr;                     // the entry the last get() returned
    // after the kernels that read stream st's entry are enqueued
    int done(hipStream_t st) {
      for (auto& x : es) {
        if (x->s != st) continue;
        if (!x->done && hipEventCreateWithFlags(&x->done, hipEventDisableTiming | fmcw::kEvDevice) != hipSuccess) {
          (void)hipGetLastError();
          return fail(FMCW_E_HIP, "per-stream scratch: hipEventCreate failed");
        }
        if (hipEventRecord(x->done, st) != hipSuccess) {
          (void)hipGetLastError();
          return fail(FMCW_E_HIP, "per-stream scratch: hipEventRecord failed");
        }
      }
      return FMCW_OK;
    }
  };
  // STFT 20-tap tables W[nfft/2+1][20] + the 20 taps they were built from, one per stream that
  // asked for one
  PerStream s_tabs;
  // a table the caller rewrites (any nfft): the entry no longer holds what a cached nfft-64 key
  // says it holds, so the key is cleared (a later stft_tab64 with the same window rebuilds)
  float2* stft_tab(hipStream_t st, size_t bytes, int* status) {
    float2* t = static_cast<float2*>(s_tabs.get(st, bytes + STFT_TAPS_BYTES, status));
    if (t) {
      s_tabs.last->key = nullptr;
      s_tabs.last->key_n = 0;
    }
    return t;
  }
  static constexpr size_t STFT_TAPS_BYTES = 20 * 4;
  // The device calls at nfft 64 (the bench's config-4 STFT, two passes per step) keep the
  // stream's table while the window pointer and nfft are unchanged: k_stft64m compares the 20
  // taps stored behind the table with the call's window and forms its W entries itself when they
  // differ (a window rewritten in place), so the table is rebuilt once, not every pass.
  // *build: the caller must launch k_stft_table into the returned table.
  float2* stft_tab64(hipStream_t st, const float* d_win, int nfft, bool* build, int* status) {
    float2* t = static_cast<float2*>(s_tabs.get(st, (size_t)(nfft / 2 + 1) * 20 * 8 + STFT_TAPS_BYTES, status));
    if (!t) return nullptr;
    PerStream::Entry* e = s_tabs.last;
    *build = !(e->key == d_win && e->key_n == nfft);
    e->key = d_win;
    e->key_n = nfft;
    return t;
  }
  int stft_tab_done(hipStream_t st) { return s_tabs.done(st); }
  // K1's per-workgroup profile maxima of fmcw_range_fft_device (config 2), one per stream: two
  // range-only calls on different streams of one context do not write over each other's partials
  PerStream k1_part;
  // k_detect_1p's arrival counter of the fused compaction (fmcw_process_slow_device), one per
  // stream; zeroed when allocated, reset by the kernel's last workgroup
  PerStream det_done;
  int64_t chunk_frames = 0;
  int64_t last_coarse_tiles = -1;     // tiles the last coarse-to-fine max(P) evaluated in full (diagnostics)
  int pipe_mode = FMCW_PIPE_AUTO;
  DevBuf op_rowpk, op_cidx, op_crows;           // single-pass schedule scratch (per chunk)
  DevBuf x_cube, x_ctr, x_err, x_tab;          // XCD-team schedule: hand-off slots, counters, sticky error, XT_* table
  DevBuf x_clk;                                // k_rdx's clock stamps of its last launch (fmcw_rdx_clock)
  int xcd_teams = -1;                          // census of the device: its XCD teams (-1 not run yet, 0 none)
  int8_t xcc_team[16] = {};                    // HW_REG_XCC_ID -> team
  bool xcd_used = false;                       // a k_rdx launch since the last error check
  int x_ctr_set = 0;                           // the counter set (0 / 1) of x_ctr the next k_rdx launch counts in
  bool x_tab_ok = false;                       // x_tab built for the current taps
  // Multi-device context (fmcw_ctx_create with n_devices > 1): this object is
  // device 0 of the context and peers[i] a full context on device i + 1.  The
  // host-pointer calls shard their frames (fmcw_process, fmcw_range_fft) or
  // spectrogram segments (fmcw_stft) over all of them; the device-pointer
  // calls act on device 0.  comms: one RCCL communicator per device
  // (ncclCommInitAll) when the device ids are distinct.
  std::vector<fmcw_ctx*> peers;
  std::vector<ncclComm_t> comms;
  int timing = 0;                    // 0 off, 1 range+Doppler span + STFT launches, 2 + every K1/K2/K3
  struct Pending {
    hipEvent_t a, b;
    int stage;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  double total_ms[kStages] = {};
  int64_t launches[kStages] = {};

  ~fmcw_ctx() {
    for (ncclComm_t m : comms) (void)rccl().comm_destroy(m);
    for (fmcw_ctx* q : peers) delete q;
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& pd : pending) { (void)hipEventDestroy(pd.a); (void)hipEventDestroy(pd.b); }
    for (auto e : pool) (void)hipEventDestroy(e);
    for (int i = 0; i < kSlots; ++i)
      for (hipEvent_t e : {ev_k1[i], ev_k2[i], ev_k3[i]})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_fork, ev_join, ev_h2d[0], ev_h2d[1], ev_comp[0], ev_comp[1], ev_d2h[0], ev_d2h[1]})
      if (e) (void)hipEventDestroy(e);
    for (hipStream_t x : {sd, sx, cin, cout})
      if (x) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); }
    if (stream) (void)hipStreamDestroy(stream);
  }

  hipEvent_t get_event() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, fmcw::kEvDevice) != hipSuccess) return nullptr;   // timing pairs
    return e;
  }
};

namespace {

// Record an event pair around one launch when timing is enabled.
struct StageTimer {
  fmcw_ctx* c;
  int stage;
  hipStream_t s;
  hipEvent_t a = nullptr;
  StageTimer(fmcw_ctx* c_, int st, hipStream_t s_, int level = 1) : c(c_), stage(st), s(s_) {
    // level 3: only the dominant kernels' launches (k_rdx, stage 8; K1 range-only, stage 6):
    // every event pair on the stream costs the step a few microseconds
    const bool on = c->timing == 3 ? (st == 6 || st == 8) : c->timing >= level;
    if (on) {
      a = c->get_event();
      if (a) (void)hipEventRecord(a, s);
    }
  }
  void done() {
    if (a) {
      hipEvent_t b = c->get_event();
      if (b) {
        (void)hipEventRecord(b, s);
        c->pending.push_back({a, b, stage});
      }
      a = nullptr;
    }
  }
};

int set_device(fmcw_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return FMCW_OK;
}

int check_params(const fmcw_params* p) {
  if (!p) return fail(FMCW_E_ARG, "params is NULL");
  if (p->nts < 1 || p->nts > 65536) return fail(FMCW_E_ARG, "nts out of range [1, 65536]");
  if (p->pn < 1 || p->pn > 65536) return fail(FMCW_E_ARG, "pn out of range [1, 65536]");
  if (!fmcw::range_size_supported(p->nr)) return fail(FMCW_E_ARG, "nr must be a power of two in [16, 2048]");
  if (!fmcw::doppler_size_supported(p->nd)) return fail(FMCW_E_ARG, "nd must be a power of two in [2, 1024]");
  if (p->max_targets < 1 || p->max_targets > 8) return fail(FMCW_E_ARG, "max_targets must be in [1, 8]");
  if (!(p->dist_per_bin > 0.f)) return fail(FMCW_E_ARG, "dist_per_bin must be > 0");
  return FMCW_OK;
}

// {cal.re, cal.im, IF_scale*w, w} per sample: one 16-byte load per sample in K1
int build_calw(fmcw_ctx* c, float if_scale, hipStream_t s) {
  const size_t n = c->h_wr.size();
  std::vector<float> t(4 * n);
  for (size_t i = 0; i < n; ++i) {
    t[4 * i] = c->h_cal[2 * i];
    t[4 * i + 1] = c->h_cal[2 * i + 1];
    t[4 * i + 2] = (float)((double)if_scale * c->h_wr[i]);
    t[4 * i + 3] = c->h_wr[i];
  }
  CHK(c->calw.ensure(t.size() * 4));
  HIPCHK(hipMemcpyAsync(c->calw.p, t.data(), t.size() * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  c->calw_scale = if_scale;
  return FMCW_OK;
}

int check_ctx(fmcw_ctx* c, const fmcw_params* p) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(check_params(p));
  if (!c->taps) return fail(FMCW_E_STATE, "fmcw_set_taps has not been called");
  if (p->nts != c->p.nts || p->pn != c->p.pn || p->nr != c->p.nr || p->nd != c->p.nd)
    return fail(FMCW_E_STATE, "nts/pn/nr/nd differ from the ones given to fmcw_set_taps");
  CHK(set_device(c));
  if (p->if_scale != c->calw_scale) {   // queued work on any stream may still read the old table
    HIPCHK(hipDeviceSynchronize());
    CHK(build_calw(c, p->if_scale, c->stream));
  }
  return FMCW_OK;
}

int upload_twiddles(DevBuf& buf, int n, hipStream_t s) {
  std::vector<float> tw(2 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    const double a = -2.0 * M_PI * (double)i / (double)n;
    tw[2 * i] = (float)std::cos(a);
    tw[2 * i + 1] = (float)std::sin(a);
  }
  CHK(buf.ensure(tw.size() * sizeof(float)));
  HIPCHK(hipMemcpyAsync(buf.p, tw.data(), tw.size() * sizeof(float), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return FMCW_OK;
}

int64_t default_chunk(const fmcw_params* p) {
  // The range cube of one chunk is the only intermediate.  Measured on MI355X
  // (tools/mall_probe.hip): re-reading a freshly written buffer is no faster
  // from the Infinity Cache than from HBM, so the chunk is sized for launch
  // efficiency (long kernels, few boundaries): 256 MiB per slot, 3 slots.
  const int64_t per_frame = (int64_t)p->pn * p->nr * 8;
  int64_t c = (256ll << 20) / std::max<int64_t>(per_frame, 1);
  return std::max<int64_t>(c, 1);
}

// Chirps per K1 team: long enough streams for the next-chirp prefetch, while
// keeping >= ~2048 workgroups per launch to fill 256 CUs.
int range_cpt(int nr, int64_t nchirps) {
  const int T = nr >= 16 ? nr / 16 : 1;
  const int teams = T >= 256 ? 1 : 256 / T;
  const int64_t c = nchirps / ((int64_t)teams * 2048);
  return (int)std::max<int64_t>(1, std::min<int64_t>(8, c));
}

hipStream_t pick(fmcw_ctx* c, void* stream) { return stream ? static_cast<hipStream_t>(stream) : c->stream; }

}  // namespace

extern "C" {

int32_t fmcw_abi_version(void) { return FMCW_ABI_VERSION; }

const char* fmcw_last_error(void) { return g_err.c_str(); }

int fmcw_device_count(int32_t* n) {
  if (!n) return fail(FMCW_E_ARG, "n is NULL");
  int d = 0;
  hipError_t e = hipGetDeviceCount(&d);
  if (e != hipSuccess) {
    *n = 0;
    return fail(FMCW_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *n = d;
  return FMCW_OK;
}

int fmcw_default_devices(int32_t cap, int32_t* ids, int32_t* n) {
  if (!ids || !n || cap < 1) return fail(FMCW_E_ARG, "ids/n NULL or cap < 1");
  *n = 0;
  const char* env = std::getenv("FMCW_DEVICES");
  std::string v = env ? env : "";
  v.erase(std::remove_if(v.begin(), v.end(), [](char ch) { return ch == ' ' || ch == '\t'; }), v.end());
  std::vector<long> want;                      // the list is parsed before any device is asked about
  if (!v.empty() && v != "all") {
    size_t pos = 0;
    while (pos <= v.size()) {
      const size_t end = std::min(v.find(',', pos), v.size());
      const std::string tok = v.substr(pos, end - pos);
      char* stop = nullptr;
      const long id = tok.empty() ? -1 : std::strtol(tok.c_str(), &stop, 10);
      if (tok.empty() || *stop != '\0' || id < 0) return fail(FMCW_E_ARG, "FMCW_DEVICES: malformed list '" + v + "'");
      want.push_back(id);
      pos = end + 1;
    }
    if ((int64_t)want.size() > cap) return fail(FMCW_E_ARG, "FMCW_DEVICES: more ids than cap");
  }
  int nd = 0;
  hipError_t e = hipGetDeviceCount(&nd);
  if (e != hipSuccess) return fail(FMCW_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  if (want.empty()) {
    if (nd < 1) return fail(FMCW_E_HIP, "no HIP device present");
    const int m = std::min<int>(nd, cap);
    for (int i = 0; i < m; ++i) ids[i] = i;
    *n = m;
    return FMCW_OK;
  }
  for (size_t i = 0; i < want.size(); ++i) {
    if (want[i] >= nd)
      return fail(FMCW_E_ARG, "FMCW_DEVICES: device " + std::to_string(want[i]) + " not present (" +
                                  std::to_string(nd) + " devices)");
    ids[i] = (int32_t)want[i];
  }
  *n = (int32_t)want.size();
  return FMCW_OK;
}

static int ctx_create_one(int32_t device_id, fmcw_ctx** out) {
  *out = nullptr;
  int nd = 0;
  HIPCHK(hipGetDeviceCount(&nd));
  if (device_id < 0 || device_id >= nd)
    return fail(FMCW_E_HIP, "device " + std::to_string(device_id) + " not present (" + std::to_string(nd) + " devices)");
  HIPCHK(hipSetDevice(device_id));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device_id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(FMCW_E_HIP, std::string("libfmcw is built for gfx950, device is ") + prop.gcnArchName);
  auto* c = new fmcw_ctx();
  c->device = device_id;
  bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->sd, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->sx, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->cin, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->cout, hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; i < 2; ++i)
    for (hipEvent_t* e : {&c->ev_h2d[i], &c->ev_comp[i], &c->ev_d2h[i]})
      ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  for (int i = 0; i < fmcw_ctx::kSlots; ++i)   // the streams schedule's joins: device scope
    for (hipEvent_t* e : {&c->ev_k1[i], &c->ev_k2[i], &c->ev_k3[i]})
      ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming | fmcw::kEvDevice) == hipSuccess;
  for (hipEvent_t* e : {&c->ev_fork, &c->ev_join})
    ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming | fmcw::kEvDevice) == hipSuccess;
  if (!ok) {
    delete c;
    return fail(FMCW_E_HIP, "stream/event creation failed");
  }
  *out = c;
  return FMCW_OK;
}

int fmcw_ctx_create(int32_t n_devices, const int32_t* device_ids, fmcw_ctx** out) {
  if (!out) return fail(FMCW_E_ARG, "out is NULL");
  *out = nullptr;
  if (n_devices < 1 || n_devices > 64) return fail(FMCW_E_ARG, "n_devices must be in [1, 64]");
  std::vector<int> ids(n_devices);
  for (int i = 0; i < n_devices; ++i) ids[i] = device_ids ? device_ids[i] : i;
  fmcw_ctx* c = nullptr;
  CHK(ctx_create_one(ids[0], &c));
  for (int i = 1; i < n_devices; ++i) {
    fmcw_ctx* q = nullptr;
    const int st = ctx_create_one(ids[i], &q);
    if (st != FMCW_OK) {
      delete c;
      return st;
    }
    c->peers.push_back(q);
  }
  std::vector<int> sorted = ids;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (n_devices > 1 && distinct) {   // one communicator per device, one process
    if (!rccl().ok) {
      delete c;
      return fail(FMCW_E_HIP, "RCCL (librccl.so.1) not found: needed for a context over several devices");
    }
    c->comms.assign(n_devices, nullptr);
    const ncclResult_t r = rccl().comm_init_all(c->comms.data(), n_devices, ids.data());
    if (r != ncclSuccess) {
      c->comms.clear();
      const std::string msg = std::string("ncclCommInitAll: ") + rccl().error_string(r);
      delete c;
      return fail(FMCW_E_HIP, msg);
    }
  }
  *out = c;
  return FMCW_OK;
}

int fmcw_ctx_devices(fmcw_ctx* c, int32_t* n_devices, int32_t* device_ids, int32_t* rccl_comms) {
  if (!c || !n_devices) return fail(FMCW_E_ARG, "NULL argument");
  *n_devices = 1 + (int32_t)c->peers.size();
  if (device_ids) {
    device_ids[0] = c->device;
    for (size_t i = 0; i < c->peers.size(); ++i) device_ids[i + 1] = c->peers[i]->device;
  }
  if (rccl_comms) *rccl_comms = c->comms.empty() ? 0 : 1;
  return FMCW_OK;
}

int fmcw_ctx_destroy(fmcw_ctx* c) {
  if (!c) return FMCW_OK;
  delete c;
  return FMCW_OK;
}

int fmcw_set_taps(fmcw_ctx* c, const fmcw_params* p, const float* range_win, const float* doppler_win,
                  const float* calib) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(check_params(p));
  if (!range_win || !doppler_win || !calib) return fail(FMCW_E_ARG, "taps pointer is NULL");
  CHK(set_device(c));
  hipStream_t s = c->stream;
  // the taps are read by work on the caller's streams, which the context's stream does not
  // order against: let queued work finish with the old taps, and finish the copies before
  // returning, so that a call on any stream afterwards reads the new ones
  HIPCHK(hipDeviceSynchronize());
  CHK(c->wd.ensure((size_t)p->pn * 4));
  CHK(c->cal.ensure((size_t)p->nts * 8));
  HIPCHK(hipMemcpyAsync(c->wd.p, doppler_win, (size_t)p->pn * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->cal.p, calib, (size_t)p->nts * 8, hipMemcpyHostToDevice, s));
  c->h_wr.assign(range_win, range_win + p->nts);
  c->h_cal.assign(calib, calib + 2 * (size_t)p->nts);
  double sr = 0, si = 0;
  for (int n = 0; n < p->nts; ++n) { sr += calib[2 * n]; si += calib[2 * n + 1]; }
  c->cal_sum = make_float2((float)sr, (float)si);
  CHK(build_calw(c, p->if_scale, s));
  CHK(upload_twiddles(c->tw_nr, p->nr, s));
  CHK(upload_twiddles(c->tw_nd, p->nd, s));
  c->p = *p;
  c->taps = true;
  c->x_tab_ok = false;
  HIPCHK(hipStreamSynchronize(s));
  for (fmcw_ctx* q : c->peers) CHK(fmcw_set_taps(q, p, range_win, doppler_win, calib));
  return FMCW_OK;
}

int fmcw_set_chunk_frames(fmcw_ctx* c, int64_t frames) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (frames < 0) return fail(FMCW_E_ARG, "frames < 0");
  c->chunk_frames = frames;
  for (fmcw_ctx* q : c->peers) q->chunk_frames = frames;
  return FMCW_OK;
}

int fmcw_set_pipeline(fmcw_ctx* c, int32_t mode) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (mode != FMCW_PIPE_AUTO && mode != FMCW_PIPE_STREAMS && mode != FMCW_PIPE_ONEPASS && mode != FMCW_PIPE_XCD)
    return fail(FMCW_E_ARG, "bad pipeline mode");
  c->pipe_mode = mode;
  for (fmcw_ctx* q : c->peers) q->pipe_mode = mode;
  return FMCW_OK;
}

// The XCD-team schedule's sticky error word (kernels_xcd.hip): read after the
// stream is idle; a set bit means the outputs of some k_rdx launch are invalid.
static int xcd_check(fmcw_ctx* c) {
  if (!c->xcd_used) return FMCW_OK;
  unsigned e = 0;
  HIPCHK(hipMemcpy(&e, c->x_err.p, sizeof(e), hipMemcpyDeviceToHost));
  c->xcd_used = false;
  if (!e) return FMCW_OK;
  HIPCHK(hipMemset(c->x_err.p, 0, sizeof(e)));
  return fail(FMCW_E_HIP, (e & 2) ? "XCD schedule: an XCD received more than 32 workgroups (outputs invalid)"
                                  : "XCD schedule: a range-cube hand-off timed out (outputs invalid)");
}

int fmcw_rdx_clock(fmcw_ctx* c, double* mhz, double* us) {
  if (!c || !mhz) return fail(FMCW_E_ARG, "ctx / mhz is NULL");
  *mhz = 0.0;
  if (us) *us = 0.0;
  CHK(set_device(c));
  if (!c->x_clk.p) return FMCW_OK;             // no k_rdx launch yet
  unsigned long long h[4] = {};
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(h, c->x_clk.p, sizeof(h), hipMemcpyDeviceToHost));
  if (h[3] > h[1] && h[2] > h[0]) {
    *mhz = (double)(h[2] - h[0]) / (double)(h[3] - h[1]) * 100.0;   // s_memrealtime: 100 MHz
    if (us) *us = (double)(h[3] - h[1]) / 100.0;
  }
  return FMCW_OK;
}

int fmcw_copy_device(fmcw_ctx* c, const void* d_src, void* d_dst, int64_t bytes, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (!d_src || !d_dst || bytes < 0) return fail(FMCW_E_ARG, "bad copy arguments");
  CHK(set_device(c));
  HIPCHK(fmcw::launch_copy16(d_src, d_dst, bytes, pick(c, stream)));
  return FMCW_OK;
}

int fmcw_synchronize(fmcw_ctx* c) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(set_device(c));
  HIPCHK(hipStreamSynchronize(c->stream));
  return xcd_check(c);
}

int fmcw_timing_enable(fmcw_ctx* c, int32_t enable) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (enable < 0 || enable > 3) return fail(FMCW_E_ARG, "timing level must be 0, 1, 2 or 3");
  c->timing = enable;
  return FMCW_OK;   // device 0 only: the timers are the device-pointer calls' (benches)
}

static int timing_collect(fmcw_ctx* c) {
  for (auto& pd : c->pending) {
    HIPCHK(hipEventSynchronize(pd.b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, pd.a, pd.b));
    c->total_ms[pd.stage] += ms;
    c->launches[pd.stage] += 1;
    c->pool.push_back(pd.a);
    c->pool.push_back(pd.b);
  }
  c->pending.clear();
  return FMCW_OK;
}

int fmcw_timing_read(fmcw_ctx* c, int32_t stage, double* total_ms, int64_t* launches) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (stage < 0 || stage >= kStages) return fail(FMCW_E_ARG, "stage out of range");
  CHK(set_device(c));
  CHK(timing_collect(c));
  if (total_ms) *total_ms = c->total_ms[stage];
  if (launches) *launches = c->launches[stage];
  return FMCW_OK;
}

int fmcw_timing_reset(fmcw_ctx* c) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(set_device(c));
  CHK(timing_collect(c));
  for (int i = 0; i < kStages; ++i) { c->total_ms[i] = 0; c->launches[i] = 0; }
  return FMCW_OK;
}

// ---------------------------------------------------------------------------
// per-frame stages
// ---------------------------------------------------------------------------
// Twiddle table of the XCD-team schedule (kernels_xcd.hip, XT_* sections, lane order [..][64]),
// built in float64 and rounded once; it depends only on NR, so it is built once per context.
static int build_xcd_tab(fmcw_ctx* c, hipStream_t s) {
  const int NR = c->p.nr;
  std::vector<double> cr(NR), ci(NR);
  for (int i = 0; i < NR; ++i) {
    const double a = -2.0 * M_PI * (double)i / (double)NR;
    cr[i] = std::cos(a);
    ci[i] = std::sin(a);
  }
  std::vector<float> xt(2 * (size_t)fmcw::XT_SIZE);
  auto xput = [&](int idx, int e1024) { xt[2 * idx] = (float)cr[e1024 & (NR - 1)]; xt[2 * idx + 1] = (float)ci[e1024 & (NR - 1)]; };
  for (int l = 0; l < 64; ++l) {
    for (int k1 = 1; k1 < 8; ++k1)
      for (int e = 0; e < 2; ++e) xput(fmcw::XT_R1 + (2 * (k1 - 1) + e) * 64 + l, (2 * l + e) * k1);   // W1024^(a k1)
    for (int s1 = 1; s1 < 16; ++s1) xput(fmcw::XT_R2 + (s1 - 1) * 64 + l, 8 * ((l & 7) * s1));      // W128^(a0 s1)
    for (int d0 = 1; d0 < 16; ++d0) xput(fmcw::XT_D1 + (d0 - 1) * 64 + l, 4 * ((l & 15) * d0));     // W256^(q d0)
    // half-frame build (-DXK_HALF)
    for (int k1 = 1; k1 < 8; ++k1) xput(fmcw::XT_H1 + (k1 - 1) * 64 + l, 2 * l * k1);              // W512^(l k1)
    for (int s1 = 1; s1 < 8; ++s1) xput(fmcw::XT_H2 + (s1 - 1) * 64 + l, 16 * ((l & 7) * s1));     // W64^(l0 s1)
    for (int s2 = 0; s2 < 8; ++s2) xput(fmcw::XT_HC + s2 * 64 + l, l + 64 * s2);                   // W1024^(l + 64 s2)
  }
  CHK(c->x_tab.ensure(xt.size() * 4));
  HIPCHK(hipMemcpyAsync(c->x_tab.p, xt.data(), xt.size() * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  c->x_tab_ok = true;
  return FMCW_OK;
}

// fp16 storage on the single pass: the 128-bin blocks of the range cube that hold no bin able
// to become a detection or slow-time candidate (k_rdx's key test: 1 <= r <= NR - 2 and
// min_d <= r * dist_per_bin <= max_d, with two bins of margin each side for the local-maximum
// test's neighbours) are handed between the CUs as c32h; the others stay c64, so the slow-time
// rows and the profile around a target come from fp32 values.  FMCW_S16=0 keeps every block c64.
static unsigned host_s16mask(const fmcw_params* p, int NR) {
  {
    const char* e = std::getenv("FMCW_S16");
    if (e && e[0] == '0') return 0u;
  }
  const double dpb = p->dist_per_bin;
  if (!(dpb > 0.0) || !std::isfinite(dpb) || !std::isfinite(p->min_d) || !std::isfinite(p->max_d)) return 0u;
  const double lo_d = std::floor((double)p->min_d / dpb) - 2, hi_d = std::ceil((double)p->max_d / dpb) + 2;
  const int lo = (int)std::max(0.0, std::min((double)NR, lo_d));
  const int hi = (int)std::max(-1.0, std::min((double)NR - 1, hi_d));
  unsigned m = 0;
  for (int b = 0; b < NR / 128; ++b)
    if (hi < lo || 128 * b + 127 < lo || 128 * b > hi) m |= 1u << b;
  return m;
}

// The slow-time leg's start, fused into the detection (fmcw_process_slow_device): the
// compaction of :257-260 (frame list, L) and the reset of the STFT's running max(P).
struct SlowLeg {
  int32_t* list;
  int64_t* len;
  float* pmax;   // may be NULL
};

// Single-pass schedule (kernels_xcd.hip): k_rdx computes range FFT, profile,
// Doppler FFT and the slow-time candidate rows of each frame, the range cube
// handed between the CUs of one XCD; k_detect_1p runs the detection (and
// recomputes the rare slow-time row that was not among a group's candidates).
// Chunks bound the candidate scratch (XCD_TILES * XCD_CAND rows of PN floats per
// frame).  The hand-off ring has XCD_MAX_SLOTS slots per XCD.
static int process_onepass(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int h, int64_t F, float* d_prof,
                           int32_t* d_count, int32_t* d_ridx, float* d_rmag, int32_t* d_didx, float* d_slow,
                           void* d_rd, int64_t probe_column, float* d_probe, const SlowLeg* leg, hipStream_t s) {
  const int C = p->pn, S = p->nts, NR = p->nr, ND = p->nd, M = p->max_targets;
  const int64_t chunk = std::min<int64_t>(F, c->chunk_frames > 0 ? c->chunk_frames : 8192);
  const int tiles = fmcw::XCD_TILES, ncand = fmcw::XCD_CAND;
  const int TC = tiles * ncand;
  const int slots = fmcw::XCD_MAX_SLOTS;
  {
#ifdef FMCW_XCUBE_PAD_AB   // A/B (tools/place_probe.py slots): the slot ring FMCW_XCUBE_PAD bytes into a larger buffer
    CHK(c->x_cube.ensure((size_t)8 * slots * fmcw::XCD_TILES * C * 32 * 8 + ((size_t)1 << 30)));
#else
    CHK(c->x_cube.ensure((size_t)8 * slots * fmcw::XCD_TILES * C * 32 * 8));
#endif
    if (!c->x_ctr.p) {                         // two counter sets, both zero before the first launch
      CHK(c->x_ctr.ensure(sizeof(unsigned) * 2 * fmcw::XCD_CTR_WORDS));
      HIPCHK(hipMemsetAsync(c->x_ctr.p, 0, sizeof(unsigned) * 2 * fmcw::XCD_CTR_WORDS, s));
      c->x_ctr_set = 0;
    }
    if (!c->x_clk.p) {
      CHK(c->x_clk.ensure(4 * sizeof(unsigned long long)));
      HIPCHK(hipMemsetAsync(c->x_clk.p, 0, 4 * sizeof(unsigned long long), s));
    }
    if (!c->x_err.p) {
      CHK(c->x_err.ensure(sizeof(unsigned)));
      HIPCHK(hipMemsetAsync(c->x_err.p, 0, sizeof(unsigned), s));
    }
  }
  CHK(c->op_rowpk.ensure((size_t)chunk * NR * 8));
  CHK(c->op_cidx.ensure((size_t)chunk * TC * 4));
  CHK(c->op_crows.ensure((size_t)chunk * TC * C * 4));
  int32_t* det_done = nullptr;
  if (leg) {
    int st = FMCW_OK;
    bool fresh = false;
    det_done = static_cast<int32_t*>(c->det_done.get(s, 9 * 128, &st, &fresh));   // 8 shards + top, 128 B apart
    CHK(st);
    if (fresh) HIPCHK(hipMemsetAsync(det_done, 0, 9 * 128, s));
  }
  const int64_t pframe = probe_column > 0 ? (probe_column - 1) / C : -1;
  const int pchirp = probe_column > 0 ? (int)((probe_column - 1) % C) : 0;
  if (!c->x_tab_ok) CHK(build_xcd_tab(c, s));
  if (pframe >= 0 && d_probe) {                // :410-411 fft_data column: one chirp by a direct DFT
    fmcw::ProbeArgs pa{};
    pa.iq = d_iq; pa.h = h;
    pa.frame = pframe; pa.chirp = pchirp; pa.C = C; pa.S = S; pa.NR = NR;
    pa.calw = c->calw.as<float4>(); pa.tw_nr = c->tw_nr.as<float2>(); pa.probe_mag = d_probe;
    HIPCHK(fmcw::launch_probe(pa, s));
  }
  StageTimer span(c, 7, s, 1);
  for (int64_t f0 = 0; f0 < F; f0 += chunk) {
    const int64_t nf = std::min(chunk, F - f0);
    fmcw::OnePassArgs a{};
    a.iq = static_cast<const char*>(d_iq) + (size_t)f0 * C * S * (h ? 4 : 8);
    a.h = h;
    a.rd_scale = h ? 1.0f / ((float)NR * ND) : 1.0f;
    a.F = nf; a.C = C; a.S = S;
    a.calw = c->calw.as<float4>();
    a.tw_nr = c->tw_nr.as<float2>(); a.tw_nd = c->tw_nd.as<float2>(); a.wd = c->wd.as<float>();
    a.rd = d_rd ? static_cast<char*>(d_rd) + (size_t)f0 * NR * ND * (h ? 4 : 8) : nullptr;
    a.profile = d_prof + f0 * NR;
    a.rowpk = c->op_rowpk.as<int2>();
    a.cand_idx = c->op_cidx.as<int32_t>();
    a.cand_rows = c->op_crows.as<float>();
    a.range_thr = p->range_thr; a.min_d = p->min_d; a.max_d = p->max_d; a.dist_per_bin = p->dist_per_bin;
    // counter sets: this launch counts in set x_ctr_set and zeroes the other one for the next launch (launches
    // of a device run one at a time, launch_xcd's chain); FMCW_XCD_MEMSET=1: set 0 and a memset per launch
    const bool xmemset = [] { const char* e = std::getenv("FMCW_XCD_MEMSET"); return e && e[0] == '1'; }();
    a.xcube = c->x_cube.as<float2>(); a.xerr = c->x_err.as<unsigned>();
    a.xctr = c->x_ctr.as<unsigned>() + (xmemset ? 0 : c->x_ctr_set * fmcw::XCD_CTR_WORDS);
    a.xclr = xmemset ? nullptr : c->x_ctr.as<unsigned>() + (1 - c->x_ctr_set) * fmcw::XCD_CTR_WORDS;
#ifdef FMCW_XCUBE_PAD_AB
    if (const char* e = std::getenv("FMCW_XCUBE_PAD")) {
      const size_t pad = std::min<size_t>((size_t)std::strtoull(e, nullptr, 0), (size_t)1 << 30) & ~(size_t)255;
      a.xcube = reinterpret_cast<float2*>(c->x_cube.as<char>() + pad);
    }
#endif
    a.slots = slots; a.xtab = c->x_tab.as<float2>(); a.cal_sum = c->cal_sum;
    a.clk = c->x_clk.as<unsigned long long>();
    a.s16mask = h ? host_s16mask(p, NR) : 0u;
    a.nteams = c->xcd_teams > 0 ? c->xcd_teams : 0;
    std::memcpy(a.xcc_team, c->xcc_team, sizeof(a.xcc_team));
    {
      const char* e = std::getenv("FMCW_ONEPASS_FORCE_FIX");
      a.force_fix = (e && e[0] == '1') ? 1 : 0;
    }
#if defined(XK_STAMPS) || defined(XK_SKEW)
    static unsigned long long* xdbg = nullptr;
    if (!xdbg) HIPCHK(hipMalloc(&xdbg, (size_t)1 << 20));
    a.dbg = xdbg;
#endif
    {
      StageTimer tm(c, 8, s, 2);
      {
        HIPCHK(fmcw::launch_xcd(a, s));
        c->xcd_used = true;
        if (a.xclr && nf > 0) c->x_ctr_set ^= 1;   // the next launch counts in the set this one zeroed
#ifdef XK_SKEW
        {   // diagnostic build: the team's skew.  Per XCD and step j: the spread of the 32 members' publish
            // times of R(j - 1), and how long after the last publish each member's poll of it returned
            // (100 MHz realtime clock, steps 8 .. 247 of the launch); which member published last how often
          constexpr int ST = 256;
          const int nblk = 32 * a.nteams;
          std::vector<unsigned long long> hh((size_t)nblk * 2 * ST);
          HIPCHK(hipStreamSynchronize(s));
          HIPCHK(hipMemcpy(hh.data(), a.dbg, hh.size() * 8, hipMemcpyDeviceToHost));
          double spread = 0, lag_min = 0, lag_max = 0, lag_mean = 0, pub_to_first_poll = 0;
          long n = 0;
          std::vector<long> last(32, 0), first(32, 0);
          for (int xx = 0; xx < a.nteams; ++xx)
            for (int j = 8; j < ST - 8; ++j) {
              unsigned long long pmin = ~0ull, pmax = 0, qmin = ~0ull, qmax = 0;
              double qs = 0;
              int kl = 0, kf = 0;
              for (int kk = 0; kk < 32; ++kk) {
                const unsigned long long p_ = hh[((size_t)(xx * 32 + kk)) * 2 * ST + 2 * j];
                const unsigned long long q_ = hh[((size_t)(xx * 32 + kk)) * 2 * ST + 2 * j + 1];
                if (p_ > pmax) { pmax = p_; kl = kk; }
                if (p_ < pmin) { pmin = p_; kf = kk; }
                qmin = std::min(qmin, q_); qmax = std::max(qmax, q_);
                qs += (double)q_;
              }
              if (!pmin || !qmin) continue;
              spread += (double)(pmax - pmin);
              lag_min += (double)qmin - (double)pmax;
              lag_max += (double)qmax - (double)pmax;
              lag_mean += qs / 32 - (double)pmax;
              pub_to_first_poll += (double)qmin - (double)pmin;
              ++last[kl]; ++first[kf]; ++n;
            }
          if (n) {
            std::fprintf(stderr, "xk-skew (us, %ld team-steps): publish spread %.2f | poll return after the last publish: "
                         "first %.2f mean %.2f last %.2f\n", n, spread / n / 100, lag_min / n / 100, lag_mean / n / 100,
                         lag_max / n / 100);
            std::fprintf(stderr, "xk-skew last publisher by member:");
            for (int kk = 0; kk < 32; ++kk) std::fprintf(stderr, " %ld", last[kk]);
            std::fprintf(stderr, "\nxk-skew first publisher by member:");
            for (int kk = 0; kk < 32; ++kk) std::fprintf(stderr, " %ld", first[kk]);
            std::fprintf(stderr, "\n");
          }
        }
#endif
#ifdef XK_STAMPS
        {   // diagnostic build: per-step phase times of k_rdx (100 MHz realtime clock), averaged over blocks
          const int nblk = 32 * a.nteams;
          std::vector<unsigned long long> hh(nblk * 32);
          HIPCHK(hipStreamSynchronize(s));
          HIPCHK(hipMemcpy(hh.data(), a.dbg, hh.size() * 8, hipMemcpyDeviceToHost));
          static const char* nm[10] = {"B1", "stage", "B2", "rows", "pubwait+B3", "cand", "R1+ld+D3",
                                       "poll+grp", "TD..R3", "RD"};
          for (int wv = 0; wv < 2; ++wv) {
            double ph[10] = {}, steps = 0;
            for (int bb = 0; bb < nblk; ++bb) {
              for (int q = 0; q < 10; ++q) ph[q] += (double)hh[(bb * 2 + wv) * 16 + q];
              steps += (double)hh[(bb * 2 + wv) * 16 + 15];
            }
            double tot = 0;
            std::fprintf(stderr, "xk-stamps wave %d (us/step):", wv * 4);
            for (int q = 0; q < 10; ++q) { std::fprintf(stderr, " %s %.2f |", nm[q], ph[q] / steps / 100); tot += ph[q]; }
            double cyc = 0, rt = 0;
            for (int bb = 0; bb < nblk; ++bb) { cyc += (double)hh[(bb * 2 + wv) * 16 + 13]; rt += (double)hh[(bb * 2 + wv) * 16 + 14]; }
            std::fprintf(stderr, " sum %.2f | clock %.3f GHz\n", tot / steps / 100, rt > 0 ? cyc / rt * 0.1 : 0.0);
          }
        }
#endif
      }
      tm.done();
    }
    fmcw::Detect1pArgs k{};
    k.profile = a.profile; k.rowpk = a.rowpk; k.rd = a.rd; k.ND = ND; k.rd_h = h; k.cand_idx = a.cand_idx; k.cand_rows = a.cand_rows;
    k.tiles = tiles; k.ncand = ncand;
    k.nframes = (int)nf; k.NR = NR; k.C = C; k.M = M;
    k.det.ND = ND; k.det.C = C; k.det.M = M;
    k.det.range_thr = p->range_thr; k.det.doppler_thr = p->doppler_thr;
    k.det.min_d = p->min_d; k.det.max_d = p->max_d; k.det.dist_per_bin = p->dist_per_bin;
    k.det.fallback = p->doppler_fallback_idx;
    k.det.cube_unscale = 1.0f; k.det.rd_unscale = 1.0f / a.rd_scale;
    k.count = d_count + f0; k.ridx = d_ridx + f0 * M; k.rmag = d_rmag + f0 * M; k.didx = d_didx + f0 * M;
    k.slow_mag = d_slow + f0 * C;
    k.iq = a.iq; k.h = h; k.S = S; k.calw = a.calw; k.tw_nr = a.tw_nr;
    if (leg && f0 + nf == F) {   // the last chunk's detection also compacts every frame of the call
      k.done = det_done; k.count_all = d_count; k.F_all = F; k.pn = C;
      k.list = leg->list; k.len = leg->len; k.pmax_reset = leg->pmax;
    }
    {
      StageTimer tm(c, 2, s, 2);
      HIPCHK(fmcw::launch_detect_1p(k, s));
      tm.done();
    }
  }
  if (leg) CHK(c->det_done.done(s));
  span.done();
  return FMCW_OK;
}

static int process_device_impl(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int32_t in_dtype, int64_t F,
                               float* d_prof, int32_t* d_count, int32_t* d_ridx, float* d_rmag, int32_t* d_didx,
                               float* d_slow, void* d_cube, void* d_rd, int32_t out_dtype, int64_t probe_column,
                               float* d_probe, const SlowLeg* leg, void* stream);

int fmcw_process_device(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int32_t in_dtype, int64_t F,
                        float* d_prof, int32_t* d_count, int32_t* d_ridx, float* d_rmag, int32_t* d_didx,
                        float* d_slow, void* d_cube, void* d_rd, int32_t out_dtype, int64_t probe_column,
                        float* d_probe, void* stream) {
  return process_device_impl(c, p, d_iq, in_dtype, F, d_prof, d_count, d_ridx, d_rmag, d_didx, d_slow, d_cube, d_rd,
                             out_dtype, probe_column, d_probe, nullptr, stream);
}

int fmcw_process_slow_device(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int32_t in_dtype, int64_t F,
                             float* d_prof, int32_t* d_count, int32_t* d_ridx, float* d_rmag, int32_t* d_didx,
                             float* d_slow, void* d_rd, int32_t out_dtype, int32_t* d_frame_list, int64_t* d_len,
                             float* d_pmax, void* stream) {
  if (!d_frame_list || !d_len) return fail(FMCW_E_ARG, "d_frame_list / d_len is NULL");
  if (F == 0 && c) {   // nothing to detect: the leg still starts (L = 0, max(P) = 0)
    CHK(check_ctx(c, p));
    hipStream_t s = pick(c, stream);
    HIPCHK(hipMemsetAsync(d_len, 0, 8, s));
    if (d_pmax) HIPCHK(hipMemsetAsync(d_pmax, 0, 4, s));
    return FMCW_OK;
  }
  const SlowLeg leg{d_frame_list, d_len, d_pmax};
  return process_device_impl(c, p, d_iq, in_dtype, F, d_prof, d_count, d_ridx, d_rmag, d_didx, d_slow, nullptr, d_rd,
                             out_dtype, 0, nullptr, &leg, stream);
}

static int process_device_impl(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int32_t in_dtype, int64_t F,
                               float* d_prof, int32_t* d_count, int32_t* d_ridx, float* d_rmag, int32_t* d_didx,
                               float* d_slow, void* d_cube, void* d_rd, int32_t out_dtype, int64_t probe_column,
                               float* d_probe, const SlowLeg* leg, void* stream) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (F == 0) return FMCW_OK;
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  if (out_dtype != FMCW_C64 && out_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad out_dtype");
  if (!d_iq || !d_prof || !d_count || !d_ridx || !d_rmag || !d_didx || !d_slow)
    return fail(FMCW_E_ARG, "required device pointer is NULL");
  const int S = p->nts, C = p->pn, NR = p->nr, ND = p->nd, M = p->max_targets;
  if (probe_column < 0 || probe_column > F * (int64_t)C) return fail(FMCW_E_ARG, "probe_column out of range");
  hipStream_t s = pick(c, stream);
  // the single pass keeps one storage type end to end: c64 in / c64 RD, or
  // fp16 storage (c32h in / c32h RD); the RD dtype is free when RD is not asked for
  const bool onepass_ok = !d_cube && (!d_rd || out_dtype == in_dtype) && fmcw::onepass_supported(S, C, NR, ND);
  // the XCD-team single pass (k_rdx) wherever it applies: half the HBM bytes of the streams
  // schedule (no range cube) and faster on MI355X; FMCW_PIPE_ONEPASS is
  // the same schedule (the 8-tile single pass of ABI 2 is retired); AUTO falls back to the
  // streams schedule where the geometry or the device does not allow it
  const bool want = c->pipe_mode == FMCW_PIPE_ONEPASS || c->pipe_mode == FMCW_PIPE_XCD;
  if (want || (c->pipe_mode == FMCW_PIPE_AUTO && onepass_ok)) {
    if (!onepass_ok)
      return fail(FMCW_E_ARG, "single-pass schedule: needs nr 1024, pn == nd == 256, even nts <= nr, "
                              "the RD map in the IQ dtype and no range cube");
    if (c->xcd_teams < 0) {
      int n = 0;
      HIPCHK(fmcw::xcd_census(&n, c->xcc_team));
      const char* e = std::getenv("FMCW_NO_XCD");
      c->xcd_teams = (e && e[0] == '1') ? 0 : n;
    }
    if (c->xcd_teams > 0)
      return process_onepass(c, p, d_iq, in_dtype == FMCW_C32H ? 1 : 0, F, d_prof, d_count, d_ridx, d_rmag, d_didx,
                             d_slow, d_rd, probe_column, d_probe, leg, s);
    if (want)
      return fail(FMCW_E_ARG, "XCD schedule: needs 32 CUs per XCD and a grid of one workgroup per CU dealt 32 per XCD");
  }
  const int64_t chunk = c->chunk_frames > 0 ? c->chunk_frames : default_chunk(p);
  const int cube_dt = d_cube ? out_dtype : FMCW_C64;
  const int rd_dt = d_rd ? out_dtype : FMCW_C64;
  // fp16 storage keeps MATLAB's values divided by the FFT sizes applied so far
  // (exact powers of two): |X|/Nr and |D|/(Nr*Nd) stay inside the fp16 range
  const float cube_scale = cube_dt == FMCW_C32H ? 1.0f / NR : 1.0f;
  const float rd_scale = rd_dt == FMCW_C32H ? 1.0f / ((float)NR * ND) : 1.0f;
  const int64_t cf = std::min(chunk, F);
  const size_t cube_slot = (size_t)cf * C * NR * 8, rd_slot = (size_t)cf * NR * ND * 8;
  constexpr int NS = fmcw_ctx::kSlots;
  // NS scratch slots: while K3(i-1) and K2(i) read slots (i-1)%NS and i%NS,
  // K1(i+1) fills slot (i+1)%NS
  if (!d_cube) CHK(c->scratch_cube.ensure(NS * cube_slot));
  if (!d_rd) CHK(c->scratch_rd.ensure(NS * rd_slot));
  const int64_t pframe = probe_column > 0 ? (probe_column - 1) / C : -1;
  const int pchirp = probe_column > 0 ? (int)((probe_column - 1) % C) : 0;
  hipStream_t sd = c->sd, sx = c->sx;
  // one chunk: K1 -> K2 -> K3 have nothing to overlap with, so they go on the caller's stream
  // without the fork / join events (a deployed 115-frame call: 9 event calls fewer)
  if (F <= chunk) sd = sx = s;
  if (const char* e = std::getenv("FMCW_ONE_STREAM"); e && e[0] == '1') sd = sx = s;   // A/B probe
  const bool split = sd != s || sx != s;
  StageTimer span(c, 7, s, 1);     // range+Doppler span: before K1(0) on s ... after the last K2 on sd
  if (split) {
    HIPCHK(hipEventRecord(c->ev_fork, s));
    HIPCHK(hipStreamWaitEvent(sd, c->ev_fork, 0));
    HIPCHK(hipStreamWaitEvent(sx, c->ev_fork, 0));
  }

  int64_t i = 0;
  for (int64_t f0 = 0; f0 < F; f0 += chunk, ++i) {
    const int b = (int)(i % NS);
    const int64_t nf = std::min(chunk, F - f0);
    if (split && i >= NS) HIPCHK(hipStreamWaitEvent(s, c->ev_k3[b], 0));   // WAR: K2/K3(i-NS) done with slot b
    char* cube = d_cube ? static_cast<char*>(d_cube) + (size_t)f0 * C * NR * esize(cube_dt)
                        : c->scratch_cube.as<char>() + b * cube_slot;
    char* rd = d_rd ? static_cast<char*>(d_rd) + (size_t)f0 * NR * ND * esize(rd_dt)
                    : c->scratch_rd.as<char>() + b * rd_slot;

    fmcw::RangeArgs ra{};
    ra.iq = static_cast<const char*>(d_iq) + (size_t)f0 * C * S * esize(in_dtype);
    ra.in_dtype = in_dtype;
    ra.nchirps = nf * C;
    ra.C = C; ra.S = S; ra.NR = NR;
    ra.calw = c->calw.as<float4>();
    ra.cal_sum = c->cal_sum;
    ra.if_scale = p->if_scale;
    ra.tw = c->tw_nr.as<float2>();
    ra.cube = cube;
    ra.cube_dtype = cube_dt;
    ra.cube_scale = cube_scale;
    ra.profile = nullptr;
    ra.cpt = range_cpt(NR, ra.nchirps);
    {
      StageTimer tm(c, 0, s, 2);
      HIPCHK(fmcw::launch_range(ra, s));
      tm.done();
    }
    if (split) {
      HIPCHK(hipEventRecord(c->ev_k1[b], s));
      HIPCHK(hipStreamWaitEvent(sd, c->ev_k1[b], 0));
    }

    fmcw::DopplerArgs da{};
    da.cube = cube; da.cube_dtype = cube_dt;
    da.cube_unscale = 1.0f / cube_scale; da.rd_scale = rd_scale;
    da.nframes = (int)nf; da.C = C; da.NR = NR; da.ND = ND;
    da.wd = c->wd.as<float>();
    da.tw = c->tw_nd.as<float2>();
    da.rd = rd; da.rd_dtype = rd_dt;
    da.profile = d_prof + f0 * NR;
    {
      StageTimer tm(c, 1, sd, 2);
      HIPCHK(fmcw::launch_doppler(da, sd));
      tm.done();
    }
    if (split) {
      HIPCHK(hipEventRecord(c->ev_k2[b], sd));
      HIPCHK(hipStreamWaitEvent(sx, c->ev_k2[b], 0));
    }

    fmcw::DetectArgs ka{};
    ka.profile = d_prof + f0 * NR;
    ka.rd = rd; ka.rd_dtype = rd_dt;
    ka.cube = cube; ka.cube_dtype = cube_dt;
    ka.cube_unscale = 1.0f / cube_scale; ka.rd_unscale = 1.0f / rd_scale;
    ka.nframes = (int)nf; ka.NR = NR; ka.ND = ND; ka.C = C; ka.M = M;
    ka.range_thr = p->range_thr; ka.doppler_thr = p->doppler_thr;
    ka.min_d = p->min_d; ka.max_d = p->max_d; ka.dist_per_bin = p->dist_per_bin;
    ka.fallback = p->doppler_fallback_idx;
    ka.count = d_count + f0;
    ka.ridx = d_ridx + f0 * M;
    ka.rmag = d_rmag + f0 * M;
    ka.didx = d_didx + f0 * M;
    ka.slow_mag = d_slow + f0 * C;
    ka.probe_frame = (pframe >= f0 && pframe < f0 + nf) ? pframe - f0 : -1;
    ka.probe_chirp = pchirp;
    ka.probe_mag = d_probe;
    {
      StageTimer tm(c, 2, sx, 2);
      HIPCHK(fmcw::launch_detect(ka, sx));
      tm.done();
    }
    if (split) HIPCHK(hipEventRecord(c->ev_k3[b], sx));
  }
  span.s = sd;
  span.done();
  // join: the caller's stream waits for the last detect (which follows every K2)
  if (split) {
    HIPCHK(hipEventRecord(c->ev_join, sx));
    HIPCHK(hipStreamWaitEvent(s, c->ev_join, 0));
  }
  if (leg) {   // the streams schedule: the slow-time leg's start as launches of its own
    HIPCHK(fmcw::launch_compact(d_count, F, C, leg->list, leg->len, s));
    if (leg->pmax) HIPCHK(hipMemsetAsync(leg->pmax, 0, 4, s));
  }
  return FMCW_OK;
}

int fmcw_range_fft_device(fmcw_ctx* c, const fmcw_params* p, const void* d_iq, int32_t in_dtype, int64_t F,
                          void* d_cube, int32_t out_dtype, float* d_prof, void* stream) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (F == 0) return FMCW_OK;
  if (!d_iq || !d_cube || !d_prof) return fail(FMCW_E_ARG, "required device pointer is NULL");
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  if (out_dtype != FMCW_C64 && out_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad out_dtype");
  hipStream_t s = pick(c, stream);
  HIPCHK(hipMemsetAsync(d_prof, 0, (size_t)F * p->nr * 4, s));   // 0.0f: identity of max over |.|
  fmcw::RangeArgs ra{};
  ra.iq = d_iq; ra.in_dtype = in_dtype;
  ra.nchirps = F * p->pn;
  ra.C = p->pn; ra.S = p->nts; ra.NR = p->nr;
  ra.calw = c->calw.as<float4>(); ra.cal_sum = c->cal_sum; ra.if_scale = p->if_scale;
  ra.tw = c->tw_nr.as<float2>();
  ra.cube = d_cube; ra.cube_dtype = out_dtype;
  ra.cube_scale = out_dtype == FMCW_C32H ? 1.0f / p->nr : 1.0f;
  ra.profile = d_prof;
  int cpt = 8;      // config 2: 2 workgroups per frame (771-782 us vs 786-787 at 16; profiles/r04_k1_profile_combine.txt)
  if (const char* e = std::getenv("FMCW_K1_CPT")) cpt = std::max(1, std::min(64, std::atoi(e)));   // A/B
  while (cpt > 1 && (p->pn % cpt) != 0) cpt >>= 1;
  ra.cpt = cpt;
  // workgroups of TEAMS teams x cpt chirps: when several share a frame evenly, their profile
  // maxima go to per-workgroup slots (plain stores) and one reduction pass forms the profile
  const int T = p->nr >= 16 ? p->nr / 16 : 1;
  const int teams = T >= 256 ? 1 : 256 / T;
  const int64_t per_wg = (int64_t)teams * cpt;
  ra.parts = (per_wg < p->pn && p->pn % per_wg == 0) ? (int)(p->pn / per_wg) : 0;
  if (ra.parts > 1) {
    int st = FMCW_OK;
    ra.prof_part = static_cast<float*>(c->k1_part.get(s, (size_t)F * ra.parts * p->nr * 4, &st));
    CHK(st);
  }
  StageTimer tm(c, 6, s);
  HIPCHK(fmcw::launch_range(ra, s));
  if (ra.parts > 1) {
    HIPCHK(fmcw::launch_profile_reduce(ra.prof_part, ra.parts, F, p->nr, d_prof, s));
    CHK(c->k1_part.done(s));
  }
  tm.done();
  return FMCW_OK;
}

// ---------------------------------------------------------------------------
// slow time + STFT
// ---------------------------------------------------------------------------
int fmcw_compact_device(fmcw_ctx* c, const int32_t* d_count, int64_t F, int32_t pn, int32_t* d_list,
                        int64_t* d_len, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (F < 0 || pn < 1) return fail(FMCW_E_ARG, "bad F / pn");
  if (!d_count || !d_list || !d_len) return fail(FMCW_E_ARG, "NULL device pointer");
  CHK(set_device(c));
  hipStream_t s = pick(c, stream);
  StageTimer tm(c, 3, s);
  HIPCHK(fmcw::launch_compact(d_count, F, pn, d_list, d_len, s));
  tm.done();
  return FMCW_OK;
}

static int check_stft_shape(int32_t wlen, int32_t noverlap, int32_t nfft) {
  if (wlen < 1 || wlen > 256) return fail(FMCW_E_ARG, "wlen must be in [1, 256]");
  if (noverlap < 0 || noverlap >= wlen) return fail(FMCW_E_ARG, "noverlap must be in [0, wlen)");
  if (nfft < wlen || (nfft % 2) != 0) return fail(FMCW_E_ARG, "nfft must be even and >= wlen");
  return FMCW_OK;
}

int fmcw_stft_power_device(fmcw_ctx* c, const float* d_slow, const int32_t* d_list, const int64_t* d_len,
                           int32_t pn, const float* d_halo, int32_t n_halo, const int64_t* d_halo_len,
                           const float* d_win, int32_t wlen,
                           int32_t noverlap, int32_t nfft, double fs, int64_t max_seg, float* d_P, float* d_pmax,
                           int64_t* d_nseg, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(check_stft_shape(wlen, noverlap, nfft));
  if (pn < 1 || n_halo < 0 || max_seg < 0 || !(fs > 0)) return fail(FMCW_E_ARG, "bad pn / n_halo / max_seg / fs");
  if (!d_slow || !d_list || !d_len || !d_win || !d_pmax || !d_nseg || (n_halo > 0 && !d_halo))
    return fail(FMCW_E_ARG, "NULL device pointer");   // d_P may be NULL: max(P) only
  // the shard split of the slow-time signal (dist.py) starts every shard's segment grid at its own
  // sample 0 and takes wlen-1 samples of right halo: that is the global grid only for hop 1
  if (n_halo > 0 && wlen - noverlap != 1)
    return fail(FMCW_E_ARG, "a halo (sharded STFT) needs hop 1, i.e. noverlap = wlen - 1");
  CHK(set_device(c));
  hipStream_t s = pick(c, stream);
  fmcw::StftArgs a{};
  a.slow_mag = d_slow; a.frame_list = d_list; a.len = d_len; a.pn = pn;
  a.halo = d_halo; a.n_halo = n_halo; a.halo_len = d_halo_len;
  a.win = d_win; a.wlen = wlen; a.hop = wlen - noverlap; a.nfft = nfft;
  a.inv_fs = (float)(1.0 / fs);
  a.max_seg = max_seg; a.P = d_P; a.pmax = d_pmax; a.nseg_out = d_nseg;
  StageTimer tm(c, 4, s);
  if (fmcw::stft_fast_path(wlen, a.hop)) {        // the reference's 20-tap window: W table + k_stft20
    int st = FMCW_OK;
    bool build = true;
    float2* tab = fmcw::stft64_form(nfft) ? c->stft_tab64(s, d_win, nfft, &build, &st)
                                          : c->stft_tab(s, (size_t)(nfft / 2 + 1) * 20 * 8, &st);
    CHK(st);
    if (build) HIPCHK(fmcw::launch_stft_table(d_win, nfft, tab, s));
    // device API: d_P is the caller's [max_seg][nfft/2+1] (fmcw.h), the table this stream's
    HIPCHK(fmcw::launch_stft20(a, tab, d_P ? 0 : 1, nullptr, s, max_seg * (int64_t)(nfft / 2 + 1),
                               (int64_t)(nfft / 2 + 1) * 20));
    CHK(c->stft_tab_done(s));
  } else {
    HIPCHK(fmcw::launch_stft_power(a, s));
  }
  tm.done();
  return FMCW_OK;
}

int fmcw_stft_db_direct_device(fmcw_ctx* c, const float* d_slow, const int32_t* d_list, const int64_t* d_len,
                               int32_t pn, const float* d_halo, int32_t n_halo, const int64_t* d_halo_len,
                               const float* d_win, int32_t wlen, int32_t noverlap, int32_t nfft, double fs,
                               int64_t max_seg, const float* d_pmax, float* d_out, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  CHK(check_stft_shape(wlen, noverlap, nfft));
  if (pn < 1 || n_halo < 0 || max_seg < 0 || !(fs > 0)) return fail(FMCW_E_ARG, "bad pn / n_halo / max_seg / fs");
  if (!d_slow || !d_list || !d_len || !d_win || !d_pmax || !d_out || (n_halo > 0 && !d_halo))
    return fail(FMCW_E_ARG, "NULL device pointer");
  if (!fmcw::stft_fast_path(wlen, wlen - noverlap))
    return fail(FMCW_E_ARG, "the direct dB STFT needs the 20-tap window and hop <= 4");
  if (n_halo > 0 && wlen - noverlap != 1)
    return fail(FMCW_E_ARG, "a halo (sharded STFT) needs hop 1, i.e. noverlap = wlen - 1");
  CHK(set_device(c));
  hipStream_t s = pick(c, stream);
  fmcw::StftArgs a{};
  a.slow_mag = d_slow; a.frame_list = d_list; a.len = d_len; a.pn = pn;
  a.halo = d_halo; a.n_halo = n_halo; a.halo_len = d_halo_len;
  a.win = d_win; a.wlen = wlen; a.hop = wlen - noverlap; a.nfft = nfft;
  a.inv_fs = (float)(1.0 / fs);
  a.max_seg = max_seg; a.P = nullptr; a.pmax = const_cast<float*>(d_pmax); a.nseg_out = nullptr;
  StageTimer tm(c, 5, s);
  int st = FMCW_OK;
  bool build = true;
  float2* tab = fmcw::stft64_form(nfft) ? c->stft_tab64(s, d_win, nfft, &build, &st)
                                        : c->stft_tab(s, (size_t)(nfft / 2 + 1) * 20 * 8, &st);
  CHK(st);
  if (build) HIPCHK(fmcw::launch_stft_table(d_win, nfft, tab, s));
  HIPCHK(fmcw::launch_stft20(a, tab, 2, d_out, s, max_seg * (int64_t)(nfft / 2 + 1), (int64_t)(nfft / 2 + 1) * 20));
  CHK(c->stft_tab_done(s));
  tm.done();
  return FMCW_OK;
}

// logspace(log10(fs/nfft), log10(fs/2), n) located on F = (0:nfft/2)*fs/nfft
static void log_table(int nfft, double fs, int n, std::vector<int32_t>& idx, std::vector<float>& wt,
                      std::vector<double>* fq_out) {
  const int nb = nfft / 2 + 1;
  const double df = fs / nfft;
  const double a = std::log10(df), b = std::log10((nb - 1) * df);
  idx.resize(n);
  wt.resize(n);
  if (fq_out) fq_out->resize(n);
  for (int j = 0; j < n; ++j) {
    const double e = (n == 1) ? b : (j == n - 1 ? b : a + j * (b - a) / (n - 1));
    const double fq = std::pow(10.0, e);
    int i0 = (int)std::floor(fq / df);
    if (i0 < 0) i0 = 0;
    if (i0 > nb - 2) i0 = nb - 2;
    idx[j] = i0;
    wt[j] = (float)((fq - i0 * df) / df);
    if (fq_out) (*fq_out)[j] = fq;
  }
}

int fmcw_stft_db_device(fmcw_ctx* c, const float* d_P, const int64_t* d_nseg, int64_t max_seg, int32_t nfft,
                        double fs, const float* d_pmax, int32_t n_log_bins, float* d_out, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (nfft < 2 || (nfft % 2) != 0 || n_log_bins < 0 || max_seg < 0 || !(fs > 0))
    return fail(FMCW_E_ARG, "bad nfft / n_log_bins / max_seg / fs");
  if (!d_P || !d_nseg || !d_pmax || !d_out) return fail(FMCW_E_ARG, "NULL device pointer");
  if (n_log_bins > 0 && d_out == d_P) return fail(FMCW_E_ARG, "d_out may alias d_P only without resampling");
  CHK(set_device(c));
  hipStream_t s = pick(c, stream);
  if (n_log_bins > 0) {
    std::vector<int32_t> idx;
    std::vector<float> wt;
    log_table(nfft, fs, n_log_bins, idx, wt, nullptr);
    CHK(c->s_lidx.ensure(idx.size() * 4));
    CHK(c->s_lw.ensure(wt.size() * 4));
    HIPCHK(hipMemcpyAsync(c->s_lidx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->s_lw.p, wt.data(), wt.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));   // host vectors go out of scope
  }
  fmcw::StftDbArgs a{};
  a.P = d_P; a.nseg = d_nseg; a.max_seg = max_seg; a.nbins_in = nfft / 2 + 1;
  a.pmax = d_pmax; a.nlog = n_log_bins;
  a.lidx = n_log_bins > 0 ? c->s_lidx.as<int32_t>() : nullptr;
  a.lw = n_log_bins > 0 ? c->s_lw.as<float>() : nullptr;
  a.out = d_out;
  StageTimer tm(c, 5, s);
  HIPCHK(fmcw::launch_stft_db(a, s));
  tm.done();
  return FMCW_OK;
}

int fmcw_stft_sizes(int64_t L, int32_t wlen, int32_t noverlap, int32_t nfft, int32_t n_log_bins, int64_t* nseg,
                    int32_t* nfft_used, int32_t* nbins_out) {
  if (L < 0 || n_log_bins < 0) return fail(FMCW_E_ARG, "L < 0 or n_log_bins < 0");
  int32_t nf = nfft;
  if (nf == 0) {                       // :273 nfft_stft = 2^nextpow2(length(iq_data(:)))
    int64_t v = 1;
    while (v < L) v <<= 1;
    if (v > (1 << 26)) return fail(FMCW_E_ARG, "2^nextpow2(L) too large");
    nf = (int32_t)v;
  }
  if (wlen < 1 || noverlap < 0 || noverlap >= wlen) return fail(FMCW_E_ARG, "need 0 <= noverlap < wlen");
  const int hop = wlen - noverlap;
  const int64_t ns = (L - noverlap) >= 0 ? (L - noverlap) / hop : 0;   // fix((nx-noverlap)/(nwind-noverlap))
  if (nseg) *nseg = ns;
  if (nfft_used) *nfft_used = nf;
  if (nbins_out) *nbins_out = n_log_bins > 0 ? n_log_bins : nf / 2 + 1;
  if (ns < 1) return fail(FMCW_E_DATA, "spectrogram: signal length " + std::to_string(L) + " is shorter than the window");
  CHK(check_stft_shape(wlen, noverlap, nf));
  return FMCW_OK;
}

int fmcw_render_spectrogram_device(fmcw_ctx* c, const float* d_Q, int32_t nq, const int64_t* d_nseg,
                                   const float* d_pmax, int32_t nfft, double fs, double t0, double dt, int32_t width,
                                   int32_t height, uint8_t* d_img, void* stream) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if (!d_Q || !d_nseg || !d_pmax || !d_img) return fail(FMCW_E_ARG, "NULL device pointer");
  if (nfft < 2 || (nfft % 2) != 0 || nq < 1 || nq > nfft / 2 || !(fs > 0) || !(dt > 0))
    return fail(FMCW_E_ARG, "bad nfft / nq / fs / dt");
  if (width < 1 || height < 1 || width > 65536 || height > 65535) return fail(FMCW_E_ARG, "bad image size");
  CHK(set_device(c));
  fmcw::RenderArgs a{};
  a.Q = d_Q; a.nq = nq; a.nseg = d_nseg; a.pmax = d_pmax;
  a.nb = nfft / 2 + 1; a.nfft = nfft; a.seam = a.nb - a.nb / 2 - 1;
  a.fs = fs; a.t0 = t0; a.dt = dt;
  a.fmax = FMCW_PNG_FMAX_HZ; a.cmin = FMCW_PNG_CMIN_DB; a.cmax = FMCW_PNG_CMAX_DB;
  a.W = width; a.H = height; a.img = d_img;
  hipStream_t s = pick(c, stream);
  StageTimer tm(c, 9, s);
  HIPCHK(fmcw::launch_render(a, s));
  tm.done();
  return FMCW_OK;
}

static int stft_impl(fmcw_ctx* c, const float* x, int64_t L, const float* win, int32_t wlen, int32_t noverlap,
                     int32_t nfft, double fs, int32_t n_log_bins, float* T, float* freq, float* intensity,
                     const char* png_path, int32_t width, int32_t height, int64_t* png_bytes);

int fmcw_stft(fmcw_ctx* c, const float* x, int64_t L, const float* win, int32_t wlen, int32_t noverlap, int32_t nfft,
              double fs, int32_t n_log_bins, float* T, float* freq, float* intensity) {
  return stft_impl(c, x, L, win, wlen, noverlap, nfft, fs, n_log_bins, T, freq, intensity, nullptr, 0, 0, nullptr);
}

int fmcw_stft_png(fmcw_ctx* c, const float* x, int64_t L, const float* win, int32_t wlen, int32_t noverlap,
                  int32_t nfft, double fs, int32_t n_log_bins, float* T, float* freq, float* intensity,
                  const char* png_path, int32_t width, int32_t height, int64_t* png_bytes) {
  if (!png_path) return fail(FMCW_E_ARG, "png_path is NULL");
  return stft_impl(c, x, L, win, wlen, noverlap, nfft, fs, n_log_bins, T, freq, intensity, png_path,
                   width > 0 ? width : FMCW_PNG_DEFAULT_W, height > 0 ? height : FMCW_PNG_DEFAULT_H, png_bytes);
}

// A large device -> pageable-host copy on stream s, through the two pinned out slots of the
// context: the DMA of piece i overlaps the host threads copying piece i-1 to the caller (and
// taking its first-touch page faults in parallel). Returns once dst holds every byte.
static int d2h_big(fmcw_ctx* c, void* dst, const void* d_src, size_t bytes, hipStream_t s) {
  constexpr size_t kPiece = 32u << 20;
  if (bytes < 2 * kPiece) {
    HIPCHK(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return FMCW_OK;
  }
  CHK(c->pin_out.ensure(2 * kPiece));
  const size_t n = (bytes + kPiece - 1) / kPiece;
  auto piece = [&](size_t i) { return std::min(kPiece, bytes - i * kPiece); };
  for (size_t i = 0; i <= n; ++i) {
    if (i < n) {
      const int b = (int)(i & 1);
      HIPCHK(hipMemcpyAsync(c->pin_out.at(b * kPiece), static_cast<const char*>(d_src) + i * kPiece, piece(i),
                            hipMemcpyDeviceToHost, s));
      HIPCHK(hipEventRecord(c->ev_d2h[b], s));
    }
    if (i >= 1) {   // piece i-1 is in its pinned slot once its event fires; slot (i-1)&1 is reused by piece i+1
      const int b = (int)((i - 1) & 1);
      HIPCHK(hipEventSynchronize(c->ev_d2h[b]));
      par_memcpy(static_cast<char*>(dst) + (i - 1) * kPiece, c->pin_out.at(b * kPiece), piece(i - 1));
    }
  }
  return FMCW_OK;
}

// max(P) of :282-283 over every bin of a large nfft without evaluating every bin of every segment.
// |X_s(w)| of a 20-tap segment is a trigonometric polynomial of degree 19, so (Bernstein) within one
// coarse step h = 2 pi / K of its peak it is at least (1 - 19 h) of the peak.  Pass 1 takes each
// segment's max over the coarse bins k = m nfft / K (exact P values of the fine grid, so their
// maximum G is a lower bound of max(P)); a segment whose coarse max is below G (1 - 19 h)^2 cannot
// hold max(P).  Pass 2 takes the max over every bin of the 256-segment tiles that hold a
// candidate: the same P values the full pass would compare, so the result is the same bits.
static int stft_coarse_max(fmcw_ctx* d, const fmcw::StftArgs& a0, hipStream_t s) {
  // The bound below holds for the 20-tap window only (a degree-19 trigonometric polynomial per
  // segment; any sign of the samples) and for a power-of-two nfft of at least 2^16, so that the
  // coarse grid (every D-th bin) holds DC, Nyquist and an interior bin within h of any peak.
  if (!fmcw::stft_fast_path(a0.wlen, a0.hop)) return fail(FMCW_E_ARG, "stft_coarse_max: not the 20-tap fast path");
  if (a0.nfft < (1 << 16) || (a0.nfft & (a0.nfft - 1))) return fail(FMCW_E_ARG, "stft_coarse_max: nfft must be a power of two >= 2^16");
  const int nf = a0.nfft, K = std::min(16384, nf / 8), D = nf / K, nc = K / 2 + 1;   // nf >= 2^16
  const int64_t ns = a0.max_seg;
  if (ns < 1 || ns > 0x7fffffffLL) return fail(FMCW_E_ARG, "stft_coarse_max: bad segment count");
  std::vector<int32_t> cb(nc);
  for (int m = 0; m < nc; ++m) cb[m] = D * m;
  CHK(d->s_cbins.ensure((size_t)nc * 4));
  CHK(d->s_segmax.ensure((size_t)ns * 4));
  int st = FMCW_OK;
  float2* tab = d->stft_tab(s, (size_t)(nf / 2 + 1) * 20 * 8, &st);
  CHK(st);
  HIPCHK(hipMemcpyAsync(d->s_cbins.p, cb.data(), (size_t)nc * 4, hipMemcpyHostToDevice, s));
  HIPCHK(fmcw::launch_stft_table(a0.win, nf, tab, s));
  fmcw::StftArgs a = a0;
  a.bins = d->s_cbins.as<int32_t>();
  a.ncol = nc;
  // mode 4 writes one float per segment: s_segmax holds ns (launch_stft20 checks the capacity)
  HIPCHK(fmcw::launch_stft20(a, tab, 4, d->s_segmax.as<float>(), s, (int64_t)(d->s_segmax.n / 4),
                             (int64_t)(nf / 2 + 1) * 20));
  std::vector<float> sm((size_t)ns);
  HIPCHK(hipMemcpyAsync(sm.data(), d->s_segmax.p, (size_t)ns * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float G = 0.f;
  for (float v : sm) G = std::max(G, v);
  const double f = 1.0 - (double)(a0.wlen - 1) * 2.0 * M_PI / K;   // degree wlen - 1 (the 20-tap fast path)
  const float thr = (float)((double)G * f * f * (1.0 - 1e-3));   // margin for the fp32 rounding of P
  std::vector<int32_t> tiles;
  for (int64_t t = 0; t * 256 < ns; ++t) {
    const int64_t e = std::min<int64_t>(ns, (t + 1) * 256);
    for (int64_t i = t * 256; i < e; ++i)
      if (sm[(size_t)i] >= thr) { tiles.push_back((int32_t)t); break; }
  }
  CHK(d->s_tiles.ensure(tiles.size() * 4));
  HIPCHK(hipMemcpyAsync(d->s_tiles.p, tiles.data(), tiles.size() * 4, hipMemcpyHostToDevice, s));
  a = a0;
  a.tiles = d->s_tiles.as<int32_t>();
  a.ntiles = (int)tiles.size();
  HIPCHK(fmcw::launch_stft20(a, tab, 1, nullptr, s, 0, (int64_t)(nf / 2 + 1) * 20));
  CHK(d->stft_tab_done(s));
  HIPCHK(hipStreamSynchronize(s));   // tiles / cb leave scope
  d->last_coarse_tiles = (int64_t)tiles.size();
  if (const char* e = std::getenv("FMCW_STFT_DEBUG"); e && e[0] == '1')
    std::fprintf(stderr, "stft_coarse_max: nfft %d, %lld segments, %zu of %lld tiles in full\n", nf, (long long)ns,
                 tiles.size(), (long long)((ns + 255) / 256));
  return FMCW_OK;
}

static int stft_impl(fmcw_ctx* c, const float* x, int64_t L, const float* win, int32_t wlen, int32_t noverlap,
                     int32_t nfft, double fs, int32_t n_log_bins, float* T, float* freq, float* intensity,
                     const char* png_path, int32_t width, int32_t height, int64_t* png_bytes) {
  if (!c) return fail(FMCW_E_ARG, "ctx is NULL");
  if ((!x && L > 0) || !win || !T || !freq || !intensity) return fail(FMCW_E_ARG, "NULL pointer");
  if (!(fs > 0)) return fail(FMCW_E_ARG, "fs must be > 0");
  if (L > 0x7fffffffLL) return fail(FMCW_E_ARG, "L too large for the host API");
  int64_t nseg = 0;
  int32_t nf = 0, nbo = 0;
  CHK(fmcw_stft_sizes(L, wlen, noverlap, nfft, n_log_bins, &nseg, &nf, &nbo));   // nfft rule on the whole signal
  const int hop = wlen - noverlap;
  const int nb = nf / 2 + 1;
  const int world = 1 + (int)c->peers.size();
  auto dev = [&](int g) { return g == 0 ? c : c->peers[g - 1]; };
  const double df = fs / nf;
  const int nq = png_path ? (int)std::min<int64_t>(nb - 1, (int64_t)std::floor(FMCW_PNG_FMAX_HZ / df) + 2) : 0;
  // With the log-frequency output (:286-299) and the 20-tap window, P is formed only for the
  // bins interp1 and the picture read: a max(P)-only pass over every bin, then those columns
  // ([seg][ncolP], ascending bins). Otherwise every bin ([seg][nb]).
  const bool sel_mode = n_log_bins > 0 && fmcw::stft_fast_path(wlen, hop);
  std::vector<int32_t> bins, lidx;
  std::vector<float> lw;
  if (sel_mode) {
    log_table(nf, fs, n_log_bins, lidx, lw, nullptr);
    std::vector<int32_t> pos(nb, 0);
    for (int32_t i0 : lidx) pos[i0] = pos[i0 + 1] = 1;
    for (int k = 0; k < nq; ++k) pos[k] = 1;
    if (png_path) pos[nb - 1] = 1;
    for (int k = 0; k < nb; ++k)
      if (pos[k]) { pos[k] = (int32_t)bins.size(); bins.push_back(k); }
    for (auto& i0 : lidx) i0 = pos[i0];   // i0 and i0+1 are both listed, so they are adjacent columns
  }
  const int ncolP = sel_mode ? (int)bins.size() : nb;
  // per device, the call's inputs (its samples, the one-entry frame list, the length, the window,
  // the listed bins and the interp1 table) in one arena: one pinned H2D copy instead of seven
  struct InOff { size_t x, list, len, win, bins, lidx, lw; };
  std::vector<InOff> io(world);
  // Segments are sharded contiguously over the devices; device g takes the
  // samples its segments cover (its halo is simply the next samples of x).
  // 1) P and the local max(P) per device
  for (int g = 0; g < world; ++g) {
    fmcw_ctx* d = dev(g);
    int64_t s0, ns;
    shard(nseg, g, world, s0, ns);
    CHK(set_device(d));
    hipStream_t s = d->stream;
    const int64_t Ld = ns > 0 ? (ns - 1) * hop + wlen : 0;
    CHK(d->s_P.ensure((size_t)std::max<int64_t>(ns, 1) * ncolP * 4));
    CHK(d->s_pmax.ensure(4));
    CHK(d->s_nseg.ensure(8));
    CHK(d->s_out.ensure((size_t)std::max<int64_t>(ns, 1) * nbo * 4));
    HIPCHK(hipMemsetAsync(d->s_pmax.p, 0, 4, s));
    if (ns == 0) continue;
    Arena ar;
    InOff& o = io[g];
    o.x = ar.add((size_t)Ld * 4); o.list = ar.add(4); o.len = ar.add(8); o.win = ar.add((size_t)wlen * 4);
    o.bins = ar.add(bins.size() * 4); o.lidx = ar.add(lidx.size() * 4); o.lw = ar.add(lw.size() * 4);
    CHK(d->s_in.ensure(ar.off));
    CHK(d->pin_sin.ensure(ar.off));
    {
      char* h = d->pin_sin.at(0);
      par_memcpy(h + o.x, x + s0 * hop, (size_t)Ld * 4);
      const int32_t zero = 0;
      std::memcpy(h + o.list, &zero, 4);
      std::memcpy(h + o.len, &Ld, 8);
      std::memcpy(h + o.win, win, (size_t)wlen * 4);
      if (!bins.empty()) std::memcpy(h + o.bins, bins.data(), bins.size() * 4);
      if (!lidx.empty()) std::memcpy(h + o.lidx, lidx.data(), lidx.size() * 4);
      if (!lw.empty()) std::memcpy(h + o.lw, lw.data(), lw.size() * 4);
    }
    HIPCHK(hipMemcpyAsync(d->s_in.p, d->pin_sin.p, ar.off, hipMemcpyHostToDevice, s));
    char* const di = d->s_in.as<char>();
    float* const d_x = reinterpret_cast<float*>(di + o.x);
    int32_t* const d_list = reinterpret_cast<int32_t*>(di + o.list);
    int64_t* const d_len = reinterpret_cast<int64_t*>(di + o.len);
    float* const d_win = reinterpret_cast<float*>(di + o.win);
    // the shard's samples are one "frame" of Ld samples in the compaction indirection
    const char* ce = std::getenv("FMCW_STFT_COARSE");   // 0: every bin of every segment (tests, A/B)
    const char* me = std::getenv("FMCW_STFT_MFMA");
    const bool coarse_ok = !(ce && ce[0] == '0') && !(me && me[0] == '0');
    if (sel_mode && coarse_ok && nf >= (1 << 16)) {   // max(P) only, over a large nfft: coarse-to-fine
      fmcw::StftArgs a{};
      a.slow_mag = d_x; a.frame_list = d_list; a.len = d_len; a.pn = (int32_t)Ld;
      a.win = d_win; a.wlen = wlen; a.hop = hop; a.nfft = nf; a.inv_fs = (float)(1.0 / fs);
      a.max_seg = ns; a.P = nullptr; a.pmax = d->s_pmax.as<float>(); a.nseg_out = d->s_nseg.as<int64_t>();
      StageTimer tm(d, 4, s);
      CHK(stft_coarse_max(d, a, s));
      tm.done();
    } else if (sel_mode) {   // max(P) only, in the table form the listed-bins pass below uses (at nfft 64
                             // too: P / max(P) of the listed bins then peaks at exactly 0 dB, as in MATLAB)
      fmcw::StftArgs a{};
      a.slow_mag = d_x; a.frame_list = d_list; a.len = d_len; a.pn = (int32_t)Ld;
      a.win = d_win; a.wlen = wlen; a.hop = hop; a.nfft = nf; a.inv_fs = (float)(1.0 / fs);
      a.max_seg = ns; a.P = nullptr; a.pmax = d->s_pmax.as<float>(); a.nseg_out = d->s_nseg.as<int64_t>();
      a.table_form = 1;
      StageTimer tm(d, 4, s);
      int st = FMCW_OK;
      float2* tab = d->stft_tab(s, (size_t)(nf / 2 + 1) * 20 * 8, &st);
      CHK(st);
      HIPCHK(fmcw::launch_stft_table(d_win, nf, tab, s));
      HIPCHK(fmcw::launch_stft20(a, tab, 1, nullptr, s, 0, (int64_t)(nf / 2 + 1) * 20));
      CHK(d->stft_tab_done(s));
      tm.done();
    } else {
      CHK(fmcw_stft_power_device(d, d_x, d_list, d_len, (int32_t)Ld, nullptr, 0, nullptr, d_win, wlen, noverlap, nf, fs, ns,
                                 d->s_P.as<float>(), d->s_pmax.as<float>(), d->s_nseg.as<int64_t>(), s));
    }
    if (sel_mode) {   // second pass: P of the listed bins (the W table the first pass built on s is reused)
      fmcw::StftArgs a{};
      a.slow_mag = d_x; a.frame_list = d_list; a.len = d_len;
      a.pn = (int32_t)Ld; a.win = d_win; a.wlen = wlen; a.hop = hop; a.nfft = nf;
      a.inv_fs = (float)(1.0 / fs); a.max_seg = ns; a.bins = reinterpret_cast<int32_t*>(di + o.bins); a.ncol = ncolP;
      StageTimer tm(d, 4, s);
      int st = FMCW_OK;
      float2* tab = d->stft_tab(s, (size_t)(nf / 2 + 1) * 20 * 8, &st);   // the first pass's table on s (both
      CHK(st);                                                             // first-pass forms built it for d_win)
      HIPCHK(fmcw::launch_stft20(a, tab, 3, d->s_P.as<float>(), s, (int64_t)(d->s_P.n / 4), (int64_t)(nf / 2 + 1) * 20));
      CHK(d->stft_tab_done(s));
      tm.done();
    }
    if (world > 1) HIPCHK(hipStreamSynchronize(s));   // local max(P) final (step 2 may read it through the host)
  }
  // 2) the global max(P) of :282-283: RCCL all_reduce(max) across the devices
  if (world > 1) {
    if (!c->comms.empty()) {
      NCCLCHK(rccl().group_start());
      for (int g = 0; g < world; ++g) {
        fmcw_ctx* d = dev(g);
        CHK(set_device(d));
        NCCLCHK(rccl().all_reduce(d->s_pmax.p, d->s_pmax.p, 1, ncclFloat32, ncclMax, c->comms[g], d->stream));
      }
      NCCLCHK(rccl().group_end());
    } else {   // several contexts on ONE device (no communicator can span them): 4 bytes through the host
      float m = 0.f;
      for (int g = 0; g < world; ++g) {
        float v = 0.f;
        CHK(set_device(dev(g)));
        HIPCHK(hipMemcpy(&v, dev(g)->s_pmax.p, 4, hipMemcpyDeviceToHost));
        m = std::max(m, v);
      }
      for (int g = 0; g < world; ++g) {
        CHK(set_device(dev(g)));
        HIPCHK(hipMemcpy(dev(g)->s_pmax.p, &m, 4, hipMemcpyHostToDevice));
      }
    }
  }
  // 2b) spectrogram.png (:331-348) from the linear-bin P before it is overwritten:
  //     the bins below ylim plus the Nyquist bin of every segment, gathered to device 0
  std::vector<uint8_t> img;
  if (png_path) {
    std::vector<float> q((size_t)std::max<int64_t>(nseg, 1) * (nq + 1));
    for (int g = 0; g < world; ++g) {
      fmcw_ctx* d = dev(g);
      int64_t s0, ns;
      shard(nseg, g, world, s0, ns);
      if (ns == 0) continue;
      CHK(set_device(d));
      // bins 0..nq-1 are the first nq columns of P and the Nyquist bin its last, in both layouts
      HIPCHK(hipMemcpy2DAsync(q.data() + s0 * (nq + 1), (nq + 1) * 4, d->s_P.p, (size_t)ncolP * 4, (size_t)nq * 4, ns,
                              hipMemcpyDeviceToHost, d->stream));
      HIPCHK(hipMemcpy2DAsync(q.data() + s0 * (nq + 1) + nq, (nq + 1) * 4, d->s_P.as<float>() + (ncolP - 1),
                              (size_t)ncolP * 4, 4, ns, hipMemcpyDeviceToHost, d->stream));
    }
    for (int g = 0; g < world; ++g) {
      CHK(set_device(dev(g)));
      HIPCHK(hipStreamSynchronize(dev(g)->stream));
    }
    CHK(set_device(c));
    hipStream_t s = c->stream;
    CHK(c->r_q.ensure(q.size() * 4));
    CHK(c->r_nseg.ensure(8));
    CHK(c->r_img.ensure((size_t)height * (width + 1)));
    HIPCHK(hipMemcpyAsync(c->r_q.p, q.data(), q.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->r_nseg.p, &nseg, 8, hipMemcpyHostToDevice, s));
    CHK(fmcw_render_spectrogram_device(c, c->r_q.as<float>(), nq, c->r_nseg.as<int64_t>(), c->s_pmax.as<float>(), nf, fs,
                                       (wlen / 2.0) / fs, hop / fs, width, height, c->r_img.as<uint8_t>(), s));
    img.resize((size_t)height * (width + 1));
    HIPCHK(hipMemcpyAsync(img.data(), c->r_img.p, img.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  // 3) dB (+ log-frequency resampling) and the rows back into intensity
  for (int g = 0; g < world; ++g) {
    fmcw_ctx* d = dev(g);
    int64_t s0, ns;
    shard(nseg, g, world, s0, ns);
    if (ns == 0) continue;
    CHK(set_device(d));
    hipStream_t s = d->stream;
    if (sel_mode) {   // interp1 over the listed columns (lidx holds column positions; uploaded in step 1)
      fmcw::StftDbArgs a{};
      a.P = d->s_P.as<float>(); a.nseg = d->s_nseg.as<int64_t>(); a.max_seg = ns; a.nbins_in = ncolP;
      a.pmax = d->s_pmax.as<float>(); a.nlog = n_log_bins;
      a.lidx = reinterpret_cast<int32_t*>(d->s_in.as<char>() + io[g].lidx);
      a.lw = reinterpret_cast<float*>(d->s_in.as<char>() + io[g].lw); a.out = d->s_out.as<float>();
      StageTimer tm(d, 5, s);
      HIPCHK(fmcw::launch_stft_db(a, s));
      tm.done();
    } else {
      CHK(fmcw_stft_db_device(d, d->s_P.as<float>(), d->s_nseg.as<int64_t>(), ns, nf, fs, d->s_pmax.as<float>(),
                              n_log_bins, n_log_bins > 0 ? d->s_out.as<float>() : d->s_P.as<float>(), s));
    }
    const float* res = n_log_bins > 0 ? d->s_out.as<float>() : d->s_P.as<float>();
    CHK(d2h_big(d, intensity + s0 * nbo, res, (size_t)ns * nbo * 4, s));
  }
  for (int g = 0; g < world; ++g) {
    CHK(set_device(dev(g)));
    HIPCHK(hipStreamSynchronize(dev(g)->stream));
  }
  if (png_path) CHK(fmcw::png_write_indexed(png_path, img.data(), width, height, 1, 0, png_bytes));
  for (int64_t i = 0; i < nseg; ++i) T[i] = (float)(((double)i * hop + wlen / 2.0) / fs);   // spectrogram T
  if (n_log_bins > 0) {
    std::vector<int32_t> idx;
    std::vector<float> wt;
    std::vector<double> fq;
    log_table(nf, fs, n_log_bins, idx, wt, &fq);
    for (int j = 0; j < n_log_bins; ++j) freq[j] = (float)fq[j];
  } else {
    for (int j = 0; j < nb; ++j) freq[j] = (float)(j * fs / nf);
  }
  return FMCW_OK;
}

// ---------------------------------------------------------------------------
// host-pointer per-frame API
// ---------------------------------------------------------------------------
}  // extern "C"

// Frames per host-path chunk: ~64 MiB of input per slot (FMCW_HOST_CHUNK
// overrides, for tests of the chunk seams).
static int64_t host_chunk(size_t frame_in_bytes, int64_t F) {
  int64_t fc = (int64_t)((64ull << 20) / std::max<size_t>(frame_in_bytes, 1));
  if (const char* e = std::getenv("FMCW_HOST_CHUNK"); e && std::atoll(e) > 0) fc = std::atoll(e);
  return std::max<int64_t>(1, std::min<int64_t>(fc, F));
}

// The host-pointer calls as a two-slot pipeline over chunks of frames:
//   host:  caller's iq chunk i -> pinned slot i%2 (once the H2D of chunk i-2 has left it)
//   cin:   pinned slot -> device slot (after chunk i-2's kernels released the device slot)
//   s:     the device-pointer call on the chunk (small outputs written in place at f0)
//   cout:  the chunk's large outputs (range cube, RD map) -> pinned out slot; the host
//          copies chunk i-2's rows to the caller before that slot is reused
// The small per-frame outputs stay on the device for all F and come back once.
// `run(d_in, f0, nf, d_big[2])` enqueues the device call for one chunk on s.
struct BigOut {
  char* host;        // caller's [F][...] array or nullptr
  size_t fbytes;     // bytes per frame
};
template <typename Run>
static int host_pipeline(fmcw_ctx* c, const void* iq, int64_t F, size_t fin, const BigOut (&big)[2], Run&& run) {
  hipStream_t s = c->stream;
  const int64_t Fc = host_chunk(fin, F);
  const size_t slot_in = (size_t)Fc * fin;
  size_t slot_big[2], off_big[2] = {0, 0}, slot_out = 0;
  bool any = false;
  for (int q = 0; q < 2; ++q) {
    slot_big[q] = big[q].host ? (size_t)Fc * big[q].fbytes : 0;
    off_big[q] = slot_out;
    slot_out += slot_big[q];
    any = any || big[q].host;
  }
  CHK(c->h_iq.ensure(2 * slot_in));
  CHK(c->pin_in.ensure(2 * slot_in));
  if (any) {
    CHK(c->h_rd.ensure(2 * slot_out));
    CHK(c->pin_out.ensure(2 * slot_out));
  }
  const int64_t n = (F + Fc - 1) / Fc;
  auto drain = [&](int64_t j) -> int {          // chunk j's large outputs: pinned slot -> caller
    const int b = (int)(j & 1);
    const int64_t f0 = j * Fc, nf = std::min(Fc, F - f0);
    HIPCHK(hipEventSynchronize(c->ev_d2h[b]));
    for (int q = 0; q < 2; ++q)
      if (big[q].host)
        par_memcpy(big[q].host + (size_t)f0 * big[q].fbytes, c->pin_out.at(b * slot_out + off_big[q]),
                   (size_t)nf * big[q].fbytes);
    return FMCW_OK;
  };
  // one chunk: its H2D copy has nothing to overlap with and goes on s (no fork / join events)
  const bool single = n == 1;
  hipStream_t cin = single ? s : c->cin;
  if (!single) {
    HIPCHK(hipEventRecord(c->ev_fork, s));          // the device buffers are free once earlier work on s is done
    HIPCHK(hipStreamWaitEvent(c->cin, c->ev_fork, 0));
  }
  for (int64_t i = 0; i < n; ++i) {
    const int b = (int)(i & 1);
    const int64_t f0 = i * Fc, nf = std::min(Fc, F - f0);
    if (i >= 2) HIPCHK(hipEventSynchronize(c->ev_h2d[b]));   // pinned slot b: chunk i-2's H2D has read it
    par_memcpy(c->pin_in.at(b * slot_in), static_cast<const char*>(iq) + (size_t)f0 * fin, (size_t)nf * fin);
    if (i >= 2) HIPCHK(hipStreamWaitEvent(c->cin, c->ev_comp[b], 0));   // device slot b: chunk i-2's kernels are done
    HIPCHK(hipMemcpyAsync(c->h_iq.as<char>() + b * slot_in, c->pin_in.at(b * slot_in), (size_t)nf * fin,
                          hipMemcpyHostToDevice, cin));
    if (!single) {
      HIPCHK(hipEventRecord(c->ev_h2d[b], c->cin));
      HIPCHK(hipStreamWaitEvent(s, c->ev_h2d[b], 0));
    }
    if (any && i >= 2) {                          // device out slot b: chunk i-2's D2H has read it
      HIPCHK(hipStreamWaitEvent(s, c->ev_d2h[b], 0));
      CHK(drain(i - 2));                          // and its rows go to the caller (pinned slot b is reused below)
    }
    char* d_big[2];
    for (int q = 0; q < 2; ++q) d_big[q] = big[q].host ? c->h_rd.as<char>() + b * slot_out + off_big[q] : nullptr;
    CHK(run(c->h_iq.as<char>() + b * slot_in, f0, nf, d_big));
    HIPCHK(hipEventRecord(c->ev_comp[b], s));
    if (any) {
      HIPCHK(hipStreamWaitEvent(c->cout, c->ev_comp[b], 0));
      for (int q = 0; q < 2; ++q)
        if (big[q].host)
          HIPCHK(hipMemcpyAsync(c->pin_out.at(b * slot_out + off_big[q]), d_big[q], (size_t)nf * big[q].fbytes,
                                hipMemcpyDeviceToHost, c->cout));
      HIPCHK(hipEventRecord(c->ev_d2h[b], c->cout));
    }
  }
  if (any)
    for (int64_t j = std::max<int64_t>(0, n - 2); j < n; ++j) CHK(drain(j));
  return FMCW_OK;
}

extern "C" {

static int process_host_one(fmcw_ctx* c, const fmcw_params* p, const void* iq, int32_t in_dtype, int64_t F,
                            float* prof, int32_t* count, int32_t* ridx, float* rmag, int32_t* didx, float* slow,
                            float* cube, float* rd, int64_t probe_column, float* probe) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (F == 0) return FMCW_OK;
  if (!iq || !prof || !count || !ridx || !rmag || !didx || !slow) return fail(FMCW_E_ARG, "required pointer is NULL");
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  const int S = p->nts, C = p->pn, NR = p->nr, ND = p->nd, M = p->max_targets;
  hipStream_t s = c->stream;
  // the small outputs in one device arena, back through one pinned copy
  Arena ar;
  const size_t o_prof = ar.add((size_t)F * NR * 4), o_count = ar.add((size_t)F * 4), o_ridx = ar.add((size_t)F * M * 4),
               o_rmag = ar.add((size_t)F * M * 4), o_didx = ar.add((size_t)F * M * 4), o_slow = ar.add((size_t)F * C * 4),
               o_probe = ar.add(probe ? (size_t)NR * 4 : 0);
  CHK(c->h_small.ensure(ar.off));
  CHK(c->pin_small.ensure(ar.off));
  char* const hs = c->h_small.as<char>();
  auto at = [&](size_t o) { return reinterpret_cast<float*>(hs + o); };
  auto ati = [&](size_t o) { return reinterpret_cast<int32_t*>(hs + o); };
  const size_t fin = (size_t)C * S * esize(in_dtype);
  const BigOut big[2] = {{reinterpret_cast<char*>(cube), (size_t)C * NR * 8}, {reinterpret_cast<char*>(rd), (size_t)NR * ND * 8}};
  CHK(host_pipeline(c, iq, F, fin, big, [&](char* d_in, int64_t f0, int64_t nf, char* const* d_big) {
    const int64_t pc = probe && probe_column > f0 * C && probe_column <= (f0 + nf) * C ? probe_column - f0 * C : 0;
    return fmcw_process_device(c, p, d_in, in_dtype, nf, at(o_prof) + f0 * NR, ati(o_count) + f0, ati(o_ridx) + f0 * M,
                               at(o_rmag) + f0 * M, ati(o_didx) + f0 * M, at(o_slow) + f0 * C, d_big[0], d_big[1], FMCW_C64,
                               pc, pc ? at(o_probe) : nullptr, s);
  }));
  HIPCHK(hipMemcpyAsync(c->pin_small.p, hs, ar.off, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipStreamSynchronize(c->cout));
  const char* ps = c->pin_small.at(0);
  par_memcpy(prof, ps + o_prof, (size_t)F * NR * 4);
  std::memcpy(count, ps + o_count, (size_t)F * 4);
  std::memcpy(ridx, ps + o_ridx, (size_t)F * M * 4);
  std::memcpy(rmag, ps + o_rmag, (size_t)F * M * 4);
  std::memcpy(didx, ps + o_didx, (size_t)F * M * 4);
  par_memcpy(slow, ps + o_slow, (size_t)F * C * 4);
  if (probe) std::memcpy(probe, ps + o_probe, (size_t)NR * 4);
  return xcd_check(c);
}

static int range_fft_host_one(fmcw_ctx* c, const fmcw_params* p, const void* iq, int32_t in_dtype, int64_t F,
                              float* cube, float* prof) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (F == 0) return FMCW_OK;
  if (!iq || !cube || !prof) return fail(FMCW_E_ARG, "required pointer is NULL");
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  const int S = p->nts, C = p->pn, NR = p->nr;
  hipStream_t s = c->stream;
  CHK(c->h_prof.ensure((size_t)F * NR * 4));
  const BigOut big[2] = {{reinterpret_cast<char*>(cube), (size_t)C * NR * 8}, {nullptr, 0}};
  CHK(host_pipeline(c, iq, F, (size_t)C * S * esize(in_dtype), big, [&](char* d_in, int64_t f0, int64_t nf, char* const* d_big) {
    return fmcw_range_fft_device(c, p, d_in, in_dtype, nf, d_big[0], FMCW_C64, c->h_prof.as<float>() + f0 * NR, s);
  }));
  HIPCHK(hipMemcpyAsync(prof, c->h_prof.p, (size_t)F * NR * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipStreamSynchronize(c->cout));
  return FMCW_OK;
}

}  // extern "C"

// Run fn(device context, shard index, f0, n) on every device of the context,
// one host thread per device (their H2D copies, kernels and D2H copies then
// overlap), over contiguous shards of `total` items.  The first failing
// device's status and message are returned.
template <typename Fn>
static int over_devices(fmcw_ctx* c, int64_t total, Fn&& fn) {
  const int world = 1 + (int)c->peers.size();
  if (world == 1) return fn(c, 0, (int64_t)0, total);
  std::vector<int> st(world, FMCW_OK);
  std::vector<std::string> msg(world);
  std::vector<std::thread> th;
  for (int g = 0; g < world; ++g) {
    th.emplace_back([&, g] {
      int64_t f0, n;
      shard(total, g, world, f0, n);
      fmcw_ctx* d = g == 0 ? c : c->peers[g - 1];
      st[g] = n > 0 ? fn(d, g, f0, n) : FMCW_OK;
      if (st[g] != FMCW_OK) msg[g] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < world; ++g)
    if (st[g] != FMCW_OK) return fail(st[g], "device " + std::to_string(g) + ": " + msg[g]);
  return FMCW_OK;
}

extern "C" {

int fmcw_process(fmcw_ctx* c, const fmcw_params* p, const void* iq, int32_t in_dtype, int64_t F, float* prof,
                 int32_t* count, int32_t* ridx, float* rmag, int32_t* didx, float* slow, float* cube, float* rd,
                 int64_t probe_column, float* probe) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  if (probe_column < 0 || probe_column > F * (int64_t)p->pn) return fail(FMCW_E_ARG, "probe_column out of range");
  const int C = p->pn, S = p->nts, NR = p->nr, ND = p->nd, M = p->max_targets;
  const size_t fin = (size_t)C * S * esize(in_dtype);
  // frames are independent: each device takes a contiguous shard and writes its
  // rows of every output in place (the range_speed concatenation of :386-389 is
  // the frame order itself); the probed column lives on one shard
  return over_devices(c, F, [&](fmcw_ctx* d, int, int64_t f0, int64_t n) {
    const int64_t pc = probe_column > f0 * C && probe_column <= (f0 + n) * C ? probe_column - f0 * C : 0;
    return process_host_one(d, p, static_cast<const char*>(iq) + f0 * fin, in_dtype, n, prof + f0 * NR, count + f0,
                            ridx + f0 * M, rmag + f0 * M, didx + f0 * M, slow + f0 * C,
                            cube ? cube + f0 * (size_t)C * NR * 2 : nullptr, rd ? rd + f0 * (size_t)NR * ND * 2 : nullptr,
                            pc, pc ? probe : nullptr);
  });
}

int fmcw_range_fft(fmcw_ctx* c, const fmcw_params* p, const void* iq, int32_t in_dtype, int64_t F, float* cube,
                   float* prof) {
  CHK(check_ctx(c, p));
  if (F < 0) return fail(FMCW_E_ARG, "F < 0");
  if (in_dtype != FMCW_C64 && in_dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad in_dtype");
  const size_t fin = (size_t)p->pn * p->nts * esize(in_dtype);
  return over_devices(c, F, [&](fmcw_ctx* d, int, int64_t f0, int64_t n) {
    return range_fft_host_one(d, p, static_cast<const char*>(iq) + f0 * fin, in_dtype, n,
                              cube + f0 * (size_t)p->pn * p->nr * 2, prof + f0 * p->nr);
  });
}

int fmcw_synth_device(fmcw_ctx* c, const fmcw_params* p, int64_t frame0, int64_t F, void* d_iq, int32_t dtype,
                      void* stream) {
  CHK(check_ctx(c, p));
  if (F < 0 || frame0 < 0) return fail(FMCW_E_ARG, "F / frame0 < 0");
  if (!d_iq) return fail(FMCW_E_ARG, "d_iq is NULL");
  if (dtype != FMCW_C64 && dtype != FMCW_C32H) return fail(FMCW_E_ARG, "bad dtype");
  fmcw::SynthArgs a{};
  a.iq = d_iq; a.dtype = dtype; a.frame0 = frame0; a.nframes = F;
  a.C = p->pn; a.S = p->nts; a.NR = p->nr; a.ND = p->nd;
  a.dist_per_bin = p->dist_per_bin;
  a.cal = c->cal.as<float2>();
  HIPCHK(fmcw::launch_synth(a, pick(c, stream)));
  return FMCW_OK;
}

}  // extern "C"
