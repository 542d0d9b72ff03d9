// sanitize_writers.cpp -- test driver for the sanitizer builds of libfmcw's host-threaded
// writers (csrc/Makefile targets asan / tsan; tests/test_sanitize.py).  It links
// json_writer.cpp and png_writer.cpp as they ship (16 formatter threads, parallel deflate
// strips) with -fsanitize=address,undefined or -fsanitize=thread, writes the spectrogram /
// range_fft JSON shapes of radar_processing.m:306-377 and a spectrogram.png-sized image of
// :331-348, and exits non-zero on a writer error.  The data are exact binary fractions from
// integer formulas, so tests/test_sanitize.py rebuilds them in numpy and compares the bytes
// with the Python mirror (matlab_json.encode) and the decoded PNG rows.
//
//   sanitize_writers <out_dir> <threads>
#include "../../include/fmcw.h"
#include "../../fmcw_radar_processing_amd/csrc/host_io.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace fmcw {
// the library's thread-local error text lives in fmcw_api.cpp (HIP); the driver keeps its own
int set_error(int code, const char* msg) {
  std::fprintf(stderr, "writer error %d: %s\n", code, msg);
  return code;
}
}  // namespace fmcw

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string dir = argv[1];
  const int threads = std::atoi(argv[2]);
  // spectrogram_data.json (:306-321): intensity is the device layout [nseg][nbins], written as
  // MATLAB's nbins x nseg through strides; NaN / +-Inf become null
  const int nseg = 3001, nb = 1024;
  std::vector<float> inten((size_t)nseg * nb), tm(nseg);
  std::vector<double> fq(nb);
  for (int s = 0; s < nseg; ++s) {
    tm[s] = (float)(s + 10) / 1250.0f;
    for (int b = 0; b < nb; ++b) {
      const int v = (s * 7 + b * 13) % 1000;
      inten[(size_t)s * nb + b] = v == 999 ? NAN : v == 998 ? INFINITY : (float)v / 8.0f - 60.0f;
    }
  }
  for (int b = 0; b < nb; ++b) fq[b] = (double)(b + 1) * 0.125;
  const char* title = "All Frames - Log-Scaled Spectrogram";
  std::vector<fmcw_json_field> f(4);
  f[0] = {"time", FMCW_JSON_F32, tm.data(), 1, nseg, 0, 1};
  f[1] = {"frequency", FMCW_JSON_F64, fq.data(), 1, nb, 0, 1};
  f[2] = {"intensity", FMCW_JSON_F32, inten.data(), nb, nseg, 1, nb};
  f[3] = {"title", FMCW_JSON_STRING, title, 0, 0, 0, 0};
  int64_t n = 0;
  if (fmcw_json_write((dir + "/spectrogram_data.json").c_str(), f.data(), 4, 1, threads, &n) != FMCW_OK) return 1;
  // radar_data_range_fft_data.json (:355-361) shapes: Nr x F profile, int and logical vectors
  const int nr = 256, F = 115;
  std::vector<float> prof((size_t)F * nr);
  std::vector<int32_t> idx(F);
  std::vector<uint8_t> det(F);
  for (int i = 0; i < F; ++i) {
    idx[i] = (i * 37) % nr;
    det[i] = (uint8_t)(i % 3 != 0);
    for (int r = 0; r < nr; ++r) prof[(size_t)i * nr + r] = (float)((i * 31 + r * 17) % 4096) / 16.0f;
  }
  std::vector<fmcw_json_field> g(4);
  g[0] = {"range_tx1rx1_max_abs", FMCW_JSON_F32, prof.data(), nr, F, 1, nr};
  g[1] = {"target_bin", FMCW_JSON_I32, idx.data(), 1, F, 0, 1};
  g[2] = {"detected", FMCW_JSON_BOOL, det.data(), 1, F, 0, 1};
  g[3] = {"filename", FMCW_JSON_STRING, "radar_data", 0, 0, 0, 0};
  if (fmcw_json_write((dir + "/range_fft_data.json").c_str(), g.data(), 4, 0, threads, &n) != FMCW_OK) return 1;
  // spectrogram.png (:331-348): 2906 x 2038 palette indices, filter byte 0 first in each row
  const int W = 2906, H = 2038;
  std::vector<uint8_t> rows((size_t)H * (W + 1));
  for (int y = 0; y < H; ++y) {
    rows[(size_t)y * (W + 1)] = 0;
    for (int x = 0; x < W; ++x) rows[(size_t)y * (W + 1) + 1 + x] = (uint8_t)((x / 7 + y / 5 + (x * y) % 3) & 255);
  }
  if (fmcw::png_write_indexed((dir + "/spectrogram.png").c_str(), rows.data(), W, H, 6, threads, &n) != FMCW_OK) return 1;
  std::printf("ok\n");
  return 0;
}
