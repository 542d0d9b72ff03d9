// png_writer.cpp -- palette PNG of the rendered spectrogram (radar_processing.m
// :344 exportgraphics(fig, 'spectrogram.png', 'Resolution', 600)).
// The image is jet(256) palette indices, so it is stored as an 8-bit indexed
// PNG (colour type 3, PLTE = the 256 jet colours): the same pixels as an RGB
// export in a third of the bytes.  The rows (filter byte 0 first, as the render
// kernel writes them) are deflated in parallel strips -- raw deflate streams
// ended by a sync flush, concatenated, with the adler32 of the whole image
// combined from the strips' -- which is one valid zlib stream (the pigz method).
#include "../../include/fmcw.h"
#include "host_io.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

namespace fmcw {

static void be32(std::string& o, uint32_t v) {
  o += (char)(v >> 24);
  o += (char)(v >> 16);
  o += (char)(v >> 8);
  o += (char)v;
}

static void chunk(std::string& o, const char* type, const std::string& data) {
  be32(o, (uint32_t)data.size());
  std::string td = std::string(type, 4) + data;
  o += td;
  be32(o, (uint32_t)crc32(0L, reinterpret_cast<const Bytef*>(td.data()), (uInt)td.size()));
}

// jet(256) exactly as MATLAB builds it (n = ceil(m/4), u = [(1:n)/n ones(1,n-1) (n:-1:1)/n]),
// colours rounded to 8 bits
void jet_palette(uint8_t* rgb) {
  const int m = 256, n = (m + 3) / 4;
  std::vector<double> u;
  for (int i = 1; i <= n; ++i) u.push_back((double)i / n);
  for (int i = 1; i < n; ++i) u.push_back(1.0);
  for (int i = n; i >= 1; --i) u.push_back((double)i / n);
  std::vector<double> J(3 * m, 0.0);
  const int g0 = (n + 1) / 2 - ((m % 4) == 1 ? 1 : 0);   // ceil(n/2) - (mod(m,4)==1)
  for (int i = 0; i < (int)u.size(); ++i) {
    const int g = g0 + 1 + i, r = g + n, b = g - n;       // 1-based rows of J
    if (g >= 1 && g <= m) J[3 * (g - 1) + 1] = u[i];
    if (r >= 1 && r <= m) J[3 * (r - 1) + 0] = u[i];
    if (b >= 1 && b <= m) J[3 * (b - 1) + 2] = u[i];
  }
  for (int i = 0; i < 3 * m; ++i) rgb[i] = (uint8_t)std::lround(J[i] * 255.0);
}

int png_write_indexed(const char* path, const uint8_t* rows, int W, int H, int level, int threads, int64_t* bytes) {
  const size_t stride = (size_t)W + 1, total = stride * (size_t)H;
  unsigned T = threads > 0 ? (unsigned)threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  T = std::max(1u, std::min<unsigned>(T, (unsigned)H));
  std::vector<std::string> part(T);
  std::vector<uLong> ad(T);
  std::vector<size_t> len(T);
  std::vector<int> st(T, Z_OK);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const int r0 = (int)((int64_t)H * t / T), r1 = (int)((int64_t)H * (t + 1) / T);
      const Bytef* src = rows + (size_t)r0 * stride;
      const size_t n = (size_t)(r1 - r0) * stride;
      len[t] = n;
      ad[t] = adler32(1L, src, (uInt)n);
      z_stream z{};
      if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { st[t] = Z_STREAM_ERROR; return; }
      part[t].resize(deflateBound(&z, (uLong)n) + 64);
      z.next_in = const_cast<Bytef*>(src);
      z.avail_in = (uInt)n;
      z.next_out = reinterpret_cast<Bytef*>(&part[t][0]);
      z.avail_out = (uInt)part[t].size();
      const int r = deflate(&z, t + 1 == T ? Z_FINISH : Z_SYNC_FLUSH);
      if (r != (t + 1 == T ? Z_STREAM_END : Z_OK)) st[t] = r == Z_OK ? Z_BUF_ERROR : r;
      part[t].resize(part[t].size() - z.avail_out);
      deflateEnd(&z);
    });
  }
  for (auto& x : th) x.join();
  for (unsigned t = 0; t < T; ++t)
    if (st[t] != Z_OK) return set_error(FMCW_E_ARG, "deflate failed");
  uLong adler = ad[0];
  for (unsigned t = 1; t < T; ++t) adler = adler32_combine(adler, ad[t], (z_off_t)len[t]);
  (void)total;
  std::string idat = "\x78\x01";                            // zlib header: deflate, 32K window, check bits ok
  for (auto& p : part) idat += p;
  be32(idat, (uint32_t)adler);
  std::string png = "\x89PNG\r\n\x1a\n";
  std::string ihdr;
  be32(ihdr, (uint32_t)W);
  be32(ihdr, (uint32_t)H);
  ihdr += (char)8;                                          // bit depth
  ihdr += (char)3;                                          // colour type: indexed
  ihdr += std::string(3, '\0');                             // deflate, adaptive filter set, no interlace
  chunk(png, "IHDR", ihdr);
  uint8_t pal[768];
  jet_palette(pal);
  chunk(png, "PLTE", std::string(reinterpret_cast<char*>(pal), 768));
  chunk(png, "IDAT", idat);
  chunk(png, "IEND", std::string());
  FILE* fh = std::fopen(path, "wb");
  if (!fh) return set_error(FMCW_E_ARG, (std::string("cannot open ") + path + " for writing").c_str());
  const size_t w = std::fwrite(png.data(), 1, png.size(), fh);
  const bool ok = std::fclose(fh) == 0 && w == png.size();
  if (!ok) return set_error(FMCW_E_ARG, (std::string("write to ") + path + " failed").c_str());
  if (bytes) *bytes = (int64_t)png.size();
  return FMCW_OK;
}

}  // namespace fmcw
