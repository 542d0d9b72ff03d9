// host_io.h -- the host-only pieces of libfmcw (no HIP): the PNG writer, the jet palette and
// the thread-local error text.  json_writer.cpp and png_writer.cpp include only this and
// include/fmcw.h, so the sanitizer builds (Makefile targets asan / tsan) compile them with
// the host compiler alone.
#pragma once
#include <stdint.h>

namespace fmcw {

// png_writer.cpp: indexed PNG of [H][1 + W] rows (filter byte first), jet(256) palette
int png_write_indexed(const char* path, const uint8_t* rows, int W, int H, int level, int threads, int64_t* bytes);
void jet_palette(uint8_t* rgb);

// thread-local error text of fmcw_last_error (fmcw_api.cpp); returns code
int set_error(int code, const char* msg);

}  // namespace fmcw
