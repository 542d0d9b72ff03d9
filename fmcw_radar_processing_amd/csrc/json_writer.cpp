// json_writer.cpp -- native jsonencode(struct, 'PrettyPrint', true) for the
// output files of radar_processing.m (:302-436 spectrogram_data.json,
// <file>_range_fft_data.json, <file>_range_speed_data.json, <file>_fft_data.json,
// and :566-593 the 'yes' branch's per-batch spectrogram JSONs).
//
// Once the DSP takes microseconds, formatting ~10^6-10^8 numbers is the host's
// cost (a 115-frame deployed file has a 1024 x 1821 intensity matrix; 256
// config-3 frames a 1024 x 65517 one).  Numbers are formatted with
// std::to_chars (shortest-path printf "%.15g" semantics) in parallel pieces
// and written in order.  The byte stream is that of the Python mirror
// fmcw_radar_processing_amd/matlab_json.py (tests/test_json_native.py):
//   struct -> object, fields in order, 2-space indent, ",\n" separators
//   1x1 -> number; 1xN / Nx1 -> flat array, one element per line;
//   MxN -> array of M row arrays; empty -> []
//   NaN / Inf -> null; integral |v| < 1e15 -> integer text; else %.15g
#include "../../include/fmcw.h"
#include "host_io.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

int jfail(int code, const std::string& m) { return fmcw::set_error(code, m.c_str()); }

double elem(const fmcw_json_field& f, int64_t i, int64_t j) {
  const int64_t o = i * f.row_stride + j * f.col_stride;
  switch (f.kind) {
    case FMCW_JSON_F32: return (double)static_cast<const float*>(f.data)[o];
    case FMCW_JSON_F64: return static_cast<const double*>(f.data)[o];
    default: return (double)static_cast<const int32_t*>(f.data)[o];
  }
}

// one number as matlab_json._num formats it
inline char* put_num(char* p, double v);

// one element: a logical prints as true / false (MATLAB jsonencode of a logical array)
inline char* put_elem(char* p, const fmcw_json_field& f, int64_t i, int64_t j) {
  if (f.kind == FMCW_JSON_BOOL) {
    const bool b = static_cast<const uint8_t*>(f.data)[i * f.row_stride + j * f.col_stride] != 0;
    std::memcpy(p, b ? "true" : "false", b ? 4 : 5);
    return p + (b ? 4 : 5);
  }
  return put_num(p, elem(f, i, j));
}

inline char* put_num(char* p, double v) {
  if (std::isnan(v) || std::isinf(v)) {
    std::memcpy(p, "null", 4);
    return p + 4;
  }
  if (std::fabs(v) < 1e15 && v == std::trunc(v)) {
    const long long iv = (long long)v;
    return std::to_chars(p, p + 24, iv).ptr;
  }
  return std::to_chars(p, p + 32, v, std::chars_format::general, 15).ptr;
}

// A piece of the output: elements [e0, e1) of one array in row-major order of
// its MATLAB shape, formatted with the indentation of the pretty layout.
struct Piece {
  const fmcw_json_field* f;
  int64_t e0, e1;
  std::string ind;       // indentation of the array's opening line
  bool matrix;
  std::string out;
};

void format_piece(Piece& pc, bool pretty) {
  const fmcw_json_field& f = *pc.f;
  const int64_t C = f.cols;
  const std::string in1 = pc.ind + "  ", in2 = pc.ind + "    ";
  // worst case per element: separator 2 + indent + number 24 + row open/close
  const size_t per = 2 + in2.size() + 32 + 2 * (in1.size() + 3);
  pc.out.resize((size_t)(pc.e1 - pc.e0) * per + 16);
  char* p = pc.out.data();
  auto lit = [&](const char* t, size_t n) {
    std::memcpy(p, t, n);
    p += n;
  };
  const char* sep = pretty ? ",\n" : ",";
  const size_t nsep = pretty ? 2 : 1;
  for (int64_t e = pc.e0; e < pc.e1; ++e) {
    const int64_t i = pc.matrix ? e / C : (f.rows == 1 ? 0 : e);
    const int64_t j = pc.matrix ? e % C : (f.rows == 1 ? e : 0);
    if (pc.matrix) {
      if (j == 0) {                       // open row i (pieces hold whole rows; the writer joins pieces)
        if (e > pc.e0) lit(sep, nsep);
        if (pretty) {
          lit(in1.data(), in1.size());
          lit("[\n", 2);
        } else {
          lit("[", 1);
        }
      } else {
        lit(sep, nsep);
      }
      if (pretty) lit(in2.data(), in2.size());
    } else {
      if (e > pc.e0) lit(sep, nsep);
      if (pretty) lit(in1.data(), in1.size());
    }
    p = put_elem(p, f, i, j);
    if (pc.matrix && j == C - 1) {        // close row i
      if (pretty) {
        lit("\n", 1);
        lit(in1.data(), in1.size());
      }
      lit("]", 1);
    }
  }
  pc.out.resize(p - pc.out.data());
}

std::string quote(const char* s) {
  std::string o = "\"";
  for (const char* p = s; *p; ++p) {
    if (*p == '\\' || *p == '"') o += '\\';
    o += *p;
  }
  o += '"';
  return o;
}

}  // namespace

extern "C" {

int fmcw_json_write(const char* path, const fmcw_json_field* fields, int32_t n_fields, int32_t pretty, int32_t threads,
                    int64_t* bytes_out) {
  if (!path || (!fields && n_fields > 0) || n_fields < 0) return jfail(FMCW_E_ARG, "NULL path / fields");
  for (int k = 0; k < n_fields; ++k) {
    const fmcw_json_field& f = fields[k];
    if (!f.name) return jfail(FMCW_E_ARG, "field " + std::to_string(k) + " has no name");
    if (f.kind == FMCW_JSON_STRING) {
      if (!f.data) return jfail(FMCW_E_ARG, std::string("string field '") + f.name + "' is NULL");
    } else if (f.kind == FMCW_JSON_F32 || f.kind == FMCW_JSON_F64 || f.kind == FMCW_JSON_I32 ||
               f.kind == FMCW_JSON_BOOL) {
      if (f.rows < 0 || f.cols < 0 || (f.rows * f.cols > 0 && !f.data))
        return jfail(FMCW_E_ARG, std::string("bad array field '") + f.name + "'");
    } else {
      return jfail(FMCW_E_ARG, std::string("bad kind of field '") + f.name + "'");
    }
  }
  const bool pp = pretty != 0;
  // head/tail text between arrays, and the pieces of every array
  std::vector<std::string> glue;          // glue[k]: text before field k's value; glue[n]: closing text
  std::vector<std::vector<Piece>> pieces(n_fields);
  std::vector<std::string> tails(n_fields);
  const std::string ind = "", in1 = "  ";
  constexpr int64_t kPiece = 1 << 16;     // elements per formatting task
  std::string open = n_fields == 0 ? "{}" : (pp ? "{\n" : "{");
  for (int k = 0; k < n_fields; ++k) {
    const fmcw_json_field& f = fields[k];
    std::string g = k == 0 ? open : (pp ? ",\n" : ",");
    g += (pp ? in1 : std::string()) + quote(f.name) + (pp ? ": " : ":");
    if (f.kind == FMCW_JSON_STRING) {
      g += quote(static_cast<const char*>(f.data));
      glue.push_back(g);
      continue;
    }
    const int64_t n = f.rows * f.cols;
    if (n == 0) {
      g += "[]";
    } else if (n == 1) {
      char buf[48];
      g.append(buf, put_elem(buf, f, 0, 0) - buf);
    } else {
      const bool matrix = f.rows > 1 && f.cols > 1;
      g += pp ? "[\n" : "[";
      const int64_t step = matrix ? std::max<int64_t>(1, kPiece / f.cols) * f.cols : kPiece;   // whole rows
      for (int64_t e = 0; e < n; e += step) pieces[k].push_back(Piece{&f, e, std::min(n, e + step), in1, matrix, {}});
      tails[k] = pp ? "\n" + in1 + "]" : "]";
    }
    glue.push_back(g);
  }
  // format all pieces in parallel
  std::vector<Piece*> work;
  for (auto& v : pieces)
    for (auto& pc : v) work.push_back(&pc);
  unsigned T = threads > 0 ? (unsigned)threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  T = std::max(1u, std::min<unsigned>(T, (unsigned)work.size()));
  if (T <= 1) {
    for (Piece* pc : work) format_piece(*pc, pp);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (size_t i = t; i < work.size(); i += T) format_piece(*work[i], pp);
      });
    for (auto& x : th) x.join();
  }
  FILE* fh = std::fopen(path, "wb");
  if (!fh) return jfail(FMCW_E_ARG, std::string("cannot open ") + path + " for writing");
  int64_t total = 0;
  auto put = [&](const std::string& s) {
    if (!s.empty()) total += (int64_t)std::fwrite(s.data(), 1, s.size(), fh);
  };
  if (n_fields == 0) put(open);
  for (int k = 0; k < n_fields; ++k) {
    put(glue[k]);
    for (auto& pc : pieces[k]) {
      if (&pc != &pieces[k].front()) put(pp ? ",\n" : ",");
      put(pc.out);
      std::string().swap(pc.out);
    }
    put(tails[k]);
  }
  if (n_fields > 0) put(pp ? "\n}" : "}");
  const bool ok = std::fflush(fh) == 0;
  std::fclose(fh);
  if (!ok) return jfail(FMCW_E_ARG, std::string("write to ") + path + " failed");
  if (bytes_out) *bytes_out = total;
  return FMCW_OK;
}

}  // extern "C"
