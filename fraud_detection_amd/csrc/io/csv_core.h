// Parsing core of the native CSV reader (csv_reader.cpp), free of Python so that the host
// sanitizer harness (csv_selftest.cpp, tools/sanitize_host.sh: ASan+UBSan and TSan builds) runs
// exactly the code the extension runs.
#pragma once
#include <charconv>
#include <cmath>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace fdx_io {

inline const char* next_line(const char* s, const char* e) {
  while (s < e && *s != '\n') ++s;
  return s < e ? s + 1 : e;
}

inline std::vector<std::string> split_header(const char* s, const char* e) {
  std::vector<std::string> out;
  std::string cur;
  for (; s < e && *s != '\n' && *s != '\r'; ++s) {
    if (*s == ',') { out.push_back(cur); cur.clear(); }
    else if (*s != '"') cur.push_back(*s);
  }
  out.push_back(cur);
  return out;
}

inline float parse_field(const char*& s, const char* e) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  float v = NAN;
  if (s < e && *s != ',' && *s != '\n' && *s != '\r') {
    const char* st = s;
    if (*st == '+') ++st;
    auto r = std::from_chars(st, e, v);
    if (r.ec != std::errc()) v = NAN;
    s = r.ptr;
  }
  while (s < e && *s != ',' && *s != '\n') ++s;  // skip closing quote / junk
  return v;
}

inline bool blank_line(const char* s, const char* nl) {
  for (const char* q = s; q < nl; ++q)
    if (*q != '\n' && *q != '\r' && *q != ' ') return false;
  return true;
}

// Parsed table: header names + row-major float32 values ([rows][ncols]).  ``alloc(rows, cols)``
// returns the destination buffer (a numpy array in the extension, a vector in the self-test).
struct Table {
  std::vector<std::string> header;
  size_t rows = 0;
};

template <class Alloc>
Table parse_csv(const char* beg, const char* end, int nthreads, Alloc alloc) {
  if (beg == end) throw std::runtime_error("empty file");
  Table tb;
  const char* body = next_line(beg, end);
  tb.header = split_header(beg, body);
  const int ncols = (int)tb.header.size();
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads < 1) nthreads = 1;
  // chunk boundaries at line starts
  std::vector<const char*> cuts{body};
  const size_t span = (size_t)(end - body);
  for (int t = 1; t < nthreads; ++t) {
    const char* c = body + span * t / nthreads;
    if (c > body) c = next_line(c - 1, end);
    if (c < cuts.back()) c = cuts.back();
    cuts.push_back(c);
  }
  cuts.push_back(end);
  const int nchunks = (int)cuts.size() - 1;
  std::vector<size_t> counts(nchunks, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nchunks; ++t)
      th.emplace_back([&, t] {
        size_t c = 0;
        for (const char* s = cuts[t]; s < cuts[t + 1];) {
          const char* nl = next_line(s, cuts[t + 1]);
          c += blank_line(s, nl) ? 0 : 1;
          s = nl;
        }
        counts[t] = c;
      });
    for (auto& x : th) x.join();
  }
  std::vector<size_t> offs(nchunks + 1, 0);
  for (int t = 0; t < nchunks; ++t) offs[t + 1] = offs[t] + counts[t];
  tb.rows = offs[nchunks];
  float* dst = alloc(tb.rows, (size_t)ncols);
  std::vector<std::thread> th;
  for (int t = 0; t < nchunks; ++t)
    th.emplace_back([&, t] {
      float* row = dst + offs[t] * ncols;
      for (const char* s = cuts[t]; s < cuts[t + 1];) {
        const char* nl = next_line(s, cuts[t + 1]);
        if (!blank_line(s, nl)) {
          const char* q = s;
          for (int c = 0; c < ncols; ++c) {
            row[c] = (q < nl) ? parse_field(q, nl) : NAN;
            if (q < nl && *q == ',') ++q;
          }
          row += ncols;
        }
        s = nl;
      }
    });
  for (auto& x : th) x.join();
  return tb;
}

}  // namespace fdx_io
