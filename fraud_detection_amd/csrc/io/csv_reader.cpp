// Native multi-threaded CSV reader for numeric tables (the creditcard.csv layout:
// header line, then rows of numbers).  Replaces pandas.read_csv on the training path
// (train_model.py:22, preprocess.py:21; SURVEY.md §7.2 data/).
//
// The file is mmap'ed, split into per-thread byte ranges aligned to line starts, each thread
// counts and then parses its lines with std::from_chars into a preallocated float32 matrix
// (row-major [n][ncols]) that is handed to Python through the buffer protocol without a copy.
// Quoted numbers ("1.0") are accepted; empty fields / unparsable fields become NaN.
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <charconv>
#include <cmath>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  explicit Mapped(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    fstat(fd, &st);
    n = (size_t)st.st_size;
    if (n) {
      void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
      p = static_cast<const char*>(m);
    }
  }
  ~Mapped() {
    if (p) munmap(const_cast<char*>(p), n);
    if (fd >= 0) ::close(fd);
  }
};

inline const char* next_line(const char* s, const char* e) {
  while (s < e && *s != '\n') ++s;
  return s < e ? s + 1 : e;
}

std::vector<std::string> split_header(const char* s, const char* e) {
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

py::tuple read_csv(const std::string& path, int nthreads) {
  Mapped m(path);
  if (m.n == 0) throw std::runtime_error("empty file " + path);
  const char* beg = m.p;
  const char* end = m.p + m.n;
  const char* body = next_line(beg, end);
  std::vector<std::string> header = split_header(beg, body);
  const int ncols = (int)header.size();
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
          bool blank = true;
          for (const char* q = s; q < nl; ++q)
            if (*q != '\n' && *q != '\r' && *q != ' ') { blank = false; break; }
          c += blank ? 0 : 1;
          s = nl;
        }
        counts[t] = c;
      });
    for (auto& x : th) x.join();
  }
  std::vector<size_t> offs(nchunks + 1, 0);
  for (int t = 0; t < nchunks; ++t) offs[t + 1] = offs[t] + counts[t];
  const size_t nrows = offs[nchunks];
  py::array_t<float> out({(py::ssize_t)nrows, (py::ssize_t)ncols});
  float* dst = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> th;
    for (int t = 0; t < nchunks; ++t)
      th.emplace_back([&, t] {
        float* row = dst + offs[t] * ncols;
        for (const char* s = cuts[t]; s < cuts[t + 1];) {
          const char* nl = next_line(s, cuts[t + 1]);
          bool blank = true;
          for (const char* q = s; q < nl; ++q)
            if (*q != '\n' && *q != '\r' && *q != ' ') { blank = false; break; }
          if (!blank) {
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
  }
  return py::make_tuple(out, header);
}

}  // namespace

PYBIND11_MODULE(_fdx_io, m) {
  m.doc() = "native CSV reader (mmap + threads + from_chars)";
  m.def("read_csv", &read_csv, py::arg("path"), py::arg("nthreads") = 0);
}
