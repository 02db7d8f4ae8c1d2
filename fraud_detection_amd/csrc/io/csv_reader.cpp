// Native multi-threaded CSV reader for numeric tables (the creditcard.csv layout:
// header line, then rows of numbers).  Replaces pandas.read_csv on the training path
// (train_model.py:22, preprocess.py:21; SURVEY.md §7.2 data/).
//
// The file is mmap'ed, split into per-thread byte ranges aligned to line starts, each thread
// counts and then parses its lines with std::from_chars into a preallocated float32 matrix
// (row-major [n][ncols]) that is handed to Python through the buffer protocol without a copy.
// Quoted numbers ("1.0") are accepted; empty fields / unparsable fields become NaN.  The parser
// itself lives in csv_core.h (shared with the host sanitizer self-test).
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "csv_core.h"

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

py::tuple read_csv(const std::string& path, int nthreads) {
  Mapped m(path);
  if (m.n == 0) throw std::runtime_error("empty file " + path);
  py::array_t<float> out;
  fdx_io::Table tb;
  {
    // the numpy allocation needs the GIL: take it only inside the allocator callback
    py::gil_scoped_release nogil;
    tb = fdx_io::parse_csv(m.p, m.p + m.n, nthreads, [&](size_t rows, size_t cols) {
      py::gil_scoped_acquire gil;
      out = py::array_t<float>({(py::ssize_t)rows, (py::ssize_t)cols});
      return out.mutable_data();
    });
  }
  return py::make_tuple(out, tb.header);
}

}  // namespace

PYBIND11_MODULE(_fdx_io, m) {
  m.doc() = "native CSV reader (mmap + threads + from_chars)";
  m.def("read_csv", &read_csv, py::arg("path"), py::arg("nthreads") = 0);
}
