// Host self-test of the CSV parsing core (csv_core.h) for the sanitizer builds
// (tools/sanitize_host.sh: -fsanitize=address,undefined and -fsanitize=thread).  Every case
// parses with 1..16 threads -- more threads than lines, boundaries inside CRLF pairs, quoted
// fields, blank lines, short rows, no trailing newline -- and must give the same table.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "csv_core.h"

namespace {

int failures = 0;

void check(bool ok, const std::string& what) {
  if (!ok) {
    ++failures;
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
  }
}

bool same(float a, float b) { return (std::isnan(a) && std::isnan(b)) || a == b; }

void run_case(const std::string& name, const std::string& text, size_t rows, size_t cols,
              const std::vector<float>& expect) {
  for (int th = 1; th <= 16; ++th) {
    // exact-size heap copy: any read past the end is an ASan heap-buffer-overflow
    std::vector<char> buf(text.begin(), text.end());
    std::vector<float> out;
    fdx_io::Table tb = fdx_io::parse_csv(buf.data(), buf.data() + buf.size(), th, [&](size_t r, size_t c) {
      out.assign(r * c, -12345.0f);
      return out.data();
    });
    check(tb.rows == rows, name + ": rows with " + std::to_string(th) + " threads");
    check(tb.header.size() == cols, name + ": cols");
    if (tb.rows != rows || tb.header.size() != cols) continue;
    for (size_t i = 0; i < expect.size(); ++i)
      if (!same(out[i], expect[i])) {
        check(false, name + ": value " + std::to_string(i) + " with " + std::to_string(th) + " threads");
        break;
      }
  }
}

}  // namespace

int main() {
  const float N = NAN;
  run_case("basic", "a,b\n1,2\n3,4\n", 2, 2, {1, 2, 3, 4});
  run_case("no trailing newline", "a,b\n1,2\n3,4", 2, 2, {1, 2, 3, 4});
  run_case("crlf", "a,b\r\n1,2\r\n3,4\r\n", 2, 2, {1, 2, 3, 4});
  run_case("quoted", "\"a\",\"b\"\n\"1.5\",\"-2\"\n", 1, 2, {1.5f, -2});
  run_case("blank lines", "a,b\n\n1,2\n   \n3,4\n\n", 2, 2, {1, 2, 3, 4});
  run_case("short and empty fields", "a,b,c\n1,,3\n4\n", 2, 3, {1, N, 3, 4, N, N});
  run_case("junk and plus", "a,b\n+1e3,x\n-0.25,7junk\n", 2, 2, {1000, N, -0.25f, 7});
  run_case("header only", "a,b\n", 0, 2, {});
  // a larger random table: boundaries fall everywhere
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1e4f, 1e4f);
  std::string big = "t,v1,v2,amount,class\n";
  std::vector<float> exp;
  for (int r = 0; r < 5000; ++r) {
    for (int c = 0; c < 5; ++c) {
      const float v = (c == 4) ? (float)(r % 2) : U(rng);
      char tmp[64];
      std::snprintf(tmp, sizeof tmp, "%.9g", v);
      float back = std::strtof(tmp, nullptr);
      exp.push_back(back);
      big += tmp;
      big += (c == 4) ? ((r % 7 == 0) ? "\r\n" : "\n") : ",";
    }
  }
  run_case("random 5000x5", big, 5000, 5, exp);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("csv_selftest: all cases passed\n");
  return 0;
}
