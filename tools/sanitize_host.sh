#!/usr/bin/env bash
# Host-side sanitizer runs for the native C++ code.  GPU sanitizers are not
# available on this pool, so the device kernels are covered by oracle + determinism tests and
# FDX_SYNC_LAUNCH=1 (synchronous launches that name the failing kernel); the host code that
# has threads and raw pointers -- the mmap CSV parser -- is built twice:
#   ASan + UBSan : out-of-bounds reads past the mapped file, UB in the parser
#   TSan         : races between the per-chunk parser threads
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/fdx_sanitize}"
mkdir -p "$OUT"
SRC="$ROOT/fraud_detection_amd/csrc/io/csv_selftest.cpp"
INC="-I$ROOT/fraud_detection_amd/csrc/io"
CXX="${CXX:-g++}"
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
  $INC "$SRC" -o "$OUT/csv_selftest_asan" -pthread
$CXX -std=c++17 -O1 -g -fsanitize=thread $INC "$SRC" -o "$OUT/csv_selftest_tsan" -pthread
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/csv_selftest_asan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/csv_selftest_tsan"
echo "sanitize_host: ASan+UBSan and TSan clean"
