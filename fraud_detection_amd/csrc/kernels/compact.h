// Label-group helpers shared by the compaction kernels (scaler.hip) and the stratified split
// (split.hip).  A group is 16 consecutive uint8 labels read with one 16-byte load; block b of a
// grid of G blocks owns groups [b*per, (b+1)*per) with per = ceil(ngroups / G), so a count
// kernel and a later write/assign kernel launched with the same G see the same ranges.
#pragma once
#include "common.h"

namespace fdx {

constexpr int kCompactThreads = 256;

// ---- vectorised compaction: 16 labels per thread (one 16-byte load) --------------------------
// Bit 7 of each byte of the result is set iff that byte of x equals the pattern byte (exact: the
// masked add cannot borrow across bytes).
__device__ __forceinline__ uint32_t match_bytes(uint32_t x, uint32_t pat) {
  const uint32_t v = x ^ pat;
  const uint32_t y = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(y | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t nibble_of(uint32_t m) {  // bits 7,15,23,31 -> bits 0..3
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
// 16-bit match mask of label group g (labels [16g, 16g+16) clipped to n)
__device__ __forceinline__ uint32_t group_mask(const uint8_t* __restrict__ labels, int64_t n, int64_t g,
                                               int target, uint32_t pat) {
  if (16 * g + 16 <= n) {
    const uint4 v = reinterpret_cast<const uint4*>(labels)[g];
    return nibble_of(match_bytes(v.x, pat)) | (nibble_of(match_bytes(v.y, pat)) << 4) |
           (nibble_of(match_bytes(v.z, pat)) << 8) | (nibble_of(match_bytes(v.w, pat)) << 12);
  }
  uint32_t m = 0;
  for (int j = 0; j < 16 && 16 * g + j < n; ++j) m |= (labels[16 * g + j] == target ? 1u : 0u) << j;
  return m;
}
__device__ __forceinline__ void group_range(int64_t ngroups, int64_t* lo, int64_t* hi) {
  const int64_t per = (ngroups + gridDim.x - 1) / gridDim.x;
  *lo = min((int64_t)blockIdx.x * per, ngroups);
  *hi = min(*lo + per, ngroups);
}

}  // namespace fdx
