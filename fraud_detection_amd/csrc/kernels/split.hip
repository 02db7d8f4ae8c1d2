// K3 strat_assign: stratified train/test split + K-fold assignment in one pass over the labels.
//
// Reference behaviour being replaced: train_test_split(stratify=y, test_size=0.2, rs=42) and
// StratifiedKFold(5, shuffle=True, rs=42) (train_model.py:31-33,49,58):
// every class is shuffled independently, a fixed share of each class goes to the test set and
// the rest is dealt into K folds whose sizes differ by at most one row.
//
// MI355X mapping: no sort.  The row's rank inside its class comes from the same block-count +
// scan as the label compaction (compact.h), and a keyed 4-round Feistel network with cycle
// walking maps that rank to a position in a pseudo-random permutation of [0, n_class) -- a
// bijection evaluated independently per row in registers (~60 integer ops), so 100M labels
// cost one 100 MB read and one 100 MB write.  The test set is the first round(frac * n_c)
// positions of each class's permutation; the remaining positions are cut into K contiguous
// folds (the first n_c' mod K folds one row larger, like StratifiedKFold).  Output code per row:
// 255 = test, 0..K-1 = fold.  ops/split.py holds the bit-identical numpy oracle.
#include "common.h"
#include "compact.h"
#include "launchers.h"

namespace fdx {

namespace {

constexpr uint8_t kTestCode = 255;

__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

struct ClassPerm {
  uint64_t n;        // class size
  uint64_t ntest;    // rows of this class in the test set
  uint64_t q, r;     // fold sizes: r folds of q+1 rows, then folds of q rows
  uint32_t mask;     // half-word mask (h bits)
  int h;
  uint32_t key[4];

  __device__ void init(uint64_t n_c, uint32_t seed, int cls, double test_frac, int k) {
    n = n_c;
    ntest = (uint64_t)floor(test_frac * (double)n_c + 0.5);
    if (ntest > n_c) ntest = n_c;
    const uint64_t m = n_c - ntest;
    const uint64_t kk = k > 1 ? (uint64_t)k : 1;
    q = m / kk;
    r = m % kk;
    int b = 2;
    while (b < 64 && (1ull << b) < n_c) ++b;  // 2^b >= n_c
    h = (b + 1) >> 1;
    mask = (h >= 32) ? 0xffffffffu : ((1u << h) - 1u);
#pragma unroll
    for (int i = 0; i < 4; ++i) key[i] = fmix32(seed ^ fmix32(0x9E3779B9u * (uint32_t)(2 * cls + 1) + (uint32_t)i));
  }

  // position of in-class rank x in the class permutation (cycle walking keeps it in [0, n))
  __device__ uint64_t apply(uint64_t x) const {
    do {
      uint32_t L = (uint32_t)(x >> h), R = (uint32_t)x & mask;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t t = L ^ (fmix32(R ^ key[i]) & mask);
        L = R;
        R = t;
      }
      x = ((uint64_t)L << h) | R;
    } while (x >= n);
    return x;
  }

  __device__ uint8_t code(uint64_t rank, int k) const {
    const uint64_t pos = apply(rank);
    if (pos < ntest) return kTestCode;
    if (k <= 1) return 0;
    const uint64_t p = pos - ntest, big = r * (q + 1);
    return (uint8_t)(p < big ? p / (q + 1) : r + (p - big) / q);
  }
};

// offsets[b] = positives before block b (exclusive scan of compact_count16 over the same grid);
// total = number of positives.
__global__ __launch_bounds__(kCompactThreads) void strat_assign_kernel(
    const uint8_t* __restrict__ labels, int64_t n, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ total, uint32_t seed, double test_frac, int k, uint8_t* __restrict__ out) {
  int64_t lo, hi;
  group_range((n + 15) / 16, &lo, &hi);
  const int64_t n1 = *total;
  ClassPerm P0, P1;
  P0.init((uint64_t)(n - n1), seed, 0, test_frac, k);
  P1.init((uint64_t)n1, seed, 1, test_frac, k);
  const uint32_t pat = 0x01010101u;
  __shared__ int wave_tot[kCompactThreads / kWave];
  const int lane = lane_id(), w = wave_id();
  int64_t base = offsets[blockIdx.x];
  for (int64_t g0 = lo; g0 < hi; g0 += kCompactThreads) {  // block-uniform trip count
    const int64_t g = g0 + threadIdx.x;
    const uint32_t m = g < hi ? group_mask(labels, n, g, 1, pat) : 0u;
    const int c = __popc(m);
    int inc = c;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int u = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += u;
    }
    if (lane == kWave - 1) wave_tot[w] = inc;
    __syncthreads();
    int64_t ones = base + inc - c;  // positives before row 16g
    int tot = 0;
    for (int i = 0; i < kCompactThreads / kWave; ++i) {
      if (i < w) ones += wave_tot[i];
      tot += wave_tot[i];
    }
    if (g < hi) {
      uint32_t word[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int64_t row = 16 * g + j;
        const bool pos = (m >> j) & 1u;
        const int64_t before = ones + __popc(m & ((1u << j) - 1u));
        uint8_t cd = 0;
        if (row < n) cd = pos ? P1.code((uint64_t)before, k) : P0.code((uint64_t)(row - before), k);
        word[j >> 2] |= (uint32_t)cd << (8 * (j & 3));
      }
      if (16 * g + 16 <= n) {
        reinterpret_cast<uint4*>(out)[g] = make_uint4(word[0], word[1], word[2], word[3]);
      } else {
        for (int j = 0; j < 16 && 16 * g + j < n; ++j) out[16 * g + j] = (uint8_t)(word[j >> 2] >> (8 * (j & 3)));
      }
    }
    base += tot;
    __syncthreads();
  }
}

}  // namespace

void launch_strat_assign(const uint8_t* labels, int64_t n, const int64_t* offsets, const int64_t* total,
                         uint32_t seed, double test_frac, int k, uint8_t* out, int nblocks, hipStream_t stream) {
  if ((reinterpret_cast<uintptr_t>(labels) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    throw std::invalid_argument("strat_assign: labels and out must be 16-byte aligned");
  if (k < 0 || k > 254) throw std::invalid_argument("strat_assign: 0 <= k <= 254");
  strat_assign_kernel<<<nblocks, kCompactThreads, 0, stream>>>(labels, n, offsets, total, seed, test_frac, k, out);
  check_launch("strat_assign");
}

}  // namespace fdx
