// K10 auc / confusion: exact ROC-AUC and confusion counts on device.
//
// Reference behaviour being replaced: sklearn roc_auc_score / roc_curve+auc / confusion_matrix
// (train_model.py:83,109; evaluate_model.py:31,45,49-50).
//
// Exact AUC = (#{(p,n): s_p > s_n} + 0.5 #{(p,n): s_p == s_n}) / (P N).
// Fraud data is heavily imbalanced, so instead of sorting all N scores we sort only the positive
// class (compacted, then bitonic-sorted in LDS chunks of <= 16384 floats = 64 KiB) and let every
// negative count its rank inside each sorted chunk by binary search in LDS.  Integer pair counts
// are reduced with 64-bit integer atomics, so the result is exact (ties averaged exactly like
// sklearn) and bitwise deterministic.  Cost ~ N log2(chunk) LDS probes per chunk.
#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void auc_compact_kernel(const float* __restrict__ scores,
                                                               const uint8_t* __restrict__ labels,
                                                               int64_t n, float* __restrict__ pos,
                                                               unsigned long long* __restrict__ counter) {
  const int lane = lane_id();
  for (int64_t i0 = (int64_t)blockIdx.x * kThreads; i0 < n; i0 += (int64_t)gridDim.x * kThreads) {
    const int64_t i = i0 + threadIdx.x;
    const bool hit = i < n && labels[i] != 0;
    const unsigned long long m = __ballot(hit);
    if (m == 0ull) continue;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(counter, (unsigned long long)__popcll(m));
    base = __shfl(base, 0, kWave);
    if (hit) pos[base + __popcll(m & ((1ull << lane) - 1ull))] = scores[i];
  }
}

// Bitonic sort of pos[c*chunk, min((c+1)*chunk, P)) ascending, in LDS (chunk = 2^k <= 16384).
__global__ __launch_bounds__(1024) void sort_chunks_kernel(float* __restrict__ pos,
                                                           const unsigned long long* __restrict__ counter,
                                                           int chunk) {
  __shared__ float s[16384];
  const int64_t P = (int64_t)*counter;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  if (lo >= P) return;
  const int len = (int)((P - lo) < chunk ? (P - lo) : chunk);
  for (int i = threadIdx.x; i < chunk; i += 1024) s[i] = i < len ? pos[lo + i] : __builtin_inff();
  __syncthreads();
  for (int k = 2; k <= chunk; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < chunk; i += 1024) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float a = s[i], b = s[ixj];
          const bool asc = (i & k) == 0;
          if ((a > b) == asc) { s[i] = b; s[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < len; i += 1024) pos[lo + i] = s[i];
}

__global__ __launch_bounds__(kThreads) void auc_count_kernel(
    const float* __restrict__ scores, const uint8_t* __restrict__ labels, int64_t n,
    const float* __restrict__ pos, const unsigned long long* __restrict__ counter, int chunk,
    int nchunks, unsigned long long* __restrict__ out_pairs) {
  __shared__ float s[16384];
  __shared__ unsigned long long red[kThreads / kWave];
  const int64_t P = (int64_t)*counter;
  unsigned long long acc = 0;  // 2 * (#greater) + #equal
  for (int c = 0; c < nchunks; ++c) {
    const int64_t lo = (int64_t)c * chunk;
    if (lo >= P) break;
    const int len = (int)((P - lo) < chunk ? (P - lo) : chunk);
    __syncthreads();
    for (int i = threadIdx.x; i < len; i += kThreads) s[i] = pos[lo + i];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads) {
      if (labels[i] != 0) continue;
      const float v = scores[i];
      int a = 0, b = len;  // lower_bound: first >= v
      while (a < b) { const int m = (a + b) >> 1; if (s[m] < v) a = m + 1; else b = m; }
      const int lb = a;
      b = len;             // upper_bound: first > v
      while (a < b) { const int m = (a + b) >> 1; if (s[m] <= v) a = m + 1; else b = m; }
      acc += 2ull * (unsigned long long)(len - a) + (unsigned long long)(a - lb);
    }
  }
  acc = wave_sum(acc);
  if (lane_id() == 0) red[wave_id()] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kThreads / kWave; ++w) t += red[w];
    atomicAdd(out_pairs, t);
  }
}

__global__ __launch_bounds__(kThreads) void confusion_kernel(const float* __restrict__ scores,
                                                             const uint8_t* __restrict__ labels,
                                                             int64_t n, float thr,
                                                             unsigned long long* __restrict__ out4) {
  unsigned long long c[4] = {0, 0, 0, 0};  // tn, fp, fn, tp
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads) {
    const int y = labels[i] != 0;
    const int p = scores[i] > thr;
    c[2 * y + p] += 1;
  }
  __shared__ unsigned long long red[kThreads / kWave][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c[k] = wave_sum(c[k]);
    if (lane_id() == 0) red[wave_id()][k] = c[k];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
    for (int w = 0; w < kThreads / kWave; ++w) t += red[w][threadIdx.x];
    atomicAdd(out4 + threadIdx.x, t);
  }
}

// ---- histogram AUC (mergeable across ranks) ---------------------------------------------------
// Order-preserving u32 key of a float: larger float -> larger key (incl. negatives, -0 < +0).
__device__ __forceinline__ uint32_t order_key(float f) {
  uint32_t b = __float_as_uint(f);
  if (b == 0x80000000u) b = 0u;  // -0 == +0 (ties, as in the exact AUC)
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// hist[label][key >> (32 - bits)] += 1 for every score; u32 global atomics on 2 x 2^bits
// counters (2^20 by default: spread enough that contention is negligible).
__global__ __launch_bounds__(kThreads) void auc_hist_kernel(const float* __restrict__ scores,
                                                            const uint8_t* __restrict__ labels, int64_t n,
                                                            int bits, unsigned* __restrict__ hist) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int sh = 32 - bits;
  const int64_t nb = (int64_t)1 << bits;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const uint32_t b = order_key(scores[i]) >> sh;
    atomicAdd(&hist[(labels[i] != 0 ? nb : 0) + b], 1u);
  }
}

// out[0] = sum_b P_b (2 N_<b + N_b)  (twice the tie-averaged pair count, exact u64),
// out[1] = P, out[2] = N.  One block of 1024 threads, each scanning a contiguous range of bins.
__global__ __launch_bounds__(1024) void auc_hist_reduce_kernel(const unsigned* __restrict__ hist, int bits,
                                                               unsigned long long* __restrict__ out) {
  __shared__ unsigned long long wsum[16];
  __shared__ unsigned long long red[3][16];
  const int64_t nb = (int64_t)1 << bits;
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const int64_t per = (nb + 1023) / 1024;
  const int64_t lo = min((int64_t)t * per, nb), hi = min(lo + per, nb);
  const unsigned* neg = hist;
  const unsigned* pos = hist + nb;
  unsigned long long nsum = 0, psum = 0;
  for (int64_t b = lo; b < hi; ++b) { nsum += neg[b]; psum += pos[b]; }
  unsigned long long inc = nsum;  // block exclusive scan of the per-thread negative counts
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned long long u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    unsigned long long x = lane < 16 ? wsum[lane] : 0ull;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const unsigned long long u = __shfl_up(x, o, kWave);
      if (lane >= o) x += u;
    }
    if (lane < 16) wsum[lane] = x;
  }
  __syncthreads();
  unsigned long long nbefore = (w > 0 ? wsum[w - 1] : 0ull) + inc - nsum;
  unsigned long long num = 0;
  for (int64_t b = lo; b < hi; ++b) {
    const unsigned long long nb_ = neg[b], pb = pos[b];
    num += pb * (2ull * nbefore + nb_);
    nbefore += nb_;
  }
  num = wave_sum(num); psum = wave_sum(psum); nsum = wave_sum(nsum);
  if (lane == 0) { red[0][w] = num; red[1][w] = psum; red[2][w] = nsum; }
  __syncthreads();
  if (t < 3) {
    unsigned long long a = 0;
    for (int i = 0; i < 16; ++i) a += red[t][i];
    out[t] = a;
  }
}

// Exact AUC for any class balance (the chunked path above costs ~N log(chunk) per 16384
// positives, quadratic in spirit once positives are common).  Input: the scores sorted ascending
// (rocPRIM radix sort through torch.sort), the inclusive prefix count of positives in that order
// and, per element, the index where its tie segment starts (inclusive max-scan of the segment-
// start positions).  The thread at each segment end adds
//     pos_in_seg * (2 * neg_before_seg + neg_in_seg)
// -- twice the pairs the segment's positives win plus the ties -- as an exact 64-bit integer:
// the sum is order independent, so the result is bitwise deterministic and equal to sklearn's
// tie-averaged AUC.  O(N) after the sort.
__global__ __launch_bounds__(kThreads) void auc_segments_kernel(const float* __restrict__ s,
                                                                const int64_t* __restrict__ pos_incl,
                                                                const int64_t* __restrict__ seg_start,
                                                                int64_t n, unsigned long long* __restrict__ out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const bool end = (i == n - 1) || !(s[i] == s[i + 1]);
    if (!end) continue;
    const int64_t st = seg_start[i];
    const int64_t pos_before = st > 0 ? pos_incl[st - 1] : 0;
    const int64_t pos_in = pos_incl[i] - pos_before;
    const int64_t neg_in = (i + 1 - st) - pos_in;
    const int64_t neg_before = st - pos_before;
    acc += (unsigned long long)pos_in * (unsigned long long)(2 * neg_before + neg_in);
  }
  acc = wave_sum(acc);
  if (lane_id() == 0 && acc != 0ull) atomicAdd(out, acc);
}

}  // namespace

void launch_auc_segments(const float* sorted_scores, const int64_t* pos_incl, const int64_t* seg_start, int64_t n,
                         unsigned long long* out_twice_pairs, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = stream_grid(n, kThreads * 4, 4096);
  auc_segments_kernel<<<grid, kThreads, 0, stream>>>(sorted_scores, pos_incl, seg_start, n, out_twice_pairs);
  check_launch("auc_segments");
}

void launch_auc_compact(const float* scores, const uint8_t* labels, int64_t n, float* pos,
                        unsigned long long* counter, hipStream_t stream) {
  const int grid = stream_grid(n, kThreads, 2048);
  auc_compact_kernel<<<grid, kThreads, 0, stream>>>(scores, labels, n, pos, counter);
  check_launch("auc_compact");
}

void launch_sort_chunks(float* pos, int64_t npos_cap, const unsigned long long* counter, int chunk,
                        int nchunks, hipStream_t stream) {
  (void)npos_cap;
  if (chunk <= 0 || chunk > 16384 || (chunk & (chunk - 1)) != 0)
    throw std::runtime_error("sort_chunks: chunk must be a power of two <= 16384");
  if (nchunks <= 0) return;
  sort_chunks_kernel<<<nchunks, 1024, 0, stream>>>(pos, counter, chunk);
  check_launch("sort_chunks");
}

void launch_auc_count(const float* scores, const uint8_t* labels, int64_t n, const float* pos,
                      const unsigned long long* counter, int chunk, int nchunks,
                      unsigned long long* out_pairs, hipStream_t stream) {
  const int grid = stream_grid(n, kThreads * 8, 1024);
  auc_count_kernel<<<grid, kThreads, 0, stream>>>(scores, labels, n, pos, counter, chunk, nchunks,
                                                  out_pairs);
  check_launch("auc_count");
}

void launch_confusion(const float* scores, const uint8_t* labels, int64_t n, float threshold,
                      unsigned long long* out4, hipStream_t stream) {
  const int grid = stream_grid(n, kThreads * 8, 1024);
  confusion_kernel<<<grid, kThreads, 0, stream>>>(scores, labels, n, threshold, out4);
  check_launch("confusion");
}

void launch_auc_hist(const float* scores, const uint8_t* labels, int64_t n, int bits, unsigned* hist,
                     hipStream_t stream) {
  if (bits < 8 || bits > 24) throw std::runtime_error("auc_hist: bits must be in [8, 24]");
  if (n <= 0) return;
  const int grid = stream_grid(n, kThreads, 4096);
  auc_hist_kernel<<<grid, kThreads, 0, stream>>>(scores, labels, n, bits, hist);
  check_launch("auc_hist");
}

void launch_auc_hist_reduce(const unsigned* hist, int bits, unsigned long long* out, hipStream_t stream) {
  auc_hist_reduce_kernel<<<1, 1024, 0, stream>>>(hist, bits, out);
  check_launch("auc_hist_reduce");
}

}  // namespace fdx
