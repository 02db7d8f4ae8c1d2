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

}  // namespace

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

}  // namespace fdx
