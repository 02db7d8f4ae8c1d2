// K11 quantile cuts: exact per-feature order statistics of the GBDT cut sample, without a sort.
//
// The cuts (ops/gbdt.py quantile_cuts, numpy oracle reference_gbdt.quantile_cuts) need, for every
// feature, the sample minimum and the values at ranks floor(t m / max_bin), t = 1 .. max_bin-1 --
// 256 order statistics out of ~1M values per feature.  A full segmented sort (torch.sort: rocPRIM
// merge sort, ~600 dispatches per call) does ~20x the work the cuts need.  Here the
// order statistics come from a three-level MSD radix select over the floats' order-preserving
// 32-bit keys (11 + 11 + 10 bits):
//   1. qsel_hist: per-(feature, 2048-bin top-11-bit digit) counts, LDS-private per block;
//   2. qsel_plan (one block per feature): scan, the digit bucket and in-bucket rank of every
//      target, and a compacted layout of just the target buckets;
//   3. qsel_scatter: the values of target buckets are copied into their bucket's run (order inside
//      a run is irrelevant: only values are kept, so LDS-atomic slots are fine);
//   4. qsel_final (one block per (feature, target)): LDS histograms of the next 11 and the last 10
//      bits over that target's run -- the run is small (a 1/2048-wide slice of the key space, and
//      of the ranks for a well-spread feature) and L2-resident.
// Every step counts exactly, so the selected values equal np.sort(sample)[rank] bit for bit (-0.0
// is taken as +0.0, which compares equal; NaN sorts last as in numpy).
#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kQBins0 = 2048;      // level 0 / 1 digit width: 11 bits
constexpr int kQBins2 = 1024;      // level 2: the last 10 bits
constexpr int kQFeatGroup = 4;     // features per histogram / scatter block
constexpr int kQChunk = 4096;      // sample rows per histogram / scatter block
constexpr int kQThreads = 256;

__device__ __forceinline__ uint32_t ordered_key(float x) {
  uint32_t u = __float_as_uint(x);
  if (x == 0.0f) u = 0u;                  // -0.0 -> +0.0
  if (x != x) u = 0x7fffffffu;            // NaN last
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Exclusive scan of an NB-bin LDS array by the block's 256 threads (NB/256 consecutive bins each).
template <int NB>
__device__ void excl_scan(const uint32_t* h, uint32_t* pre) {
  constexpr int kPer = NB / kQThreads;
  __shared__ uint32_t part[kQThreads];
  const int t = threadIdx.x;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) s += h[t * kPer + j];
  part[t] = s;
  __syncthreads();
  if (t < kWave) {  // one wave: exclusive scan of the 256 partial sums (4 per lane)
    uint32_t v[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = part[4 * t + j]; tot += v[j]; }
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, kWave);
      if (t >= o) inc += y;
    }
    uint32_t run = inc - tot;
#pragma unroll
    for (int j = 0; j < 4; ++j) { const uint32_t c = v[j]; part[4 * t + j] = run; run += c; }
  }
  __syncthreads();
  uint32_t run = part[t];
#pragma unroll
  for (int j = 0; j < kPer; ++j) { pre[t * kPer + j] = run; run += h[t * kPer + j]; }
  __syncthreads();
}

// The bin of an NB-bin LDS histogram holding rank r (0 <= r < total) and r's rank inside it: the
// largest bin whose exclusive prefix is <= r (it is non-empty).  Uniform: every thread gets it.
template <int NB>
__device__ void find_rank(const uint32_t* h, uint32_t* pre, uint32_t r, int& bin, uint32_t& rin) {
  excl_scan<NB>(h, pre);
  int lo = 0;
#pragma unroll
  for (int half = NB / 2; half >= 1; half >>= 1)
    if (pre[lo + half] <= r) lo += half;
  bin = lo;
  rin = r - pre[lo];
  __syncthreads();
}

__device__ __forceinline__ float sample_at(const float* X, int64_t row, int64_t stride, int ld, int f) {
  return X[row * stride * ld + f];
}

__global__ __launch_bounds__(kQThreads) void qsel_hist_kernel(const float* __restrict__ X, int64_t m,
                                                              int64_t stride, int ld, int d,
                                                              uint32_t* __restrict__ hist0) {
  __shared__ uint32_t h[kQFeatGroup][kQBins0];  // 32 KiB
  const int f0 = blockIdx.y * kQFeatGroup;
  for (int i = threadIdx.x; i < kQFeatGroup * kQBins0; i += kQThreads) (&h[0][0])[i] = 0u;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kQChunk, r1 = min(m, r0 + kQChunk);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kQThreads) {
#pragma unroll
    for (int j = 0; j < kQFeatGroup; ++j)
      if (f0 + j < d) atomicAdd(&h[j][ordered_key(sample_at(X, r, stride, ld, f0 + j)) >> 21], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kQFeatGroup * kQBins0; i += kQThreads) {
    const int j = i / kQBins0, b = i % kQBins0;
    const uint32_t c = h[j][b];
    if (c != 0u && f0 + j < d) atomicAdd(hist0 + (int64_t)(f0 + j) * kQBins0 + b, c);
  }
}

// One block per feature.  Targets: t = 0 -> rank 0 (the minimum), t >= 1 -> floor(t m / max_bin).
// Out: per target its top digit, in-bucket rank, and its bucket's run [off, off + cnt) inside the
// feature's compacted area; cursor[f][b] = run start of a target bucket, -1 for the others.
__global__ __launch_bounds__(kQThreads) void qsel_plan_kernel(const uint32_t* __restrict__ hist0, int64_t m,
                                                              int max_bin, int* __restrict__ cursor,
                                                              int* __restrict__ tdig, int64_t* __restrict__ trank,
                                                              int64_t* __restrict__ toff, int64_t* __restrict__ tcnt) {
  __shared__ uint32_t h[kQBins0];
  __shared__ uint32_t pre[kQBins0];
  __shared__ uint32_t flag[kQBins0];
  const int f = blockIdx.x;
  for (int i = threadIdx.x; i < kQBins0; i += kQThreads) {
    h[i] = hist0[(int64_t)f * kQBins0 + i];
    flag[i] = 0u;
  }
  __syncthreads();
  excl_scan<kQBins0>(h, pre);
  // target t: the largest bin with pre[b] <= r is non-empty and holds rank r (r < m = total)
  for (int t = threadIdx.x; t < max_bin; t += kQThreads) {
    const uint32_t r = t == 0 ? 0u : (uint32_t)(((int64_t)t * m) / max_bin);
    int lo = 0;
#pragma unroll
    for (int half = kQBins0 / 2; half >= 1; half >>= 1)
      if (pre[lo + half] <= r) lo += half;
    tdig[f * kQThreads + t] = lo;
    trank[f * kQThreads + t] = (int64_t)(r - pre[lo]);
    flag[lo] = h[lo];  // same value from every target of the bucket
  }
  __syncthreads();
  excl_scan<kQBins0>(flag, pre);  // compacted runs of the target buckets only
  for (int i = threadIdx.x; i < kQBins0; i += kQThreads)
    cursor[(int64_t)f * kQBins0 + i] = flag[i] ? (int)pre[i] : -1;
  for (int t = threadIdx.x; t < max_bin; t += kQThreads) {
    const int b = tdig[f * kQThreads + t];
    toff[f * kQThreads + t] = pre[b];
    tcnt[f * kQThreads + t] = h[b];
  }
}

__global__ __launch_bounds__(kQThreads) void qsel_scatter_kernel(const float* __restrict__ X, int64_t m,
                                                                 int64_t stride, int ld, int d,
                                                                 int* __restrict__ cursor,
                                                                 uint32_t* __restrict__ runs) {
  __shared__ uint32_t cnt[kQFeatGroup][kQBins0];   // 32 KiB
  __shared__ int lbase[kQFeatGroup][kQBins0];      // 32 KiB
  const int f0 = blockIdx.y * kQFeatGroup;
  for (int i = threadIdx.x; i < kQFeatGroup * kQBins0; i += kQThreads) {
    const int j = i / kQBins0, b = i % kQBins0;
    (&cnt[0][0])[i] = 0u;
    (&lbase[0][0])[i] = f0 + j < d ? cursor[(int64_t)(f0 + j) * kQBins0 + b] : -1;  // -1: not a target
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kQChunk, r1 = min(m, r0 + kQChunk);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kQThreads) {
#pragma unroll
    for (int j = 0; j < kQFeatGroup; ++j) {
      if (f0 + j >= d) continue;
      const uint32_t b = ordered_key(sample_at(X, r, stride, ld, f0 + j)) >> 21;
      if (lbase[j][b] >= 0) atomicAdd(&cnt[j][b], 1u);
    }
  }
  __syncthreads();
  // reserve this block's slice of every target run it touches
  for (int i = threadIdx.x; i < kQFeatGroup * kQBins0; i += kQThreads) {
    const int j = i / kQBins0, b = i % kQBins0;
    const uint32_t c = cnt[j][b];
    if (c != 0u) lbase[j][b] = atomicAdd(cursor + (int64_t)(f0 + j) * kQBins0 + b, (int)c);
    cnt[j][b] = 0u;
  }
  __syncthreads();
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kQThreads) {
#pragma unroll
    for (int j = 0; j < kQFeatGroup; ++j) {
      if (f0 + j >= d) continue;
      const uint32_t k = ordered_key(sample_at(X, r, stride, ld, f0 + j));
      const uint32_t b = k >> 21;
      const int lb = lbase[j][b];
      if (lb >= 0) {
        const uint32_t s = atomicAdd(&cnt[j][b], 1u);
        runs[(int64_t)(f0 + j) * m + lb + s] = k;
      }
    }
  }
}

// One block per (target, feature): the next 11 bits, then the last 10, over the target's run.
__global__ __launch_bounds__(kQThreads) void qsel_final_kernel(const uint32_t* __restrict__ runs, int64_t m,
                                                               int max_bin, const int* __restrict__ tdig,
                                                               const int64_t* __restrict__ trank,
                                                               const int64_t* __restrict__ toff,
                                                               const int64_t* __restrict__ tcnt,
                                                               float* __restrict__ out) {
  __shared__ uint32_t h[kQBins0];
  __shared__ uint32_t pre[kQBins0];
  const int t = blockIdx.x, f = blockIdx.y;
  if (t >= max_bin) return;
  const int ti = f * kQThreads + t;
  const uint32_t* run = runs + (int64_t)f * m + toff[ti];
  const int64_t n = tcnt[ti];
  const uint32_t top = (uint32_t)tdig[ti];
  const uint32_t r = (uint32_t)trank[ti];
  for (int i = threadIdx.x; i < kQBins0; i += kQThreads) h[i] = 0u;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += kQThreads) atomicAdd(&h[(run[i] >> 10) & (kQBins0 - 1)], 1u);
  __syncthreads();
  int b1;
  uint32_t r1;
  find_rank<kQBins0>(h, pre, r, b1, r1);
  for (int i = threadIdx.x; i < kQBins2; i += kQThreads) h[i] = 0u;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += kQThreads) {
    const uint32_t k = run[i];
    if (((k >> 10) & (kQBins0 - 1)) == (uint32_t)b1) atomicAdd(&h[k & (kQBins2 - 1)], 1u);
  }
  __syncthreads();
  int b2;
  uint32_t r2;
  find_rank<kQBins2>(h, pre, r1, b2, r2);
  if (threadIdx.x == 0) out[(int64_t)t * gridDim.y + f] = key_value((top << 21) | ((uint32_t)b1 << 10) | (uint32_t)b2);
}

}  // namespace

int64_t quantile_select_ws_bytes(int64_t m, int d) {
  // hist0 | cursor | tdig | trank | toff | tcnt | runs
  return (int64_t)d * kQBins0 * 4 * 2 + (int64_t)d * kQThreads * (4 + 8 * 3) + (int64_t)d * m * 4 + 256;
}

void launch_quantile_select(const float* X, int64_t m, int64_t stride, int ld, int d, int max_bin, void* ws,
                            float* out, hipStream_t stream) {
  if (d < 1 || d > 32 || max_bin < 2 || max_bin > kQThreads || m < 1)
    throw std::runtime_error("quantile_select: need 1 <= d <= 32, 2 <= max_bin <= 256, m >= 1");
  if (m > (int64_t)INT32_MAX) throw std::runtime_error("quantile_select: at most 2^31 - 1 sample rows");
  char* p = static_cast<char*>(ws);
  uint32_t* hist0 = reinterpret_cast<uint32_t*>(p); p += (int64_t)d * kQBins0 * 4;
  int* cursor = reinterpret_cast<int*>(p); p += (int64_t)d * kQBins0 * 4;
  int64_t* trank = reinterpret_cast<int64_t*>(p); p += (int64_t)d * kQThreads * 8;
  int64_t* toff = reinterpret_cast<int64_t*>(p); p += (int64_t)d * kQThreads * 8;
  int64_t* tcnt = reinterpret_cast<int64_t*>(p); p += (int64_t)d * kQThreads * 8;
  int* tdig = reinterpret_cast<int*>(p); p += (int64_t)d * kQThreads * 4;
  uint32_t* runs = reinterpret_cast<uint32_t*>(p);
  if (hipMemsetAsync(hist0, 0, (size_t)d * kQBins0 * 4, stream) != hipSuccess)
    throw std::runtime_error("quantile_select: memset failed");
  const dim3 grid((unsigned)((m + kQChunk - 1) / kQChunk), (unsigned)((d + kQFeatGroup - 1) / kQFeatGroup));
  qsel_hist_kernel<<<grid, kQThreads, 0, stream>>>(X, m, stride, ld, d, hist0);
  qsel_plan_kernel<<<d, kQThreads, 0, stream>>>(hist0, m, max_bin, cursor, tdig, trank, toff, tcnt);
  qsel_scatter_kernel<<<grid, kQThreads, 0, stream>>>(X, m, stride, ld, d, cursor, runs);
  qsel_final_kernel<<<dim3(max_bin, d), kQThreads, 0, stream>>>(runs, m, max_bin, tdig, trank, toff, tcnt, out);
  check_launch("quantile_select");
}

}  // namespace fdx
