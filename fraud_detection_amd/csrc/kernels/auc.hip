// K10 auc / confusion: exact ROC-AUC and confusion counts on device.
//
// Reference behaviour being replaced: sklearn roc_auc_score / roc_curve+auc / confusion_matrix
// (train_model.py:83,109; evaluate_model.py:31,45,49-50).
//
// Exact AUC = (#{(p,n): s_p > s_n} + 0.5 #{(p,n): s_p == s_n}) / (P N).
// Fraud data is heavily imbalanced, so (small positive class) instead of sorting all N scores we
// sort only the positive class (compacted, then bitonic-sorted in LDS chunks of <= 16384 floats = 64 KiB) and let every
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

// ---- exact AUC for any class balance: native LSD radix sort + one counting pass -------------
// The chunked path above costs ~N log(chunk) per 16384 positives (quadratic in spirit once
// positives are common).  Here the (score, label) pairs are sorted by (score, label) -- a stable
// LSD radix sort of the 32-bit order-preserving score key, with the label as the least significant
// "digit" (pass 0) so inside a tie the negatives come first -- and then, with i the sorted index:
//   sum over positives of #neg with key <= key_i  =  sum_pos (i - #pos before i)
//                                                  =  S1 - P (P - 1) / 2,   S1 = sum_pos i
//   twice_pairs = 2 (S1 - P (P - 1) / 2) - T,      T = sum over tie segments of P_seg N_seg
// (2 #{s_p > s_n} + #{s_p == s_n} = sum_pos (2 #neg< + #neg=) = 2 sum_pos #neg<= - sum_pos #neg=).
// T needs the segment bounds only where a segment mixes the classes: at its first positive (its
// predecessor is a negative of the same key) two binary searches find [lo, hi).  All counts are
// 64-bit integers (order independent): bitwise deterministic and equal to sklearn's tie-averaged
// roc_auc_score.  Each radix pass = digit histogram per block -> one-block exclusive scan (digit-
// major, so offsets are stable across blocks) -> stable scatter (per 256-key sub-chunk: wave-level
// match of equal digits by 8 ballots, ranks = popcount of lower peers, waves ordered through LDS).
constexpr int kRadixBlocks = 1024;

__device__ __forceinline__ uint32_t radix_digit(uint32_t k, uint8_t l, int shift) {
  return shift < 0 ? (uint32_t)l : ((k >> shift) & 255u);
}

__global__ __launch_bounds__(kThreads) void radix_init_kernel(const float* __restrict__ s,
                                                              const uint8_t* __restrict__ y, int64_t n,
                                                              uint32_t* __restrict__ key, uint8_t* __restrict__ lab) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    key[i] = order_key(s[i]);
    lab[i] = y[i] != 0 ? 1 : 0;
  }
}

__global__ __launch_bounds__(kThreads) void radix_hist_kernel(const uint32_t* __restrict__ key,
                                                              const uint8_t* __restrict__ lab, int64_t n,
                                                              int shift, int64_t per_blk,
                                                              uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_blk, b1 = min(n, b0 + per_blk);
  for (int64_t i = b0 + t; i < b1; i += kThreads) atomicAdd(&h[radix_digit(key[i], lab[i], shift)], 1u);
  __syncthreads();
  hist[(int64_t)t * gridDim.x + blockIdx.x] = h[t];  // digit-major: the scan order = stable order
}

// Exclusive scan of one wave's values (inclusive shuffle scan minus the own value); *tot = sum.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* tot) {
  const int lane = lane_id();
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  *tot = __shfl(inc, kWave - 1, kWave);
  return inc - v;
}

// Per-digit scan of the digit-major [256][nblk] block counts: block d scans row d in place
// (within-digit offsets, stable across blocks) and writes the digit's total; the scatter kernel
// adds the exclusive scan of the 256 totals.  (Was one 1024-thread block walking 1024-element
// runs per thread -- uncoalesced, 256 dependent loads per thread: ~330 us per radix pass at 2M
// scores, profiles/r4_i/timeline_cv_job.txt; now two parallel scans of <= 1024 elements.)
__global__ __launch_bounds__(1024) void radix_rowscan_kernel(uint32_t* __restrict__ hist, int nblk,
                                                             uint32_t* __restrict__ tot) {
  __shared__ uint32_t wsum[16];
  const int t = threadIdx.x, w = wave_id();
  uint32_t* row = hist + (int64_t)blockIdx.x * nblk;
  const uint32_t v = t < nblk ? row[t] : 0u;
  uint32_t wt;
  const uint32_t ex = wave_excl_scan(v, &wt);
  if (lane_id() == 0) wsum[w] = wt;
  __syncthreads();
  uint32_t wb = 0, all = 0;
  for (int i = 0; i < 16; ++i) {
    const uint32_t x = wsum[i];
    wb += i < w ? x : 0u;
    all += x;
  }
  if (t < nblk) row[t] = wb + ex;
  if (t == 0) tot[blockIdx.x] = all;
}

__global__ __launch_bounds__(kThreads) void radix_scatter_kernel(const uint32_t* __restrict__ key,
                                                                 const uint8_t* __restrict__ lab, int64_t n,
                                                                 int shift, int64_t per_blk,
                                                                 const uint32_t* __restrict__ offs,
                                                                 const uint32_t* __restrict__ tot,
                                                                 uint32_t* __restrict__ key_out,
                                                                 uint8_t* __restrict__ lab_out) {
  __shared__ uint32_t run[256];
  __shared__ uint32_t wc[kThreads / kWave][256];
  __shared__ uint32_t dsum[kThreads / kWave];
  const int t = threadIdx.x, w = wave_id(), lane = lane_id();
  {  // digit base = exclusive scan of the 256 digit totals (kThreads == 256: one digit per thread)
    uint32_t wt;
    const uint32_t ex = wave_excl_scan(tot[t], &wt);
    if (lane == 0) dsum[w] = wt;
    __syncthreads();
    uint32_t wb = 0;
    for (int i = 0; i < w; ++i) wb += dsum[i];
    run[t] = wb + ex + offs[(int64_t)t * gridDim.x + blockIdx.x];
  }
#pragma unroll
  for (int v = 0; v < kThreads / kWave; ++v) wc[v][t] = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t b0 = (int64_t)blockIdx.x * per_blk, b1 = min(n, b0 + per_blk);
  for (int64_t base = b0; base < b1; base += kThreads) {
    const int64_t i = base + t;
    const bool valid = i < b1;
    const uint32_t k = valid ? key[i] : 0u;
    const uint8_t l = valid ? lab[i] : (uint8_t)0;
    const uint32_t dg = valid ? radix_digit(k, l, shift) : 0u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot(valid && ((dg >> b) & 1u));
      peers &= ((dg >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt);
    __syncthreads();  // previous sub-chunk's run update / wc reset is visible
    if (valid && rank == 0) wc[w][dg] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[dg] + rank;
      for (int v = 0; v < w; ++v) pos += wc[v][dg];
      key_out[pos] = k;
      lab_out[pos] = l;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int v = 0; v < kThreads / kWave; ++v) {
      add += wc[v][t];
      wc[v][t] = 0;
    }
    run[t] += add;
  }
}

__device__ __forceinline__ int64_t lower_bound_u32(const uint32_t* a, int64_t lo, int64_t hi, uint32_t v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t upper_bound_u32(const uint32_t* a, int64_t lo, int64_t hi, uint32_t v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// out[0] += S1 = sum of sorted positions of positives, out[1] += T, out[2] += P
__global__ __launch_bounds__(kThreads) void auc_sorted_count_kernel(const uint32_t* __restrict__ key,
                                                                    const uint8_t* __restrict__ lab, int64_t n,
                                                                    unsigned long long* __restrict__ out) {
  unsigned long long s1 = 0, tt = 0, p = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    if (!lab[i]) continue;
    s1 += (unsigned long long)i;
    p += 1;
    if (i > 0 && lab[i - 1] == 0 && key[i - 1] == key[i]) {  // first positive of a mixed tie segment
      const uint32_t kv = key[i];
      const int64_t lo = lower_bound_u32(key, 0, i, kv);
      const int64_t hi = upper_bound_u32(key, i, n, kv);
      tt += (unsigned long long)(hi - i) * (unsigned long long)(i - lo);
    }
  }
  s1 = wave_sum(s1);
  tt = wave_sum(tt);
  p = wave_sum(p);
  if (lane_id() == 0) {
    if (s1) atomicAdd(out, s1);
    if (tt) atomicAdd(out + 1, tt);
    if (p) atomicAdd(out + 2, p);
  }
}

// res[0] = twice_pairs, res[1] = P, res[2] = N (int64); auc[0] = twice / (2 P N) (NaN if a class is empty)
__global__ void auc_sorted_finalize_kernel(const unsigned long long* __restrict__ cnt, int64_t n,
                                           int64_t* __restrict__ res, double* __restrict__ auc) {
  const long long P = (long long)cnt[2], N = n - P;
  const long long twice = 2 * ((long long)cnt[0] - P * (P - 1) / 2) - (long long)cnt[1];
  res[0] = (P > 0 && N > 0) ? twice : 0;
  res[1] = P;
  res[2] = N;
  auc[0] = (P > 0 && N > 0) ? (double)twice / (2.0 * (double)P * (double)N) : __builtin_nan("");
}

}  // namespace

// Workspace layout, every region 256-byte aligned (the u64 counters take 64-bit atomics; an odd n
// must not shift them off alignment): k0 | k1 (u32 [n]) | l0 | l1 (u8 [n]) | hist (u32 [256][blocks])
// | cnt (u64 [3]) | tot (u32 [256]).  Offsets in bytes; [7] = total.
static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
void auc_radix_layout(int64_t n, size_t off[8]) {
  const size_t nn = (size_t)(n > 0 ? n : 0);
  off[0] = 0;
  off[1] = align256(off[0] + nn * 4);
  off[2] = align256(off[1] + nn * 4);
  off[3] = align256(off[2] + nn);
  off[4] = align256(off[3] + nn);
  off[5] = align256(off[4] + (size_t)256 * kRadixBlocks * 4);
  off[6] = align256(off[5] + 3 * sizeof(unsigned long long));
  off[7] = align256(off[6] + 256 * 4);  // per-digit totals
}

size_t auc_radix_workspace_bytes(int64_t n) {
  size_t off[8];
  auc_radix_layout(n, off);
  return off[7];
}

void launch_auc_radix(const float* scores, const uint8_t* labels, int64_t n, void* ws, int64_t* res, double* auc,
                      hipStream_t stream) {
  if (reinterpret_cast<uintptr_t>(ws) % 256 != 0) throw std::runtime_error("auc_radix: workspace must be 256-byte aligned");
  size_t off[8];
  auc_radix_layout(n, off);
  char* p = static_cast<char*>(ws);
  uint32_t* k0 = reinterpret_cast<uint32_t*>(p + off[0]);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(p + off[1]);
  uint8_t* l0 = reinterpret_cast<uint8_t*>(p + off[2]);
  uint8_t* l1 = reinterpret_cast<uint8_t*>(p + off[3]);
  uint32_t* hist = reinterpret_cast<uint32_t*>(p + off[4]);
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(p + off[5]);
  uint32_t* tot = reinterpret_cast<uint32_t*>(p + off[6]);
  if (hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), stream) != hipSuccess)
    throw std::runtime_error("auc_radix: memset failed");
  if (n > 0) {
    if (n > 0xFFFFFFFFll) throw std::runtime_error("auc_radix: at most 2^32 scores");
    radix_init_kernel<<<stream_grid(n, kThreads, 4096), kThreads, 0, stream>>>(scores, labels, n, k0, l0);
    // fewer blocks for small inputs (each owns a contiguous, 256-aligned range)
    int64_t per_blk = (n + kRadixBlocks - 1) / kRadixBlocks;
    per_blk = std::max<int64_t>(kThreads, (per_blk + kThreads - 1) / kThreads * kThreads);
    const int nblk = (int)((n + per_blk - 1) / per_blk);
    const int shifts[5] = {-1, 0, 8, 16, 24};  // label digit first (least significant), then key bytes
    for (int ps = 0; ps < 5; ++ps) {
      radix_hist_kernel<<<nblk, kThreads, 0, stream>>>(k0, l0, n, shifts[ps], per_blk, hist);
      radix_rowscan_kernel<<<256, 1024, 0, stream>>>(hist, nblk, tot);
      radix_scatter_kernel<<<nblk, kThreads, 0, stream>>>(k0, l0, n, shifts[ps], per_blk, hist, tot, k1, l1);
      std::swap(k0, k1);
      std::swap(l0, l1);
    }
    auc_sorted_count_kernel<<<stream_grid(n, kThreads * 4, 2048), kThreads, 0, stream>>>(k0, l0, n, cnt);
  }
  auc_sorted_finalize_kernel<<<1, 1, 0, stream>>>(cnt, n, res, auc);
  check_launch("auc_radix");
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
