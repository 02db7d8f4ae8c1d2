// K1 scaler_stats / K2 scale_cast / stable label compaction.
//
// Reference behaviour being replaced: sklearn StandardScaler.fit / transform called from
// train_model.py:36-40, preprocess.py:32-33, api/app.py:194, predict_single.py:25
// (SURVEY.md §2.3 rows K1, K2).  Semantics: population variance (ddof=0), float64 accumulation,
// near-constant columns get scale 1 (sklearn/preprocessing/_data.py:76-89,1046-1051).
//
// MI355X mapping: the raw matrix is row-major fp32 [n][ld] (ld >= d, d <= 30).  A wave reads
// 8 rows per instruction with 8 lanes per row, each lane owning 4 fixed columns, so 64 lanes
// touch 8 consecutive rows (960 B contiguous for ld = 30): coalesced without LDS staging, and
// each lane's per-column accumulators live in registers with static indices.  Sums are taken
// relative to a pivot row in fp64 (exact zero variance for constant columns, no cancellation
// for the Time column whose mean is ~1e5), block partials are reduced in a fixed order by a
// second kernel, so results are bitwise deterministic.
#include "common.h"
#include "compact.h"
#include "launchers.h"

namespace fdx {

namespace {

constexpr int kThreads = 256;  // 4 waves
constexpr int kUnroll = 4;     // row groups in flight per lane

// Load the (up to) 4 columns [c0, c0+4) of row r, masking columns >= d.
template <int VEC>
__device__ __forceinline__ void load_row4(const float* __restrict__ X, int64_t r, int ld, int c0,
                                          int d, float (&v)[4]) {
  const float* p = X + r * (int64_t)ld + c0;
  if constexpr (VEC == 4) {
    if (c0 + 4 <= d) {
      float4 t = *reinterpret_cast<const float4*>(p);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
      return;
    }
  }
  if constexpr (VEC >= 2) {
    if (c0 + 2 <= d) {
      float2 t = *reinterpret_cast<const float2*>(p);
      v[0] = t.x; v[1] = t.y;
      if (c0 + 4 <= d) {
        float2 u = *reinterpret_cast<const float2*>(p + 2);
        v[2] = u.x; v[3] = u.y;
      } else {
        v[2] = (c0 + 2 < d) ? p[2] : 0.0f;
        v[3] = 0.0f;
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (c0 + j < d) ? p[j] : 0.0f;
}

template <int VEC>
__global__ __launch_bounds__(kThreads) void scaler_partial_kernel(const float* __restrict__ X,
                                                                  int64_t n, int ld, int d,
                                                                  const float* __restrict__ pivot,
                                                                  double* __restrict__ partial) {
  const int lane = lane_id();
  const int c0 = (lane & 7) * 4;
  const int rsub = lane >> 3;
  double piv[4], s[4], q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    piv[j] = (c0 + j < d) ? (double)pivot[c0 + j] : 0.0;
    s[j] = 0.0;
    q[j] = 0.0;
  }
  const int64_t ngroups = (n + 7) >> 3;  // groups of 8 rows
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t g = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); g < ngroups;
       g += nwaves * kUnroll) {
    float v[kUnroll][4];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t r = (g + u * nwaves) * 8 + rsub;
      ok[u] = (g + u * nwaves) < ngroups && r < n;
      if (ok[u]) {
        load_row4<VEC>(X, r, ld, c0, d, v[u]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double dd = (double)v[u][j] - piv[j];
        s[j] += dd;
        q[j] = fma(dd, dd, q[j]);
      }
    }
  }
  // reduce over the 8 row-lanes that share a column set (lane bits 3..5)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s[j] = strided_sum<8>(s[j]);
    q[j] = strided_sum<8>(q[j]);
  }
  __shared__ double red[kThreads / kWave][8][8];
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[wave_id()][lane][j] = s[j];
      red[wave_id()][lane][4 + j] = q[j];
    }
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = threadIdx.x, l8 = c >> 2, j = c & 3;
    double ss = 0.0, qq = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / kWave; ++w) {  // fixed order
      ss += red[w][l8][j];
      qq += red[w][l8][4 + j];
    }
    partial[(int64_t)blockIdx.x * 64 + c] = ss;
    partial[(int64_t)blockIdx.x * 64 + 32 + c] = qq;
  }
}

// Fast path for contiguous rows (ld == d, 16 B aligned): 128-row tiles arrive through fully
// coalesced 16 B loads into LDS; thread (column c = tid & 31, row group tid >> 5) then walks
// its column of the tile (consecutive lanes read consecutive floats: conflict-free).
constexpr int kStatTileRows = 128;

__global__ __launch_bounds__(kThreads) void scaler_partial_tiled_kernel(const float* __restrict__ X,
                                                                        int64_t n, int d,
                                                                        const float* __restrict__ pivot,
                                                                        double* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) float tile[kStatTileRows * 30];
  __shared__ double red[2][8][32];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const double piv = (c < d) ? (double)pivot[c] : 0.0;
  double s = 0.0, q = 0.0;
  const int64_t ntiles = (n + kStatTileRows - 1) / kStatTileRows;
  const int64_t total = n * (int64_t)d;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t f0 = t * kStatTileRows * (int64_t)d;
    const int nf = (int)((total - f0) < (int64_t)kStatTileRows * d ? (total - f0) : (int64_t)kStatTileRows * d);
    const int nf4 = nf >> 2;
    const float4* src = reinterpret_cast<const float4*>(X + f0);
    for (int i = threadIdx.x; i < nf4; i += kThreads) reinterpret_cast<float4*>(tile)[i] = src[i];
    for (int i = (nf4 << 2) + threadIdx.x; i < nf; i += kThreads) tile[i] = X[f0 + i];
    __syncthreads();
    const int rows = nf / d;
    if (c < d) {
      for (int r = rg; r < rows; r += 8) {
        const double dd = (double)tile[r * d + c] - piv;
        s += dd;
        q = fma(dd, dd, q);
      }
    }
    __syncthreads();
  }
  red[0][rg][c] = s;
  red[1][rg][c] = q;
  __syncthreads();
  if (threadIdx.x < 32) {
    double ss = 0.0, qq = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) { ss += red[0][g][c]; qq += red[1][g][c]; }  // fixed order
    partial[(int64_t)blockIdx.x * 64 + c] = ss;
    partial[(int64_t)blockIdx.x * 64 + 32 + c] = qq;
  }
}

// One 128-row tile of the raw matrix into registers: 4 float4 slots + 1 tail float per thread
// (960 float4 per tile with d = 30 over 256 threads).  Returns the tile's float count.
__device__ __forceinline__ int stats_fetch(const float* __restrict__ X, int64_t t, int d, int64_t total,
                                           float4& b0, float4& b1, float4& b2, float4& b3, float& tail) {
  const int64_t f0 = t * kStatTileRows * (int64_t)d;
  const int nf = (int)((total - f0) < (int64_t)kStatTileRows * d ? (total - f0) : (int64_t)kStatTileRows * d);
  const int nf4 = nf >> 2, i = threadIdx.x;
  const float4* src = reinterpret_cast<const float4*>(X + f0);
  if (i < nf4) b0 = src[i];
  if (i + kThreads < nf4) b1 = src[i + kThreads];
  if (i + 2 * kThreads < nf4) b2 = src[i + 2 * kThreads];
  if (i + 3 * kThreads < nf4) b3 = src[i + 3 * kThreads];
  const int ti = (nf4 << 2) + i;
  if (ti < nf) tail = X[f0 + ti];
  return nf;
}

// K1+K2 fused (bf16 training rows, standardization folded into the solver): one read of the raw
// tile feeds both the shifted fp64 column sums (as scaler_partial_tiled) and the padded bf16 row
// s = x - pivot (col 30 = bias_value, col 31 = label).  The standardization z = (s - c) / sigma
// is applied later as an exact affine map on the solver's 32x32 sums (newton_update with aff),
// so the raw matrix is read once instead of twice (stats, then cast) per fit.
// FP8: the row is written as OCP e4m3 of (x - pivot) * colscale * out_scale (32 B/row, half the
// bf16 bytes).  e4m3 needs values near unit scale, so the host passes a sample estimate of the
// mean as the pivot and of 1/sigma as colscale (ops/scaler.py fp8_fused_prescale); the exact
// statistics from this same pass turn that into the solver's affine map, so the prescale only
// has to be roughly right.
// Scatter form (IDX: cross-validation, models/cv.py): row i is written to output row idx[i] -- the
// fold-sorted training table is cast from the raw table read in order (64-byte rows land whole at
// scattered positions; gathering the 120-byte raw rows instead ran at a third of the stream rate).
template <bool NT, bool FP8, bool IDX = false>
__global__ __launch_bounds__(kThreads, FP8 ? 6 : 8) void scaler_stats_cast_kernel(
    const float* __restrict__ X, int64_t n, int d, const float* __restrict__ pivot,
    const uint8_t* __restrict__ labels, float bias_value, void* __restrict__ outv,
    double* __restrict__ partial, const float* __restrict__ colscale, float out_scale,
    const int64_t* __restrict__ idx) {
  __shared__ __attribute__((aligned(16))) float tile[kStatTileRows * 30];
  __shared__ double red[2][8][32];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const double piv = (c < d) ? (double)pivot[c] : 0.0;
  const int q = threadIdx.x & 3;  // cast: column group of both of this lane's row slots
  float pv[8], ks[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pv[j] = (8 * q + j < d) ? pivot[8 * q + j] : 0.0f;
    ks[j] = (FP8 && 8 * q + j < d) ? colscale[8 * q + j] * out_scale : 1.0f;
  }
  double s = 0.0, sq = 0.0;
  const int64_t ntiles = (n + kStatTileRows - 1) / kStatTileRows;
  const int64_t total = n * (int64_t)d;
  // Register double buffer: tile t+G's global loads (<= 4 float4 + 1 tail float per thread) are
  // in flight while tile t is reduced and cast out of LDS.
  float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0, b2 = b0, b3 = b0;
  float tail = 0.0f;
  int64_t t = blockIdx.x;
  int nf = 0;
  if (t < ntiles) nf = stats_fetch(X, t, d, total, b0, b1, b2, b3, tail);
  for (; t < ntiles; t += gridDim.x) {
    {
      const int nf4 = nf >> 2, i = threadIdx.x;
      float4* t4 = reinterpret_cast<float4*>(tile);
      if (i < nf4) t4[i] = b0;
      if (i + kThreads < nf4) t4[i + kThreads] = b1;
      if (i + 2 * kThreads < nf4) t4[i + 2 * kThreads] = b2;
      if (i + 3 * kThreads < nf4) t4[i + 3 * kThreads] = b3;
      const int ti = (nf4 << 2) + threadIdx.x;
      if (ti < nf) tile[ti] = tail;
    }
    __syncthreads();
    const int rows = nf / d;
    if (t + gridDim.x < ntiles) nf = stats_fetch(X, t + gridDim.x, d, total, b0, b1, b2, b3, tail);
    if (c < d) {
      for (int r = rg; r < rows; r += 8) {
        const double dd = (double)tile[r * d + c] - piv;
        s += dd;
        sq = fma(dd, dd, sq);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int slot = threadIdx.x + k * kThreads;  // 512 slots = 128 rows x 4 column groups
      const int r = slot >> 2;
      if (r >= rows) continue;
      const int64_t grow = t * kStatTileRows + r;
      const int64_t orow = IDX ? idx[grow] : grow;  // destination row
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cc = 8 * q + j;
        if (cc < d) o[j] = FP8 ? (tile[r * d + cc] - pv[j]) * ks[j] : tile[r * d + cc] - pv[j];
        else if (cc == kBiasCol) o[j] = bias_value;
        else if (cc == kLabelCol) o[j] = labels ? (float)labels[grow] : 0.0f;
        else o[j] = 0.0f;
      }
      if constexpr (FP8) {
        const uint2 pk = make_uint2(f32x4_to_fp8(o[0], o[1], o[2], o[3]), f32x4_to_fp8(o[4], o[5], o[6], o[7]));
        if constexpr (NT) __builtin_nontemporal_store(u32x2_t{pk.x, pk.y}, reinterpret_cast<u32x2_t*>(outv) + orow * 4 + q);
        else reinterpret_cast<uint2*>(outv)[orow * 4 + q] = pk;
      } else {
        uint4 pk;
        pk.x = pack_bf16x2(o[0], o[1]); pk.y = pack_bf16x2(o[2], o[3]);
        pk.z = pack_bf16x2(o[4], o[5]); pk.w = pack_bf16x2(o[6], o[7]);
        if constexpr (NT) __builtin_nontemporal_store(u32x4_t{pk.x, pk.y, pk.z, pk.w}, reinterpret_cast<u32x4_t*>(outv) + orow * 4 + q);
        else reinterpret_cast<uint4*>(outv)[orow * 4 + q] = pk;
      }
    }
    __syncthreads();
  }
  red[0][rg][c] = s;
  red[1][rg][c] = sq;
  __syncthreads();
  if (threadIdx.x < 32) {
    double ss = 0.0, qq = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) { ss += red[0][g][c]; qq += red[1][g][c]; }  // fixed order
    partial[(int64_t)blockIdx.x * 64 + c] = ss;
    partial[(int64_t)blockIdx.x * 64 + 32 + c] = qq;
  }
}

// Fixed-order fp64 reduction of [nblocks][64] block partials.  Block g folds partials
// [g * kRedSpan, (g + 1) * kRedSpan) into out[g][64]: 64 columns x 16 row-groups, every thread's
// <= 8 loads in flight at once.  The partials come from a whole-device pass (dirty in other XCDs'
// L2s), so a load round is a long latency: a single 1024-thread block over 2048 partials needed
// 4 rounds of 32 loads (15.7-19 us in the step timeline); two launches of one round each
// (2048 -> 16 -> 1) replace it.  The tree is fixed by nblocks only: run-to-run deterministic.
constexpr int kRedSpan = 128;
__global__ __launch_bounds__(1024) void scaler_reduce_kernel(const double* __restrict__ partial,
                                                             int nblocks, double* __restrict__ out) {
  __shared__ double red[16][64];
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int b0 = blockIdx.x * kRedSpan, b1 = min(nblocks, b0 + kRedSpan);
  double v[kRedSpan / 16];
#pragma unroll
  for (int u = 0; u < kRedSpan / 16; ++u) {
    const int b = b0 + grp + 16 * u;
    v[u] = b < b1 ? partial[(int64_t)b * 64 + e] : 0.0;
  }
  double acc = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  red[grp][e] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    double s = 0.0;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g][e];
    out[(int64_t)blockIdx.x * 64 + e] = s;
  }
}

// mean / var / scale from (possibly all-reduced) shifted sums.  One wave.
// aff (optional, [64]): the map from pivot-shifted rows s = x - pivot to standardized ones,
// z = (s - aff[c]) * aff[32 + c]; identity (0, 1) beyond d, so the intercept/label columns pass.
__global__ void scaler_finalize_kernel(const double* __restrict__ sums, double n,
                                       const float* __restrict__ pivot, int d,
                                       double* __restrict__ mean64, double* __restrict__ var64,
                                       double* __restrict__ scale64, float* __restrict__ mean32,
                                       float* __restrict__ inv32, double* __restrict__ aff,
                                       const float* __restrict__ colscale, int nparts) {
  const int c = threadIdx.x;
  if (c >= kCols) return;
  // nparts > 1: `sums` holds the first-level reduce's [nparts][64] rows, summed here in order
  // (the order of the second-level reduce launch this replaces: bit-identical sums)
  double s1 = 0.0, s2 = 0.0, sn = 0.0;
  for (int p = 0; p < nparts; ++p) {
    s1 += sums[64 * p + c];
    s2 += sums[64 * p + 32 + c];
    sn += sums[64 * p + kCols - 1];
  }
  // n < 0: the (all-reduced) row count rides in the unused slot sums[31] (one collective for the
  // sums and the count, and no host round trip for n)
  if (n < 0.0) n = sn;
  if (c < d) {
    const double m = s1 / n;
    const double mean = (double)pivot[c] + m;
    double var = s2 / n - m * m;
    if (var < 0.0) var = 0.0;
    const double eps = 2.220446049250313e-16;
    const double ub = n * eps * var + (n * mean * eps) * (n * mean * eps);
    const double scale = (var <= ub) ? 1.0 : sqrt(var);
    mean64[c] = mean;
    var64[c] = var;
    scale64[c] = scale;
    mean32[c] = (float)mean;
    inv32[c] = (float)(1.0 / scale);
    if (aff) {
      // mean - pivot, without the cancellation of (pivot + m) - pivot; fp8 rows store v = s * k
      // (colscale), so z = (s - m) / scale = (v - k m) * (1 / (scale k))
      const double k = colscale ? (double)colscale[c] : 1.0;
      aff[c] = m * k;
      aff[32 + c] = 1.0 / scale / k;
    }
  } else {
    mean64[c] = 0.0; var64[c] = 0.0; scale64[c] = 1.0;
    mean32[c] = 0.0f; inv32[c] = 0.0f;
    if (aff) {
      aff[c] = 0.0;
      aff[32 + c] = 1.0;
    }
  }
}

// fp8 prescale sample (ops/scaler.fp8_fused_prescale): fp64 sums of ns rows strided by `stride`
// (rows 0, stride, 2 stride, ...), shifted by row 0, in the [nblocks][64] partial layout that
// scaler_reduce_kernel folds.  Thread (column c = tid & 31, row lane tid >> 5): the 32 lanes of a
// half-wave read one row's d floats contiguously.
// 1024 blocks x 8 row lanes: the 65536 sampled rows are 8 per thread, all loads in flight at
// once (the sampled rows are a page apart: each load is a DRAM + TLB miss)
constexpr int kSampleBlocks = 1024;

__global__ __launch_bounds__(kThreads) void sample_partial_kernel(const float* __restrict__ X, int d, int64_t ns,
                                                                  int64_t stride, double* __restrict__ partial) {
  const int c = threadIdx.x & 31, rl = threadIdx.x >> 5;
  double s = 0.0, q = 0.0;
  if (c < d) {
    const double piv = (double)X[c];
    // every strided row load of a thread in flight before any use: the sampled rows are far
    // apart (no locality); a one-load-at-a-time loop over 128 blocks paid ~64 memory latencies
    // in a row per thread (~70 us in front of every fp8 fit)
    constexpr int U = 8;
    const int64_t rs = (int64_t)gridDim.x * 8;
    for (int64_t i0 = (int64_t)blockIdx.x * 8 + rl; i0 < ns; i0 += rs * U) {
      float x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * rs;
        x[u] = i < ns ? X[i * stride * d + c] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + u * rs < ns) {
          const double v = (double)x[u] - piv;
          s += v;
          q = fma(v, v, q);
        }
      }
    }
  }
  __shared__ double red[8][64];
  red[rl][c] = s;
  red[rl][32 + c] = q;
  __syncthreads();
  if (threadIdx.x < 64) {
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += red[r][threadIdx.x];  // fixed order
    partial[(int64_t)blockIdx.x * 64 + threadIdx.x] = a;
  }
}

// mean and 1 / std (population; constant columns -> 1) of the sample, as float32 prescale vectors
__global__ void sample_finalize_kernel(const double* __restrict__ sums, const float* __restrict__ X, int d,
                                       double ns, float* __restrict__ mu, float* __restrict__ k) {
  const int c = threadIdx.x;
  if (c >= d) return;
  const double m = sums[c] / ns;
  double var = sums[32 + c] / ns - m * m;
  if (var < 0.0) var = 0.0;
  mu[c] = (float)((double)X[c] + m);
  k[c] = var > 0.0 ? (float)(1.0 / sqrt(var)) : 1.0f;
}

// K2: standardize + pad to 32 columns + cast.  OUT: 0 = bf16, 1 = fp32, 2 = fp8 e4m3fn.
// Optional row gather (idx != nullptr): output row i reads input row idx[i].
template <int VEC, int OUT>
__global__ __launch_bounds__(kThreads) void scale_cast_kernel(
    const float* __restrict__ X, int64_t n, int ld, int d, const int64_t* __restrict__ idx,
    const float* __restrict__ mean32, const float* __restrict__ inv32,
    const uint8_t* __restrict__ labels, float bias_value, float out_scale, void* __restrict__ out) {
  const int lane = lane_id();
  const int c0 = (lane & 7) * 4;
  const int rsub = lane >> 3;
  float mu[4], inv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mu[j] = mean32[c0 + j];
    inv[j] = inv32[c0 + j];
  }
  const int64_t ngroups = (n + 7) >> 3;
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t g = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); g < ngroups;
       g += nwaves * kUnroll) {
    float v[kUnroll][4];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t row = (g + u * nwaves) * 8 + rsub;
      ok[u] = (g + u * nwaves) < ngroups && row < n;
      if (ok[u]) {
        const int64_t src = idx ? idx[row] : row;
        load_row4<VEC>(X, src, ld, c0, d, v[u]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = 0.0f;  // defined on every path: v stays in VGPRs
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (!ok[u]) continue;
      const int64_t row = (g + u * nwaves) * 8 + rsub;  // recomputed: no int64 array to spill
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c < d) o[j] = (v[u][j] - mu[j]) * inv[j];
        else if (c == kBiasCol) o[j] = bias_value;
        else if (c == kLabelCol) {
          const int64_t src = idx ? idx[row] : row;
          o[j] = labels ? (float)labels[src] : 0.0f;
        } else o[j] = 0.0f;
      }
      const int64_t base = row * kCols + c0;
      if constexpr (OUT == 0) {
        uint2 pk;
        pk.x = pack_bf16x2(o[0], o[1]);
        pk.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + base) = pk;
      } else if constexpr (OUT == 1) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + base) =
            make_float4(o[0], o[1], o[2], o[3]);
      } else {
        // fp8 storage: features are multiplied by out_scale (per-tensor) before encoding;
        // bias / label columns are stored unscaled (1.0 and 0/1 are exact in e4m3).
        uint32_t pk = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float val = (c0 + j < d) ? o[j] * out_scale : o[j];
          pk |= (uint32_t)f32_to_fp8e4m3(val) << (8 * j);
        }
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(out) + base) = pk;
      }
    }
  }
}

// K2 fast path for contiguous rows (ld == d, 16 B aligned base): a 128-row tile is one
// contiguous block of 128*d floats, loaded with fully coalesced 16 B loads into LDS (the 120 B
// rows of the creditcard layout are not 16 B aligned individually), then re-read row-wise so
// every lane emits 8 output columns: one 16 B bf16 store (64 lanes = 16 rows = 1 KiB contiguous).
constexpr int kTileRows = 128;

template <int OUT>
__global__ __launch_bounds__(kThreads) void scale_cast_tiled_kernel(
    const float* __restrict__ X, int64_t n, int d, const float* __restrict__ mean32,
    const float* __restrict__ inv32, const uint8_t* __restrict__ labels, float bias_value,
    float out_scale, void* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float tile[kTileRows * 30];
  const int64_t ntiles = (n + kTileRows - 1) / kTileRows;
  const int64_t total = n * (int64_t)d;
  const int q = threadIdx.x & 3;  // column group of both of this lane's slots
  float mu[8], inv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean32[8 * q + j];
    inv[j] = inv32[8 * q + j];
  }
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t f0 = t * kTileRows * (int64_t)d;  // first float of the tile
    const int nf = (int)((total - f0) < (int64_t)kTileRows * d ? (total - f0) : (int64_t)kTileRows * d);
    const int nf4 = nf >> 2;
    const float4* src = reinterpret_cast<const float4*>(X + f0);
    for (int i = threadIdx.x; i < nf4; i += kThreads) reinterpret_cast<float4*>(tile)[i] = src[i];
    for (int i = (nf4 << 2) + threadIdx.x; i < nf; i += kThreads) tile[i] = X[f0 + i];
    __syncthreads();
    const int rows = (int)((n - t * kTileRows) < kTileRows ? (n - t * kTileRows) : kTileRows);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int slot = threadIdx.x + k * kThreads;  // 512 slots = 128 rows x 4 column groups
      const int r = slot >> 2;
      if (r >= rows) continue;
      const int64_t grow = t * kTileRows + r;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * q + j;
        if (c < d) o[j] = (tile[r * d + c] - mu[j]) * inv[j];
        else if (c == kBiasCol) o[j] = bias_value;
        else if (c == kLabelCol) o[j] = labels ? (float)labels[grow] : 0.0f;
        else o[j] = 0.0f;
      }
      if constexpr (OUT == 0) {
        uint4 pk;
        pk.x = pack_bf16x2(o[0], o[1]); pk.y = pack_bf16x2(o[2], o[3]);
        pk.z = pack_bf16x2(o[4], o[5]); pk.w = pack_bf16x2(o[6], o[7]);
        reinterpret_cast<uint4*>(out)[grow * 4 + q] = pk;
      } else if constexpr (OUT == 1) {
        float4* dst = reinterpret_cast<float4*>(out) + grow * 8 + 2 * q;
        dst[0] = make_float4(o[0], o[1], o[2], o[3]);
        dst[1] = make_float4(o[4], o[5], o[6], o[7]);
      } else {
        uint2 pk = make_uint2(0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (8 * q + j < d) ? o[j] * out_scale : o[j];
          const uint32_t b = f32_to_fp8e4m3(v);
          if (j < 4) pk.x |= b << (8 * j); else pk.y |= b << (8 * (j - 4));
        }
        reinterpret_cast<uint2*>(out)[grow * 4 + q] = pk;
      }
    }
    __syncthreads();
  }
}

// ---- stable compaction of row indices whose label == target -------------------------------
// Blocks own contiguous row ranges so the output order equals the input order.
__device__ __forceinline__ void block_range(int64_t n, int64_t* lo, int64_t* hi) {
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + kCompactThreads - 1) / kCompactThreads *
                      kCompactThreads;
  *lo = (int64_t)blockIdx.x * per;
  *hi = *lo + per < n ? *lo + per : n;
}

__global__ __launch_bounds__(kCompactThreads) void compact_count_kernel(
    const uint8_t* __restrict__ labels, int64_t n, int target, int64_t* __restrict__ counts) {
  int64_t lo, hi;
  block_range(n, &lo, &hi);
  int64_t c = 0;
  for (int64_t r = lo + threadIdx.x; r < hi; r += kCompactThreads) c += (labels[r] == target);
  c = wave_sum(c);
  __shared__ int64_t red[kCompactThreads / kWave];
  if (lane_id() == 0) red[wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kCompactThreads / kWave; ++w) t += red[w];
    counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kCompactThreads) void compact_count16_kernel(
    const uint8_t* __restrict__ labels, int64_t n, int target, int64_t* __restrict__ counts) {
  int64_t lo, hi;
  group_range((n + 15) / 16, &lo, &hi);
  const uint32_t pat = 0x01010101u * (uint32_t)(target & 0xff);
  int64_t c = 0;
  for (int64_t g = lo + threadIdx.x; g < hi; g += kCompactThreads) c += __popc(group_mask(labels, n, g, target, pat));
  c = wave_sum(c);
  __shared__ int64_t red[kCompactThreads / kWave];
  if (lane_id() == 0) red[wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kCompactThreads / kWave; ++w) t += red[w];
    counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kCompactThreads) void compact_write16_kernel(
    const uint8_t* __restrict__ labels, int64_t n, int target, const int64_t* __restrict__ offsets,
    int64_t* __restrict__ out_idx) {
  int64_t lo, hi;
  group_range((n + 15) / 16, &lo, &hi);
  const uint32_t pat = 0x01010101u * (uint32_t)(target & 0xff);
  __shared__ int wave_tot[kCompactThreads / kWave];
  const int lane = lane_id(), w = wave_id();
  int64_t base = offsets[blockIdx.x];
  for (int64_t g0 = lo; g0 < hi; g0 += kCompactThreads) {  // block-uniform trip count
    const int64_t g = g0 + threadIdx.x;
    uint32_t m = g < hi ? group_mask(labels, n, g, target, pat) : 0u;
    const int c = __popc(m);
    int inc = c;  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int u = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += u;
    }
    if (lane == kWave - 1) wave_tot[w] = inc;
    __syncthreads();
    int64_t off = base + inc - c;
    int total = 0;
    for (int i = 0; i < kCompactThreads / kWave; ++i) {
      if (i < w) off += wave_tot[i];
      total += wave_tot[i];
    }
    while (m) {
      const int j = __builtin_ctz(m);
      m &= m - 1;
      out_idx[off++] = 16 * g + j;
    }
    base += total;
    __syncthreads();
  }
}

// In-place exclusive scan of a small int64 array (n <= 4096), one block of 1024 threads; writes
// the total to tot.  Each thread owns 4 consecutive elements; lane totals are scanned with wave
// shuffles, wave totals by wave 0 -- integer adds, so the result is exact and order-free.
// host_tot (nullable): device address of a mapped pinned word that also receives the total
// (system-scope store): the host polls it instead of waiting for a D2H copy and its event.
__global__ __launch_bounds__(1024) void exclusive_scan_small_kernel(int64_t* __restrict__ a, int n,
                                                                    int64_t* __restrict__ tot,
                                                                    int64_t* __restrict__ host_tot) {
  __shared__ int64_t wsum[16];
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  int64_t v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (4 * t + j < n) ? a[4 * t + j] : 0;
  const int64_t mine = (v[0] + v[1]) + (v[2] + v[3]);
  int64_t inc = mine;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int64_t u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    int64_t x = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int64_t u = __shfl_up(x, o, kWave);
      if (lane >= o) x += u;
    }
    if (lane < 16) wsum[lane] = x;  // inclusive scan of wave totals
  }
  __syncthreads();
  int64_t run = (w > 0 ? wsum[w - 1] : 0) + inc - mine;  // exclusive prefix of this thread
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (4 * t + j < n) a[4 * t + j] = run;
    run += v[j];
  }
  if (t == 0) {
    *tot = wsum[15];
    if (host_tot != nullptr)
      __hip_atomic_store(host_tot, wsum[15], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(kCompactThreads) void compact_write_kernel(
    const uint8_t* __restrict__ labels, int64_t n, int target,
    const int64_t* __restrict__ offsets, int64_t* __restrict__ out_idx) {
  int64_t lo, hi;
  block_range(n, &lo, &hi);
  __shared__ int64_t wave_cnt[kCompactThreads / kWave];
  int64_t base = offsets[blockIdx.x];
  const int lane = lane_id(), w = wave_id();
  for (int64_t r0 = lo; r0 < hi; r0 += kCompactThreads) {
    const int64_t r = r0 + threadIdx.x;
    const bool hit = (r < hi) && labels[r] == target;
    const unsigned long long m = __ballot(hit);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_cnt[w] = __popcll(m);
    __syncthreads();
    int64_t off = base;
    for (int i = 0; i < w; ++i) off += wave_cnt[i];
    if (hit) out_idx[off + before] = r;
    int64_t total = 0;
    for (int i = 0; i < kCompactThreads / kWave; ++i) total += wave_cnt[i];
    base += total;
    __syncthreads();
  }
}

// Hardware fp8 codec self-check: decode all 256 codes, encode n floats (4 per thread).
__global__ void fp8_hw_check_kernel(float* __restrict__ dec, const float* __restrict__ vals, int n,
                                    uint8_t* __restrict__ enc) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 64) {
    const uint32_t w = (uint32_t)(4 * t) | ((uint32_t)(4 * t + 1) << 8) | ((uint32_t)(4 * t + 2) << 16) |
                       ((uint32_t)(4 * t + 3) << 24);
    fp8x4_to_f32(w, dec + 4 * t);
  }
  if (4 * t + 3 < n) {
    const uint32_t e = f32x4_to_fp8(vals[4 * t], vals[4 * t + 1], vals[4 * t + 2], vals[4 * t + 3]);
    *reinterpret_cast<uint32_t*>(enc + 4 * t) = e;
  }
}

inline int vec_for(const void* p, int ld) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if ((ld % 4) == 0 && (a % 16) == 0) return 4;
  if ((ld % 2) == 0 && (a % 8) == 0) return 2;
  return 1;
}

}  // namespace

void launch_scaler_partial(const float* X, int64_t n, int ld, int d, const float* pivot,
                           double* partial, int nblocks, hipStream_t stream) {
  if (ld == d && d <= 30 && (reinterpret_cast<uintptr_t>(X) % 16) == 0) {
    scaler_partial_tiled_kernel<<<nblocks, kThreads, 0, stream>>>(X, n, d, pivot, partial);
    check_launch("scaler_partial_tiled");
    return;
  }
  switch (vec_for(X, ld)) {
    case 4: scaler_partial_kernel<4><<<nblocks, kThreads, 0, stream>>>(X, n, ld, d, pivot, partial); break;
    case 2: scaler_partial_kernel<2><<<nblocks, kThreads, 0, stream>>>(X, n, ld, d, pivot, partial); break;
    default: scaler_partial_kernel<1><<<nblocks, kThreads, 0, stream>>>(X, n, ld, d, pivot, partial); break;
  }
  check_launch("scaler_partial");
}

int scaler_reduce_scratch_rows(int nblocks) {
  return nblocks > kRedSpan ? (nblocks + kRedSpan - 1) / kRedSpan : 0;
}

int launch_scaler_reduce_level1(const double* partial, int nblocks, double* mid, hipStream_t stream) {
  // the first level only: [nblocks][64] -> [g][64] rows at `mid` (g returned), which
  // scaler_finalize(nparts = g) sums in the order the second level would
  if (nblocks > kRedSpan * kRedSpan) throw std::runtime_error("scaler_reduce: too many block partials");
  const int g = (nblocks + kRedSpan - 1) / kRedSpan;
  scaler_reduce_kernel<<<g, 1024, 0, stream>>>(partial, nblocks, mid);
  check_launch("scaler_reduce");
  return g;
}

void launch_scaler_reduce(const double* partial, int nblocks, double* sums, hipStream_t stream) {
  // nblocks > kRedSpan: `partial` holds scaler_reduce_scratch_rows(nblocks) more [64] rows after
  // the block partials for the first level's outputs
  if (nblocks > kRedSpan * kRedSpan) throw std::runtime_error("scaler_reduce: too many block partials");
  if (nblocks > kRedSpan) {
    const int g = scaler_reduce_scratch_rows(nblocks);
    double* mid = const_cast<double*>(partial) + (int64_t)nblocks * 64;
    scaler_reduce_kernel<<<g, 1024, 0, stream>>>(partial, nblocks, mid);
    scaler_reduce_kernel<<<1, 1024, 0, stream>>>(mid, g, sums);
  } else {
    scaler_reduce_kernel<<<1, 1024, 0, stream>>>(partial, nblocks, sums);
  }
  check_launch("scaler_reduce");
}

void launch_scaler_finalize(const double* sums, double n, const float* pivot, int d,
                            double* mean64, double* var64, double* scale64, float* mean32,
                            float* inv32, double* aff, hipStream_t stream, const float* colscale, int nparts) {
  if (nparts < 1 || nparts > kRedSpan) throw std::runtime_error("scaler_finalize: 1 <= nparts <= 128");
  scaler_finalize_kernel<<<1, 64, 0, stream>>>(sums, n, pivot, d, mean64, var64, scale64, mean32,
                                               inv32, aff, colscale, nparts);
  check_launch("scaler_finalize");
}

int fp8_prescale_blocks() { return kSampleBlocks; }

void launch_fp8_prescale(const float* X, int64_t n, int d, int64_t ns, int64_t stride, double* partial,
                         double* sums, float* mu, float* k, hipStream_t stream) {
  if (d < 1 || d > kCols - 2) throw std::runtime_error("fp8_prescale: 1 <= d <= 30");
  if (ns < 1 || stride < 1 || (ns - 1) * stride >= n) throw std::runtime_error("fp8_prescale: sample out of range");
  // partial: (kSampleBlocks + scaler_reduce_scratch_rows(kSampleBlocks)) x 64 doubles
  sample_partial_kernel<<<kSampleBlocks, kThreads, 0, stream>>>(X, d, ns, stride, partial);
  launch_scaler_reduce(partial, kSampleBlocks, sums, stream);
  sample_finalize_kernel<<<1, 64, 0, stream>>>(sums, X, d, (double)ns, mu, k);
  check_launch("fp8_prescale");
}

// Each format's own occupancy: the fp8 instantiation holds more VGPRs (74 vs 68: 6 vs 7 blocks
// per CU), and a grid sized for bf16 ran 256 fp8 blocks in a second round (+25 us per pass).
int scaler_stats_cast_blocks(int fp8) {
  static const int cap16 = resident_cap(scaler_stats_cast_kernel<false, false>, kThreads);
  static const int cap8 = resident_cap(scaler_stats_cast_kernel<false, true>, kThreads);
  return fp8 ? cap8 : cap16;
}

void launch_scaler_stats_cast(const float* X, int64_t n, int d, const float* pivot, const uint8_t* labels,
                              float bias_value, void* out, double* partial, int nblocks, hipStream_t stream,
                              const float* colscale, float out_scale, const int64_t* idx) {
  if (d > 30 || (reinterpret_cast<uintptr_t>(X) % 16) != 0 || (reinterpret_cast<uintptr_t>(out) % 16) != 0)
    throw std::invalid_argument("scaler_stats_cast: contiguous 16-byte aligned rows, d <= 30");
  // every block must be resident at once (a second round of blocks would double the span);
  // nblocks is fixed by the caller (partial buffer), the grid-stride loop covers the rest
#define FDX_SSC(NT, F8, I)                                                                                 \
  scaler_stats_cast_kernel<NT, F8, I><<<nblocks, kThreads, 0, stream>>>(X, n, d, pivot, labels, bias_value, \
                                                                        out, partial, colscale, out_scale, idx)
  // plain row stores (launchers.h: nontemporal ones measured slower for this pass)
  if (idx != nullptr) {
    if (colscale != nullptr) FDX_SSC(false, true, true);
    else FDX_SSC(false, false, true);
  } else if (colscale != nullptr) {
    FDX_SSC(false, true, false);
  } else {
    FDX_SSC(false, false, false);
  }
#undef FDX_SSC
  check_launch("scaler_stats_cast");
}

void launch_scale_cast(const float* X, int64_t n, int ld, int d, const int64_t* idx,
                       const float* mean32, const float* inv32, const uint8_t* labels,
                       float bias_value, float out_scale, int out_kind, void* out,
                       hipStream_t stream) {
  if (idx == nullptr && ld == d && d <= 30 && (reinterpret_cast<uintptr_t>(X) % 16) == 0 &&
      (reinterpret_cast<uintptr_t>(out) % 16) == 0) {
    const int grid = stream_grid((n + kTileRows - 1) / kTileRows, 1, 2048);
    if (out_kind == 0)
      scale_cast_tiled_kernel<0><<<grid, kThreads, 0, stream>>>(X, n, d, mean32, inv32, labels, bias_value, out_scale, out);
    else if (out_kind == 1)
      scale_cast_tiled_kernel<1><<<grid, kThreads, 0, stream>>>(X, n, d, mean32, inv32, labels, bias_value, out_scale, out);
    else
      scale_cast_tiled_kernel<2><<<grid, kThreads, 0, stream>>>(X, n, d, mean32, inv32, labels, bias_value, out_scale, out);
    check_launch("scale_cast_tiled");
    return;
  }
  const int grid = stream_grid((n + 7) / 8, (kThreads / kWave) * kUnroll, 2048);
  const int vec = vec_for(X, ld);
#define FDX_SC(V, O)                                                                              \
  scale_cast_kernel<V, O><<<grid, kThreads, 0, stream>>>(X, n, ld, d, idx, mean32, inv32, labels, \
                                                         bias_value, out_scale, out)
  if (out_kind == 0) {
    if (vec == 4) FDX_SC(4, 0); else if (vec == 2) FDX_SC(2, 0); else FDX_SC(1, 0);
  } else if (out_kind == 1) {
    if (vec == 4) FDX_SC(4, 1); else if (vec == 2) FDX_SC(2, 1); else FDX_SC(1, 1);
  } else {
    if (vec == 4) FDX_SC(4, 2); else if (vec == 2) FDX_SC(2, 2); else FDX_SC(1, 2);
  }
#undef FDX_SC
  check_launch("scale_cast");
}

// Vector path when the label array is 16-byte aligned (torch allocations are); count and write
// make the same choice from the same pointer, so their per-block ranges agree.
static inline bool compact_vec(const uint8_t* labels) { return (reinterpret_cast<uintptr_t>(labels) & 15) == 0; }

void launch_fp8_hw_check(float* dec, const float* vals, int n, uint8_t* enc, hipStream_t stream) {
  const int threads = 256, blocks = (n / 4 + threads - 1) / threads + 1;
  fp8_hw_check_kernel<<<blocks, threads, 0, stream>>>(dec, vals, n, enc);
  check_launch("fp8_hw_check");
}

void launch_compact_count(const uint8_t* labels, int64_t n, int target, int64_t* counts,
                          int nblocks, hipStream_t stream) {
  if (compact_vec(labels))
    compact_count16_kernel<<<nblocks, kCompactThreads, 0, stream>>>(labels, n, target, counts);
  else
    compact_count_kernel<<<nblocks, kCompactThreads, 0, stream>>>(labels, n, target, counts);
  check_launch("compact_count");
}
void launch_exclusive_scan_small(int64_t* a, int n, int64_t* total, hipStream_t stream, int64_t* host_total) {
  exclusive_scan_small_kernel<<<1, 1024, 0, stream>>>(a, n, total, host_total);
  check_launch("exclusive_scan_small");
}
void launch_compact_write(const uint8_t* labels, int64_t n, int target, const int64_t* offsets,
                          int64_t* out_idx, int nblocks, hipStream_t stream) {
  if (compact_vec(labels))
    compact_write16_kernel<<<nblocks, kCompactThreads, 0, stream>>>(labels, n, target, offsets, out_idx);
  else
    compact_write_kernel<<<nblocks, kCompactThreads, 0, stream>>>(labels, n, target, offsets, out_idx);
  check_launch("compact_write");
}

}  // namespace fdx
