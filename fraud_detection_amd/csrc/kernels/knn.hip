// K8 knn_topk: the k-nearest-neighbour search inside SMOTE.
//
// Reference behaviour being replaced: imblearn SMOTE(k_neighbors=5) fits
// NearestNeighbors(n_neighbors=6) on the minority rows and drops each row's self match
// (train_model.py:65-66,91-92; preprocess.py:43-44).
//
// MI355X mapping: distance ranking via score(c, q) = q.c - 0.5 ||c||^2 (argmax score == argmin
// squared L2).  A workgroup owns 32 queries; each of its 4 waves sweeps every 4th 32-candidate
// tile.  The 32x32 score tile is one chain of 16 v_mfma_f32_32x32x2_f32 (exact fp32, a k-ordered
// fmaf chain, so rankings match an fp32 CPU oracle) with the accumulator pre-loaded with
// -0.5||c||^2.  Candidates sit on the MFMA row axis, so each lane holds 16 scores of ONE query
// (its column) and keeps a sorted top-k of (score, index) in registers with static indices
// (insertion network); the n x n distance matrix never exists.  Lane pairs (l, l^32) and then
// the 4 waves merge their lists through LDS.  Ties break on the smaller candidate index.
// K-index layout: MFMA step s, slot h <-> feature 16h + s, so each lane's operand for all 16
// steps is 16 CONTIGUOUS floats of one row (four 16 B loads).
#include <cmath>

#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kMaxK = 8;
constexpr float kNegBig = -3.0e38f;

__device__ __forceinline__ bool better(float s, int i, float s2, int i2) {
  return s > s2 || (s == s2 && i < i2);
}

template <int K>
__device__ __forceinline__ void topk_insert(float (&bs)[K], int (&bi)[K], float s, int i) {
  if (!better(s, i, bs[K - 1], bi[K - 1])) return;
  bs[K - 1] = s;
  bi[K - 1] = i;
#pragma unroll
  for (int k = K - 1; k > 0; --k) {
    if (better(bs[k], bi[k], bs[k - 1], bi[k - 1])) {
      const float ts = bs[k]; bs[k] = bs[k - 1]; bs[k - 1] = ts;
      const int ti = bi[k]; bi[k] = bi[k - 1]; bi[k - 1] = ti;
    }
  }
}

__global__ void row_half_norms_kernel(const float* __restrict__ X, int m, float* __restrict__ out,
                                      int m_pad) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m_pad) return;
  if (r >= m) {
    out[r] = -3.0e38f;  // padding candidates can never be selected
    return;
  }
  const float4* p = reinterpret_cast<const float4*>(X + (int64_t)r * kCols);
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < kCols / 4; ++k) {
    const float4 v = p[k];
    s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
  }
  out[r] = -0.5f * s;  // stored negated: it initialises the MFMA accumulator directly
}

// Q: [mq_pad][32] fp32 queries, C: [mc_pad][32] fp32 candidates, chalf: [mc_pad] 0.5||c||^2.
// Query row q is candidate row (self_offset + q) when self_offset >= 0 (self excluded).
template <int K>
__global__ __launch_bounds__(kThreads) void knn_topk_kernel(const float* __restrict__ Q, int mq,
                                                            const float* __restrict__ C,
                                                            const float* __restrict__ chalf,
                                                            int mc_pad, int mc,
                                                            int64_t self_offset,
                                                            int* __restrict__ out_idx,
                                                            float* __restrict__ out_score) {
  const int lane = lane_id(), wv = wave_id();
  const int h = lane >> 5, j = lane & 31;
  const int q0 = blockIdx.x * 32;
  const int qg = q0 + j;  // this lane's query (column of the score tile)
  const int64_t self_c = self_offset >= 0 ? self_offset + qg : -1;
  float bq[16];
  {
    const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)qg * kCols + 16 * h);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = p[k];
      bq[4 * k] = v.x; bq[4 * k + 1] = v.y; bq[4 * k + 2] = v.z; bq[4 * k + 3] = v.w;
    }
  }
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }

  // per-lane parking row for one tile's 16 scores (stride 17 floats: conflict-free column reads)
  __shared__ float park_all[kWaves][kWave * 17];
  float* park = park_all[wv];
  // blockIdx.y selects a contiguous slice of candidate tiles (split-K over candidates: enough
  // workgroups to fill 256 CUs and several waves per SIMD to hide the top-k VALU work behind
  // other waves' MFMA); slices write partial lists merged by knn_merge_kernel.
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  const int ntiles = t_hi;
  // Register double buffer: the next candidate tile (16 floats of one row + 16 norms per lane,
  // L2-resident) is fetched while the current tile's MFMA chain and top-k run.
  float4 cv[4], nv[4];
  auto fetch = [&](int t, float4 (&a)[4], float4 (&b)[4]) {
    const int cb = t * 32;
    const float4* p = reinterpret_cast<const float4*>(C + (int64_t)(cb + j) * kCols + 16 * h);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = p[k];
      // accumulator rows (k&3)+8(k>>2)+4h -> 4 contiguous candidates per register group
      b[k] = *reinterpret_cast<const float4*>(chalf + cb + 8 * k + 4 * h);
    }
  };
  if (t_lo + wv < ntiles) fetch(t_lo + wv, cv, nv);
  for (int t = t_lo + wv; t < ntiles; t += kWaves) {
    const int c0 = t * 32;
    float ac[16];
    f32x16_t acc;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ac[4 * k] = cv[k].x; ac[4 * k + 1] = cv[k].y; ac[4 * k + 2] = cv[k].z; ac[4 * k + 3] = cv[k].w;
      acc[4 * k] = nv[k].x; acc[4 * k + 1] = nv[k].y; acc[4 * k + 2] = nv[k].z; acc[4 * k + 3] = nv[k].w;
    }
    if (t + kWaves < ntiles) fetch(t + kWaves, cv, nv);
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[s], bq[s], acc, 0, 0, 0);
    // Fast path: the tile's best score (v_max3 tree) against this lane's current k-th best.  Once
    // the lists are warm almost every tile fails for every lane, costing ~10 VALU instead of the
    // exact masked filter below (the max includes self/padding, which can only cause a harmless
    // trip into the exact path).
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
    if (!__any(mx >= bs[K - 1])) continue;
    // Exact filter: a candidate can only enter the list if it beats the CURRENT k-th best (which
    // only improves), so 16 compares build a bitmask; the tile's scores are parked in this lane's
    // LDS row and only set bits are inserted (dynamic index via LDS, not register arrays).
    unsigned mask = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = c0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const float sc = (ci == self_c || ci >= mc) ? kNegBig : acc[r];
      acc[r] = sc;
      mask |= better(sc, ci, bs[K - 1], bi[K - 1]) ? (1u << r) : 0u;
    }
    if (__any(mask != 0)) {
      float* my = park + lane * 17;
#pragma unroll
      for (int r = 0; r < 16; ++r) my[r] = acc[r];
      while (__any(mask != 0)) {
        if (mask) {
          const int r = __builtin_ctz(mask);
          mask &= mask - 1;
          const int ci = c0 + (r & 3) + 8 * (r >> 2) + 4 * h;
          topk_insert<K>(bs, bi, my[r], ci);
        }
      }
    }
  }
  // merge with the other half-wave (same query, other candidate rows)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s2 = __shfl_xor(bs[k], 32, kWave);
    const int i2 = __shfl_xor(bi[k], 32, kWave);
    if (h == 0) topk_insert<K>(bs, bi, s2, i2);
  }
  __shared__ float ls[kWaves][32][K];
  __shared__ int li[kWaves][32][K];
  if (h == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) { ls[wv][j][k] = bs[k]; li[wv][j][k] = bi[k]; }
  }
  __syncthreads();
  if (wv == 0 && h == 0) {
#pragma unroll
    for (int w2 = 1; w2 < kWaves; ++w2) {
#pragma unroll
      for (int k = 0; k < K; ++k) topk_insert<K>(bs, bi, ls[w2][j][k], li[w2][j][k]);
    }
    if (qg < mq) {
      // gridDim.y > 1: partial list of this slice at [blockIdx.y][q][k] of the workspace
      const int64_t o = ((int64_t)blockIdx.y * mq + qg) * K;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        out_idx[o + k] = bi[k];
        if (out_score) out_score[o + k] = bs[k];
      }
    }
  }
}

// Merge the per-slice top-k lists of every query (same ordering: score desc, index asc).
template <int K>
__global__ __launch_bounds__(256) void knn_merge_kernel(const float* __restrict__ ps, const int* __restrict__ pi,
                                                        int nsplit, int mq, int* __restrict__ out_idx,
                                                        float* __restrict__ out_score) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= mq) return;
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  for (int s = 0; s < nsplit; ++s) {
    const int64_t o = ((int64_t)s * mq + q) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) topk_insert<K>(bs, bi, ps[o + k], pi[o + k]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    out_idx[(int64_t)q * K + k] = bi[k];
    if (out_score) out_score[(int64_t)q * K + k] = bs[k];
  }
}

}  // namespace

void launch_row_half_norms(const float* X, int m, float* out, int m_pad, hipStream_t stream) {
  row_half_norms_kernel<<<(m_pad + 255) / 256, 256, 0, stream>>>(X, m, out, m_pad);
  check_launch("row_half_norms");
}

int knn_splits(int mq_pad, int mc_pad) {
  // Candidate slices restart their top-k lists (fill cost), so use the fewest slices that give
  // >= 2 workgroups per CU with the best whole-round balance over the CUs.
  const int qblocks = mq_pad / 32, tiles = mc_pad / 32;
  const int cus = device_cu_count();
  int max_s = tiles / (kWaves * 8);
  if (max_s > 16) max_s = 16;
  if (max_s < 1) max_s = 1;
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= max_s; ++s) {
    const double blocks = (double)qblocks * s;
    const double rounds = std::ceil(blocks / cus);
    double eff = blocks / (rounds * cus);     // load balance of the last round
    if (blocks < 2.0 * cus) eff *= 0.5;       // too few waves per SIMD to overlap VALU with MFMA
    eff -= 0.01 * (s - 1);                    // fill cost of every extra slice
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return best;
}

void launch_knn_topk(const float* Q, int mq_pad, int mq, const float* C, const float* chalf,
                     int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                     float* out_score, float* ws_score, int* ws_idx, int nsplit, hipStream_t stream) {
  if (mq_pad % 32 != 0 || mc_pad % 32 != 0) throw std::runtime_error("knn_topk: pads must be x32");
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 1 && (ws_score == nullptr || ws_idx == nullptr))
    throw std::runtime_error("knn_topk: split search needs the [nsplit][mq][k] workspaces");
  const dim3 grid(mq_pad / 32, nsplit);
  int* oi = nsplit > 1 ? ws_idx : out_idx;
  float* os = nsplit > 1 ? ws_score : out_score;
#define FDX_KNN(KK)                                                                             \
  knn_topk_kernel<KK><<<grid, kThreads, 0, stream>>>(Q, mq, C, chalf, mc_pad, mc, self_offset, oi, \
                                                     os);                                        \
  if (nsplit > 1)                                                                               \
    knn_merge_kernel<KK><<<(mq + 255) / 256, 256, 0, stream>>>(ws_score, ws_idx, nsplit, mq, out_idx, out_score)
  switch (k) {
    case 1: FDX_KNN(1); break;
    case 2: FDX_KNN(2); break;
    case 3: FDX_KNN(3); break;
    case 4: FDX_KNN(4); break;
    case 5: FDX_KNN(5); break;
    case 6: FDX_KNN(6); break;
    case 7: FDX_KNN(7); break;
    case 8: FDX_KNN(8); break;
    default: throw std::runtime_error("knn_topk: k must be in [1, 8]");
  }
#undef FDX_KNN
  check_launch("knn_topk");
}

}  // namespace fdx
