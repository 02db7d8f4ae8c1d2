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
constexpr int kQFlush = 4;               // flush a wave's queues once any lane holds this many
constexpr int kQCap = kQFlush - 1 + 16 + 1;  // + one tile's worth of appends + the dump slot

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

// Rows for the score GEMM, padded to 32 floats.  Feature columns 0..29 are copied; the
// squared-norm term rides in column 30 so that one MFMA chain yields the whole score:
//   candidate: [c_0..c_29, -0.5 ||c||^2, 0]      (padding rows: [0.., -3e38, 0] -> never chosen)
//   query:     [q_0..q_29, 1, 0]                  (padding rows: zeros)
// so  score(c, q) = q.c - 0.5 ||c||^2  with no norm loads and a zero-initialised accumulator.
__global__ void knn_prep_kernel(const float* __restrict__ X, int m, int m_pad, int role,
                                float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m_pad) return;
  float4* o = reinterpret_cast<float4*>(out + (int64_t)r * kCols);
  if (r >= m) {
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) o[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (role == 0) out[(int64_t)r * kCols + 30] = -3.0e38f;
    return;
  }
  const float4* p = reinterpret_cast<const float4*>(X + (int64_t)r * kCols);
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < kCols / 4; ++k) {
    float4 v = p[k];
    if (k == kCols / 4 - 1) {  // columns 28..31: keep 28, 29; 30 = norm term / 1, 31 = 0
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s);
      v.z = 0.0f; v.w = 0.0f;
    } else {
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
    o[k] = v;
  }
  out[(int64_t)r * kCols + 30] = role == 0 ? -0.5f * s : 1.0f;
}

// Q: [mq_pad][32] query rows and C: [mc_pad][32] candidate rows, both from knn_prep_kernel.
// Query row q is candidate row (self_offset + q) when self_offset >= 0 (self excluded).
//
// One wave per workgroup: blockIdx.x owns 32 queries, blockIdx.y a contiguous slice of the
// candidate tiles (the per-slice lists are merged by knn_merge_kernel).  Per 32-candidate tile:
//   * 16 v_mfma_f32_32x32x2_f32 give lane (j, h) the scores of query j against the 16 candidate
//     rows of half h (exact fp32: score = q.c - 0.5||c||^2, the norm term is column 30);
//   * a branch-free filter appends every score >= the lane's threshold to a per-lane LDS queue
//     (non-passing lanes store into a private dump slot instead: no exec-mask juggling);
//   * once any lane holds kQFlush entries the queues are inserted into the per-lane top-k
//     (exact score-then-index order, self/padding excluded) and the threshold becomes the k-th
//     best of the UNION of the two half-lists of the query (lanes j and j+32), which is a valid
//     filter for both halves and about twice as tight.
template <int K>
__global__ __launch_bounds__(kWave) void knn_topk_kernel(const float* __restrict__ Q, int mq,
                                                         const float* __restrict__ C,
                                                         int mc_pad, int mc,
                                                         int64_t self_offset,
                                                         int* __restrict__ out_idx,
                                                         float* __restrict__ out_score) {
  const int lane = threadIdx.x;
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
  float thr = kNegBig;

  // Per-lane queue, [slot][lane]: same-slot stores of a wave hit 64 distinct banks.  Slot
  // kQCap - 1 is the lane's dump slot.
  __shared__ int2 qent[kQCap * kWave];  // (score bits, candidate index) at [slot * 64 + lane]
  int qn = 0;
  auto flush = [&]() {
    for (int e = 0; __any(e < qn); ++e) {
      if (e < qn) {
        const int2 v = qent[e * kWave + lane];
        const int ci = v.y;
        if (ci != self_c && ci < mc) topk_insert<K>(bs, bi, __int_as_float(v.x), ci);
      }
    }
    qn = 0;
    // k-th best of the union of this lane's and its partner's (other half) sorted lists
    float ps[K];
#pragma unroll
    for (int k = 0; k < K; ++k) ps[k] = __shfl_xor(bs[k], 32, kWave);
    int ia = 0, ib = 0;
    float kth = kNegBig;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float a = kNegBig, b = kNegBig;
#pragma unroll
      for (int u = 0; u < K; ++u) { if (u == ia) a = bs[u]; if (u == ib) b = ps[u]; }
      const bool ta = a >= b;
      kth = ta ? a : b;
      ia += ta ? 1 : 0;
      ib += ta ? 0 : 1;
    }
    thr = kth;
  };
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  // register double buffer: the next tile's 16 floats per lane (L2-resident) are in flight
  // while the current tile's MFMA chain and filter run
  float4 cv[4];
  auto fetch = [&](int t, float4 (&a)[4]) {
    const float4* p = reinterpret_cast<const float4*>(C + (int64_t)(t * 32 + j) * kCols + 16 * h);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = p[k];
  };
  if (t_lo < t_hi) fetch(t_lo, cv);
  for (int t = t_lo; t < t_hi; ++t) {
    const int c0 = t * 32;
    float ac[16];
    f32x16_t acc = {};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ac[4 * k] = cv[k].x; ac[4 * k + 1] = cv[k].y; ac[4 * k + 2] = cv[k].z; ac[4 * k + 3] = cv[k].w;
    }
    if (t + 1 < t_hi) fetch(t + 1, cv);
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[s], bq[s], acc, 0, 0, 0);
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
    if (!__any(mx >= thr)) continue;
    const int cbase = c0 + 4 * h;
    int qe = qn * kWave + lane;                     // element of this lane's next free slot
    const int de = (kQCap - 1) * kWave + lane;      // this lane's dump slot
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool pass = acc[r] >= thr;
      qent[pass ? qe : de] = make_int2(__float_as_int(acc[r]), cbase + (r & 3) + 8 * (r >> 2));
      qe += pass ? kWave : 0;
    }
    qn = (qe - lane) / kWave;
    if (__any(qn >= kQFlush)) flush();
  }
  flush();
  // merge with the other half (same query, other candidate rows); lanes h == 0 write
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s2 = __shfl_xor(bs[k], 32, kWave);
    const int i2 = __shfl_xor(bi[k], 32, kWave);
    if (h == 0) topk_insert<K>(bs, bi, s2, i2);
  }
  if (h == 0 && qg < mq) {
    // gridDim.y > 1: partial list of this slice at [blockIdx.y][q][k] of the workspace
    const int64_t o = ((int64_t)blockIdx.y * mq + qg) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[o + k] = bi[k];
      if (out_score) out_score[o + k] = bs[k];
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

void launch_knn_prep(const float* X, int m, int m_pad, int role, float* out, hipStream_t stream) {
  knn_prep_kernel<<<(m_pad + 255) / 256, 256, 0, stream>>>(X, m, m_pad, role, out);
  check_launch("knn_prep");
}

int knn_splits(int mq_pad, int mc_pad) {
  // Candidate slices restart their top-k lists (fill cost), so use the fewest slices that fill
  // the resident capacity (one-wave workgroups) with the best whole-round balance.
  static const int cap = resident_cap(knn_topk_kernel<5>, kWave);
  const int qblocks = mq_pad / 32, tiles = mc_pad / 32;
  int max_s = tiles / 8;
  if (max_s > 32) max_s = 32;
  if (max_s < 1) max_s = 1;
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= max_s; ++s) {
    const double blocks = (double)qblocks * s;
    const double rounds = std::ceil(blocks / cap);
    double eff = blocks / (rounds * cap);            // occupancy of the resident slots over all rounds
    eff -= 0.004 * (s - 1);                          // fill cost of every extra slice
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return best;
}

void launch_knn_topk(const float* Q, int mq_pad, int mq, const float* C,
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
  knn_topk_kernel<KK><<<grid, kWave, 0, stream>>>(Q, mq, C, mc_pad, mc, self_offset, oi,           \
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
