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
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kMaxK = 8;
constexpr float kNegBig = -3.0e38f;
constexpr int kQFlush = 4;  // flush a wave's queues once any lane holds this many (2 / 8 / 12 measured
                             // slower at both bench shapes: profiles/r4_l/knn_flush*.json)
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
// role 2 (queries == candidates, the SMOTE self-search): one read of X writes both operands,
// candidates to `out` and queries to `outq`.  P != nullptr (candidate roles): the same launch also
// writes the bf16 SMOTE parents of smote_parents_kernel (smote.hip), bit for bit.
// chl / qhl / tmax (role 2 only, nullable): the hi/lo bf16 split of both operands in the same
// launch -- knn_split_kernel's role 2 (candidates, fragment order, per-tile norm bound) and role 1
// (queries, row order) on the values this thread just wrote, bitwise the same -- so the self-search
// of the bf16x3 engines needs no split launches.
__device__ __forceinline__ void split_row(const float (&x)[32], uint32_t (&h)[16], uint32_t (&l)[16]);
__global__ void knn_prep_kernel(const float* __restrict__ X, int m, int m_pad, int role,
                                float* __restrict__ out, float* __restrict__ outq,
                                const double* __restrict__ aff, uint16_t* __restrict__ P,
                                uint4* __restrict__ chl = nullptr, uint4* __restrict__ qhl = nullptr,
                                float* __restrict__ tmax = nullptr) {
#pragma clang fp contract(off)  // the parents' mul-then-add must match smote_parents_kernel
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (chl != nullptr) {  // the fused split (blockDim 256, m_pad % 32 == 0: whole tiles per wave half)
    const bool ok = r < m_pad;
    float x[32];
    if (ok && r < m) {
      const float4* p = reinterpret_cast<const float4*>(X + (int64_t)r * kCols);
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < kCols / 4; ++k) {
        float4 v = p[k];
        if (k == kCols / 4 - 1) {
          s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s);
          v.z = 0.0f; v.w = 0.0f;
        } else {
          s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
        }
        x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
      }
      x[30] = -0.5f * s;  // the candidate row; the query row has 1 there
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) x[k] = 0.0f;
      x[30] = -3.0e38f;  // padding candidate
    }
    uint32_t h[16], l[16];
    split_row(x, h, l);
    if (ok) {
      const int64_t tb = (int64_t)(r >> 5) * 256 + (r & 31);
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int k = v & 3;
        const uint4 c = v < 4 ? make_uint4(h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3])
                              : make_uint4(l[4 * k], l[4 * k + 1], l[4 * k + 2], l[4 * k + 3]);
        chl[tb + (v >> 1) * 64 + (v & 1) * 32] = c;
      }
    }
    float n2 = (ok && x[30] > -1.0e37f) ? -2.0f * x[30] : 0.0f;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) n2 = fmaxf(n2, __shfl_xor(n2, o, kWave));
    if (ok && (r & 31) == 0) tmax[r >> 5] = sqrtf(n2) * 1.0001f;
    x[30] = (ok && r < m) ? 1.0f : 0.0f;  // the query row (padding queries: zeros)
    split_row(x, h, l);
    if (ok) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        qhl[(int64_t)r * 8 + k] = make_uint4(h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]);
        qhl[(int64_t)r * 8 + 4 + k] = make_uint4(l[4 * k], l[4 * k + 1], l[4 * k + 2], l[4 * k + 3]);
      }
    }
  }
  if (r >= m_pad) return;
  float4* o = reinterpret_cast<float4*>(out + (int64_t)r * kCols);
  float4* oq = role == 2 ? reinterpret_cast<float4*>(outq + (int64_t)r * kCols) : nullptr;
  if (r >= m) {
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) {
      o[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (oq) oq[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (role != 1) out[(int64_t)r * kCols + 30] = -3.0e38f;
    return;
  }
  const float4* p = reinterpret_cast<const float4*>(X + (int64_t)r * kCols);
  uint2* pp = P ? reinterpret_cast<uint2*>(P + (int64_t)r * kCols) : nullptr;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < kCols / 4; ++k) {
    float4 v = p[k];
    if (pp) {
      float4 u = v;
      if (aff != nullptr) {
        const int c = 4 * k;
        u.x = u.x * (float)(1.0 / aff[32 + c]) + (float)aff[c];
        u.y = u.y * (float)(1.0 / aff[32 + c + 1]) + (float)aff[c + 1];
        if (c + 2 < kBiasCol) {
          u.z = u.z * (float)(1.0 / aff[32 + c + 2]) + (float)aff[c + 2];
          u.w = u.w * (float)(1.0 / aff[32 + c + 3]) + (float)aff[c + 3];
        }
      }
      pp[k] = make_uint2(pack_bf16x2(u.x, u.y), pack_bf16x2(u.z, u.w));
    }
    if (k == kCols / 4 - 1) {  // columns 28..31: keep 28, 29; 30 = norm term / 1, 31 = 0
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s);
      v.z = 0.0f; v.w = 0.0f;
    } else {
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
    o[k] = v;
    if (oq) oq[k] = v;
  }
  out[(int64_t)r * kCols + 30] = role == 1 ? 1.0f : -0.5f * s;
  if (oq) outq[(int64_t)r * kCols + 30] = 1.0f;
}

// Q: [mq_pad][32] query rows and C: [mc_pad][32] candidate rows, both from knn_prep_kernel.
// Query row q is candidate row (self_offset + q) when self_offset >= 0 (self excluded).
//
// One wave per workgroup: blockIdx.x owns 32 queries, blockIdx.y a contiguous slice of the
// candidate tiles (the per-slice lists are merged by knn_merge_kernel).  Per 32-candidate tile:
//   * 16 v_mfma_f32_32x32x2_f32 give lane (j, h) the scores of query j against the 16 candidate
//     rows of half h (exact fp32: score = q.c - 0.5||c||^2, the norm term is column 30);
//   * every score >= the lane's threshold is appended to a per-lane LDS queue (a wave-uniform
//     branch per accumulator row skips the rows no lane passes);
//   * once any lane holds kQFlush entries the queues are inserted into the per-lane top-k
//     (exact score-then-index order, self/padding excluded) and the threshold becomes the k-th
//     best of the UNION of the two half-lists of the query (lanes j and j+32), which is a valid
//     filter for both halves and about twice as tight.
template <int K, int QF = kQFlush>
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
  // padding queries (qg >= mq: zero rows, every score equal) never pass the filter: a lane that
  // appended every candidate made its wave the slowest of the grid (r5_r: 17k minority rows)
  float thr = qg < mq ? kNegBig : __builtin_inff();

  // Per-lane queue, [slot][lane]: same-slot stores of a wave hit 64 distinct banks (the last
  // slot is spare: kept from the select-and-store form's dump slot).
  constexpr int kCap = QF - 1 + 16 + 1;
  __shared__ int2 qent[kCap * kWave];  // (score bits, candidate index) at [slot * 64 + lane]
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
    thr = qg < mq ? kth : __builtin_inff();
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
    // quad maxima first (rows 4q .. 4q+3 = 4 consecutive candidates), then the tile's
    float m4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) m4[q] = fmaxf(fmaxf(acc[4 * q], acc[4 * q + 1]), fmaxf(acc[4 * q + 2], acc[4 * q + 3]));
    const float mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
    if (!__any(mx >= thr)) continue;
    const int cbase = c0 + 4 * h;
    // Append: a wave-uniform branch per passing quad, then per accumulator row of it, skips the rows
    // no lane passes (usually all but one or two once the lists are full); the passing lanes store
    // under their exec mask.  The per-row select-and-store of every row (dump slot for non-passing
    // lanes) was ~110 of the ~135 VALU instructions per tile whenever ANY lane passed (r5_n PMC).
    int qe = qn * kWave + lane;                     // element of this lane's next free slot
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!__any(m4[q] >= thr)) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = 4 * q + rr;
        const bool pass = acc[r] >= thr;
        if (__any(pass)) {
          if (pass) {
            qent[qe] = make_int2(__float_as_int(acc[r]), cbase + rr + 8 * q);
            qe += kWave;
          }
        }
      }
    }
    qn = (qe - lane) / kWave;
    if (__any(qn >= QF)) flush();
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

// ---- LDS-tiled fp32 engine --------------------------------------------------------------------
// At config-5 scale (170k minority rows of a 100M-row table) the candidate set (21.8 MB of prepped
// rows) lives in the Infinity Cache, not L2, and the one-wave kernel above re-streams it for every
// 32-query block: 116 GB at ~5.3 TB/s, 21.7 ms, MFMA ~54% busy (profiles/r2_s3h).  Here a
// workgroup of kLW waves owns 32 kLW queries and stages each chunk of kCh candidate tiles ONCE
// into LDS for all of its waves (double-buffered: the next chunk's global loads are in flight
// while the waves run the MFMA chains of this one), cutting the streamed bytes kLW-fold.  Rows sit
// at a 36-float stride: the ds_read_b128 operand reads (row j, 16 floats of half h) hit 16
// distinct 16-B slots in every lane group, and the cooperative 8-lane row stores are contiguous.
// Per wave the score/filter/top-k logic is the one-wave kernel's.
constexpr int kLW = 4;         // waves (query blocks) per workgroup
constexpr int kCh = 2;         // candidate tiles per staged chunk
constexpr int kLdC = kCols + 4;

template <int K>
__global__ __launch_bounds__(kLW * kWave) void knn_topk_lds_kernel(const float* __restrict__ Q, int mq,
                                                                   const float* __restrict__ C, int mc_pad, int mc,
                                                                   int64_t self_offset, int* __restrict__ out_idx,
                                                                   float* __restrict__ out_score) {
  const int lane = lane_id(), wv = wave_id();
  const int h = lane >> 5, j = lane & 31;
  const int qg = (blockIdx.x * kLW + wv) * 32 + j;
  const int64_t self_c = self_offset >= 0 ? self_offset + qg : -1;
  __shared__ __attribute__((aligned(16))) float cbuf[2][kCh * 32 * kLdC];
  __shared__ int2 qall[kLW][kQCap * kWave];
  int2* qent = qall[wv];
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
  // padding queries (qg >= mq: zero rows, every score equal) never pass the filter: a lane that
  // appended every candidate made its wave the slowest of the grid (r5_r: 17k minority rows)
  float thr = qg < mq ? kNegBig : __builtin_inff();
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
    thr = qg < mq ? kth : __builtin_inff();
  };
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  // chunk c covers tiles [t_lo + kCh c, min(t_hi, t_lo + kCh (c + 1))): kCh * 32 rows * 8 float4
  // = 2 kCh float4 per thread (rows past the slice are not read: their tiles are not processed)
  constexpr int kVec = kCh * 32 * 8 / (kLW * kWave);
  float4 st[kVec];
  auto load = [&](int c) {
    const int64_t r0 = (int64_t)(t_lo + kCh * c) * 32;
    const int64_t rmax = (int64_t)t_hi * 32;
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const int e = threadIdx.x + i * kLW * kWave;  // float4 index in the chunk: row e >> 3
      const int64_t r = r0 + (e >> 3);
      st[i] = r < rmax ? reinterpret_cast<const float4*>(C + r * kCols)[e & 7] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int b) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const int e = threadIdx.x + i * kLW * kWave;
      *reinterpret_cast<float4*>(&cbuf[b][(e >> 3) * kLdC + 4 * (e & 7)]) = st[i];
    }
  };
  const int nch = (t_hi - t_lo + kCh - 1) / kCh;
  if (nch > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) load(c + 1);
    const float* cb = cbuf[c & 1];
    const int ntile = min(kCh, t_hi - (t_lo + kCh * c));
    for (int tt = 0; tt < ntile; ++tt) {
      const int c0 = (t_lo + kCh * c + tt) * 32;
      const float* crow = cb + (tt * 32 + j) * kLdC + 16 * h;
      float ac[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(crow + 4 * k);
        ac[4 * k] = v.x; ac[4 * k + 1] = v.y; ac[4 * k + 2] = v.z; ac[4 * k + 3] = v.w;
      }
      f32x16_t acc = {};
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[s], bq[s], acc, 0, 0, 0);
      float mx = acc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
      if (!__any(mx >= thr)) continue;
      const int cbase = c0 + 4 * h;
      int qe = qn * kWave + lane;
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // knn_topk_kernel's uniform-skip append
        const bool pass = acc[r] >= thr;
        if (__any(pass)) {
          if (pass) {
            qent[qe] = make_int2(__float_as_int(acc[r]), cbase + (r & 3) + 8 * (r >> 2));
            qe += kWave;
          }
        }
      }
      qn = (qe - lane) / kWave;
      if (__any(qn >= kQFlush)) flush();
    }
    if (c + 1 < nch) store((c + 1) & 1);  // that buffer was last read in chunk c - 1 (barrier since)
    __syncthreads();
  }
  flush();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s2 = __shfl_xor(bs[k], 32, kWave);
    const int i2 = __shfl_xor(bi[k], 32, kWave);
    if (h == 0) topk_insert<K>(bs, bi, s2, i2);
  }
  if (h == 0 && qg < mq) {
    const int64_t o = ((int64_t)blockIdx.y * mq + qg) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[o + k] = bi[k];
      if (out_score) out_score[o + k] = bs[k];
    }
  }
}

// ---- bf16x3 MFMA filter + exact fp32 re-score ---------------------------------------------
// The fp32 MFMA chain above is 16 x v_mfma_f32_32x32x2_f32 = 1024 SIMD cycles per 32x32 tile
// (profiles/r1_s31: 206 us of the bench step at 13.6k minority rows).  Here every prepped row x
// is split x = hi + lo (two bf16 rows) and the tile score is hi.hi + hi.lo + lo.hi on
// v_mfma_f32_32x32x16_bf16 (6 MFMAs = 192 cycles), |approx - exact| <= 2^-16 sum|q_f c_f| (the
// omitted lo.lo term, the split residuals and fp32 accumulation).  That approximate score only
// FILTERS: a candidate passes when approx >= thr - margin, margin = 2^-13 (||q|| tmax +
// 0.5 tmax^2) >= 8x the error bound (tmax = largest ||c|| of the tile); a tile with any pass is
// staged to LDS in fp32 and its passing rows are re-scored exactly before the top-k insertion
// -- no true neighbour can be filtered out, and lists, threshold and returned scores are exact
// fp32 (ties -> smaller index).

__device__ __forceinline__ void split_row(const float (&x)[32], uint32_t (&h)[16], uint32_t (&l)[16]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float a = x[2 * k], b = x[2 * k + 1];
    const uint32_t ph = pack_bf16x2(a, b);
    h[k] = ph;
    l[k] = pack_bf16x2(a - bf16lo(ph), b - bf16hi(ph));
  }
}

// hi/lo bf16 split of prepped rows: hl[r] = 8 x uint4 (hi cols 0..31, then lo cols 0..31);
// role 0 (candidates) also writes tmax[r / 32] = max feature norm over the 32-row tile; role 2 = role 0
// with hl in the b3top fragment order (below).
__global__ __launch_bounds__(256) void knn_split_kernel(const float* __restrict__ Xp, int m_pad, int role,
                                                        uint4* __restrict__ hl, float* __restrict__ tmax) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  const bool ok = r < m_pad;
  float x[32];
  const float4* p = reinterpret_cast<const float4*>(Xp + (int64_t)(ok ? r : 0) * kCols);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float4 v = p[k];
    x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
  }
  uint32_t h[16], l[16];
  split_row(x, h, l);
  if (ok && role == 2) {
    // fragment order (b3top): tile r / 32 as [u 0..3][lane 64] uint4, lane (half hh, row j) of load u
    // holding chunk 2u + hh of row j (chunks 0..3 hi, 4..7 lo) -- each of the tile loop's four
    // loads is one contiguous 1 KiB per wave instead of 16 B pieces of 32 rows
    const int64_t tb = (int64_t)(r >> 5) * 256 + (r & 31);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int k = v & 3;
      const uint4 c = v < 4 ? make_uint4(h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3])
                            : make_uint4(l[4 * k], l[4 * k + 1], l[4 * k + 2], l[4 * k + 3]);
      hl[tb + (v >> 1) * 64 + (v & 1) * 32] = c;
    }
  } else if (ok) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hl[(int64_t)r * 8 + k] = make_uint4(h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]);
      hl[(int64_t)r * 8 + 4 + k] = make_uint4(l[4 * k], l[4 * k + 1], l[4 * k + 2], l[4 * k + 3]);
    }
  }
  if (role == 0 || role == 2) {
    // candidate rows carry -0.5 ||c||^2 in column 30 (padding rows: -3e38 -> norm 0)
    float n2 = (ok && x[30] > -1.0e37f) ? -2.0f * x[30] : 0.0f;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) n2 = fmaxf(n2, __shfl_xor(n2, o, kWave));
    if (ok && (r & 31) == 0) tmax[r >> 5] = sqrtf(n2) * 1.0001f;
  }
}

template <int K>
__global__ __launch_bounds__(kWave) void knn_topk3_kernel(const float* __restrict__ Q, const uint4* __restrict__ Qhl,
                                                          int mq, const float* __restrict__ C,
                                                          const uint4* __restrict__ Chl,
                                                          const float* __restrict__ tmax, int mc_pad, int mc,
                                                          int64_t self_offset, int* __restrict__ out_idx,
                                                          float* __restrict__ out_score) {
  const int lane = threadIdx.x;
  const int h = lane >> 5, j = lane & 31;
  const int q0 = blockIdx.x * 32;
  const int qg = q0 + j;
  const int64_t self_c = self_offset >= 0 ? self_offset + qg : -1;
  // the block's 32 query rows and the current candidate tile, fp32 (prepped), for the exact
  // re-score from LDS (row stride 36 floats: 16 B aligned, b128 reads of 8 consecutive rows
  // spread over the banks)
  constexpr int kLd = kCols + 4;
  __shared__ __attribute__((aligned(16))) float qs[32 * kLd];
  __shared__ __attribute__((aligned(16))) float cs[32 * kLd];
  {
    const float4* src = reinterpret_cast<const float4*>(Q + (int64_t)q0 * kCols);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane + 64 * i;  // float4 index: row e >> 3, cols 4 (e & 7) ..
      *reinterpret_cast<float4*>(&qs[(e >> 3) * kLd + 4 * (e & 7)]) = src[e];
    }
  }
  __syncthreads();
  float qn2 = 0.0f;
#pragma unroll
  for (int f = 0; f < 30; ++f) qn2 = fmaf(qs[j * kLd + f], qs[j * kLd + f], qn2);
  const float qn = sqrtf(qn2);
  // B operand (query j): MFMA 0 covers columns 8h..8h+7, MFMA 1 columns 16+8h..16+8h+7
  const uint4* qr = Qhl + (int64_t)qg * 8;
  const bf16x8_t qh0 = __builtin_bit_cast(bf16x8_t, qr[h]), qh1 = __builtin_bit_cast(bf16x8_t, qr[2 + h]);
  const bf16x8_t ql0 = __builtin_bit_cast(bf16x8_t, qr[4 + h]), ql1 = __builtin_bit_cast(bf16x8_t, qr[6 + h]);

  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  // padding queries (qg >= mq: zero rows, every score equal) never pass the filter: a lane that
  // appended every candidate made its wave the slowest of the grid (r5_r: 17k minority rows)
  float thr = qg < mq ? kNegBig : __builtin_inff();
  // exact fp32 score of tile row rl against this lane's query (a k-ordered fmaf chain)
  auto rescore = [&](int rl) -> float {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float4 c = *reinterpret_cast<const float4*>(&cs[rl * kLd + 4 * k]);
      const float4 q = *reinterpret_cast<const float4*>(&qs[j * kLd + 4 * k]);
      acc = fmaf(q.x, c.x, acc);
      acc = fmaf(q.y, c.y, acc);
      acc = fmaf(q.z, c.z, acc);
      acc = fmaf(q.w, c.w, acc);
    }
    return acc;
  };
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  // register double buffer of the next tile: hi/lo bf16 operands of candidate row j (this lane's
  // K half), 64 B per lane.  The fp32 rows are fetched only for a tile with a passing score (once
  // the lists are full that is rare: half the streamed bytes of fetching them with every tile)
  uint4 cv[4];
  auto fetch = [&](int t, uint4 (&a)[4]) {
    const uint4* p = Chl + (int64_t)(t * 32 + j) * 8;
    a[0] = p[h]; a[1] = p[2 + h]; a[2] = p[4 + h]; a[3] = p[6 + h];
  };
  if (t_lo < t_hi) fetch(t_lo, cv);
  for (int t = t_lo; t < t_hi; ++t) {
    const int c0 = t * 32;
    const bf16x8_t ch0 = __builtin_bit_cast(bf16x8_t, cv[0]), ch1 = __builtin_bit_cast(bf16x8_t, cv[1]);
    const bf16x8_t cl0 = __builtin_bit_cast(bf16x8_t, cv[2]), cl1 = __builtin_bit_cast(bf16x8_t, cv[3]);
    const float tm = tmax[t];
    if (t + 1 < t_hi) fetch(t + 1, cv);
    f32x16_t acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, qh1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, ql0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, ql1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, qh1, acc, 0, 0, 0);
    const float cut = thr - 0x1p-13f * fmaf(qn, tm, 0.5f * tm * tm);
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
    if (!__any(mx >= cut)) continue;
    // stage the tile's fp32 rows (lane j, h: row j, columns 16h..16h+15) and re-score exactly
    {
      const float4* pf = reinterpret_cast<const float4*>(C + (int64_t)(c0 + j) * kCols + 16 * h);
      const float4 f0 = pf[0], f1 = pf[1], f2 = pf[2], f3 = pf[3];
      float* crow = &cs[j * kLd + 16 * h];
      *reinterpret_cast<float4*>(crow) = f0;
      *reinterpret_cast<float4*>(crow + 4) = f1;
      *reinterpret_cast<float4*>(crow + 8) = f2;
      *reinterpret_cast<float4*>(crow + 12) = f3;
    }
    __builtin_amdgcn_wave_barrier();  // one wave: LDS ops retire in order
    uint32_t pm = 0;  // passing accumulator rows of this lane (static indices -> no acc spill)
#pragma unroll
    for (int r = 0; r < 16; ++r) pm |= (acc[r] >= cut ? 1u : 0u) << r;
    while (pm) {
      const int r = __builtin_ctz(pm);
      pm &= pm - 1;
      const int rl = 4 * h + (r & 3) + 8 * (r >> 2);
      const int ci = c0 + rl;
      if (ci != self_c && ci < mc) topk_insert<K>(bs, bi, rescore(rl), ci);
    }
    __builtin_amdgcn_wave_barrier();  // cs is rewritten by the next staging tile
    // threshold = k-th best of the union of this lane's and its partner's (other half) lists
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
    thr = qg < mq ? kth : __builtin_inff();
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s2 = __shfl_xor(bs[k], 32, kWave);
    const int i2 = __shfl_xor(bi[k], 32, kWave);
    if (h == 0) topk_insert<K>(bs, bi, s2, i2);
  }
  if (h == 0 && qg < mq) {
    const int64_t o = ((int64_t)blockIdx.y * mq + qg) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[o + k] = bi[k];
      if (out_score) out_score[o + k] = bs[k];
    }
  }
}

// ---- bf16x3 collect + exact re-rank (two phases) ---------------------------------------------
// The engines above run the top-k on the critical path of every tile: the fp32 chain costs 1024
// MFMA cycles per 32x32 tile plus the filter's VALU (serial per wave: ~200 us at 13.6k minority
// rows, profiles/r4_g), and knn_topk3 stalls on a dependent fp32 tile load + LDS re-score whenever
// a lane passes.  Here phase 1 (knn_collect_kernel) never touches fp32 candidate rows: per tile it
// runs the 6 bf16 MFMAs of knn_topk3 and a max test, and a passing candidate only APPENDS its index
// to a per-lane global list.  The running threshold is the k-th best LOWER bound approx - m of the
// union of the query's two half-lists, where m = 2^-14 (||q|| tmax + 0.5 tmax^2) >= 4x the bf16x3
// error bound 2^-16 sum|q_f c_f| (see knn_topk3; fp32 accumulation of the 96 products and the
// exact fmaf chain add < 0.6 x 2^-16 more); a candidate is appended when its UPPER bound approx + m
// reaches it.
// Since k distinct candidates have exact >= lower bound >= thr, the exact k-th best s_k >= thr
// at every moment, so every candidate with exact >= s_k (upper bound >= s_k >= thr) is on a list.
// Phase 2 (knn_rerank_kernel, 8 lanes per query) re-scores the listed candidates exactly (the
// k-ordered fp32 fmaf chain of knn_topk3's re-score) and keeps the top-k (ties -> smaller index):
// the exact fp32 ranking.  A full lane list is compacted in place first: an entry (lower bound
// lb) whose upper bound -- at most lb + 2 m_max, m_max the largest margin the lane has used -- is
// below the current threshold cannot reach s_k and is dropped.  A list still full after that
// sends its query to a brute-force exact scan in phase 2 (correct, slow: r5_q measured the config-5
// shard, 17k x 17k, at 0.67 ms before the compaction).
constexpr int kListCap = 64;
constexpr int kSeedTiles = 2;             // seed candidates per slice > 0: 64
constexpr float kMarginScale = 0x1p-14f;  // m = 2^-14 (||q|| tmax + 0.5 tmax^2): >= 4x the error bound

template <int K>
__global__ __launch_bounds__(kWave) void knn_collect_kernel(const float* __restrict__ Q, const uint4* __restrict__ Qhl,
                                                            const uint4* __restrict__ Chl,
                                                            const float* __restrict__ tmax, int mq, int mc_pad, int mc,
                                                            int64_t self_offset, int2* __restrict__ lists,
                                                            int* __restrict__ counts) {
  const int lane = threadIdx.x;
  const int h = lane >> 5, j = lane & 31;
  const int qg = blockIdx.x * 32 + j;
  const int64_t self_c = self_offset >= 0 ? self_offset + qg : -1;
  float qn;
  {  // ||q|| over the 30 feature columns: half h sums columns 16h .. 16h + 15
    const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)qg * kCols + 16 * h);
    float s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = p[k];
      s2 = fmaf(v.x, v.x, s2);
      s2 = fmaf(v.y, v.y, s2);
      if (h == 0 || k < 3) {  // columns 30, 31 (query 1 / 0) are not features
        s2 = fmaf(v.z, v.z, s2);
        s2 = fmaf(v.w, v.w, s2);
      }
    }
    s2 += __shfl_xor(s2, 32, kWave);
    qn = sqrtf(s2) * 1.0001f;
  }
  const uint4* qr = Qhl + (int64_t)qg * 8;
  const bf16x8_t qh0 = __builtin_bit_cast(bf16x8_t, qr[h]), qh1 = __builtin_bit_cast(bf16x8_t, qr[2 + h]);
  const bf16x8_t ql0 = __builtin_bit_cast(bf16x8_t, qr[4 + h]), ql1 = __builtin_bit_cast(bf16x8_t, qr[6 + h]);
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  // padding queries (qg >= mq: zero rows, every score equal) never pass the filter: a lane that
  // appended every candidate made its wave the slowest of the grid (r5_r: 17k minority rows)
  float thr = qg < mq ? kNegBig : __builtin_inff();
  float mgmax = 0.0f;  // the largest margin this lane has used (list compaction bound)
  constexpr int kCap = kQFlush - 1 + 16 + 1;
  __shared__ int2 qent[kCap * kWave];  // (lower-bound bits, candidate index) at [slot * 64 + lane]
  int qc = 0, cnt = 0;
  const int64_t lbase = (int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * kListCap * kWave + lane;
  auto union_thr = [&]() {  // k-th best lower bound of the union of this lane's and its partner's lists
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
    thr = qg < mq ? kth : __builtin_inff();
  };
  auto flush = [&]() {
    for (int e = 0; __any(e < qc); ++e) {
      if (e < qc) {
        const int2 v = qent[e * kWave + lane];
        const int ci = v.y;
        if (ci != self_c && ci < mc) {
          if (cnt == kListCap) {  // full: drop the entries that can no longer reach s_k (rare path)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's list stores have landed
            int w = 0;
            for (int e2 = 0; e2 < kListCap; ++e2) {
              const int2 o = lists[lbase + (int64_t)e2 * kWave];
              if (__int_as_float(o.x) + 2.0f * mgmax >= thr) lists[lbase + (int64_t)(w++) * kWave] = o;
            }
            cnt = w;
          }
          if (cnt < kListCap) lists[lbase + (int64_t)cnt * kWave] = v;
          ++cnt;
          topk_insert<K>(bs, bi, __int_as_float(v.x), ci);
        }
      }
    }
    qc = 0;
    union_thr();
  };
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  // Chl in the fragment order of knn_split role 2: each of a tile's four loads is one contiguous
  // 1 KiB per wave (lane (h, j) of load u holds chunk 2u + h of row j -- the same registers as the
  // row layout's p[h], p[2 + h], p[4 + h], p[6 + h]) instead of 32 rows' 16-byte pieces
  auto fetch = [&](int t, uint4 (&a)[4], float& tmv) {
    const uint4* p = Chl + (int64_t)t * 256 + lane;
    a[0] = p[0]; a[1] = p[64]; a[2] = p[128]; a[3] = p[192];
    tmv = tmax[t];
  };
  auto approx = [&](const uint4 (&c)[4]) -> f32x16_t {
    const bf16x8_t ch0 = __builtin_bit_cast(bf16x8_t, c[0]), ch1 = __builtin_bit_cast(bf16x8_t, c[1]);
    const bf16x8_t cl0 = __builtin_bit_cast(bf16x8_t, c[2]), cl1 = __builtin_bit_cast(bf16x8_t, c[3]);
    f32x16_t acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, qh1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, ql0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, ql1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, qh1, acc, 0, 0, 0);
    return acc;
  };
  // Seed (slices > 0): the lower bounds of the first kSeedTiles tiles of the candidate set -- slice
  // 0's, so distinct from this slice's candidates -- fill the top-k before the slice starts.  They
  // are never appended (slice 0 lists them), but the threshold they give is valid (k distinct
  // candidates with exact >= lower bound >= thr) and spares every slice its fill phase: with
  // thr = -inf the first tile appends all 16 candidates of every lane (r5_j: 62 list entries per
  // query and slice at 13.6k x 13.6k, 4 slices, a 124 us re-rank).
  if (blockIdx.y > 0) {
    const int ns0 = (int)((int64_t)all_tiles / gridDim.y);  // slice 0's tile count
    const int nseed = ns0 < kSeedTiles ? ns0 : kSeedTiles;
    for (int t = 0; t < nseed; ++t) {
      uint4 c[4];
      float tm;
      fetch(t, c, tm);
      const f32x16_t acc = approx(c);
      const float mg = kMarginScale * fmaf(qn, tm, 0.5f * tm * tm);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = t * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
        if (ci != self_c && ci < mc) topk_insert<K>(bs, bi, acc[r] - mg, ci);
      }
    }
    union_thr();
  }
  // The filter of one scored tile (knn_topk_kernel's quad-then-row uniform-skip append).
  auto filter = [&](int t, const f32x16_t& acc, float tm) {
    const float mg = kMarginScale * fmaf(qn, tm, 0.5f * tm * tm);
    mgmax = fmaxf(mgmax, mg);
    const float cut = thr - mg;  // upper bound approx + mg >= thr
    float m4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) m4[q] = fmaxf(fmaxf(acc[4 * q], acc[4 * q + 1]), fmaxf(acc[4 * q + 2], acc[4 * q + 3]));
    const float mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
    if (!__any(mx >= cut)) return;
    const int cbase = t * 32 + 4 * h;
    int qe = qc * kWave + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!__any(m4[q] >= cut)) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = 4 * q + rr;
        const bool pass = acc[r] >= cut;
        if (__any(pass)) {
          if (pass) {
            qent[qe] = make_int2(__float_as_int(acc[r] - mg), cbase + rr + 8 * q);
            qe += kWave;
          }
        }
      }
    }
    qc = (qe - lane) / kWave;
    if (__any(qc >= kQFlush)) flush();
  };
  // Tiles in PAIRS: the two tiles' 6-MFMA chains are interleaved (independent accumulators), so one
  // chain's result latency is covered by the other's issue -- at ~1.7 waves per SIMD a lone chain's
  // latency was exposed on every tile.  The next pair's loads are in flight meanwhile.
  uint4 ca[4], cb[4];
  float tma = 0.0f, tmb = 0.0f;
  if (t_lo < t_hi) fetch(t_lo, ca, tma);
  if (t_lo + 1 < t_hi) fetch(t_lo + 1, cb, tmb);
  for (int t = t_lo; t < t_hi; t += 2) {
    const bool two = t + 1 < t_hi;  // wave-uniform
    f32x16_t acc0 = {}, acc1 = {};
    {
      const bf16x8_t ah0 = __builtin_bit_cast(bf16x8_t, ca[0]), ah1 = __builtin_bit_cast(bf16x8_t, ca[1]);
      const bf16x8_t al0 = __builtin_bit_cast(bf16x8_t, ca[2]), al1 = __builtin_bit_cast(bf16x8_t, ca[3]);
      const bf16x8_t bh0 = __builtin_bit_cast(bf16x8_t, cb[0]), bh1 = __builtin_bit_cast(bf16x8_t, cb[1]);
      const bf16x8_t bl0 = __builtin_bit_cast(bf16x8_t, cb[2]), bl1 = __builtin_bit_cast(bf16x8_t, cb[3]);
      // approx()'s order per tile (bitwise the same sums), the two chains alternating
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al0, qh0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl0, qh0, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al1, qh1, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl1, qh1, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, ql0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh0, ql0, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, ql1, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh1, ql1, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, qh0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh0, qh0, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, qh1, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh1, qh1, acc1, 0, 0, 0);
    }
    const float ta = tma, tb = tmb;
    if (t + 2 < t_hi) fetch(t + 2, ca, tma);  // the next pair
    if (t + 3 < t_hi) fetch(t + 3, cb, tmb);
    filter(t, acc0, ta);
    if (two) filter(t + 1, acc1, tb);
  }
  flush();
  // counts holds three planes of gridDim.x * gridDim.y * 64 ints: the list length, then this lane's
  // final threshold (the union's k-th best lower bound) and largest margin -- the re-rank skips
  // every entry whose upper bound cannot reach the best of the slices' final thresholds
  const int64_t ci0 = (int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * kWave + lane;
  const int64_t plane = (int64_t)gridDim.x * gridDim.y * kWave;
  counts[ci0] = cnt;
  counts[plane + ci0] = __float_as_int(thr);
  counts[2 * plane + ci0] = __float_as_int(mgmax);
}

// Phase 2: 8 lanes per query (lane l takes every 8th listed candidate), exact re-score, per-lane
// top-k, then a 3-round butterfly merge of the 8 sorted lists (knn_merge_kernel's merge).
template <int K>
__global__ __launch_bounds__(256) void knn_rerank_kernel(const float* __restrict__ Q, const float* __restrict__ C,
                                                         int mq, int mc, int qblocks, int nsplit, int64_t self_offset,
                                                         const int2* __restrict__ lists,
                                                         const int* __restrict__ counts, int* __restrict__ out_idx,
                                                         float* __restrict__ out_score) {
  const int gl = blockIdx.x * 256 + threadIdx.x;
  const int q = gl >> 3, l = gl & 7;
  const bool live = q < mq;
  const int qq = live ? q : 0;
  const int blk = qq >> 5, j = qq & 31;
  const int64_t self_c = self_offset >= 0 ? self_offset + qq : -1;
  float qv[kCols];
  {
    const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)qq * kCols);
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) {
      const float4 v = p[k];
      qv[4 * k] = v.x; qv[4 * k + 1] = v.y; qv[4 * k + 2] = v.z; qv[4 * k + 3] = v.w;
    }
  }
  auto exact = [&](int ci) -> float {  // knn_topk3's re-score: columns 0..31 in order
    const float4* c = reinterpret_cast<const float4*>(C + (int64_t)ci * kCols);
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) {
      const float4 v = c[k];
      acc = fmaf(qv[4 * k], v.x, acc);
      acc = fmaf(qv[4 * k + 1], v.y, acc);
      acc = fmaf(qv[4 * k + 2], v.z, acc);
      acc = fmaf(qv[4 * k + 3], v.w, acc);
    }
    return acc;
  };
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  if (live) {
    bool over = false;
    const int64_t plane = (int64_t)nsplit * qblocks * kWave;
    float T = kNegBig;  // the best slice threshold: a lower bound of the exact k-th best s_k
    for (int s = 0; s < nsplit; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h) over |= counts[((int64_t)s * qblocks + blk) * kWave + j + 32 * h] > kListCap;
      T = fmaxf(T, __int_as_float(counts[plane + ((int64_t)s * qblocks + blk) * kWave + j]));
    }
    if (!over) {
      for (int s = 0; s < nsplit; ++s) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t cb = ((int64_t)s * qblocks + blk) * kWave + j + 32 * h;
          const int n = counts[cb];
          // an entry's upper bound is at most lb + 2 m_max; below T <= s_k it cannot be in the top-k
          // (not even on a tie), so its fp32 row is never gathered
          const float skip = T - 2.0f * __int_as_float(counts[2 * plane + cb]);
          const int2* li = lists + ((int64_t)s * qblocks + blk) * kListCap * kWave + j + 32 * h;
          for (int e = l; e < n; e += 8) {
            const int2 v = li[(int64_t)e * kWave];
            if (__int_as_float(v.x) < skip) continue;
            topk_insert<K>(bs, bi, exact(v.y), v.y);
          }
        }
      }
    } else {  // a list overflowed: exact scan of every candidate
      for (int ci = l; ci < mc; ci += 8)
        if (ci != self_c) topk_insert<K>(bs, bi, exact(ci), ci);
    }
  }
#pragma unroll
  for (int off = 1; off < 8; off <<= 1) {
    float os[K];
    int oi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      os[k] = __shfl_xor(bs[k], off, kWave);
      oi[k] = __shfl_xor(bi[k], off, kWave);
    }
    float ns[K];
    int ni[K];
    int ia = 0, ib = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float a = kNegBig, b = kNegBig;
      int ai = 0x7fffffff, bj = 0x7fffffff;
#pragma unroll
      for (int u = 0; u < K; ++u) {
        if (u == ia) { a = bs[u]; ai = bi[u]; }
        if (u == ib) { b = os[u]; bj = oi[u]; }
      }
      const bool ta = !better(b, bj, a, ai);
      ns[k] = ta ? a : b;
      ni[k] = ta ? ai : bj;
      ia += ta ? 1 : 0;
      ib += ta ? 0 : 1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) { bs[k] = ns[k]; bi[k] = ni[k]; }
  }
  if (live && l == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[(int64_t)q * K + k] = bi[k];
      if (out_score) out_score[(int64_t)q * K + k] = bs[k];
    }
  }
}

// Merge the per-slice top-k lists of every query (same ordering: score desc, index asc).
// lps (a power of two >= nsplit, <= 64) lanes per query: lane s loads slice s's sorted list, then
// log2(lps) butterfly rounds merge lists pairwise through shuffles (a static-index merge of two
// sorted K-lists).  The order is total (candidate indices are unique across slices), so the
// result equals sequential insertion -- but 13.6k queries x 9 slices take ~4 us instead of the
// ~30 us of one thread walking all slices of a query.
template <int K>
__global__ __launch_bounds__(256) void knn_merge_kernel(const float* __restrict__ ps, const int* __restrict__ pi,
                                                        int nsplit, int lps_log2, int mq, int* __restrict__ out_idx,
                                                        float* __restrict__ out_score) {
  const int gl = blockIdx.x * 256 + threadIdx.x;
  const int q = gl >> lps_log2, sl = gl & ((1 << lps_log2) - 1);
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  if (q < mq && sl < nsplit) {
    const int64_t o = ((int64_t)sl * mq + q) * K;
#pragma unroll
    for (int k = 0; k < K; ++k) { bs[k] = ps[o + k]; bi[k] = pi[o + k]; }
  }
  for (int off = 1; off < (1 << lps_log2); off <<= 1) {
    float os[K];
    int oi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      os[k] = __shfl_xor(bs[k], off, kWave);
      oi[k] = __shfl_xor(bi[k], off, kWave);
    }
    float ns[K];
    int ni[K];
    int ia = 0, ib = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float a = kNegBig, b = kNegBig;
      int ai = 0x7fffffff, bj = 0x7fffffff;
#pragma unroll
      for (int u = 0; u < K; ++u) {
        if (u == ia) { a = bs[u]; ai = bi[u]; }
        if (u == ib) { b = os[u]; bj = oi[u]; }
      }
      const bool ta = !better(b, bj, a, ai);
      ns[k] = ta ? a : b;
      ni[k] = ta ? ai : bj;
      ia += ta ? 1 : 0;
      ib += ta ? 0 : 1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) { bs[k] = ns[k]; bi[k] = ni[k]; }
  }
  if (sl == 0 && q < mq) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[(int64_t)q * K + k] = bi[k];
      if (out_score) out_score[(int64_t)q * K + k] = bs[k];
    }
  }
}


// ---- bf16x3 scores + register top-K' + exact verification ("b3top") -------------------------
// The fp32 engine's structure (one wave = 32 queries x 32-candidate tiles, per-lane LDS queue and
// top list, the union threshold of the two half-lists) on the bf16x3 approximate score of
// knn_collect_kernel (6 x v_mfma_f32_32x32x16_bf16 per tile = 192 SIMD cycles instead of the fp32
// chain's 1024), with NO per-candidate fp32 work and no global lists in the tile loop: the per-lane
// lists hold APPROXIMATE scores, kTopP = 8 of them (more than k).  Exactness comes at the end
// (knn_b3top_final_kernel): the per-slice lists are merged to the query's top kTopP approximate
// candidates, those are re-scored exactly (knn_rerank_kernel's fmaf chain) and their exact top k is
// returned when it is PROVABLY the exact top k of every candidate:
//   a candidate outside the merged list was filtered against, or evicted by, kTopP entries at least
//   as good (seeds included: slice 0 lists them or kTopP better ones), so its approx <= a_P (the
//   merged list's last approximate score); its exact score is within its tile's margin m_t =
//   2^-14 (||q|| tmax_t + 0.5 tmax_t^2) (>= 4x the bf16x3 error bound, knn_collect_kernel) of that.
//   Per lane and tile: a tile none of whose 16 entries reached the threshold bounds its candidates
//   by U = max (tile max approx + m_t); a tile with an entry at or above it by a_P + M, M = max m_t
//   over such tiles (the tiles near the query -- a far outlier tile, whose norm sets a large margin,
//   lands in U with its low scores).  If the exact k-th best s_k > max(U, a_P + M), nothing outside
//   the list can reach it -- ties included.
// Otherwise (near-ties within the margin) the query is queued for knn_b3top_scan_kernel: one
// workgroup re-scans every candidate exactly.  Slices > 0 seed their threshold with slice 0's first kSeedTiles tiles (flagged
// entries, never output), sparing each slice its fill phase, so the grid can hold enough slices to
// put ~6 waves on every SIMD.
constexpr int kTopP = 8;
constexpr int kSeedFlag = 0x40000000;

// Merge two sorted (score desc, index asc) lists of N into the best N (static indices).
template <int N>
__device__ __forceinline__ void merge_sorted(float (&bs)[N], int (&bi)[N], const float (&os)[N], const int (&oi)[N]) {
  float ns[N];
  int ni[N];
  int ia = 0, ib = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float a = kNegBig, b = kNegBig;
    int ai = 0x7fffffff, bj = 0x7fffffff;
#pragma unroll
    for (int u = 0; u < N; ++u) {
      if (u == ia) { a = bs[u]; ai = bi[u]; }
      if (u == ib) { b = os[u]; bj = oi[u]; }
    }
    const bool ta = !better(b, bj, a, ai);
    ns[k] = ta ? a : b;
    ni[k] = ta ? ai : bj;
    ia += ta ? 1 : 0;
    ib += ta ? 0 : 1;
  }
#pragma unroll
  for (int k = 0; k < N; ++k) { bs[k] = ns[k]; bi[k] = ni[k]; }
}

template <int QF = kQFlush>
__global__ __launch_bounds__(kWave) void knn_b3top_kernel(const float* __restrict__ Q, const uint4* __restrict__ Qhl,
                                                          const uint4* __restrict__ Chl,
                                                          const float* __restrict__ tmax, int mq, int mc_pad, int mc,
                                                          int64_t self_offset, float* __restrict__ ws_s,
                                                          int* __restrict__ ws_i, float* __restrict__ ws_m) {
  const int lane = threadIdx.x;
  const int h = lane >> 5, j = lane & 31;
  const int qg = blockIdx.x * 32 + j;
  const int64_t self_c = self_offset >= 0 ? self_offset + qg : -1;
  float qn;
  {  // ||q|| over the 30 feature columns: half h sums columns 16h .. 16h + 15
    const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)qg * kCols + 16 * h);
    float s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = p[k];
      s2 = fmaf(v.x, v.x, s2);
      s2 = fmaf(v.y, v.y, s2);
      if (h == 0 || k < 3) {  // columns 30, 31 (query 1 / 0) are not features
        s2 = fmaf(v.z, v.z, s2);
        s2 = fmaf(v.w, v.w, s2);
      }
    }
    s2 += __shfl_xor(s2, 32, kWave);
    qn = sqrtf(s2) * 1.0001f;
  }
  const uint4* qr = Qhl + (int64_t)qg * 8;
  const bf16x8_t qh0 = __builtin_bit_cast(bf16x8_t, qr[h]), qh1 = __builtin_bit_cast(bf16x8_t, qr[2 + h]);
  const bf16x8_t ql0 = __builtin_bit_cast(bf16x8_t, qr[4 + h]), ql1 = __builtin_bit_cast(bf16x8_t, qr[6 + h]);
  float bs[kTopP];
  int bi[kTopP];
#pragma unroll
  for (int k = 0; k < kTopP; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
  float thr = qg < mq ? kNegBig : __builtin_inff();
  float ub_f = kNegBig;  // U: max over this lane's fully filtered tiles of (tile max approx + m_t)
  float mg_p = 0.0f;     // M: max m_t over this lane's tiles with an entry at or above the threshold
  constexpr int kCap = QF - 1 + 16 + 1;
  __shared__ int2 qent[kCap * kWave];  // (approx bits, candidate index) at [slot * 64 + lane]
  int qn_ = 0;
  auto flush = [&]() {
    for (int e = 0; __any(e < qn_); ++e) {
      if (e < qn_) {
        const int2 v = qent[e * kWave + lane];
        topk_insert<kTopP>(bs, bi, __int_as_float(v.x), v.y);
      }
    }
    qn_ = 0;
    // max of the two half-lists' kTopP-th best: one of them holds kTopP entries at or above it, so
    // it is a valid threshold -- one shuffle instead of a kTopP x kTopP union merge (the flush
    // ran ~500 VALU per call, the kernel's dominant cost, r6_e)
    const float kth = fmaxf(bs[kTopP - 1], __shfl_xor(bs[kTopP - 1], 32, kWave));
    thr = qg < mq ? kth : __builtin_inff();
  };
  const int all_tiles = mc_pad / 32;
  const int t_lo = (int)(((int64_t)all_tiles * blockIdx.y) / gridDim.y);
  const int t_hi = (int)(((int64_t)all_tiles * (blockIdx.y + 1)) / gridDim.y);
  auto fetch = [&](int t, uint4 (&a)[4], float& tmv) {  // Chl in fragment order (knn_split role 2)
    const uint4* p = Chl + (int64_t)t * 256 + lane;
    a[0] = p[0]; a[1] = p[64]; a[2] = p[128]; a[3] = p[192];
    tmv = tmax[t];
  };
  auto approx = [&](const uint4 (&c)[4]) -> f32x16_t {
    const bf16x8_t ch0 = __builtin_bit_cast(bf16x8_t, c[0]), ch1 = __builtin_bit_cast(bf16x8_t, c[1]);
    const bf16x8_t cl0 = __builtin_bit_cast(bf16x8_t, c[2]), cl1 = __builtin_bit_cast(bf16x8_t, c[3]);
    f32x16_t acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, qh1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, ql0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, ql1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, qh0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, qh1, acc, 0, 0, 0);
    return acc;
  };
  // seed: slice 0's first tiles (flagged: they set the threshold, slice 0 outputs them)
  if (blockIdx.y > 0) {
    const int ns0 = (int)((int64_t)all_tiles / gridDim.y);
    const int nseed = ns0 < kSeedTiles ? ns0 : kSeedTiles;
    for (int t = 0; t < nseed; ++t) {
      uint4 c[4];
      float tm;
      fetch(t, c, tm);
      const f32x16_t acc = approx(c);
      (void)tm;  // seeds are slice 0's candidates: slice 0's bookkeeping bounds them
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = t * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
        if (ci != self_c && ci < mc) topk_insert<kTopP>(bs, bi, acc[r], ci | kSeedFlag);
      }
    }
    const float kth = fmaxf(bs[kTopP - 1], __shfl_xor(bs[kTopP - 1], 32, kWave));
    thr = qg < mq ? kth : __builtin_inff();
  }
  // kBufs tiles in flight in separate registers, the loop unrolled by kBufs: a buffer is refilled
  // right after its 6 MFMAs consumed it, kBufs tiles (~kBufs x 200 cycles) ahead of its next use.
  // (A rotating copy cv = cv2 made the compiler wait for the newest loads every tile: one tile of
  // prefetch distance against an L2 round trip of several, r6_d.)
  constexpr int kBufs = 3;
  uint4 cb[kBufs][4];
  float tb[kBufs];
  const int tlast = t_hi > 0 ? t_hi - 1 : 0;  // a valid tile even for an empty slice
#pragma unroll
  for (int u = 0; u < kBufs; ++u) {  // in buffer order (the loop head's vmcnt assumes it)
    fetch(t_lo + u < t_hi ? t_lo + u : tlast, cb[u], tb[u]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // Every step issues its refill (clamped to the slice's last tile), so every path has the same
  // loads in the same order and the compiler's vmcnt waits stay exact (a conditional refill made it
  // wait for all outstanding loads at the loop head).
  for (int t0 = t_lo; t0 < t_hi; t0 += kBufs) {
#pragma unroll
    for (int u = 0; u < kBufs; ++u) {
      const int t = t0 + u;
      const f32x16_t acc = approx(cb[u]);
      const float tm = tb[u];
      fetch(t + kBufs < t_hi ? t + kBufs : tlast, cb[u], tb[u]);
      if (t >= t_hi) continue;  // wave-uniform: the last group's spare steps
      const int c0 = t * 32;
      float mx = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, acc[r]), acc[r + 1]);
      mx = fmaxf(mx, acc[15]);
      {
        const float mt = kMarginScale * fmaf(qn, tm, 0.5f * tm * tm);
        if (mx >= thr) mg_p = fmaxf(mg_p, mt);
        else ub_f = fmaxf(ub_f, mx + mt);  // the self row stays in mx: a valid (if loose) bound
      }
      if (!__any(mx >= thr)) continue;
      // With 64 queries per wave SOME lane passes on most tiles, so the append must cost little
      // when few rows pass: a 16-bit pass mask per lane, OR-reduced over the wave, and a loop over
      // just the rows some lane passed (uniform row index: one indexed register read each).  The
      // per-row uniform branch over all 16 rows ran ~245 VALU + ~140 SALU per tile (r6_f PMC).
      uint32_t pm = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) pm |= (acc[r] >= thr ? 1u : 0u) << r;
      uint32_t wm = pm;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) wm |= (uint32_t)__shfl_xor((int)wm, o, kWave);
      wm = __builtin_amdgcn_readfirstlane(wm);
      const int cbase = c0 + 4 * h;
      int qe = qn_ * kWave + lane;
      while (wm) {
        const int r = __builtin_ctz(wm);  // wave-uniform
        wm &= wm - 1;
        const int ci = cbase + (r & 3) + 8 * (r >> 2);
        if (((pm >> r) & 1u) && ci != self_c && ci < mc) {
          qent[qe] = make_int2(__float_as_int(acc[r]), ci);
          qe += kWave;
        }
      }
      qn_ = (qe - lane) / kWave;
      if (__any(qn_ >= QF)) flush();
    }
  }
  flush();
  ub_f = fmaxf(ub_f, __shfl_xor(ub_f, 32, kWave));
  mg_p = fmaxf(mg_p, __shfl_xor(mg_p, 32, kWave));
  // merge the two halves; drop the seeds (lanes h == 0 write)
  float os[kTopP];
  int oi[kTopP];
#pragma unroll
  for (int k = 0; k < kTopP; ++k) {
    os[k] = __shfl_xor(bs[k], 32, kWave);
    oi[k] = __shfl_xor(bi[k], 32, kWave);
  }
  merge_sorted<kTopP>(bs, bi, os, oi);
  if (h == 0 && qg < mq) {  // the non-seed entries, still sorted, then empty slots
    const int64_t o = ((int64_t)blockIdx.y * mq + qg) * kTopP;
    int w = 0;
#pragma unroll
    for (int k = 0; k < kTopP; ++k) {
      if (bi[k] != 0x7fffffff && !(bi[k] & kSeedFlag)) {
        ws_s[o + w] = bs[k];
        ws_i[o + w] = bi[k];
        ++w;
      }
    }
    for (; w < kTopP; ++w) {
      ws_s[o + w] = kNegBig;
      ws_i[o + w] = 0x7fffffff;
    }
    ws_m[2 * ((int64_t)blockIdx.y * mq + qg)] = ub_f;
    ws_m[2 * ((int64_t)blockIdx.y * mq + qg) + 1] = mg_p;
  }
}

// Per query: lps lanes (a power of two >= max(nsplit, kTopP)) merge the slices' approximate lists,
// re-score the best kTopP exactly and verify (see above); a query that fails the check is appended
// to `fail` (count in fail[0]) for knn_b3top_scan_kernel.
template <int K>
__global__ __launch_bounds__(256) void knn_b3top_final_kernel(const float* __restrict__ Q, const float* __restrict__ C,
                                                              int mq, int mc, int nsplit, int lps_log2,
                                                              int64_t self_offset, const float* __restrict__ ws_s,
                                                              const int* __restrict__ ws_i,
                                                              const float* __restrict__ ws_m,
                                                              int* __restrict__ out_idx, float* __restrict__ out_score,
                                                              int* __restrict__ fail) {
  const int lps = 1 << lps_log2;
  const int gl = blockIdx.x * 256 + threadIdx.x;
  const int q = gl >> lps_log2, sl = gl & (lps - 1);
  const bool live = q < mq;
  const int qq = live ? q : 0;
  const int64_t self_c = self_offset >= 0 ? self_offset + qq : -1;
  float as[kTopP];
  int ai[kTopP];
  float ub = kNegBig, mg = 0.0f;
#pragma unroll
  for (int k = 0; k < kTopP; ++k) { as[k] = kNegBig; ai[k] = 0x7fffffff; }
  if (live && sl < nsplit) {
    const int64_t o = ((int64_t)sl * mq + qq) * kTopP;
#pragma unroll
    for (int k = 0; k < kTopP; ++k) { as[k] = ws_s[o + k]; ai[k] = ws_i[o + k]; }
    ub = ws_m[2 * ((int64_t)sl * mq + qq)];
    mg = ws_m[2 * ((int64_t)sl * mq + qq) + 1];
  }
  for (int off = 1; off < lps; off <<= 1) {
    float os[kTopP];
    int oi[kTopP];
#pragma unroll
    for (int k = 0; k < kTopP; ++k) {
      os[k] = __shfl_xor(as[k], off, kWave);
      oi[k] = __shfl_xor(ai[k], off, kWave);
    }
    merge_sorted<kTopP>(as, ai, os, oi);
    mg = fmaxf(mg, __shfl_xor(mg, off, kWave));
    ub = fmaxf(ub, __shfl_xor(ub, off, kWave));
  }
  float qv[kCols];
  {
    const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)qq * kCols);
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) {
      const float4 v = p[k];
      qv[4 * k] = v.x; qv[4 * k + 1] = v.y; qv[4 * k + 2] = v.z; qv[4 * k + 3] = v.w;
    }
  }
  auto exact = [&](int ci) -> float {  // knn_rerank_kernel's re-score: columns 0..31 in order
    const float4* c = reinterpret_cast<const float4*>(C + (int64_t)ci * kCols);
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < kCols / 4; ++k) {
      const float4 v = c[k];
      acc = fmaf(qv[4 * k], v.x, acc);
      acc = fmaf(qv[4 * k + 1], v.y, acc);
      acc = fmaf(qv[4 * k + 2], v.z, acc);
      acc = fmaf(qv[4 * k + 3], v.w, acc);
    }
    return acc;
  };
  // lane sl < kTopP re-scores merged entry sl; every lane of the query then ranks all kTopP
  int my = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < kTopP; ++u) if (u == sl) my = ai[u];
  const float ex = (my != 0x7fffffff && sl < kTopP) ? exact(my) : kNegBig;
  const int base = threadIdx.x & ~(lps - 1) & (kWave - 1);
  float bs[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
#pragma unroll
  for (int u = 0; u < kTopP; ++u) {
    const float e = __shfl(ex, base + u, kWave);
    if (ai[u] != 0x7fffffff) topk_insert<K>(bs, bi, e, ai[u]);
  }
  // proof of exactness: the exact k-th best beats every unlisted candidate's upper bound
  const float bound = fmaxf(ub, as[kTopP - 1] > kNegBig ? as[kTopP - 1] + mg : kNegBig);
  const bool ok = bs[K - 1] > bound;
  if (live && !ok && sl == 0) fail[1 + atomicAdd(fail, 1)] = q;  // answered by the scan kernel
  if (live && sl == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      out_idx[(int64_t)q * K + k] = bi[k];
      if (out_score) out_score[(int64_t)q * K + k] = bs[k];
    }
  }
}

// The queries whose approximate lists could not prove their exact top k (fail[1 .. fail[0]]): one
// workgroup per query (grid-stride over the list; an empty list exits at once) scans every candidate
// with the exact fmaf chain -- 256 lanes, then a butterfly merge per wave and a 4-way merge in LDS.
template <int K>
__global__ __launch_bounds__(256) void knn_b3top_scan_kernel(const float* __restrict__ Q, const float* __restrict__ C,
                                                             int mc, int64_t self_offset, const int* __restrict__ fail,
                                                             int* __restrict__ out_idx, float* __restrict__ out_score) {
  const int nf = fail[0];
  __shared__ float ls[4][K];
  __shared__ int li[4][K];
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (int f = blockIdx.x; f < nf; f += gridDim.x) {
    const int q = fail[1 + f];
    const int64_t self_c = self_offset >= 0 ? self_offset + q : -1;
    float qv[kCols];
    {
      const float4* p = reinterpret_cast<const float4*>(Q + (int64_t)q * kCols);
#pragma unroll
      for (int k = 0; k < kCols / 4; ++k) {
        const float4 v = p[k];
        qv[4 * k] = v.x; qv[4 * k + 1] = v.y; qv[4 * k + 2] = v.z; qv[4 * k + 3] = v.w;
      }
    }
    float bs[K];
    int bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { bs[k] = kNegBig; bi[k] = 0x7fffffff; }
    // 4 candidates per lane in flight (every row load issued before the first fma)
    for (int c0 = threadIdx.x; c0 < mc; c0 += 4 * 256) {
      float4 rv[4][kCols / 4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ci = c0 + u * 256;
        const float4* c = reinterpret_cast<const float4*>(C + (int64_t)(ci < mc ? ci : 0) * kCols);
#pragma unroll
        for (int k = 0; k < kCols / 4; ++k) rv[u][k] = c[k];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ci = c0 + u * 256;
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < kCols / 4; ++k) {
          acc = fmaf(qv[4 * k], rv[u][k].x, acc);
          acc = fmaf(qv[4 * k + 1], rv[u][k].y, acc);
          acc = fmaf(qv[4 * k + 2], rv[u][k].z, acc);
          acc = fmaf(qv[4 * k + 3], rv[u][k].w, acc);
        }
        if (ci < mc && ci != self_c) topk_insert<K>(bs, bi, acc, ci);
      }
    }
    for (int off = 1; off < kWave; off <<= 1) {
      float os[K];
      int oi[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        os[k] = __shfl_xor(bs[k], off, kWave);
        oi[k] = __shfl_xor(bi[k], off, kWave);
      }
      merge_sorted<K>(bs, bi, os, oi);
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) { ls[wv][k] = bs[k]; li[wv][k] = bi[k]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 4; ++w) {
        float os[K];
        int oi[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { os[k] = ls[w][k]; oi[k] = li[w][k]; }
        merge_sorted<K>(bs, bi, os, oi);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        out_idx[(int64_t)q * K + k] = bi[k];
        if (out_score) out_score[(int64_t)q * K + k] = bs[k];
      }
    }
    __syncthreads();
  }
}

}  // namespace

int merge_log2(int nsplit) {
  if (nsplit > kWave) throw std::runtime_error("knn merge: at most 64 candidate slices");
  int l = 0;
  while ((1 << l) < nsplit) ++l;
  return l;
}

unsigned merge_blocks(int mq, int nsplit) {
  return (unsigned)(((int64_t)mq << merge_log2(nsplit)) + 255) / 256;
}

void launch_knn_prep(const float* X, int m, int m_pad, int role, float* out, float* outq,
                     const double* aff, uint16_t* P, hipStream_t stream, void* chl, void* qhl, float* tmax) {
  if (role < 0 || role > 2 || (role == 2) != (outq != nullptr) || (role == 1 && P != nullptr))
    throw std::invalid_argument("knn_prep: role 2 needs outq (and only it); parents need a candidate role");
  if ((chl != nullptr || qhl != nullptr || tmax != nullptr) &&
      (role != 2 || chl == nullptr || qhl == nullptr || tmax == nullptr || m_pad % 32 != 0))
    throw std::invalid_argument("knn_prep: the fused split needs role 2, all three outputs and m_pad % 32 == 0");
  knn_prep_kernel<<<(m_pad + 255) / 256, 256, 0, stream>>>(X, m, m_pad, role, out, outq, aff, P,
                                                            static_cast<uint4*>(chl), static_cast<uint4*>(qhl), tmax);
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

int knn_lds_splits(int mq_pad, int mc_pad) {
  static const int cap = resident_cap(knn_topk_lds_kernel<5>, kLW * kWave);
  const int qblocks = mq_pad / (32 * kLW), tiles = mc_pad / 32;
  int max_s = tiles / (8 * kCh);
  if (max_s > 64) max_s = 64;
  if (max_s < 1) max_s = 1;
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= max_s; ++s) {
    const double blocks = (double)qblocks * s;
    const double rounds = std::ceil(blocks / cap);
    double eff = blocks / (rounds * cap);
    eff -= 0.004 * (s - 1);
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return best;
}

void launch_knn_topk_lds(const float* Q, int mq_pad, int mq, const float* C, int mc_pad, int mc,
                         int64_t self_offset, int k, int* out_idx, float* out_score, float* ws_score, int* ws_idx,
                         int nsplit, hipStream_t stream) {
  if (mq_pad % (32 * kLW) != 0 || mc_pad % 32 != 0)
    throw std::runtime_error("knn_topk_lds: query pad must be x128, candidate pad x32");
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 1 && (ws_score == nullptr || ws_idx == nullptr))
    throw std::runtime_error("knn_topk_lds: split search needs the [nsplit][mq][k] workspaces");
  const dim3 grid(mq_pad / (32 * kLW), nsplit);
  int* oi = nsplit > 1 ? ws_idx : out_idx;
  float* os = nsplit > 1 ? ws_score : out_score;
#define FDX_KNNL(KK)                                                                                          \
  knn_topk_lds_kernel<KK><<<grid, kLW * kWave, 0, stream>>>(Q, mq, C, mc_pad, mc, self_offset, oi, os);       \
  if (nsplit > 1)                                                                                             \
    knn_merge_kernel<KK><<<merge_blocks(mq, nsplit), 256, 0, stream>>>(ws_score, ws_idx, nsplit, merge_log2(nsplit), mq, out_idx, out_score)
  switch (k) {
    case 1: FDX_KNNL(1); break;
    case 2: FDX_KNNL(2); break;
    case 3: FDX_KNNL(3); break;
    case 4: FDX_KNNL(4); break;
    case 5: FDX_KNNL(5); break;
    case 6: FDX_KNNL(6); break;
    case 7: FDX_KNNL(7); break;
    case 8: FDX_KNNL(8); break;
    default: throw std::runtime_error("knn_topk_lds: k must be in [1, 8]");
  }
#undef FDX_KNNL
  check_launch("knn_topk_lds");
}

void launch_knn_split(const float* Xp, int m_pad, int role, uint4* hl, float* tmax, hipStream_t stream) {
  knn_split_kernel<<<(m_pad + 255) / 256, 256, 0, stream>>>(Xp, m_pad, role, hl, tmax);
  check_launch("knn_split");
}

int knn3_splits(int mq_pad, int mc_pad) {
  static const int cap = resident_cap(knn_topk3_kernel<5>, kWave);
  const int qblocks = mq_pad / 32, tiles = mc_pad / 32;
  int max_s = tiles / 8;
  if (max_s > 32) max_s = 32;
  if (max_s < 1) max_s = 1;
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= max_s; ++s) {
    const double blocks = (double)qblocks * s;
    const double rounds = std::ceil(blocks / cap);
    double eff = blocks / (rounds * cap);
    eff -= 0.004 * (s - 1);
    if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
  }
  return best;
}

void launch_knn_topk3(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                      const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                      float* out_score, float* ws_score, int* ws_idx, int nsplit, hipStream_t stream) {
  if (mq_pad % 32 != 0 || mc_pad % 32 != 0) throw std::runtime_error("knn_topk3: pads must be x32");
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 1 && (ws_score == nullptr || ws_idx == nullptr))
    throw std::runtime_error("knn_topk3: split search needs the [nsplit][mq][k] workspaces");
  const dim3 grid(mq_pad / 32, nsplit);
  int* oi = nsplit > 1 ? ws_idx : out_idx;
  float* os = nsplit > 1 ? ws_score : out_score;
  const uint4* qh = reinterpret_cast<const uint4*>(Qhl);
  const uint4* chl = reinterpret_cast<const uint4*>(Chl);
#define FDX_KNN3(KK)                                                                            \
  knn_topk3_kernel<KK><<<grid, kWave, 0, stream>>>(Q, qh, mq, C, chl, tmax, mc_pad, mc, self_offset, oi, os); \
  if (nsplit > 1)                                                                               \
    knn_merge_kernel<KK><<<merge_blocks(mq, nsplit), 256, 0, stream>>>(ws_score, ws_idx, nsplit, merge_log2(nsplit), mq, out_idx, out_score)
  switch (k) {
    case 1: FDX_KNN3(1); break;
    case 2: FDX_KNN3(2); break;
    case 3: FDX_KNN3(3); break;
    case 4: FDX_KNN3(4); break;
    case 5: FDX_KNN3(5); break;
    case 6: FDX_KNN3(6); break;
    case 7: FDX_KNN3(7); break;
    case 8: FDX_KNN3(8); break;
    default: throw std::runtime_error("knn_topk3: k must be in [1, 8]");
  }
#undef FDX_KNN3
  check_launch("knn_topk3");
}

int knn3r_list_cap() { return kListCap; }

int knn3r_splits(int mq_pad, int mc_pad) {
  // Six slices (fewer on small candidate sets: >= 16 tiles each).  Round 5 measured 4 best (r5_o:
  // every slice adds its own list entries and re-rank work); with the fragment-order fetch, the
  // re-rank's final-threshold skip and the seeded slices, 6 edges it (profiles/r6_knn
  // slice_sweep.json: 0.162 vs 0.170 ms at DP=1, 0.485 vs 0.491 at the DP=8 rank; 2, 3, 5, 8 slower).
  (void)mq_pad;
  const int tiles = mc_pad / 32;
  int s = tiles / 16;
  if (s > 6) s = 6;
  if (s < 1) s = 1;
  return s;
}

void launch_knn_topk3r(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                       const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                       float* out_score, int* lists, int* counts, int nsplit, hipStream_t stream) {
  int2* lists2 = reinterpret_cast<int2*>(lists);  // [.. ][cap][64] (lower bound, index) pairs
  if (mq_pad % 32 != 0 || mc_pad % 32 != 0) throw std::runtime_error("knn_topk3r: pads must be x32");
  if (mq > mq_pad || mc > mc_pad || nsplit < 1 || lists == nullptr || counts == nullptr)
    throw std::runtime_error("knn_topk3r: bad shapes or missing list workspaces");
  const dim3 grid(mq_pad / 32, nsplit);
  const uint4* qh = reinterpret_cast<const uint4*>(Qhl);
  const uint4* chl = reinterpret_cast<const uint4*>(Chl);
  const unsigned rblocks = (unsigned)(((int64_t)mq * 8 + 255) / 256);
#define FDX_KNN3R(KK)                                                                                       \
  knn_collect_kernel<KK><<<grid, kWave, 0, stream>>>(Q, qh, chl, tmax, mq, mc_pad, mc, self_offset, lists2, counts); \
  knn_rerank_kernel<KK><<<rblocks, 256, 0, stream>>>(Q, C, mq, mc, mq_pad / 32, nsplit, self_offset, lists2, counts, \
                                                     out_idx, out_score)
  switch (k) {
    case 1: FDX_KNN3R(1); break;
    case 2: FDX_KNN3R(2); break;
    case 3: FDX_KNN3R(3); break;
    case 4: FDX_KNN3R(4); break;
    case 5: FDX_KNN3R(5); break;
    case 6: FDX_KNN3R(6); break;
    case 7: FDX_KNN3R(7); break;
    case 8: FDX_KNN3R(8); break;
    default: throw std::runtime_error("knn_topk3r: k must be in [1, 8]");
  }
#undef FDX_KNN3R
  check_launch("knn_topk3r");
}

int knn_b3top_splits(int mq_pad, int mc_pad) {
  // As many slices as fill the resident one-wave workgroups in ONE round (the seeds spare each slice
  // its fill phase; 108 VGPRs: 4 waves per SIMD), >= 8 tiles each, <= 32 (the final merge's lanes per
  // query).  FDX_KNN_B3_SPLITS: lab override.
  static const int cap = resident_cap(knn_b3top_kernel<>, kWave);
  static const int forced = [] {
    const char* e = std::getenv("FDX_KNN_B3_SPLITS");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  const int qblocks = mq_pad / 32, tiles = mc_pad / 32;
  int s = forced > 0 ? forced : cap / (qblocks > 0 ? qblocks : 1);
  if (s > 32) s = 32;
  if (s > tiles / 8) s = tiles / 8;
  if (s < 1) s = 1;
  return s;
}

void launch_knn_b3top(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                      const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                      float* out_score, float* ws_s, int* ws_i, float* ws_m, int* fail, int nsplit,
                      hipStream_t stream) {
  if (mq_pad % 32 != 0 || mc_pad % 32 != 0) throw std::runtime_error("knn_b3top: pads must be x32");
  if (mq > mq_pad || mc > mc_pad || nsplit < 1 || nsplit > 32 || ws_s == nullptr || ws_i == nullptr || ws_m == nullptr)
    throw std::runtime_error("knn_b3top: bad shapes or missing [nsplit][mq][8] workspaces");
  if (fail == nullptr) throw std::runtime_error("knn_b3top: missing the [1 + mq] failed-query list");
  if (hipMemsetAsync(fail, 0, sizeof(int), stream) != hipSuccess) throw std::runtime_error("knn_b3top: memset");
  if (k < 1 || k > kTopP) throw std::runtime_error("knn_b3top: k must be in [1, 8]");
  const dim3 grid(mq_pad / 32, nsplit);
  knn_b3top_kernel<><<<grid, kWave, 0, stream>>>(Q, reinterpret_cast<const uint4*>(Qhl),
                                                  reinterpret_cast<const uint4*>(Chl), tmax, mq, mc_pad, mc,
                                                  self_offset, ws_s, ws_i, ws_m);
  int lg = merge_log2(nsplit);
  if (lg < 3) lg = 3;  // >= kTopP lanes per query: lane u re-scores merged entry u
  const unsigned fb = (unsigned)((((int64_t)mq << lg) + 255) / 256);
#define FDX_KNNB3(KK)                                                                                         \
  knn_b3top_final_kernel<KK><<<fb, 256, 0, stream>>>(Q, C, mq, mc, nsplit, lg, self_offset, ws_s, ws_i, ws_m, \
                                                     out_idx, out_score, fail);                                   \
  knn_b3top_scan_kernel<KK><<<256, 256, 0, stream>>>(Q, C, mc, self_offset, fail, out_idx, out_score)
  switch (k) {
    case 1: FDX_KNNB3(1); break;
    case 2: FDX_KNNB3(2); break;
    case 3: FDX_KNNB3(3); break;
    case 4: FDX_KNNB3(4); break;
    case 5: FDX_KNNB3(5); break;
    case 6: FDX_KNNB3(6); break;
    case 7: FDX_KNNB3(7); break;
    default: FDX_KNNB3(8); break;
  }
#undef FDX_KNNB3
  check_launch("knn_b3top");
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
  knn_topk_kernel<KK><<<grid, kWave, 0, stream>>>(Q, mq, C, mc_pad, mc, self_offset, oi, os); \
  if (nsplit > 1)                                                                               \
    knn_merge_kernel<KK><<<merge_blocks(mq, nsplit), 256, 0, stream>>>(ws_score, ws_idx, nsplit, merge_log2(nsplit), mq, out_idx, out_score)
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
