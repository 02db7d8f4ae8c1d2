// K11 gbdt_*: histogram gradient-boosted trees (XGBoost "hist" semantics) on MI355X.
//
// Reference behaviour being replaced: XGBClassifier(objective='binary:logistic',
// n_estimators=100, learning_rate=0.1, max_depth=5, scale_pos_weight=neg/pos) fitted in
// train_model.py:69-80 (per CV fold) and :95-106 (final), SURVEY.md §2.3 row K11.
//
// Design (MI355X-first, not a port of xgboost's CPU/CUDA updaters):
//  * Features are quantised once to u8 bins (<= 256 quantile cuts per feature; row = 32 bytes),
//    so the per-level data stream is 32 B/row instead of 120 B of fp32.
//  * Gradients/Hessians are quantised per boosting round to fixed point (power-of-two scale,
//    |g|, h <= 2^14) and histograms accumulate exactly: ONE packed 64-bit LDS atomic per
//    (row, feature) carries h in the high word and g (signed) in the low word -- exact while a
//    block's partial sums stay below 2^31, i.e. for <= 2^16 rows between flushes -- then one
//    global int64 atomic flush per (block, node, g|h).  Integer addition is associative, so histograms -- and
//    therefore every split decision -- are bitwise deterministic regardless of scheduling, the
//    sibling histogram is an exact parent - child subtraction, and the data-parallel
//    all-reduce of histograms over RCCL is exact too.
//  * Rows stay node-partitioned (a permutation `ridx` with contiguous per-node segments, stable
//    partition per level), so a histogram block touches only the rows of the nodes it builds.
//    Only the smaller child of every split is histogrammed; the larger one is parent - sibling.
//  * Trees are complete heaps of depth D: a node that does not split becomes a pass-through
//    ("everything goes left", threshold +inf), so training and inference walk exactly D levels
//    with no divergence on tree shape, and leaves sit at heap ids [2^D - 1, 2^(D+1) - 1).
//  * Split search: one wave per feature, 4 bins per lane, int64 prefix scan, gain in fp64 with
//    contraction disabled (the numpy oracle in ops/reference.py reproduces it bit-for-bit).
//  * No host synchronisation inside a fit: segment sizes, build flags and leaf values stay on
//    device, so a boosting round is a fixed launch sequence (hipGraph-capturable).
#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kGBBins = 256;
constexpr int kGBRowBytes = 32;
constexpr int kGBMaxFeat = 30;
constexpr int kGBMaxNodes = 127;  // internal nodes of a depth-7 tree (node ids fit a byte)
constexpr int kHistEntries = kGBMaxFeat * kGBBins * 2;  // per node: [feature][bin][g, h]
constexpr int kHistThreads = 1024;
constexpr int kPartThreads = 256;

__device__ __forceinline__ int heap_first(int level) { return (1 << level) - 1; }

// Level 0 walks the fit's rows in order without reading ridx.  A cross-validation fold fits the
// table minus one contiguous block [hole_at, hole_at + hole_len) (the fold's validation rows, whose
// margins the round's margin update scores for free): position p of the root is row
// p + (p >= hole_at ? hole_len : 0).  Deeper levels read ridx, which holds those row ids.
__device__ __forceinline__ int64_t hole_row(int64_t p, int64_t hole_at, int64_t hole_len) {
  return p + (p >= hole_at ? hole_len : 0);
}

// Build flag of a node at level >= 1: the smaller child of each split (ties: the left one) is
// histogrammed; its sibling is derived.  `gcnt` holds global (all-rank) row counts.
__device__ __forceinline__ bool is_built(int node, const int64_t* gcnt) {
  if (node == 0) return true;
  const bool left = (node & 1) != 0;
  const int sib = left ? node + 1 : node - 1;
  const int64_t c = gcnt[node], s = gcnt[sib];
  return left ? (c <= s) : (c < s);
}

// ---- quantisation ----------------------------------------------------------------------------
// 8 lanes per row, 4 features per lane: the 8 lanes write one 32-byte binned row.
//  * VEC (rows 16-byte aligned, ld % 4 == 0 -- the pipeline's [n, 32] fp32 rows): each lane reads
//    its 4 features with ONE 16-byte load, so a row is one coalesced 128-byte read (the scalar
//    form issued 4 loads per lane);
//  * the upper-bound search is branchless over the 256 cut slots (cuts past nbins are +inf):
//    8 dependent LDS reads with the lane's 4 features as 4 independent chains, and a NaN lands in
//    the last bin exactly as the branchy search did (!(cut > x) holds);
//  * the LDS cut table is bin-major with a 33-float row (sc[b][f]): the 8 features a wave reads at
//    the same search depth sit in distinct banks instead of all in bank (mid mod 64).
//  * the first three search levels compare against registers (7 cuts per feature), the last five
//    read LDS.
// (2.78 ms in round 3; 0.94 ms with the vector loads and the LDS-only search, profiles/r4_k)
constexpr int kCutLd = 33;
template <bool VEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void gbdt_bin_kernel(const float* __restrict__ X, int64_t n, int ld,
                                                       int d, const float* __restrict__ cuts,
                                                       const int* __restrict__ nbins,
                                                       uint8_t* __restrict__ bins) {
  __shared__ float sc[kGBBins * kCutLd];
  __shared__ int snb[32];
  for (int i = threadIdx.x; i < kGBBins * 32; i += blockDim.x) {
    const int b = i >> 5, f = i & 31;
    sc[b * kCutLd + f] = f < d ? cuts[f * kGBBins + b] : __builtin_inff();
  }
  if (threadIdx.x < 32) snb[threadIdx.x] = threadIdx.x < d ? nbins[threadIdx.x] : 1;
  __syncthreads();
  const int sub = threadIdx.x & 7;
  int nbm1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) nbm1[j] = snb[sub * 4 + j] - 1;
  // the top three levels of every search from registers: the 7 cuts of the implicit tree's first
  // three levels (indices 127 | 63, 191 | 31, 95, 159, 223) per feature, 28 VGPRs -- the dependent
  // LDS chain is 5 reads instead of 8, and LDS traffic drops by 3/8
  float t1[4], t2[4][2], t3[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = sub * 4 + j;
    t1[j] = sc[127 * kCutLd + f];
    t2[j][0] = sc[63 * kCutLd + f];
    t2[j][1] = sc[191 * kCutLd + f];
#pragma unroll
    for (int u = 0; u < 4; ++u) t3[j][u] = sc[(31 + 64 * u) * kCutLd + f];
  }
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 8);
  const int64_t r0 = (int64_t)blockIdx.x * (blockDim.x / 8) + (threadIdx.x >> 3);
  // VEC: the rows of the next two iterations are in flight while this one is searched -- the
  // grid is resident-capped (16 waves per CU), and with one 16-byte load per lane outstanding the
  // whole chip kept ~4 MB in flight, ~2.9 TB/s (0.87 ms at 16M rows, profiles/r4_q; 0.79 ms with
  // the two-deep prefetch, profiles/r4_v)
  const float4 zero4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float4 pf0 = zero4, pf1 = zero4;
  if constexpr (VEC) {
    if (r0 < n) pf0 = reinterpret_cast<const float4*>(X + r0 * ld)[sub];
    if (r0 + stride < n) pf1 = reinterpret_cast<const float4*>(X + (r0 + stride) * ld)[sub];
  }
  for (int64_t r = r0; r < n; r += stride) {
    float x[4];
    if constexpr (VEC) {
      const float4 v = pf0;
      pf0 = pf1;
      if (r + 2 * stride < n) pf1 = reinterpret_cast<const float4*>(X + (r + 2 * stride) * ld)[sub];
      x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (sub * 4 + j < d) ? X[r * ld + sub * 4 + j] : 0.0f;
    }
    int b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int bb = !(t1[j] > x[j]) ? 128 : 0;
      bb += !((bb ? t2[j][1] : t2[j][0]) > x[j]) ? 64 : 0;
      const float c3 = (bb & 128) ? ((bb & 64) ? t3[j][3] : t3[j][2]) : ((bb & 64) ? t3[j][1] : t3[j][0]);
      b[j] = bb + (!(c3 > x[j]) ? 32 : 0);
    }
#pragma unroll
    for (int half = kGBBins / 16; half >= 1; half >>= 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = sc[(b[j] + half - 1) * kCutLd + sub * 4 + j];
        b[j] += !(c > x[j]) ? half : 0;
      }
    }
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int bb = (sub * 4 + j < d) ? min(b[j], nbm1[j]) : 0;
      packed |= (uint32_t)bb << (8 * j);
    }
    reinterpret_cast<uint32_t*>(bins + r * kGBRowBytes)[sub] = packed;
  }
}

// ---- per-round gradients ---------------------------------------------------------------------
// logistic: g = (p - y) w, h = max(p (1 - p), 1e-16) w, w = scale_pos_weight for positives.
// fp64 so the quantised values match the numpy oracle except at measure-zero ties.
// (g, h) of a row packed into one 32-bit word, g in the low int16 and h in the high half
// (|g|, h <= 2^14): the histogram passes read 4 bytes of gradients per row instead of 8.
__device__ __forceinline__ uint32_t pack_gh(int2 q) {
  return (uint32_t)(uint16_t)(int16_t)q.x | ((uint32_t)(uint16_t)q.y << 16);
}
__device__ __forceinline__ int2 quantised_grad(float margin, bool pos, float spw, float gscale, float hscale) {
  const double m = (double)margin;
  const double p = 1.0 / (1.0 + exp(-m));
  const double w = pos ? (double)spw : 1.0;
  const double g = (p - (pos ? 1.0 : 0.0)) * w;
  const double h = fmax(p * (1.0 - p), 1e-16) * w;
  return make_int2((int)rint(g * (double)gscale), (int)rint(h * (double)hscale));
}

// First round of a fit only: later rounds get their gradients from gbdt_margin_kernel<true>.
__global__ __launch_bounds__(256) void gbdt_grad_kernel(const float* __restrict__ margin,
                                                        const uint8_t* __restrict__ label, int64_t n,
                                                        float spw, float gscale, float hscale,
                                                        uint32_t* __restrict__ gh) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    gh[i] = pack_gh(quantised_grad(margin[i], label[i] != 0, spw, gscale, hscale));
}

// ---- histograms ------------------------------------------------------------------------------
// Grid: resident blocks (2 per CU: 60 KiB of LDS each).  The rows of this level's *built* nodes
// are concatenated in node order into a virtual range that the grid splits evenly, so the work
// per block is balanced whatever the segment sizes are.
//
// LDS: one packed u64 per [feature][bin]: (h << 32) + g with g sign-extended.  Integer addition
// of packed words is the pair of additions as long as the low word's true sum stays inside
// int32 (|sum g| < 2^31, sum h < 2^31): at |g|, h <= 2^14 per row that holds for any 2^16 rows,
// so a block flushes every kFlushRows rows.
//
// Flush: NO global atomics from the histogram blocks.  Each (node, block) pair owns a slot of
// int64 [feature][bin][g, h] that the block writes with plain coalesced stores; a reduce kernel
// then sums each node's slots (16-way split of the slot axis, one int64 atomic per split).  With
// 512 blocks all adding 15k int64 atomics to the SAME node words, the flush was a fixed ~140 us
// per level whatever the row count (profiles/r3_v: 157 us at 2M rows, 322 us at 16M).
constexpr int kHistWords = kGBMaxFeat * kGBBins;  // 7680 u64 = 60 KiB
constexpr int64_t kFlushRows = 1 << 16;
constexpr int kHistBatch = 4;
constexpr int kSlotSplit = 16;

// Node k's place in the level's virtual row range and its slot range: blocks [b0, b0 + cnt)
// touch it, their slots are [base, base + cnt).  Same arithmetic in the histogram and the
// reduce kernels.
struct NodeSlots {
  int64_t off, sc;
  int b0, cnt, base;
};
// The level's node table (segment sizes, global row counts) staged in LDS by all threads at once:
// the per-node walks below then read LDS -- they were chains of dependent global loads, 2^level
// long, in every block (the slot reduce took 15 us at level 1 and 90 us at level 4, r4_l).
constexpr int kMaxLevelNodes = (kGBMaxNodes + 1) / 2;  // 64 nodes at the deepest level
struct LevelNodes {
  int64_t sc[kMaxLevelNodes];   // row count of node h0 + k
  int64_t gc[kMaxLevelNodes];   // global (all-rank) row count of node h0 + k
};
__device__ __forceinline__ void load_level(LevelNodes& L, const int64_t* seg, const int64_t* gcnt, int level) {
  const int h0 = heap_first(level), nn = 1 << level;
  for (int k = threadIdx.x; k < nn; k += blockDim.x) {
    L.sc[k] = seg[2 * (h0 + k) + 1];
    L.gc[k] = gcnt[h0 + k];
  }
  __syncthreads();
}
// is_built on the staged table: node h0 + k of a level >= 1 is a left child iff k is even, and
// its sibling is h0 + (k ^ 1)
__device__ __forceinline__ bool built_l(const LevelNodes& L, int level, int k) {
  if (level == 0) return true;
  const int64_t c = L.gc[k], s = L.gc[k ^ 1];
  return (k & 1) == 0 ? (c <= s) : (c < s);
}
__device__ __forceinline__ int64_t level_chunk(const LevelNodes& L, int level, int nblocks, int64_t* total_out) {
  const int nn = 1 << level;
  int64_t total = 0;
  for (int k = 0; k < nn; ++k)
    if (built_l(L, level, k)) total += L.sc[k];
  *total_out = total;
  return (total + nblocks - 1) / nblocks;
}

// ROT: the 64 lanes of a wave do not add into the same feature at the same time.  Lane l walks the
// 32 feature slots starting at slot (l mod 32) -- its 32-byte bin row rotated by that many bytes
// once per row (a 3-stage dword barrel shift + one byte funnel), so every bin byte is still
// extracted with a static shift -- and feature f's sub-histogram starts at f * kHistStrideRot (an
// odd number of u64: consecutive features start in different bank pairs).  A wave's concurrent
// atomics then hit 32 different sub-histograms instead of one: no same-address collisions within
// a feature and no lockstep on one 2 KiB region.  Integer adds: every histogram bit is unchanged.
constexpr int kHistStrideRot = kGBBins + 1;
constexpr int kHistWordsRot = 32 * kHistStrideRot;  // 8224 u64 = 64.25 KiB (two blocks per CU fit)
constexpr int kHistBatchRot = 4;  // rows in flight per thread
// SPLIT (lab variant 2): g and h in two int32 sub-histograms, two ds_add_u32 per (row, feature)
// instead of one 64-bit packed add -- a wave's 64 lanes then spread over 64 single-dword banks
// rather than 32 bank pairs.  Same sums (int32 exact within a flush), same flush layout.
// LANE (variant 3, the default): EIGHT lanes per row instead of one -- lane j of a row owns its
// bins dword j (features 4j .. 4j + 3), so a wave instruction adds 8 rows x 8 features, and every
// lane of a 16-lane group (and of a 32-lane group) adds into a DIFFERENT bank pair by construction.
// Words are bin-major, [bin][slot] with 32 slots, slot(f) = 8 (f & 3) + (f >> 2), i.e. feature
// 4j + kk at slot 8 kk + j (bank pair = slot mod 16 with 32 banks, mod 32 with 64).  At step k the
// row r-th of a 32-lane group (r = 0..3) adds its byte kk = k ^ r: rows 0..3 take the four kk, so
// the 32 lanes hit slots 8 kk + j = all 32 residues -- no bank conflict in any lane grouping, and
// no same-address collision (r5 PMC of the lockstep form: 8.4 bank-conflict + 2.6 address-conflict
// cycles per LDS instruction, 64 lanes adding random bins of ONE feature).  One row's (g, h) word is
// read by its 8 lanes (one broadcast fetch), its 32 bin bytes as 8 coalesced dwords.  Integer adds
// into the same packed words: every histogram -- and tree -- bit is unchanged.
constexpr int kHistWordsLane = kGBBins * 32;  // 8192 u64 = 64 KiB (two 1024-thread blocks per CU fit)
constexpr int kHistBatchLane = 4;             // row groups in flight per lane
enum HistVariant : int { kHistLockstep = 0, kHistRot = 1, kHistSplit = 2, kHistLane = 3 };
// L0 (LANE only): level 0, whose rows are the fit's rows in order (hole skipped): no ridx reads and
// no per-row level test.
template <int VAR, bool L0 = false>
__global__ __launch_bounds__(kHistThreads, VAR == kHistRot ? 4 : 8) void gbdt_hist_kernel(  // 8 waves/SIMD = 2 blocks/CU: <= 64 VGPRs
                                                                           // (ROT: 1 block/CU, <= 128 VGPRs)
    const uint8_t* __restrict__ bins, const uint32_t* __restrict__ gh, const int* __restrict__ ridx,
    const int64_t* __restrict__ seg, const int64_t* __restrict__ gcnt, int level, int d,
    long long* __restrict__ slots, int64_t flush_rows, int64_t hole_at, int64_t hole_len) {
  constexpr bool ROT = VAR == kHistRot, SPLIT = VAR == kHistSplit, LANE = VAR == kHistLane;
  constexpr int kStride = ROT ? kHistStrideRot : kGBBins;
  constexpr int kBatch = ROT ? kHistBatchRot : (LANE ? kHistBatchLane : kHistBatch);
  __shared__ unsigned long long sh[ROT ? kHistWordsRot : (LANE ? kHistWordsLane : kHistWords)];
  int* const shg = reinterpret_cast<int*>(sh);  // SPLIT: g at [f * 256 + b], h kHistWords ints later
  int* const shh = shg + kHistWords;
  __shared__ LevelNodes lv;
  const int h0 = heap_first(level), nn = 1 << level;
  load_level(lv, seg, gcnt, level);
  int64_t total;
  const int64_t chunk = level_chunk(lv, level, gridDim.x, &total);
  const int64_t vb = (int64_t)blockIdx.x * chunk;
  const int64_t ve = min(vb + chunk, total);
  if (vb >= ve) return;
  const int nw = d * kGBBins;
  int64_t off = 0;
  int slot_base = 0;
  for (int k = 0; k < nn; ++k) {
    const int node = h0 + k;
    if (!built_l(lv, level, k)) continue;
    const int64_t sc = lv.sc[k];
    const int64_t lo = max(off, vb), hi = min(off + sc, ve);
    const int64_t sb = lo < hi ? seg[2 * node] : 0;  // the node's first row (only where it is used)
    const int b0 = sc > 0 ? (int)(off / chunk) : 0;
    const int cnt = sc > 0 ? (int)((off + sc - 1) / chunk) - b0 + 1 : 0;
    off += sc;
    const int my_slot = slot_base + ((int)blockIdx.x - b0);
    slot_base += cnt;
    if (lo >= hi) continue;
    long long* dst = slots + (int64_t)my_slot * kHistEntries;
    for (int64_t c0 = lo; c0 < hi; c0 += flush_rows) {
      const int64_t c1 = min(hi, c0 + flush_rows);
      if constexpr (LANE) {
        for (int i = threadIdx.x; i < kHistWordsLane; i += kHistThreads) sh[i] = 0ull;
      } else {
        for (int i = threadIdx.x; i < nw; i += kHistThreads) {
          if constexpr (SPLIT) {
            shg[i] = 0;
            shh[i] = 0;
          } else {
            sh[ROT ? (i >> 8) * kStride + (i & 255) : i] = 0ull;
          }
        }
      }
      __syncthreads();
      // kBatch rows per thread in flight: every row index, then every row's bins and (g, h),
      // are loaded before the first atomic.  Level 0 reads rows in order (ridx is the identity
      // after the round init).
      const int64_t pbase = sb - (off - sc);
      if constexpr (LANE) {
        const int lane = lane_id();
        const int j = lane & 7, r4 = (lane >> 3) & 3;
        constexpr int kRowsPerIter = kHistThreads / 8;  // 128 rows per block per batch slot
        // Step k adds byte kk = k ^ r4 of the row's dword j.  One v_perm per row puts byte kk at
        // position k, so every step extracts a STATIC byte (the k = 1 step is a single and-or), and
        // its slot offset 8 kk is a per-lane base pointer.  Rows past the range add 0 (no branch).
        const uint32_t sel = (uint32_t)(0 ^ r4) | ((uint32_t)(1 ^ r4) << 8) | ((uint32_t)(2 ^ r4) << 16) |
                             ((uint32_t)(3 ^ r4) << 24);
        unsigned long long* hk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) hk[k] = sh + j + 8 * (k ^ r4);  // slot 8 kk + j of bin b: hk[k][b * 32]
        for (int64_t v0 = c0 + (threadIdx.x >> 3); v0 < c1; v0 += (int64_t)kRowsPerIter * kBatch) {
          int rows[kBatch];
          bool ok[kBatch];
#pragma unroll
          for (int u = 0; u < kBatch; ++u) {
            const int64_t v = v0 + (int64_t)u * kRowsPerIter;
            ok[u] = v < c1;
            const int64_t p = ok[u] ? pbase + v : pbase + c0;  // in range either way
            rows[u] = L0 ? (int)hole_row(p, hole_at, hole_len) : ridx[p];
          }
          uint32_t bw[kBatch], gw[kBatch];
#pragma unroll
          for (int u = 0; u < kBatch; ++u) {
            bw[u] = reinterpret_cast<const uint32_t*>(bins + (int64_t)rows[u] * kGBRowBytes)[j];
            gw[u] = gh[rows[u]];
          }
#pragma unroll
          for (int u = 0; u < kBatch; ++u) {
            const uint32_t g = ok[u] ? gw[u] : 0u;
            const unsigned long long pk =
                ((unsigned long long)(g >> 16) << 32) + (unsigned long long)(long long)(int16_t)(g & 0xffffu);
            const uint32_t b = __builtin_amdgcn_perm(bw[u], bw[u], sel);
#pragma unroll
            for (int k = 0; k < 4; ++k) atomicAdd(hk[k] + ((b >> (8 * k)) & 0xffu) * 32, pk);
          }
        }
      } else
      for (int64_t v0 = c0 + threadIdx.x; v0 < c1; v0 += kHistThreads * kBatch) {
        int64_t rows[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int64_t v = v0 + (int64_t)u * kHistThreads;
          rows[u] = v < c1 ? (level == 0 ? hole_row(pbase + v, hole_at, hole_len) : (int64_t)ridx[pbase + v]) : -1;
        }
        uint32_t words[kBatch][8];
        unsigned long long pk[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int64_t row = rows[u] < 0 ? 0 : rows[u];
          const uint4* br = reinterpret_cast<const uint4*>(bins + row * kGBRowBytes);
          const uint4 b0v = br[0], b1v = br[1];
          const uint32_t w = gh[row];
          const int2 q = make_int2((int)(int16_t)(w & 0xffffu), (int)(w >> 16));
          words[u][0] = b0v.x; words[u][1] = b0v.y; words[u][2] = b0v.z; words[u][3] = b0v.w;
          words[u][4] = b1v.x; words[u][5] = b1v.y; words[u][6] = b1v.z; words[u][7] = b1v.w;
          pk[u] = ((unsigned long long)(uint32_t)q.y << 32) + (unsigned long long)(long long)q.x;
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          if (rows[u] < 0) continue;
          if constexpr (ROT) {
            const int rot = lane_id() & 31;
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = words[u][i];
#pragma unroll
            for (int stage = 0; stage < 3; ++stage) {  // dwords rotated left by rot >> 2
              const int sh_d = 1 << stage;
              const bool on = ((rot >> 2) >> stage) & 1;
              uint32_t t[8];
#pragma unroll
              for (int i = 0; i < 8; ++i) t[i] = on ? w[(i + sh_d) & 7] : w[i];
#pragma unroll
              for (int i = 0; i < 8; ++i) w[i] = t[i];
            }
            uint32_t rw[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) rw[i] = __builtin_amdgcn_alignbyte(w[(i + 1) & 7], w[i], rot & 3);
            // feature of slot jj: jj + rot, minus 32 past the end (the LDS offset of slot jj is an
            // immediate; one wrapped base register)
            unsigned long long* s0 = sh + rot * kStride;
            unsigned long long* s1 = s0 - 32 * kStride;
#pragma unroll
            for (int jj = 0; jj < 32; ++jj) {
              const int f = (jj + rot) & 31;
              if (f < d) {
                const int b = (rw[jj >> 2] >> (8 * (jj & 3))) & 0xff;
                atomicAdd((jj + rot < 32 ? s0 : s1) + jj * kStride + b, pk[u]);
              }
              if ((jj & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // keep the live ranges short
            }
          } else if constexpr (SPLIT) {
            const int qg = (int)(uint32_t)(pk[u] & 0xffffffffull);  // the packed word's (g, h)
            const int qh = (int)((pk[u] - (unsigned long long)(long long)qg) >> 32);
#pragma unroll
            for (int f = 0; f < kGBMaxFeat; ++f) {
              if (f < d) {
                const int b = (words[u][f >> 2] >> (8 * (f & 3))) & 0xff;
                atomicAdd(shg + f * kGBBins + b, qg);
                atomicAdd(shh + f * kGBBins + b, qh);
              }
            }
          } else {
#pragma unroll
            for (int f = 0; f < kGBMaxFeat; ++f) {
              if (f < d) {
                const int b = (words[u][f >> 2] >> (8 * (f & 3))) & 0xff;
                atomicAdd(sh + f * kGBBins + b, pk[u]);
              }
            }
          }
        }
      }
      __syncthreads();
      const bool first = c0 == lo;  // later flushes of the same slot accumulate (block-private)
      for (int i = threadIdx.x; i < nw; i += kHistThreads) {
        long long sg, sgh;
        if constexpr (SPLIT) {
          sg = shg[i];
          sgh = shh[i];
        } else if constexpr (LANE) {
          const int f = i >> 8, b = i & 255;
          const unsigned long long x = sh[b * 32 + 8 * (f & 3) + (f >> 2)];
          sg = (long long)(int32_t)(uint32_t)(x & 0xffffffffull);
          sgh = (long long)(x - (unsigned long long)sg) >> 32;
        } else {
          const unsigned long long x = sh[ROT ? (i >> 8) * kStride + (i & 255) : i];
          sg = (long long)(int32_t)(uint32_t)(x & 0xffffffffull);
          sgh = (long long)(x - (unsigned long long)sg) >> 32;
        }
        long long* e = dst + 2 * i;
        if (first) {
          e[0] = sg;
          e[1] = sgh;
        } else {
          e[0] += sg;
          e[1] += sgh;
        }
      }
      __syncthreads();
    }
  }
}

// Level 0 of a boosting round with the previous round's margin walk and gradients fused in (every
// round of a fit after its first).  Per step of 1024 root positions: phase A, one thread per row,
// walks the previous tree on the row's 32 bin bytes (two 16-byte loads; the walk selects bytes in
// registers), updates the row's margin and writes its quantised (g, h) to gh (the deeper levels)
// and to LDS; phase B adds the same rows into the LANE histogram (8 lanes per row, the bins
// re-read from L2).  The separate margin kernel's pass over the table (140 us per tree at the bench
// shape) disappears; the decisions, margins and (g, h) are bitwise those of gbdt_margin_kernel<true>.
// Hole rows (a CV fold's validation block) get phase A only, after the histogram.
constexpr int kFuseStep = kHistThreads;
// byte f of a 32-byte bin row held as two 16-byte words (a 3-level select: no array, no stack)
__device__ __forceinline__ int row_byte(const uint4& a, const uint4& b, int f) {
  const int q = f >> 2;
  const uint32_t lo = (q & 2) ? ((q & 1) ? a.w : a.z) : ((q & 1) ? a.y : a.x);
  const uint32_t hi = (q & 2) ? ((q & 1) ? b.w : b.z) : ((q & 1) ? b.y : b.x);
  return (int)((((q & 4) ? hi : lo) >> (8 * (f & 3))) & 0xffu);
}
// Phase A of one row: the previous tree's leaf by a walk on the row's bins, the margin update, the
// row's packed quantised (g, h) -- gbdt_margin_kernel<true>'s arithmetic on the same bytes.
__device__ __forceinline__ uint32_t fused_margin_row(const uint8_t* __restrict__ bins, int64_t row, int depth,
                                                     const int* sf, const int* sbn, const float* sl, int ni,
                                                     float* __restrict__ margin, const uint8_t* __restrict__ label,
                                                     float spw, float gscale, float hscale) {
  const uint4* br = reinterpret_cast<const uint4*>(bins + row * kGBRowBytes);
  const uint4 a = br[0], b = br[1];
  int node = 0;
  for (int l = 0; l < depth; ++l) {
    const int f = sf[node];
    node = 2 * node + 1 + (int)(f >= 0 && row_byte(a, b, f) > sbn[node]);
  }
  const float m = margin[row] + sl[node - ni];
  margin[row] = m;
  return pack_gh(quantised_grad(m, label[row] != 0, spw, gscale, hscale));
}
__global__ __launch_bounds__(kHistThreads, 8) void gbdt_hist_l0_fused_kernel(
    const uint8_t* __restrict__ bins, uint32_t* __restrict__ gh, const int64_t* __restrict__ seg,
    const int64_t* __restrict__ gcnt, int d, long long* __restrict__ slots, int64_t flush_rows, int64_t hole_at,
    int64_t hole_len, const int* __restrict__ feat, const int* __restrict__ bin, const float* __restrict__ leaf,
    int depth, float* __restrict__ margin, const uint8_t* __restrict__ label, float spw, float gscale,
    float hscale) {
  __shared__ unsigned long long sh[kHistWordsLane];
  __shared__ LevelNodes lv;
  __shared__ int sf[kGBMaxNodes], sbn[kGBMaxNodes];
  __shared__ float sl[kGBMaxNodes + 1];
  __shared__ uint32_t ghs[kFuseStep];
  __shared__ int rws[kFuseStep];
  const int ni = heap_first(depth);
  for (int i = threadIdx.x; i < ni; i += blockDim.x) {
    sf[i] = feat[i];
    sbn[i] = bin[i];
  }
  for (int i = threadIdx.x; i <= ni; i += blockDim.x) sl[i] = leaf[i];
  load_level(lv, seg, gcnt, 0);  // its barrier also covers the tree tables
  int64_t total;
  const int64_t chunk = level_chunk(lv, 0, gridDim.x, &total);
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(lo + chunk, total);
  const int64_t sb = seg[0];  // the root's first position
  long long* dst = slots + (int64_t)blockIdx.x * kHistEntries;  // level 0: block b owns slot b
  const int lane = lane_id();
  const int j = lane & 7, r4 = (lane >> 3) & 3;
  const uint32_t sel = (uint32_t)(0 ^ r4) | ((uint32_t)(1 ^ r4) << 8) | ((uint32_t)(2 ^ r4) << 16) |
                       ((uint32_t)(3 ^ r4) << 24);
  unsigned long long* const hk0 = sh + j + 8 * (0 ^ r4);
  unsigned long long* const hk1 = sh + j + 8 * (1 ^ r4);
  unsigned long long* const hk2 = sh + j + 8 * (2 ^ r4);
  unsigned long long* const hk3 = sh + j + 8 * (3 ^ r4);
  for (int64_t c0 = lo; c0 < hi; c0 += flush_rows) {
    const int64_t c1 = min(hi, c0 + flush_rows);
    for (int i = threadIdx.x; i < kHistWordsLane; i += kHistThreads) sh[i] = 0ull;
    for (int64_t s0 = c0; s0 < c1; s0 += kFuseStep) {  // block-uniform
      {  // phase A
        const int64_t v = s0 + threadIdx.x;
        uint32_t g = 0u;
        int row = 0;
        if (v < c1) {
          row = (int)hole_row(sb + v, hole_at, hole_len);
          g = fused_margin_row(bins, row, depth, sf, sbn, sl, ni, margin, label, spw, gscale, hscale);
          gh[row] = g;
        }
        ghs[threadIdx.x] = g;  // rows past the range add 0 in phase B
        rws[threadIdx.x] = row;
      }
      __syncthreads();  // also orders the zeroing above before the first atomic
      // phase B: 8 passes of 128 rows, kHistBatchLane passes' loads in flight at once
#pragma unroll
      for (int p0 = 0; p0 < kHistThreads / kHistBatchLane / 128 * kHistBatchLane; p0 += kHistBatchLane) {
        uint32_t bw[kHistBatchLane], gw[kHistBatchLane];
#pragma unroll
        for (int u = 0; u < kHistBatchLane; ++u) {
          const int i = (p0 + u) * 128 + (threadIdx.x >> 3);
          gw[u] = ghs[i];
          bw[u] = reinterpret_cast<const uint32_t*>(bins + (int64_t)rws[i] * kGBRowBytes)[j];
        }
#pragma unroll
        for (int u = 0; u < kHistBatchLane; ++u) {
          const uint32_t g = gw[u];
          const unsigned long long pk =
              ((unsigned long long)(g >> 16) << 32) + (unsigned long long)(long long)(int16_t)(g & 0xffffu);
          const uint32_t b = __builtin_amdgcn_perm(bw[u], bw[u], sel);
          atomicAdd(hk0 + (b & 0xffu) * 32, pk);
          atomicAdd(hk1 + ((b >> 8) & 0xffu) * 32, pk);
          atomicAdd(hk2 + ((b >> 16) & 0xffu) * 32, pk);
          atomicAdd(hk3 + (b >> 24) * 32, pk);
        }
      }
      __syncthreads();  // ghs / rws reused by the next step
    }
    const bool first = c0 == lo;
    for (int i = threadIdx.x; i < d * kGBBins; i += kHistThreads) {
      const int f = i >> 8, b = i & 255;
      const unsigned long long x = sh[b * 32 + 8 * (f & 3) + (f >> 2)];
      const long long sg = (long long)(int32_t)(uint32_t)(x & 0xffffffffull);
      const long long sgh = (long long)(x - (unsigned long long)sg) >> 32;
      long long* e = dst + 2 * i;
      if (first) {
        e[0] = sg;
        e[1] = sgh;
      } else {
        e[0] += sg;
        e[1] += sgh;
      }
    }
    __syncthreads();
  }
  // the hole rows: margins (and (g, h), unused) only
  for (int64_t r = hole_at + (int64_t)blockIdx.x * kHistThreads + threadIdx.x; r < hole_at + hole_len;
       r += (int64_t)gridDim.x * kHistThreads)
    gh[r] = fused_margin_row(bins, r, depth, sf, sbn, sl, ni, margin, label, spw, gscale, hscale);
}

// Sum each built node's slots into its histogram: grid (entries / 256, kSlotSplit, sibling pairs).
__global__ __launch_bounds__(256) void gbdt_hist_reduce_kernel(const long long* __restrict__ slots,
                                                               const int64_t* __restrict__ seg,
                                                               const int64_t* __restrict__ gcnt, int level,
                                                               int d, int hist_blocks,
                                                               unsigned long long* __restrict__ hist) {
  const int h0 = heap_first(level);
  __shared__ LevelNodes lv;
  load_level(lv, seg, gcnt, level);
  int64_t total;
  const int64_t chunk = level_chunk(lv, level, hist_blocks, &total);
  if (total == 0) return;
  // blockIdx.z = sibling pair: exactly one node of each pair is histogrammed (level 0: the root)
  const int kk = level == 0 ? 0 : (built_l(lv, level, 2 * (int)blockIdx.z) ? 2 * (int)blockIdx.z : 2 * (int)blockIdx.z + 1);
  int64_t off = 0;
  int base = 0, cnt = 0;
  bool mine = false;
  for (int k = 0; k <= kk; ++k) {
    if (!built_l(lv, level, k)) continue;
    const int64_t sc = lv.sc[k];
    const int c = sc > 0 ? (int)((off + sc - 1) / chunk) - (int)(off / chunk) + 1 : 0;
    if (k == kk) {
      mine = true;
      cnt = c;
    } else {
      base += c;
    }
    off += sc;
  }
  // >= 32 slots per split: deep levels have many small nodes, whose few slots need no split (each
  // split costs one int64 device atomic per entry).  With >= 8 slots per split the level-4 reduce
  // ran 43.9 us, with >= 32 41.9 (profiles/r4_z, r4_aa) against 13 us at level 0 for the same
  // bytes: the rest is the 60 x 16 x 16 grid, every block staging the node table before it can
  // tell that it has no slots -- z now runs over sibling pairs, not nodes: 26.4 us (profiles/r4_ab).
  const int split = min(kSlotSplit, (cnt + 31) / 32);
  if (!mine || cnt == 0 || (int)blockIdx.y >= split) return;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= d * kGBBins * 2) return;
  long long acc = 0;
  // 8 slot loads in flight per lane (a load -> wait -> add chain per slot otherwise)
#pragma unroll 8
  for (int j = blockIdx.y; j < cnt; j += split) acc += slots[(int64_t)(base + j) * kHistEntries + e];
  if (acc) atomicAdd(hist + (int64_t)(h0 + kk) * kHistEntries + e, (unsigned long long)acc);
}

// ---- split search ----------------------------------------------------------------------------
struct SplitOut {
  int* feat;       // [heap]  -1: no split (pass-through)
  int* bin;        // [heap]
  float* thr;      // [heap]  cut value; rows with x < thr go left; +inf when not split
  double* gain;    // [heap]
  long long* cg;   // [heap]  node sums (int64 fixed point), written for the children
  long long* ch;
};

__global__ __launch_bounds__(kHistThreads) void gbdt_split_kernel(
    unsigned long long* __restrict__ hist, const int64_t* __restrict__ gcnt, int level, int d,
    const int* __restrict__ nbins, const float* __restrict__ cuts, double ginv, double hinv,
    double lambda, double min_child_weight, double gamma, int* __restrict__ tfeat,
    int* __restrict__ tbin, float* __restrict__ tthr, double* __restrict__ tgain,
    long long* __restrict__ ng, long long* __restrict__ nh) {
#pragma clang fp contract(off)
  const int node = heap_first(level) + blockIdx.x;
  const int lane = lane_id(), wv = wave_id();
  constexpr int kW = kHistThreads / kWave;
  long long* H = reinterpret_cast<long long*>(hist) + (int64_t)node * kHistEntries;
  // A node that was not histogrammed gets the exact sibling subtraction H = parent - built
  // sibling, computed by the wave that scans the feature (every feature has exactly one wave) and
  // stored for the children's subtraction -- no block-wide pass + barrier + re-read of H.
  const bool derived = !is_built(node, gcnt);
  const int parent = derived ? (node - 1) >> 1 : node, sib = derived ? ((node & 1) ? node + 1 : node - 1) : node;
  const long long* P = reinterpret_cast<long long*>(hist) + (int64_t)parent * kHistEntries;
  const long long* S = reinterpret_cast<long long*>(hist) + (int64_t)sib * kHistEntries;
  __shared__ double fgain[32];
  __shared__ int fbin[32];
  __shared__ long long fgl[32], fhl[32];
  __shared__ long long tot[2];
  for (int f = wv; f < d; f += kW) {
    const int e0 = f * kGBBins * 2 + lane * 8;  // this lane's 4 bins x (g, h)
    long long g[4], h[4];
    if (derived) {
      long long pv[8], sv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { pv[j] = P[e0 + j]; sv[j] = S[e0 + j]; }
#pragma unroll
      for (int j = 0; j < 8; ++j) H[e0 + j] = pv[j] - sv[j];
#pragma unroll
      for (int j = 0; j < 4; ++j) { g[j] = pv[2 * j] - sv[2 * j]; h[j] = pv[2 * j + 1] - sv[2 * j + 1]; }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[j] = H[e0 + 2 * j];
        h[j] = H[e0 + 2 * j + 1];
      }
    }
#pragma unroll
    for (int j = 1; j < 4; ++j) { g[j] += g[j - 1]; h[j] += h[j - 1]; }
    long long eg = g[3], eh = h[3];  // inclusive scan of lane totals
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long ug = __shfl_up(eg, o, kWave), uh = __shfl_up(eh, o, kWave);
      if (lane >= o) { eg += ug; eh += uh; }
    }
    const long long Gq = __shfl(eg, 63, kWave), Hq = __shfl(eh, 63, kWave);
    const long long pg = eg - g[3], ph = eh - h[3];  // exclusive prefix of this lane
    const double G = (double)Gq * ginv, Hs = (double)Hq * hinv;
    const double root = G * G / (Hs + lambda);
    const int nb = nbins[f];
    double best = -1.0e300;
    int bb = 0x7fffffff;
    long long bgl = 0, bhl = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = lane * 4 + j;
      const long long GLq = pg + g[j], HLq = ph + h[j];
      const double GL = (double)GLq * ginv, HL = (double)HLq * hinv;
      const double GR = (double)(Gq - GLq) * ginv, HR = (double)(Hq - HLq) * hinv;
      if (b < nb - 1 && HL >= min_child_weight && HR >= min_child_weight) {
        const double gain = (GL * GL / (HL + lambda) + GR * GR / (HR + lambda)) - root;
        if (gain > best) { best = gain; bb = b; bgl = GLq; bhl = HLq; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // argmax, ties -> lowest bin
      const double og = __shfl_xor(best, o, kWave);
      const int ob = __shfl_xor(bb, o, kWave);
      const long long ogl = __shfl_xor(bgl, o, kWave), ohl = __shfl_xor(bhl, o, kWave);
      if (og > best || (og == best && ob < bb)) { best = og; bb = ob; bgl = ogl; bhl = ohl; }
    }
    if (lane == 0) {
      fgain[f] = best;
      fbin[f] = bb;
      fgl[f] = bgl;
      fhl[f] = bhl;
      if (f == 0) { tot[0] = Gq; tot[1] = Hq; }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double best = -1.0e300;
    int bf = -1;
    for (int f = 0; f < d; ++f)  // ties -> lowest feature
      if (fgain[f] > best) { best = fgain[f]; bf = f; }
    const long long Gq = tot[0], Hq = tot[1];
    // xgboost: a split needs loss_chg > kRtEps (1e-6) and is pruned when loss_chg < gamma
    const bool split = bf >= 0 && best > 1e-6 && !(best < gamma);
    const int l = 2 * node + 1, r = 2 * node + 2;
    if (split) {
      tfeat[node] = bf;
      tbin[node] = fbin[bf];
      tthr[node] = cuts[bf * kGBBins + fbin[bf]];
      tgain[node] = best;
      ng[l] = fgl[bf]; nh[l] = fhl[bf];
      ng[r] = Gq - fgl[bf]; nh[r] = Hq - fhl[bf];
    } else {
      tfeat[node] = -1;
      tbin[node] = 255;
      tthr[node] = __builtin_inff();
      tgain[node] = 0.0;
      ng[l] = Gq; nh[l] = Hq;
      ng[r] = 0; nh[r] = 0;
    }
    if (node == 0) { ng[0] = Gq; nh[0] = Hq; }
  }
}

// ---- stable partition of every node segment --------------------------------------------------
__device__ __forceinline__ void part_range(int64_t n, int64_t* lo, int64_t* hi) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  *lo = min((int64_t)blockIdx.x * per, n);
  *hi = min(*lo + per, n);
}

// binsT: FEATURE-major u8 bins [d][ldt].  The partition reads one feature byte per row: from the
// row-major [n][32] layout every such byte costs a whole sector (~205 MB of traffic per level at
// 6.4M rows); a feature column is 1 B/row and stays L2 / Infinity Cache resident.
__device__ __forceinline__ bool goes_right(const uint8_t* binsT, int64_t ldt, int64_t row, int node,
                                           const int* feat, const int* bin) {
  const int f = feat[node];
  return f >= 0 && binsT[(int64_t)f * ldt + row] > bin[node];
}

// Row-major [n][32] -> feature-major [d][ldt] (ldt % 4 == 0): a 256-row tile through LDS, each
// thread writes 4 consecutive rows of one feature as one 32-bit word.  Once per fit.
__global__ __launch_bounds__(256) void gbdt_transpose_kernel(const uint8_t* __restrict__ bins, int64_t n, int d,
                                                             uint8_t* __restrict__ binsT, int64_t ldt) {
  __shared__ uint32_t tile[256][kGBRowBytes / 4 + 1];
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int t = threadIdx.x;
  {
    const int64_t r = r0 + t;
    const uint4* src = reinterpret_cast<const uint4*>(bins + r * kGBRowBytes);
    uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
    if (r < n) {
      a = src[0];
      b = src[1];
    }
    tile[t][0] = a.x; tile[t][1] = a.y; tile[t][2] = a.z; tile[t][3] = a.w;
    tile[t][4] = b.x; tile[t][5] = b.y; tile[t][6] = b.z; tile[t][7] = b.w;
  }
  __syncthreads();
  const int q = t & 63;  // rows 4q .. 4q+3 of the tile
  for (int f = t >> 6; f < d; f += 4) {
    uint32_t w = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) w |= ((tile[4 * q + i][f >> 2] >> (8 * (f & 3))) & 0xffu) << (8 * i);
    const int64_t r = r0 + 4 * q;
    if (r < ldt) *reinterpret_cast<uint32_t*>(binsT + (int64_t)f * ldt + r) = w;
  }
}

// 4 consecutive rows per thread per step with every load of the step issued before the first
// use (the one-row loop was a chain of dependent load latencies: ~45 us per level at 6.4M rows)
constexpr int kPartRows = 4;
constexpr int kPartMaxNodes = 64;  // nodes of one partitioned level (levels <= 5 for depth <= 7)

// Level partition = count + scatter, two launches.  The count pass writes the go-right flag of
// every row, its block's right count (counts[block]) and adds each node's right count into
// node_r[node] (one agent atomic per (block, node) present; node_r is zeroed by the round init).
// Rows are grouped by node, so the scatter derives every segment offset from node_r alone: the
// rights before a segment are the prefix of node_r over the earlier nodes of the level, and the
// block's base is the prefix of counts -- no scan launch and no per-node seg launch
// (exclusive_scan_small + gbdt_seg were 4.8 + 7.2 us plus two launch gaps per level,
// profiles/r4_o/gbdt_kernel_stats.csv).
__global__ __launch_bounds__(kPartThreads) void gbdt_part_count_kernel(
    const uint8_t* __restrict__ binsT, int64_t ldt, const int* __restrict__ ridx, const uint8_t* __restrict__ nid,
    int64_t n, const int* __restrict__ feat, const int* __restrict__ bin, int level,
    uint8_t* __restrict__ flag, int64_t* __restrict__ counts, int64_t* __restrict__ node_r, int64_t hole_at,
    int64_t hole_len) {
  __shared__ int lcnt[kPartMaxNodes];
  __shared__ int64_t red[kPartThreads / kWave];
  const int h0 = heap_first(level), nn = 1 << level;
  if (threadIdx.x < kPartMaxNodes) lcnt[threadIdx.x] = 0;
  __syncthreads();
  int64_t lo, hi;
  part_range(n, &lo, &hi);
  int64_t c = 0;
  // per-node right counts: segments are contiguous, so a thread's rows form a few runs of one node;
  // a run's count goes to LDS when the node changes, and the last runs once per wave at the end
  int cn = -1, cc = 0;
  // software pipeline over the thread's steps: the row indices / node ids of step i+1 and then
  // their split feature / bin are loaded while the bins gather of step i is in flight (the
  // unpipelined loop paid ridx -> feat -> binsT -> flag as three dependent round trips per step)
  const int64_t step = (int64_t)kPartRows * kPartThreads;
  int row[kPartRows], nd[kPartRows], f[kPartRows], bv[kPartRows];
  // level 0: every row is in the root in row order -- ridx / nid are not read (nor initialised)
  auto load_ids = [&](int64_t p, int* rw, int* ndv) {
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const bool ok = p + u < hi;
      rw[u] = !ok ? 0 : (level == 0 ? (int)hole_row(p + u, hole_at, hole_len) : ridx[p + u]);
      ndv[u] = (ok && level != 0) ? (int)nid[p + u] : h0;
    }
  };
  auto load_split = [&](const int* ndv, int* fv, int* bvv) {
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      fv[u] = feat[ndv[u]];
      bvv[u] = bin[ndv[u]];
    }
  };
  int64_t p0 = lo + (int64_t)kPartRows * threadIdx.x;
  if (p0 < hi) {
    load_ids(p0, row, nd);
    load_split(nd, f, bv);
  }
  for (; p0 < hi; p0 += step) {
    int rowN[kPartRows], ndN[kPartRows], fN[kPartRows], bvN[kPartRows];
    const bool more = p0 + step < hi;
    if (more) load_ids(p0 + step, rowN, ndN);
    uint8_t v[kPartRows];
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) v[u] = f[u] >= 0 ? binsT[(int64_t)f[u] * ldt + row[u]] : 0;
    if (more) load_split(ndN, fN, bvN);
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      if (p0 + u < hi) {
        const int r = f[u] >= 0 && (int)v[u] > bv[u];
        flag[p0 + u] = (uint8_t)r;
        c += r;
        if (nd[u] != cn) {
          if (cc != 0) atomicAdd(&lcnt[cn - h0], cc);
          cn = nd[u];
          cc = 0;
        }
        cc += r;
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < kPartRows; ++u) {
        row[u] = rowN[u];
        nd[u] = ndN[u];
        f[u] = fN[u];
        bv[u] = bvN[u];
      }
    }
  }
  {
    const unsigned long long has = __ballot(cn >= 0);
    if (has != 0ull) {  // wave-uniform
      const int lead = __builtin_amdgcn_readlane(cn, __builtin_ctzll(has));
      if (__ballot(cn >= 0 && cn != lead) == 0ull) {
        const int s = wave_sum(cc);
        if (lane_id() == 0 && s != 0) atomicAdd(&lcnt[lead - h0], s);
      } else if (cc != 0) {
        atomicAdd(&lcnt[cn - h0], cc);
      }
    }
  }
  c = wave_sum(c);
  if (lane_id() == 0) red[wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kPartThreads / kWave; ++w) t += red[w];
    counts[blockIdx.x] = t;
  }
  if ((int)threadIdx.x < nn && lcnt[threadIdx.x] != 0)
    __hip_atomic_fetch_add(node_r + h0 + threadIdx.x, (int64_t)lcnt[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Stable scatter of this block's range into the children's segments, kPartRows consecutive rows
// per thread per step (one block-wide exclusive prefix of the right-going counts per 1024 rows).
// Block 0 also writes the children's segments and (local) row counts for the next level.
__global__ __launch_bounds__(kPartThreads) void gbdt_part_scatter_kernel(
    const uint8_t* __restrict__ flag, const int64_t* __restrict__ counts, const int* __restrict__ ridx,
    const uint8_t* __restrict__ nid, int64_t n, int level, const int64_t* __restrict__ node_r,
    int64_t* __restrict__ seg, int* __restrict__ ridx_out, uint8_t* __restrict__ nid_out,
    int64_t* __restrict__ gcnt, int64_t hole_at, int64_t hole_len) {
  __shared__ int wave_cnt[kPartThreads / kWave];
  __shared__ int64_t s_red[kPartThreads / kWave];
  __shared__ int64_t s_sb[kPartMaxNodes], s_left[kPartMaxNodes], s_rb[kPartMaxNodes];
  const int lane = lane_id(), w = wave_id();
  const int h0 = heap_first(level), nn = 1 << level;
  {
    // this block's base: rights in the rows of the earlier blocks
    int64_t b = 0;
    for (int i = threadIdx.x; i < (int)blockIdx.x; i += kPartThreads) b += counts[i];
    b = wave_sum(b);
    if (lane == 0) s_red[w] = b;
    if (w == 0) {  // the level's node table: segment start, left-child size, rights before it
      const int64_t nr = lane < nn ? node_r[h0 + lane] : 0;
      int64_t incl = nr;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int64_t t = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += t;
      }
      if (lane < nn) {
        const int node = h0 + lane;
        const int64_t sb = seg[2 * node], sc = seg[2 * node + 1];
        s_sb[lane] = sb;
        s_left[lane] = sc - nr;
        s_rb[lane] = incl - nr;
        if (blockIdx.x == 0) {  // children of the next level (distinct heap slots from the parents)
          seg[2 * (2 * node + 1)] = sb;
          seg[2 * (2 * node + 1) + 1] = sc - nr;
          seg[2 * (2 * node + 2)] = sb + sc - nr;
          seg[2 * (2 * node + 2) + 1] = nr;
          if (gcnt != nullptr) {  // the children's (global, once all-reduced) row counts
            gcnt[2 * node + 1] = sc - nr;
            gcnt[2 * node + 2] = nr;
          }
        }
      }
    }
  }
  __syncthreads();
  int64_t base = 0;
#pragma unroll
  for (int i = 0; i < kPartThreads / kWave; ++i) base += s_red[i];
  int64_t lo, hi;
  part_range(n, &lo, &hi);
  // the next step's flags / row indices / node ids are loaded while this step is scanned and
  // scattered
  const int64_t step = (int64_t)kPartRows * kPartThreads;
  int rf[kPartRows], ri[kPartRows], nd[kPartRows];
  auto load_step = [&](int64_t p0, int* rfv, int* riv, int* ndv) {
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const bool ok = p0 + u < hi;
      rfv[u] = ok ? (int)flag[p0 + u] : 0;
      riv[u] = !ok ? 0 : (level == 0 ? (int)hole_row(p0 + u, hole_at, hole_len) : ridx[p0 + u]);  // level 0: in order
      ndv[u] = (ok && level != 0) ? (int)nid[p0 + u] : h0;
    }
  };
  if (lo < hi) load_step(lo + (int64_t)kPartRows * threadIdx.x, rf, ri, nd);
  for (int64_t s0 = lo; s0 < hi; s0 += step) {  // block-uniform trip count (barriers inside)
    const int64_t p0 = s0 + (int64_t)kPartRows * threadIdx.x;
    int rfN[kPartRows], riN[kPartRows], ndN[kPartRows];
    const bool more = s0 + step < hi;
    if (more) load_step(p0 + step, rfN, riN, ndN);
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) cnt += rf[u];
    int incl = cnt;  // inclusive wave scan of the per-thread counts (thread order = row order)
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int t = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += t;
    }
    if (lane == kWave - 1) wave_cnt[w] = incl;
    __syncthreads();
    int64_t R = base + (incl - cnt);  // global rights before row p0
    int64_t total = 0;
#pragma unroll
    for (int i = 0; i < kPartThreads / kWave; ++i) {
      if (i < w) R += wave_cnt[i];
      total += wave_cnt[i];
    }
#pragma unroll
    for (int u = 0; u < kPartRows; ++u) {
      const int64_t p = p0 + u;
      if (p < hi) {
        const int k = nd[u] - h0;
        const int64_t rin = R - s_rb[k];  // rights before p inside the segment
        int64_t dst;
        uint8_t child;
        if (rf[u]) { dst = s_sb[k] + s_left[k] + rin; child = (uint8_t)(2 * nd[u] + 2); }
        else { dst = p - rin; child = (uint8_t)(2 * nd[u] + 1); }
        ridx_out[dst] = ri[u];
        nid_out[dst] = child;
      }
      R += rf[u];
    }
    base += total;
    if (more) {
#pragma unroll
      for (int u = 0; u < kPartRows; ++u) {
        rf[u] = rfN[u];
        ri[u] = riN[u];
        nd[u] = ndN[u];
      }
    }
    __syncthreads();
  }
}

// ---- per-round state -------------------------------------------------------------------------
// One launch instead of five torch fills/copies at the start of every boosting round: zero the
// level histograms and per-node right counts, root segment [0, n) and its global count.  ridx /
// nid are not filled: level 0 (histogram and partition) takes row p = position p in the root,
// which saved the 80 MB iota / root fill at 16M rows (profiles/r4_z).
__global__ __launch_bounds__(256) void gbdt_round_init_kernel(unsigned long long* __restrict__ hist,
                                                              int64_t hist_words, int64_t* __restrict__ seg,
                                                              int64_t* __restrict__ gcnt, int64_t n,
                                                              int64_t n_global,
                                                              int64_t* __restrict__ node_r, int n_nodes) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < hist_words; i += stride) hist[i] = 0ull;
  if (i0 < n_nodes) node_r[i0] = 0;
  if (i0 == 0) {
    seg[0] = 0;
    seg[1] = n;
    gcnt[0] = n_global;
  }
}

// ---- leaves ----------------------------------------------------------------------------------
// xgboost CalcWeight: 0 if H < min_child_weight or H <= 0, else -G / (H + lambda); the stored
// leaf value is eta * weight.
__global__ void gbdt_leaf_kernel(const long long* __restrict__ ng, const long long* __restrict__ nh,
                                 int depth, double ginv, double hinv, double lambda,
                                 double min_child_weight, double eta, float* __restrict__ leaf) {
#pragma clang fp contract(off)
  const int nl = 1 << depth;
  for (int i = threadIdx.x; i < nl; i += blockDim.x) {
    const int node = heap_first(depth) + i;
    const double G = (double)ng[node] * ginv, H = (double)nh[node] * hinv;
    double w = 0.0;
    if (!(H < min_child_weight || H <= 0.0)) w = -G / (H + lambda);
    leaf[i] = (float)(eta * w);
  }
}

// margin += leaf of the new tree, in row order, plus (GRAD) the next round's quantised gradients
// from the updated margin.  Each row re-walks the tree through the feature-major bins with the
// partition's own goes_right, so it reaches the leaf the partition would have put it in, and
// the last level needs no partition at all (ops/gbdt.py).  The earlier update went through the
// partition order (margin[ridx[p]] += leaf[nid[p]]: a random 4-B read-modify-write per row) after
// a last-level partition, and a separate gradient pass re-read every margin: 50-78 + ~65 + 20 us
// per round at 6.4M rows against 61 us for this walk (profiles/r2_s4b).  The walk is bound by
// the bins' line traffic -- the rows of a wave read up to 2^l feature columns at level l, ~200 MB
// over a depth-5 walk -- so walking 4 rows per thread in lockstep measured slower (68-71 us).
template <bool GRAD>
__global__ __launch_bounds__(256) void gbdt_margin_kernel(const uint8_t* __restrict__ binsT, int64_t ldt,
                                                          int64_t n, const int* __restrict__ feat,
                                                          const int* __restrict__ bin,
                                                          const float* __restrict__ leaf, int depth,
                                                          float* __restrict__ margin,
                                                          const uint8_t* __restrict__ label, float spw,
                                                          float gscale, float hscale, uint32_t* __restrict__ gh) {
  __shared__ int sf[kGBMaxNodes], sb[kGBMaxNodes];
  __shared__ float sl[kGBMaxNodes + 1];
  const int ni = heap_first(depth);
  for (int i = threadIdx.x; i < ni; i += blockDim.x) {
    sf[i] = feat[i];
    sb[i] = bin[i];
  }
  for (int i = threadIdx.x; i <= ni; i += blockDim.x) sl[i] = leaf[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
    int node = 0;
    for (int l = 0; l < depth; ++l) node = 2 * node + 1 + (int)goes_right(binsT, ldt, r, node, sf, sb);
    const float m = margin[r] + sl[node - ni];
    margin[r] = m;
    if constexpr (GRAD) gh[r] = pack_gh(quantised_grad(m, label[r] != 0, spw, gscale, hscale));
  }
}

// ---- inference on fp32 rows ------------------------------------------------------------------
// One thread per row; the row sits in LDS (dynamic feature index without scratch), the trees of
// the current chunk in LDS; every row walks exactly `depth` levels per tree.
constexpr int kPredThreads = 256;
constexpr int kPredLdsFloats = 12288;  // 48 KiB of trees per chunk

__global__ __launch_bounds__(kPredThreads) void gbdt_predict_kernel(
    const float* __restrict__ X, int64_t n, int ld, int d, const int* __restrict__ feat,
    const float* __restrict__ thr, const float* __restrict__ leaf, int ntrees, int depth,
    float base_margin, float* __restrict__ out) {
  __shared__ float xr[kPredThreads][kGBMaxFeat + 1];
  __shared__ float tl[kPredLdsFloats];
  const int ni = (1 << depth) - 1, nl = 1 << depth;
  const int per_tree = 2 * ni + nl;
  const int chunk = kPredLdsFloats / per_tree;
  const int64_t r = (int64_t)blockIdx.x * kPredThreads + threadIdx.x;
  const bool ok = r < n;
  for (int j = 0; j < d; ++j) xr[threadIdx.x][j] = ok ? X[r * ld + j] : 0.0f;
  float acc = base_margin;
  for (int t0 = 0; t0 < ntrees; t0 += chunk) {
    const int nt = min(chunk, ntrees - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt * ni; i += kPredThreads) {
      const int t = i / ni, k = i % ni;
      tl[t * per_tree + k] = __int_as_float(feat[(int64_t)(t0 + t) * ni + k]);
      tl[t * per_tree + ni + k] = thr[(int64_t)(t0 + t) * ni + k];
    }
    for (int i = threadIdx.x; i < nt * nl; i += kPredThreads) {
      const int t = i / nl, k = i % nl;
      tl[t * per_tree + 2 * ni + k] = leaf[(int64_t)(t0 + t) * nl + k];
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const float* T = tl + t * per_tree;
      int node = 0;
      for (int l = 0; l < depth; ++l) {
        const int f = __float_as_int(T[node]);
        const bool right = f >= 0 && !(xr[threadIdx.x][f] < T[ni + node]);
        node = 2 * node + 1 + (right ? 1 : 0);
      }
      acc += T[2 * ni + node - ni];
    }
  }
  if (ok) out[r] = acc;
}

}  // namespace

void launch_gbdt_bin(const float* X, int64_t n, int ld, int d, const float* cuts, const int* nbins,
                     uint8_t* bins, hipStream_t stream) {
  if (d > kGBMaxFeat) throw std::runtime_error("gbdt: at most 30 features");
  const bool vec = (ld % 4) == 0 && (reinterpret_cast<uintptr_t>(X) % 16) == 0 && d <= 32;
  if (vec) {
    static const int cap = resident_cap(gbdt_bin_kernel<true>, 256);
    gbdt_bin_kernel<true><<<capped_grid(n, 256 / 8, cap), 256, 0, stream>>>(X, n, ld, d, cuts, nbins, bins);
  } else {
    static const int cap = resident_cap(gbdt_bin_kernel<false>, 256);
    gbdt_bin_kernel<false><<<capped_grid(n, 256 / 8, cap), 256, 0, stream>>>(X, n, ld, d, cuts, nbins, bins);
  }
  check_launch("gbdt_bin");
}

void launch_gbdt_grad(const float* margin, const uint8_t* label, int64_t n, float spw, float gscale,
                      float hscale, uint32_t* gh, hipStream_t stream) {
  const int grid = stream_grid(n, 256, 4096);
  gbdt_grad_kernel<<<grid, 256, 0, stream>>>(margin, label, n, spw, gscale, hscale, gh);
  check_launch("gbdt_grad");
}

int gbdt_hist_blocks() {
  static int cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  }
  cached = 2 * cus;  // 60 KiB of LDS per block: two resident blocks per CU
  return cached;
}

int64_t gbdt_hist_slot_words() { return (int64_t)(gbdt_hist_blocks() + 2 * kGBMaxNodes) * kHistEntries; }

static int g_hist_variant = -1;  // set_gbdt_hist_variant (tests / labs); -1: the environment's choice
void set_gbdt_hist_variant(int v) {
  if (v < -1 || v > 3) throw std::invalid_argument("gbdt hist variant: -1 (env), 0 lockstep, 1 rot, 2 split, 3 lane");
  g_hist_variant = v;
}

void launch_gbdt_hist(const uint8_t* bins, const uint32_t* gh, const int* ridx, const int64_t* seg,
                      const int64_t* gcnt, int level, int d, unsigned long long* hist, long long* slots,
                      hipStream_t stream, int64_t flush_rows, int64_t hole_at, int64_t hole_len) {
  if (hole_at < 0 || hole_len < 0) throw std::runtime_error("gbdt_hist: bad row hole");
  // flush_rows <= kFlushRows (the packed-word exactness bound); smaller values only for tests of
  // the multi-flush path
  if (flush_rows <= 0 || flush_rows > kFlushRows) flush_rows = kFlushRows;
  // slots: gbdt_hist_slot_words() int64 (one [feature][bin][g, h] slot per (node, block) pair:
  // at most blocks + nodes pairs)
  if (level < 0 || (1 << level) > kGBMaxNodes + 1) throw std::runtime_error("gbdt_hist: level out of range");
  const int nb = gbdt_hist_blocks();
  static const int env_var = [] {  // lab switch FDX_GBDT_HIST_VAR: 0 lockstep, 1 rotated, 2 split, 3 lane (default)
    const char* e = std::getenv("FDX_GBDT_HIST_VAR");
    const char* r = std::getenv("FDX_GBDT_HIST_ROT");  // older spelling of variant 1
    if (e != nullptr && e[0] >= '0' && e[0] <= '3') return e[0] - '0';
    return (r != nullptr && r[0] == '1') ? 1 : (int)kHistLane;
  }();
  const int var = g_hist_variant >= 0 ? g_hist_variant : env_var;
  const bool rot = var == kHistRot;
  if (rot)  // one block per CU (its rotation registers): half the blocks of the lockstep form
    gbdt_hist_kernel<kHistRot><<<nb / 2, kHistThreads, 0, stream>>>(bins, gh, ridx, seg, gcnt, level, d, slots,
                                                                    flush_rows, hole_at, hole_len);
  else if (var == kHistLane && level == 0)
    gbdt_hist_kernel<kHistLane, true><<<nb, kHistThreads, 0, stream>>>(bins, gh, ridx, seg, gcnt, level, d, slots,
                                                                       flush_rows, hole_at, hole_len);
  else if (var == kHistLane)
    gbdt_hist_kernel<kHistLane><<<nb, kHistThreads, 0, stream>>>(bins, gh, ridx, seg, gcnt, level, d, slots,
                                                                 flush_rows, hole_at, hole_len);
  else if (var == kHistSplit)
    gbdt_hist_kernel<kHistSplit><<<nb, kHistThreads, 0, stream>>>(bins, gh, ridx, seg, gcnt, level, d, slots,
                                                                  flush_rows, hole_at, hole_len);
  else
    gbdt_hist_kernel<kHistLockstep><<<nb, kHistThreads, 0, stream>>>(bins, gh, ridx, seg, gcnt, level, d, slots,
                                                                     flush_rows, hole_at, hole_len);
  check_launch("gbdt_hist");
  const dim3 rg((unsigned)((d * kGBBins * 2 + 255) / 256), kSlotSplit, level == 0 ? 1u : 1u << (level - 1));
  gbdt_hist_reduce_kernel<<<rg, 256, 0, stream>>>(slots, seg, gcnt, level, d, rot ? nb / 2 : nb, hist);
  check_launch("gbdt_hist_reduce");
}

void launch_gbdt_hist_l0_fused(const uint8_t* bins, uint32_t* gh, const int64_t* seg, const int64_t* gcnt, int d,
                               unsigned long long* hist, long long* slots, hipStream_t stream, int64_t flush_rows,
                               int64_t hole_at, int64_t hole_len, const int* feat, const int* bin, const float* leaf,
                               int depth, float* margin, const uint8_t* label, float spw, float gscale, float hscale) {
  if (hole_at < 0 || hole_len < 0) throw std::runtime_error("gbdt_hist_l0_fused: bad row hole");
  if (depth < 1 || depth > 7) throw std::runtime_error("gbdt_hist_l0_fused: depth must be in [1, 7]");
  if (d < 1 || d > kGBMaxFeat) throw std::runtime_error("gbdt_hist_l0_fused: bad feature count");
  if (flush_rows <= 0 || flush_rows > kFlushRows) flush_rows = kFlushRows;
  const int nb = gbdt_hist_blocks();
  gbdt_hist_l0_fused_kernel<<<nb, kHistThreads, 0, stream>>>(bins, gh, seg, gcnt, d, slots, flush_rows, hole_at,
                                                             hole_len, feat, bin, leaf, depth, margin, label, spw,
                                                             gscale, hscale);
  check_launch("gbdt_hist_l0_fused");
  const dim3 rg((unsigned)((d * kGBBins * 2 + 255) / 256), kSlotSplit, 1u);
  gbdt_hist_reduce_kernel<<<rg, 256, 0, stream>>>(slots, seg, gcnt, 0, d, nb, hist);
  check_launch("gbdt_hist_reduce");
}

void launch_gbdt_split(unsigned long long* hist, const int64_t* gcnt, int level, int d, const int* nbins,
                       const float* cuts, double ginv, double hinv, double lambda,
                       double min_child_weight, double gamma, int* feat, int* bin, float* thr,
                       double* gain, long long* ng, long long* nh, hipStream_t stream) {
  gbdt_split_kernel<<<1 << level, kHistThreads, 0, stream>>>(hist, gcnt, level, d, nbins, cuts, ginv, hinv,
                                                             lambda, min_child_weight, gamma, feat, bin,
                                                             thr, gain, ng, nh);
  check_launch("gbdt_split");
}

void launch_gbdt_transpose(const uint8_t* bins, int64_t n, int d, uint8_t* binsT, int64_t ldt, hipStream_t stream) {
  if (ldt < n || ldt % 4 != 0) throw std::runtime_error("gbdt_transpose: ldt must be >= n and a multiple of 4");
  if (n <= 0) return;
  gbdt_transpose_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(bins, n, d, binsT, ldt);
  check_launch("gbdt_transpose");
}

void launch_gbdt_partition(const uint8_t* binsT, int64_t ldt, const int* ridx, const uint8_t* nid, int64_t n,
                           const int* feat, const int* bin, int level, uint8_t* flag, int64_t* counts,
                           int nblocks, int64_t* seg, int64_t* node_r, int* ridx_out, uint8_t* nid_out,
                           hipStream_t stream, int64_t* gcnt, int64_t hole_at, int64_t hole_len) {
  if (nblocks > 4096 || nblocks < 1) throw std::runtime_error("gbdt: 1..4096 partition blocks");
  if (hole_at < 0 || hole_len < 0) throw std::runtime_error("gbdt_partition: bad row hole");
  if (level < 0 || (1 << level) > kPartMaxNodes) throw std::runtime_error("gbdt: partition level out of range");
  gbdt_part_count_kernel<<<nblocks, kPartThreads, 0, stream>>>(binsT, ldt, ridx, nid, n, feat, bin, level, flag,
                                                               counts, node_r, hole_at, hole_len);
  check_launch("gbdt_part_count");
  gbdt_part_scatter_kernel<<<nblocks, kPartThreads, 0, stream>>>(flag, counts, ridx, nid, n, level, node_r, seg,
                                                                 ridx_out, nid_out, gcnt, hole_at, hole_len);
  check_launch("gbdt_part_scatter");
}

void launch_gbdt_round_init(unsigned long long* hist, int64_t hist_words, int64_t* seg, int64_t* gcnt, int64_t n,
                            int64_t n_global, hipStream_t stream, int64_t* node_r, int n_nodes) {
  if (n_nodes > 256) throw std::runtime_error("gbdt_round_init: at most 256 nodes");
  gbdt_round_init_kernel<<<device_cu_count() * 4, 256, 0, stream>>>(hist, hist_words, seg, gcnt, n, n_global, node_r,
                                                                    n_nodes);
  check_launch("gbdt_round_init");
}

void launch_gbdt_leaf(const long long* ng, const long long* nh, int depth, double ginv, double hinv,
                      double lambda, double min_child_weight, double eta, float* leaf, hipStream_t stream) {
  gbdt_leaf_kernel<<<1, 256, 0, stream>>>(ng, nh, depth, ginv, hinv, lambda, min_child_weight, eta, leaf);
  check_launch("gbdt_leaf");
}

void launch_gbdt_margin(const uint8_t* binsT, int64_t ldt, int64_t n, const int* feat, const int* bin,
                        const float* leaf, int depth, float* margin, const uint8_t* label, float spw, float gscale,
                        float hscale, uint32_t* gh, hipStream_t stream) {
  if (depth < 1 || depth > 7) throw std::runtime_error("gbdt_margin: depth must be in [1, 7]");
  const int grid = stream_grid(n, 256, 4096);
  if (gh)
    gbdt_margin_kernel<true><<<grid, 256, 0, stream>>>(binsT, ldt, n, feat, bin, leaf, depth, margin, label, spw,
                                                       gscale, hscale, gh);
  else
    gbdt_margin_kernel<false><<<grid, 256, 0, stream>>>(binsT, ldt, n, feat, bin, leaf, depth, margin, label,
                                                        spw, gscale, hscale, gh);
  check_launch("gbdt_margin");
}

void launch_gbdt_predict(const float* X, int64_t n, int ld, int d, const int* feat, const float* thr,
                         const float* leaf, int ntrees, int depth, float base_margin, float* out,
                         hipStream_t stream) {
  if (depth < 1 || depth > 8) throw std::runtime_error("gbdt: depth must be in [1, 8]");
  if (d > kGBMaxFeat) throw std::runtime_error("gbdt: at most 30 features");
  const int64_t grid = (n + kPredThreads - 1) / kPredThreads;
  if (grid == 0) return;
  gbdt_predict_kernel<<<(unsigned)grid, kPredThreads, 0, stream>>>(X, n, ld, d, feat, thr, leaf, ntrees, depth,
                                                                   base_margin, out);
  check_launch("gbdt_predict");
}

}  // namespace fdx
