// K9 smote_generate: synthetic minority rows x_new = x_i + lambda (x_nn - x_i).
//
// Reference behaviour being replaced: imblearn SMOTE._generate_samples (random row i among the
// minority rows, random neighbour among its k nearest, lambda ~ U[0,1) -- here on a 2^-16 grid, so
// a draw packs into 8 bytes: common.h smote_draw) used at
// train_model.py:65-66,91-92 and preprocess.py:43-44.  imblearn draws
// from numpy MT19937; here draws are counter-based Philox4x32-10 with one call per PAIR of
// samples (in 128-sample block m, counter (64 m + L, counter_base) serves samples 128 m + L and
// 128 m + 64 + L; common.h smote_pack_draw), so the output is independent of launch geometry and
// the CPU oracle (ops/reference.py smote_plan) reproduces it bit for bit before the bf16
// rounding.  ``sample_offset`` (a multiple of 128) places this launch's samples at global sample
// indices [sample_offset, sample_offset + n_new): data-parallel ranks each generate a 128-aligned
// slice of ONE global draw sequence, so the union equals the single-process output exactly.
// Row indices are packed in 24 bits: the host refuses parent sets >= 2^24 rows
// (ops/reference.py smote_check_ranges).
//
// MI355X mapping: write-bound stream.  4 lanes per synthetic row, 8 columns (two 16 B gathers of
// each parent row, L2-resident) per lane, one 16 B store per lane: 16 rows = 1 KiB per
// wave-instruction, written straight into the training buffer after the real rows (bf16 with
// col 30 = 1 and col 31 = label, or fp8).
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;

// OUT: 0 = bf16 rows (64 B), 1 = fp32 (GBDT input), 2 = fp8 e4m3 (32 B).
// PB: parents are bf16 rows already in output space (smote_parents_kernel: the affine map applied
// once per parent instead of once per sample; half the gather bytes); else fp32 rows (+ aff).
template <int OUT, bool NT = false, bool PB = false, bool G2 = false>
__global__ __launch_bounds__(kThreads) void smote_generate_kernel(
    const void* __restrict__ Cv, const int* __restrict__ nbr, int mq, int k, int64_t q_offset,
    int64_t n_new, int64_t s_off, uint32_t key0, uint32_t key1, uint32_t cb0, uint32_t cb1, float label,
    float out_scale, const double* __restrict__ aff, void* __restrict__ out) {
#pragma clang fp contract(off)  // affine map = mul then add (the oracle); the interpolation is an explicit fmaf
  const int lane = lane_id();
  const int q = lane & 3, rr = lane >> 2;
  // aff (optional): the parents are standardized rows z but the training buffer holds
  // pivot-shifted rows s = z * sigma + c (scaler folded into the solver); interpolation commutes
  // with the affine map, so it is applied to the output (mul then add, as the numpy oracle).
  const float* C = reinterpret_cast<const float*>(Cv);
  const uint4* Cb = reinterpret_cast<const uint4*>(Cv);
  float sig[8], cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool feat = !PB && aff != nullptr && 8 * q + j < kBiasCol;
    sig[j] = feat ? (float)(1.0 / aff[32 + 8 * q + j]) : 1.0f;
    cc[j] = feat ? (float)aff[8 * q + j] : 0.0f;
  }
  const uint32_t range = (uint32_t)mq * (uint32_t)k;
  const float inv_k = 1.0f / (float)k;
  const bool small = range < (1u << 22);
  const int64_t step = (int64_t)gridDim.x * (kThreads / kWave) * 128;
  // One Philox call per lane = two samples per lane (128 samples per wave-iteration, two halves
  // of 64 rows).  Software pipeline: the NEXT iteration's draws and neighbour-index loads are
  // issued behind this iteration's first row gathers, so the dependent nbr -> row chain costs one
  // memory latency per iteration instead of two.
  auto draw2 = [&](int64_t b, int (&di)[2], int (&dj)[2], float (&dl)[2]) {
    const int64_t c = ((s_off + b) >> 1) + lane;  // s_off and b are multiples of 128
    const Philox4 r = philox4x32_10((uint32_t)c, (uint32_t)(c >> 32), cb0, cb1, key0, key1);
    const uint32_t wp[2] = {r.x, r.z}, wl[2] = {r.y, r.w};
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint2 d = (b + 64 * hh + lane < n_new) ? smote_pack_draw(wp[hh], wl[hh], range, (uint32_t)k, inv_k, small, nbr)
                                                   : make_uint2(0, 0);
      di[hh] = (int)(d.x & 0xffffffu);
      dj[hh] = (int)(d.y & 0xffffffu);
      dl[hh] = smote_lambda(d.x, d.y);
    }
  };
  int64_t base = ((int64_t)blockIdx.x * (kThreads / kWave) + wave_id()) * 128;
  int my_i[2] = {0, 0}, my_j[2] = {0, 0};
  float my_lam[2] = {0.0f, 0.0f};
  if (base < n_new) draw2(base, my_i, my_j, my_lam);
  for (; base < n_new; base += step) {
    int nx_i[2] = {0, 0}, nx_j[2] = {0, 0};
    float nx_lam[2] = {0.0f, 0.0f};
    if constexpr (G2 && PB && OUT == 0) {
      // both halves' parent gathers issued up front (16 loads in flight per lane, kept packed:
      // 64 VGPRs), then the next draws, then interpolate + store: one exposed gather latency per
      // iteration instead of two.  Same arithmetic as below: bit-identical rows.
      uint4 pi[2][4], pj[2][4];
      float lam[2][4];
  #pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
  #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = 16 * u + rr;
          const int i = __shfl(my_i[hh], src, kWave);
          const int jn = __shfl(my_j[hh], src, kWave);
          lam[hh][u] = __shfl(my_lam[hh], src, kWave);
          pi[hh][u] = Cb[(q_offset + i) * 4 + q];
          pj[hh][u] = Cb[(int64_t)jn * 4 + q];
        }
      }
      if (base + step < n_new) draw2(base + step, nx_i, nx_j, nx_lam);
  #pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
  #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t s = base + 64 * hh + 16 * u + rr;
          if (s >= n_new) continue;
          const float l = lam[hh][u];
          const uint4 a = pi[hh][u], b = pj[hh][u];
          const float av[8] = {bf16lo(a.x), bf16hi(a.x), bf16lo(a.y), bf16hi(a.y),
                               bf16lo(a.z), bf16hi(a.z), bf16lo(a.w), bf16hi(a.w)};
          const float bv[8] = {bf16lo(b.x), bf16hi(b.x), bf16lo(b.y), bf16hi(b.y),
                               bf16lo(b.z), bf16hi(b.z), bf16lo(b.w), bf16hi(b.w)};
          float o[8];
  #pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = fmaf(l, bv[j] - av[j], av[j]);
          if (q == 3) {
            o[6] = 1.0f;   // col 30: intercept column
            o[7] = label;  // col 31: label
          }
          uint4 pk;
          pk.x = pack_bf16x2(o[0], o[1]);
          pk.y = pack_bf16x2(o[2], o[3]);
          pk.z = pack_bf16x2(o[4], o[5]);
          pk.w = pack_bf16x2(o[6], o[7]);
          if constexpr (NT) __builtin_nontemporal_store(u32x4_t{pk.x, pk.y, pk.z, pk.w}, reinterpret_cast<u32x4_t*>(out) + s * 4 + q);
          else reinterpret_cast<uint4*>(out)[s * 4 + q] = pk;
        }
      }
    } else {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int64_t hbase = base + 64 * hh;
      // 4 row groups of 16 samples: 4 lanes per sample, 8 columns per lane; gathers issued first
      float4 a0[4], a1[4], b0[4], b1[4];
      float lam[4];
  #pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int src = 16 * u + rr;
        const int i = __shfl(my_i[hh], src, kWave);
        const int jn = __shfl(my_j[hh], src, kWave);
        lam[u] = __shfl(my_lam[hh], src, kWave);
        if constexpr (PB) {
          const uint4 pi = Cb[(q_offset + i) * 4 + q], pj = Cb[(int64_t)jn * 4 + q];
          a0[u] = make_float4(bf16lo(pi.x), bf16hi(pi.x), bf16lo(pi.y), bf16hi(pi.y));
          a1[u] = make_float4(bf16lo(pi.z), bf16hi(pi.z), bf16lo(pi.w), bf16hi(pi.w));
          b0[u] = make_float4(bf16lo(pj.x), bf16hi(pj.x), bf16lo(pj.y), bf16hi(pj.y));
          b1[u] = make_float4(bf16lo(pj.z), bf16hi(pj.z), bf16lo(pj.w), bf16hi(pj.w));
        } else {
          const float4* xi = reinterpret_cast<const float4*>(C + (q_offset + i) * kCols + 8 * q);
          const float4* xj = reinterpret_cast<const float4*>(C + (int64_t)jn * kCols + 8 * q);
          a0[u] = xi[0]; a1[u] = xi[1]; b0[u] = xj[0]; b1[u] = xj[1];
        }
      }
      // next iteration's draws + neighbour-index loads, issued AFTER the first half's gathers:
      // vector loads return in issue order, so waiting for the gathers does not wait for them
      if (hh == 0 && base + step < n_new) draw2(base + step, nx_i, nx_j, nx_lam);
  #pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t s = hbase + 16 * u + rr;
        if (s >= n_new) continue;
        const float l = lam[u];
        float o[8] = {fmaf(l, b0[u].x - a0[u].x, a0[u].x), fmaf(l, b0[u].y - a0[u].y, a0[u].y),
                      fmaf(l, b0[u].z - a0[u].z, a0[u].z), fmaf(l, b0[u].w - a0[u].w, a0[u].w),
                      fmaf(l, b1[u].x - a1[u].x, a1[u].x), fmaf(l, b1[u].y - a1[u].y, a1[u].y),
                      fmaf(l, b1[u].z - a1[u].z, a1[u].z), fmaf(l, b1[u].w - a1[u].w, a1[u].w)};
        if (!PB && aff) {
  #pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = o[j] * sig[j] + cc[j];
        }
        if (q == 3) {
          o[6] = 1.0f;   // col 30: intercept column
          o[7] = label;  // col 31: label
        }
        if constexpr (OUT == 0) {
          uint4 pk;
          pk.x = pack_bf16x2(o[0], o[1]);
          pk.y = pack_bf16x2(o[2], o[3]);
          pk.z = pack_bf16x2(o[4], o[5]);
          pk.w = pack_bf16x2(o[6], o[7]);
          // NT: streaming store (nt policy) so the output stream does not evict the L2-resident
          // parent rows every gather reads
          if constexpr (NT) __builtin_nontemporal_store(u32x4_t{pk.x, pk.y, pk.z, pk.w}, reinterpret_cast<u32x4_t*>(out) + s * 4 + q);
          else reinterpret_cast<uint4*>(out)[s * 4 + q] = pk;
        } else if constexpr (OUT == 1) {
          float4* dst = reinterpret_cast<float4*>(out) + s * 8 + 2 * q;
          dst[0] = make_float4(o[0], o[1], o[2], o[3]);
          dst[1] = make_float4(o[4], o[5], o[6], o[7]);
        } else {
          float v8[8];
  #pragma unroll
          for (int jj = 0; jj < 8; ++jj) v8[jj] = (8 * q + jj) < kBiasCol ? o[jj] * out_scale : o[jj];
          // hardware e4m3 (v_cvt_pk_fp8_f32, RNE + satfinite): 4 instructions per 8 values
          // instead of the ~20-op software encoder per value (this kernel was VALU-bound on it)
          const uint2 pk = make_uint2(f32x4_to_fp8(v8[0], v8[1], v8[2], v8[3]),
                                      f32x4_to_fp8(v8[4], v8[5], v8[6], v8[7]));
          reinterpret_cast<uint2*>(out)[s * 4 + q] = pk;
        }
      }
    }
    }  // G2 else
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      my_i[hh] = nx_i[hh];
      my_j[hh] = nx_j[hh];
      my_lam[hh] = nx_lam[hh];
    }
  }
}

// Output-space parents: P = bf16(z * sigma + c) on the feature columns (the pivot-shifted layout of
// the training rows; identity without aff), columns 30/31 copied.  One thread per element.
__global__ __launch_bounds__(kThreads) void smote_parents_kernel(const float* __restrict__ C, int64_t m,
                                                                 const double* __restrict__ aff,
                                                                 uint16_t* __restrict__ P) {
#pragma clang fp contract(off)  // mul then add, two roundings (= the numpy oracle), never an fma
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= m * kCols) return;
  const int c = (int)(e & (kCols - 1));
  float v = C[e];
  if (aff != nullptr && c < kBiasCol) v = v * (float)(1.0 / aff[32 + c]) + (float)aff[c];
  P[e] = f32_to_bf16(v);
}

// Group this launch's samples by pick (virtual SMOTE rows, launchers.h SmoteView) with a
// two-level counting sort that keeps every global write coalesced.  Measured dead ends
// (profiles/r3_v*): one global atomic per sample (318 us to count + 714 us to fill 8M samples
// into 68k buckets: contended L2 atomics), and a bin-major level-1 scatter (83 us: 2128 bins x 256
// blocks of open partial lines thrash L2 into partial-line HBM writes).
// Draws: one Philox call per pair of samples exactly as smote_generate_kernel draws them (pair
// t = (m, L) of the launch's 128-sample block m serves samples 128 m + L with words (x, y) and
// 128 m + 64 + L with (z, w)); pick = u32_range(word_pick, mq k), lambda = word_lam >> 16.
//   level 1: coarse bin = pick >> fb (2^fb picks per bin, ~4k samples per bin).  Block blk
//            histograms its contiguous range of pairs into table[blk][bin] (block-major); after
//            an inclusive scan, the same block redraws, places 4-byte records
//            (pick & (2^fb - 1) | lambda << 16) sorted by bin in LDS and stores its whole range
//            coalesced (its records are one contiguous run, bins in order).
//   level 2: one block per coarse bin gathers its segment of every level-1 block into LDS,
//            counts its fine picks, takes room for the bin with one global bump-allocator atomic,
//            writes each pick's (start, count), assembles the lambdas in LDS and stores them
//            coalesced (a bin too big for the stage takes the same steps through global memory).
// Order inside a bucket follows LDS atomics; the pass sums a bucket in fixed point.
constexpr int kBucketThreads = 1024;
constexpr int kBucketPairs = 8192;    // pairs per level-1 block: <= 16384 records staged (64 KiB)
constexpr int kFineMax = 128;
constexpr int kStageRecs = 8192;      // level 2: 32 KiB of records + 16 KiB of lambdas
constexpr int kSegMax = 2048;         // level 2: segment table of <= 2048 level-1 blocks in LDS
// level 2 block size: 1024 threads (57-60 us at the bench shape) -- 256-thread blocks at 3 per CU
// measured 84 us (profiles/r3_virt/timeline_r3_v9.txt)
constexpr int kL2Threads = 1024;
constexpr int kL2Waves = kL2Threads / 64;


// Samples of one global draw sequence before level-1 block b: every block covers kBucketPairs
// whole Philox pairs (128-sample blocks of the sequence), so the count is closed-form -- the
// record array needs no global scan to place a block's run.
__device__ __forceinline__ int64_t l1_block_base(int64_t b, int64_t n_new) {
  const int64_t s = b * 2 * (int64_t)kBucketPairs;
  return s < n_new ? s : n_new;
}

template <bool SCATTER>
__global__ __launch_bounds__(kBucketThreads) void smote_bucket_l1_kernel(uint32_t range, int fb, int nbins, int64_t n_new,
                                                                         int64_t blk0, uint32_t key0, uint32_t key1,
                                                                         uint32_t cb0, uint32_t cb1,
                                                                         int* __restrict__ table,
                                                                         uint32_t* __restrict__ rec,
                                                                         unsigned long long* __restrict__ bump) {
  extern __shared__ int h[];  // [nbins] counts / cursors, then (SCATTER) [2 kBucketPairs] records
  __shared__ int wtot[kBucketThreads / kWave];
  uint32_t* srec = reinterpret_cast<uint32_t*>(h + nbins);
  const int64_t tb = (int64_t)blockIdx.x * nbins;
  if constexpr (SCATTER) {
    // this block's row of counts -> exclusive prefix in LDS (block-wide scan: each thread a run of
    // consecutive bins), written back over the counts for level 2 (the within-block start of
    // every bin; level 2 adds the block's closed-form base)
    const int per = (nbins + kBucketThreads - 1) / kBucketThreads;
    const int b0 = threadIdx.x * per, b1 = min(nbins, b0 + per);
    int run = 0;
    for (int b = b0; b < b1; ++b) run += table[tb + b];
    int inc = run;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int v = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += v;
    }
    if (lane == kWave - 1) wtot[wv] = inc;
    __syncthreads();
    int off = inc - run;
    for (int w = 0; w < wv; ++w) off += wtot[w];
    for (int b = b0; b < b1; ++b) {
      const int c = table[tb + b];
      h[b] = off;
      table[tb + b] = off;
      off += c;
    }
  } else {
    for (int b = threadIdx.x; b < nbins; b += kBucketThreads) h[b] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *bump = 0ull;  // level 2's allocator
  }
  __syncthreads();
  const int64_t npairs = ((n_new + 127) >> 7) << 6;
  const uint32_t fmask = (1u << fb) - 1u;
  const int64_t lo = min((int64_t)blockIdx.x * kBucketPairs, npairs), hi = min(lo + kBucketPairs, npairs);
  for (int64_t t = lo + threadIdx.x; t < hi; t += kBucketThreads) {
    const int64_t m = t >> 6, L = t & 63;
    const int64_t c = ((blk0 + m) << 6) + L;
    const Philox4 r = philox4x32_10((uint32_t)c, (uint32_t)(c >> 32), cb0, cb1, key0, key1);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if ((m << 7) + 64 * hh + L >= n_new) continue;
      const uint32_t pick = u32_range(hh ? r.z : r.x, range);
      if constexpr (SCATTER) {
        const int pos = atomicAdd(h + (pick >> fb), 1);
        srec[pos] = (pick & fmask) | (((hh ? r.w : r.y) >> 16) << 16);
      } else {
        atomicAdd(h + (pick >> fb), 1);
      }
    }
  }
  __syncthreads();
  if constexpr (SCATTER) {
    const int64_t base = l1_block_base(blockIdx.x, n_new);
    const int cnt = (int)(l1_block_base(blockIdx.x + 1, n_new) - base);
    for (int i = threadIdx.x; i < cnt; i += kBucketThreads) rec[base + i] = srec[i];
  } else {  // every entry written: the table needs no fill
    for (int b = threadIdx.x; b < nbins; b += kBucketThreads) table[tb + b] = h[b];
  }
}

__global__ __launch_bounds__(kL2Threads) void smote_bucket_l2_kernel(const int* __restrict__ pref, int nblk, int nbins,
                                                               uint32_t range, int fb, int64_t n_new,
                                                               const uint32_t* __restrict__ rec,
                                                               uint32_t* __restrict__ tmp, int* __restrict__ pstart,
                                                               int* __restrict__ pcnt, uint16_t* __restrict__ lam,
                                                               unsigned long long* __restrict__ bump) {
  __shared__ int cnt[kFineMax], cur[kFineMax];
  __shared__ int whist[kL2Waves][kFineMax];  // per-wave fine counts, then per-wave cursors (less
                                             // same-address LDS atomic contention)
  __shared__ int gbase, wsum[kL2Waves];
  __shared__ int sstart[kSegMax], spre[kSegMax + 1];
  __shared__ uint32_t srec[kStageRecs];
  __shared__ uint16_t slam[kStageRecs];
  const int bin = blockIdx.x, fine = 1 << fb;
  const uint32_t fmask = (uint32_t)fine - 1u;
  const int lane = lane_id(), wv = wave_id();
  for (int i = threadIdx.x; i < kL2Waves * kFineMax; i += blockDim.x) whist[i / kFineMax][i % kFineMax] = 0;
  // this bin's segment of every level-1 block (start, length), lengths scanned in LDS: then every
  // thread copies records in parallel (one thread per segment was a chain of dependent loads)
  constexpr int kPer = kSegMax / kL2Threads;
  int len[kPer], tot = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int b = threadIdx.x * kPer + u;
    int l = 0;
    if (b < nblk) {  // pref: level 1's within-block exclusive prefix of the bins
      const int64_t e = (int64_t)b * nbins + bin;
      const int64_t base = l1_block_base(b, n_new);
      const int p0 = pref[e];
      const int p1 = bin + 1 < nbins ? pref[e + 1] : (int)(l1_block_base(b + 1, n_new) - base);
      sstart[b] = (int)(base + p0);
      l = p1 - p0;
    }
    len[u] = l;
    tot += l;
  }
  int inc = tot;  // block-wide exclusive scan of the per-thread totals
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int v = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += v;
  }
  if (lane == kWave - 1) wsum[wv] = inc;
  __syncthreads();
  int before = 0, n = 0;
  for (int w = 0; w < kL2Waves; ++w) {
    if (w < wv) before += wsum[w];
    n += wsum[w];
  }
  int run = before + inc - tot;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int b = threadIdx.x * kPer + u;
    if (b < nblk) spre[b] = run;
    run += len[u];
  }
  if (threadIdx.x == 0) {
    spre[nblk] = n;
    gbase = n ? (int)atomicAdd(bump, (unsigned long long)n) : 0;  // the bin's room in lam
  }
  __syncthreads();
  const int g0 = gbase;
  const bool staged = n <= kStageRecs;
  uint32_t* R = staged ? srec : tmp + g0;  // unstaged: the bin's records gathered in global scratch
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int lo = 0, hi = nblk;  // the segment holding record i: spre[lo] <= i < spre[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (spre[mid] <= i) lo = mid;
      else hi = mid;
    }
    const uint32_t r = rec[sstart[lo] + (i - spre[lo])];
    R[i] = r;
    atomicAdd(&whist[wv][r & fmask], 1);  // fine count in the same pass (same record -> wave map
                                          // as the scatter below)
  }
  __syncthreads();
  if (threadIdx.x < fine) {
    int c = 0;
    for (int w = 0; w < kL2Waves; ++w) c += whist[w][threadIdx.x];
    cnt[threadIdx.x] = c;
  }
  __syncthreads();
  if (threadIdx.x < kWave) {  // exclusive scan of <= 128 fine counts by one wave (2 per lane)
    const int l = threadIdx.x;
    const int a = 2 * l < fine ? cnt[2 * l] : 0, b = 2 * l + 1 < fine ? cnt[2 * l + 1] : 0;
    int inc = a + b;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int v = __shfl_up(inc, o, kWave);
      if (l >= o) inc += v;
    }
    const int ex = inc - (a + b);
    if (2 * l < fine) cur[2 * l] = ex;
    if (2 * l + 1 < fine) cur[2 * l + 1] = ex + a;
  }
  __syncthreads();
  if (threadIdx.x < fine) {
    const uint32_t pick = ((uint32_t)bin << fb) + threadIdx.x;
    if (pick < range) {
      pstart[pick] = g0 + cur[threadIdx.x];
      pcnt[pick] = cnt[threadIdx.x];
    }
  }
  __syncthreads();
  if (threadIdx.x < fine) {  // wave w's records of pick f go to [cur[f] + sum_{w' < w} whist[w'][f], ...)
    int run = cur[threadIdx.x];
    for (int w = 0; w < kL2Waves; ++w) {
      const int c = whist[w][threadIdx.x];
      whist[w][threadIdx.x] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {  // same record -> wave mapping as the count
    const uint32_t r = R[i];
    const int pos = atomicAdd(&whist[wv][r & fmask], 1);
    if (staged) slam[pos] = (uint16_t)(r >> 16);
    else lam[g0 + pos] = (uint16_t)(r >> 16);
  }
  if (staged) {
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) lam[g0 + i] = slam[i];
  }
}

}  // namespace

// 2^fb picks per coarse bin: ~kTarget samples per bin for the level-2 stage, <= 16384 bins for
// the level-1 LDS histogram, <= kFineMax picks per bin.
int smote_bucket_fine_bits(int64_t range, int64_t n_new) {
  // ~4096 samples per level-2 bin: 2048 measured 117 vs 91 us for the whole sort at the bench
  // shape (tools/bucket_lab.py, profiles/r4_m/bucket*.log)
  constexpr double kTarget = 4096.0;
  int fb = 0;
  while (fb < 7 && ((range + (1ll << fb) - 1) >> fb) > 16384) ++fb;
  while (fb < 7 && (double)n_new * (double)(1ll << (fb + 1)) / (double)range <= kTarget) ++fb;
  return fb;
}
int smote_bucket_bins(int64_t range, int64_t n_new) {
  const int fb = smote_bucket_fine_bits(range, n_new);
  return (int)((range + (1ll << fb) - 1) >> fb);
}
int64_t smote_bucket_max_samples() { return (int64_t)kSegMax * 2 * kBucketPairs; }
int smote_bucket_blocks(int64_t n_new) {
  const int64_t npairs = ((n_new + 127) >> 7) << 6;
  return (int)std::max<int64_t>(1, (npairs + kBucketPairs - 1) / kBucketPairs);
}

void launch_smote_bucket(int stage, int mq, int k, int64_t n_new, int64_t sample_offset, uint64_t seed,
                         uint64_t counter_base, int* table, uint32_t* rec, uint32_t* tmp, int* pstart, int* pcnt,
                         uint16_t* lam, unsigned long long* bump, hipStream_t stream) {
  if (n_new <= 0) return;
  if (sample_offset < 0 || (sample_offset & 127) != 0)
    throw std::runtime_error("smote_bucket: sample_offset must be a non-negative multiple of 128");
  const uint64_t R = (uint64_t)mq * (uint64_t)k;
  if (mq <= 0 || k <= 0 || R > kSmoteBucketMaxPicks || n_new >= (1ll << 31))
    throw std::runtime_error("smote_bucket: pick range or sample count out of bounds");
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t c0 = (uint32_t)counter_base, c1 = (uint32_t)(counter_base >> 32);
  const int fb = smote_bucket_fine_bits((int64_t)R, n_new);
  const int nbins = smote_bucket_bins((int64_t)R, n_new);
  const int nblk = smote_bucket_blocks(n_new);
  if (nblk > kSegMax) throw std::runtime_error("smote_bucket: too many samples for the level-2 segment table");
  if (stage == 0) {
    smote_bucket_l1_kernel<false><<<nblk, kBucketThreads, (size_t)nbins * sizeof(int), stream>>>(
        (uint32_t)R, fb, nbins, n_new, sample_offset >> 7, k0, k1, c0, c1, table, rec, bump);
  } else if (stage == 1) {
    const size_t lds = (size_t)nbins * sizeof(int) + 2 * (size_t)kBucketPairs * sizeof(uint32_t);
    static bool attr = false;
    if (!attr) {  // > 64 KiB of dynamic LDS (gfx950: 160 KiB per workgroup)
      hipFuncSetAttribute((const void*)smote_bucket_l1_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)(16384 * sizeof(int) + 2 * (size_t)kBucketPairs * sizeof(uint32_t)));
      attr = true;
    }
    smote_bucket_l1_kernel<true><<<nblk, kBucketThreads, lds, stream>>>(
        (uint32_t)R, fb, nbins, n_new, sample_offset >> 7, k0, k1, c0, c1, table, rec, bump);
  } else {
    smote_bucket_l2_kernel<<<nbins, kL2Threads, 0, stream>>>(table, nblk, nbins, (uint32_t)R, fb, n_new, rec, tmp,
                                                             pstart, pcnt, lam, bump);
  }
  check_launch("smote_bucket");
}

void launch_smote_parents(const float* C, int64_t m, const double* aff, uint16_t* P, hipStream_t stream) {
  if (m <= 0) return;
  smote_parents_kernel<<<(int)((m * kCols + kThreads - 1) / kThreads), kThreads, 0, stream>>>(C, m, aff, P);
  check_launch("smote_parents");
}

void launch_smote_generate(const void* C, int parents_bf16, const int* nbr, int mq, int k, int64_t q_offset,
                           int64_t n_new, int64_t sample_offset, uint64_t seed, uint64_t counter_base, float label,
                           int out_kind, float out_scale, const double* aff, void* out, hipStream_t stream) {
  if (n_new <= 0) return;
  if (sample_offset < 0 || (sample_offset & 127) != 0)
    throw std::runtime_error("smote_generate: sample_offset must be a non-negative multiple of 128");
  const int64_t per_block = (kThreads / kWave) * 128;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t c0 = (uint32_t)counter_base, c1 = (uint32_t)(counter_base >> 32);
#define FDX_SG(O, NT, PB, ...)                                                                        \
  do {                                                                                                \
    static const int cap = resident_cap(smote_generate_kernel<O, NT, PB, ##__VA_ARGS__>, kThreads);   \
    smote_generate_kernel<O, NT, PB, ##__VA_ARGS__><<<capped_grid(n_new, per_block, cap), kThreads, 0, \
                                                      stream>>>(                                      \
        C, nbr, mq, k, q_offset, n_new, sample_offset, k0, k1, c0, c1, label, out_scale, aff, out);   \
  } while (0)
  const bool pb = parents_bf16 != 0;
  // bf16 parents: both halves' gathers up front (125.7 -> 122.4 us at 8M samples, profiles/r2_s6/
  // smote_g2_ab.txt); nontemporal output stores (launchers.h nt_stores)
  if (out_kind == 0 && pb) FDX_SG(0, true, true, true);
  else if (out_kind == 0) FDX_SG(0, true, false);
  else if (out_kind == 1) { if (pb) FDX_SG(1, false, true); else FDX_SG(1, false, false); }
  else { if (pb) FDX_SG(2, false, true); else FDX_SG(2, false, false); }
#undef FDX_SG
  check_launch("smote_generate");
}

}  // namespace fdx
