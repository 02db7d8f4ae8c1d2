// K7 KernelSHAP on MI355X: batched coalition evaluation + efficiency-constrained WLS projection.
//
// Reference: shap.KernelExplainer semantics (BASELINE.json config 4), the
// north-star "coalition-masked batched GEMM" XAI path the async worker runs
// (reference xai_tasks.py:103-115, api/worker.py:53-75).  Host side (models/explainers.py): the
// coalition design Z [S][M] and the WLS operator A [M-1][S] are built once per design.
//
// Work decomposition (both model families): workgroup (e, p) = explanation e, coalition part p of
// P.  A part evaluates f(z_s) for its coalition tiles, forms y_s = link(f_s) - link(f0) in LDS and
// projects it, acc_i = sum_{s in part} A[i][s] y_s.  P = 1 finishes in place; P > 1 writes the
// partial to a workspace and the LAST part to arrive (device-scope counter) sums the partials in
// part order -- deterministic -- and finishes: phi_{<M} = acc - (A z_M) delta,
// phi_M = delta - sum(phi_{<M}), delta = link(f(x)) - link(f0).  P is chosen on the host so that
// E x P workgroups fill the 256 CUs in whole dispatch rounds (ops/kernelshap.py).
//
// Linear model (kernelshap_linear_kernel): the coalition logits are linear in z,
//   logit(z_s, b) = sum_k z_sk u_bk + c_b,   u_b = a * x_e - W_b,   W_b = a * B_b,
// a (n_bg x 32) x (32 x S) product per explanation.  v_mfma_f32_32x32x16_bf16 with the background
// row on M and the coalition on N; Z is exact in bf16, u is split into hi + lo bf16 halves (two
// MFMAs, ~16 mantissa bits per product, fp32 accumulation) and the background intercepts ride in
// K column 31 (Z[:,31] = 1, U[:,31] = c_b).  The U fragments of an explanation are built ONCE per
// workgroup into LDS (conflict-free 16 B per lane) instead of per wave in registers: 4x less build
// work and ~60 fewer VGPRs, so all 1000 workgroups of a 1k-explanation batch are resident in one
// dispatch round.  Sigmoid epilogue: u is pre-scaled by -log2(e) so sigma = 1 / (1 + exp2(acc)),
// and two background rows share one reciprocal, 1/d0 + 1/d1 = (d0 + d1) / (d0 d1): per pair one
// v_exp_f32 + 1/2 v_rcp_f32 instead of one of each (the phase is VALU-issue bound); the exp2
// argument is shifted by -40 so the pair product cannot overflow while either sigma matters.
// exp2 overflow (logit < ~-116) turns a pair into NaN; that tile is re-summed per element.
//
// Tree ensemble (kernelshap_tree_kernel, model-agnostic path for the GBDT family): the model is
// evaluated on the masked rows z * x + (1 - z) * B_b without materialising them.  Per tree t the
// host precomputes bw[t][b] = nodes where background row b goes right; the kernel computes
// xw[t] for x and, per (coalition, tree), Zt = the z-bit of each node's feature.  The effective
// direction bits are then ONE bitfield insert, R = (Zt & xw) | (~Zt & bw), and the walk is 2 VALU
// ops per level on a 1-based heap.  xw / bw are wave-uniform (a wave holds 64 coalitions x one
// background row), leaves sit in LDS.
//
// MFMA operand maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) supplies
// A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7 -> both are 16 contiguous bytes of a
// row (U row b for A, Z row s for B); accumulator row = (i & 3) + 8 (i >> 2) + 4 h, col = r.
#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kMaxBg = 128;      // 4 background tiles of 32
constexpr int kMaxS = 4096;      // coalitions per design
constexpr int kMaxParts = 8;
constexpr float kNullAcc = 70.0f;     // exact in bf16; sigma = 1 / (1 + 2^70)
constexpr float kPairShift = 40.0f;   // exp2 argument shift of the paired-reciprocal epilogue
constexpr int kTreeLdsLeaves = 8192;  // leaves (floats) staged in LDS by the tree kernel
constexpr int kMaxTrees = 2048;

__device__ __forceinline__ short bf16_bits(float f) { return (short)f32_to_bf16(f); }

// STAMP (tools/kernelshap_stamps.py): s_memtime of thread 0 at the phase boundaries -> stamps[e][8]
#define FDX_STAMP(i)                                                                              \
  do {                                                                                            \
    if constexpr (STAMP) {                                                                        \
      __builtin_amdgcn_sched_barrier(0);                                                          \
      unsigned long long t_;                                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
      __builtin_amdgcn_sched_barrier(0);                                                          \
      tsv[i] = t_;                                                                                \
    }                                                                                             \
  } while (0)

// link: 0 = identity on probabilities (shap default), 1 = logit of the mean probability,
//       2 = model log-odds (mean of logits; for the linear model KernelSHAP == LinearSHAP exactly)
__device__ __forceinline__ void link_pair(int link, float f0m, float logit_x, float& f0l, float& fxl) {
  if (link == 2) {
    f0l = f0m;
    fxl = logit_x;
  } else if (link == 1) {
    const float p0 = fminf(fmaxf(f0m, 1e-12f), 1.0f - 1e-7f);
    f0l = __logf(p0 / (1.0f - p0));
    fxl = logit_x;
  } else {
    f0l = f0m;
    fxl = fast_sigmoid(logit_x);
  }
}

// y_s = link(f_s) - f0l over the part's coalitions (in place in LDS), padded coalitions -> 0.
__device__ __forceinline__ void form_y(float* ys, int s0, int ns, int S, int link, float f0l) {
  for (int s = threadIdx.x; s < ns; s += kThreads) {
    float v = ys[s];
    if (link == 1) {
      v = fminf(fmaxf(v, 1e-12f), 1.0f - 1e-7f);
      v = __logf(v / (1.0f - v));
    }
    ys[s] = s0 + s < S ? v - f0l : 0.0f;  // A is zero-padded there too
  }
}

// One thread's share (lanes part, part + 8, ...) of sum_{s < ns} Ai[s] y_s: float4 steps, 4
// independent accumulators.  ns % 32 == 0, Ai and ys 16-B aligned.
__device__ __forceinline__ float seg_dot(const float* __restrict__ Ai_, const float* ys, int ns, int part) {
  const float4* Ai = reinterpret_cast<const float4*>(Ai_);
  const float4* fv = reinterpret_cast<const float4*>(ys);
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
  const int nq = ns >> 2;  // ns % 32 == 0 -> nq % 8 == 0
  int q = part;
  // 8 A loads in flight per round: the phase is L2-latency bound (every workgroup of the single
  // dispatch round reaches it at about the same time, so nothing else hides the latency)
  for (; q + 56 < nq; q += 64) {
    float4 av[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) av[u] = Ai[q + 8 * u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 yv = fv[q + 8 * u];
      a4[u & 3] = fmaf(av[u].x, yv.x, fmaf(av[u].y, yv.y, fmaf(av[u].z, yv.z, fmaf(av[u].w, yv.w, a4[u & 3]))));
    }
  }
  for (; q < nq; q += 8) {
    const float4 av = Ai[q], yv = fv[q];
    a4[0] = fmaf(av.x, yv.x, fmaf(av.y, yv.y, fmaf(av.z, yv.z, fmaf(av.w, yv.w, a4[0]))));
  }
  return (a4[0] + a4[1]) + (a4[2] + a4[3]);
}

// Partial projection acc_i = sum_{s < ns} A[i][s0 + s] y_s for i < d-1 into ph[i]: 8 threads per
// output over the (S_pad-strided, zero-padded) A row.  off2 >= 0: a second segment of ns
// coalitions at A column off2 + s0 with values ys[ns..2 ns) (the complement half of a paired design).
__device__ __forceinline__ void project_part(const float* ys, int s0, int ns, const float* __restrict__ Amat,
                                             int S_pad, int d, float* ph, int off2 = -1) {
  const int i = threadIdx.x >> 3, part = threadIdx.x & 7;
  float acc = 0.0f;
  if (i < d - 1) {
    const float* Ai = Amat + (int64_t)i * S_pad;
    acc = seg_dot(Ai + s0, ys, ns, part);
    if (off2 >= 0) acc += seg_dot(Ai + off2 + s0, ys + ns, ns, part);
  }
  acc = group_sum<8>(acc);
  if (part == 0 && i < d - 1) ph[i] = acc;
}

// Finish explanation e from its part's projection ph (LDS).  P > 1: publish the partial, the last
// part to arrive sums all partials in part order.  Returns after the phi row is written (or not,
// for a part that is not last).
__device__ __forceinline__ void finish(int e, int p, int P, int d, float* ph, const float* __restrict__ Az,
                                       float delta, float fxl, float f0l, float* __restrict__ phi,
                                       float* __restrict__ fx_out, float* __restrict__ f0_out,
                                       float* __restrict__ ws, unsigned* __restrict__ cnt, int* flag) {
  __syncthreads();
  if (P > 1) {
    // Partials move through agent-coherent stores / loads, ordered by vmcnt(0) before the arrival:
    // no __threadfence, whose L2 write-back (buffer_wbl2) per workgroup made every P > 1 launch
    // 2-4x slower than P = 1 (profiles/r6_ks).
    if (threadIdx.x < d - 1)
      __hip_atomic_store(ws + ((int64_t)e * kMaxParts + p) * 32 + threadIdx.x, ph[threadIdx.x], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(cnt + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == (unsigned)(P - 1);
      // self-cleaning for the next launch (no other part touches it now)
      if (last) __hip_atomic_store(cnt + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return;
    if (threadIdx.x < d - 1) {
      float s = 0.0f;
      for (int q = 0; q < P; ++q)  // fixed part order: deterministic
        s += __hip_atomic_load(ws + ((int64_t)e * kMaxParts + q) * 32 + threadIdx.x, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      ph[threadIdx.x] = s;
    }
    __syncthreads();
  }
  if (threadIdx.x < d - 1) ph[threadIdx.x] -= Az[threadIdx.x] * delta;
  __syncthreads();
  if (threadIdx.x == 0) {
    float sum = 0.0f;
    for (int k = 0; k < d - 1; ++k) sum += ph[k];
    ph[d - 1] = delta - sum;
    fx_out[e] = fxl;
    f0_out[e] = f0l;
  }
  __syncthreads();
  if (threadIdx.x < d) phi[(int64_t)e * d + threadIdx.x] = ph[threadIdx.x];
}

// ------------------------------------------------------------------------------------------------
// Linear model
// ------------------------------------------------------------------------------------------------
// amdgpu_waves_per_eu(4): <= 128 VGPRs (126, no scratch) so 4 workgroups share a CU and a
// 1000-explanation batch is ONE dispatch round of 1024 slots; left to itself the compiler took
// 152 VGPRs (3 workgroups per CU: 768 + a 232-workgroup second round, 57 us vs ~35 us).
template <int NTB, int NGL, bool LOGITS, bool STAMP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void kernelshap_linear_kernel(
    const float* __restrict__ X, int d, const float* __restrict__ a, float bias,
    const float* __restrict__ Bg, const float* __restrict__ cb, int n_bg,
    const uint16_t* __restrict__ Z, int S, int S_pad, int P, const float* __restrict__ Amat,
    const float* __restrict__ Az, int link, float* __restrict__ phi, float* __restrict__ fx_out,
    float* __restrict__ f0_out, float* __restrict__ ws, unsigned* __restrict__ cnt,
    unsigned long long* __restrict__ stamps) {
  unsigned long long tsv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  FDX_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) float ys[];  // this part's coalitions
  __shared__ uint4 Uhi[4 * 2 * 2 * 32], Ulo[4 * 2 * 2 * 32];  // [tile][kstep][half][row]
  __shared__ float xs[32];
  __shared__ float red[8];
  __shared__ float ph[32];
  __shared__ int flag;
  const int e = blockIdx.x / P, p = blockIdx.x - e * P;
  const int lane = lane_id(), wv = wave_id();
  const int r = lane & 31, h = lane >> 5;
  const int nst = S_pad >> 5;
  const int st0 = (p * nst) / P, st1 = ((p + 1) * nst) / P;
  // v = a o x (col 31: 0); u_b = v - W_b with W = [a o B_b, 0.., -c_b] precomputed per design
  if (threadIdx.x < 32) xs[threadIdx.x] = threadIdx.x < d ? a[threadIdx.x] * X[(int64_t)e * d + threadIdx.x] : 0.0f;
  __syncthreads();
  // sigmoid links: u is pre-scaled by -log2(e), so the accumulator is -z log2(e)
  const float us = LOGITS ? 1.0f : -1.4426950408889634f;
  // cooperative U build: entry q = ((t * 2 + ks) * 2 + hh) * 32 + rr holds the 8 bf16 values lane
  // (rr, hh) feeds for background tile t, k-step ks (two entries per thread)
  for (int q = threadIdx.x; q < 512; q += kThreads) {
    const int rr = q & 31, hh = (q >> 5) & 1, ks = (q >> 6) & 1, t = q >> 7;
    const int b = 32 * t + rr, k0 = 16 * ks + 8 * hh;
    float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
    const bool okb = b < n_bg;
    if (okb) {
      const float4* wr = reinterpret_cast<const float4*>(Bg + (int64_t)b * kCols + k0);
      w0 = wr[0];
      w1 = wr[1];
    }
    const float wv8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float uu[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        // rows past n_bg are NULL rows: u = 0 except the intercept column, where the sigmoid
        // links get acc = kNullAcc (2^-70 ~ 0 after the sigmoid, finite in the paired
        // reciprocal) and the logit link gets 0 -- every background tile is then a full tile
        const bool icpt = k0 + j + jj == kCols - 1;
        // column 30 (never a feature: d <= 30) carries the epilogue's -kPairShift, exact in bf16,
        // against Z[:, 30] = 1: acc = -log2(e) L - 40 without touching the intercept's precision
        const bool shift = !LOGITS && k0 + j + jj == kBiasCol;
        uu[jj] = shift ? -kPairShift
                       : okb ? (xs[k0 + j + jj] - wv8[j + jj]) * us : (!LOGITS && icpt ? kNullAcc : 0.0f);
      }
      const uint16_t h0 = f32_to_bf16(uu[0]), h1 = f32_to_bf16(uu[1]);
      const float r0 = uu[0] - __uint_as_float(((uint32_t)h0) << 16);
      const float r1 = uu[1] - __uint_as_float(((uint32_t)h1) << 16);
      hw[j >> 1] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lw[j >> 1] = pack_bf16x2(r0, r1);
    }
    Uhi[q] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    Ulo[q] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  }
  __syncthreads();
  FDX_STAMP(1);
  const float inv_nb = 1.0f / (float)n_bg;
  for (int st = st0 + wv; st < st1; st += kWaves) {
    const uint4* zr = reinterpret_cast<const uint4*>(Z + (int64_t)(32 * st + r) * kCols);
    const bf16x8_t zb0 = __builtin_bit_cast(bf16x8_t, zr[h]), zb1 = __builtin_bit_cast(bf16x8_t, zr[2 + h]);
    auto mfma_tile = [&](int t) {
      const int q0 = (t * 2 + 0) * 64 + h * 32 + r, q1 = (t * 2 + 1) * 64 + h * 32 + r;
      const bf16x8_t uh0 = __builtin_bit_cast(bf16x8_t, Uhi[q0]), ul0 = __builtin_bit_cast(bf16x8_t, Ulo[q0]);
      const bf16x8_t uh1 = __builtin_bit_cast(bf16x8_t, Uhi[q1]), ul1 = __builtin_bit_cast(bf16x8_t, Ulo[q1]);
      f32x16_t acc = {};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh0, zb0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul0, zb0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh1, zb1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul1, zb1, acc, 0, 0, 0);
      return acc;
    };
    // NG: 8-row accumulator groups holding a real background row (group j = acc[4j..4j+3],
    // rows 8j + {0..3} + 4h).  The partial last background tile evaluates only its leading NGL
    // groups (compile-time, so the MFMA chain of the next tile still interleaves): 100 rows run
    // 13 of 16 groups instead of 4 full tiles (the padded rows were 22% of the epilogue work).
    auto epilogue = [&](const f32x16_t& acc, auto ngc) {
      constexpr int ng = decltype(ngc)::value;
      if constexpr (LOGITS) {
        float ts = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i >> 2) < ng) ts += acc[i];
        return ts;
      } else {
        // 4 background rows per step in packed f32: rows (i, i+2) and (i+1, i+3) pair up so
        // that the sums d0 + d1 and products d0 d1 of both pairs are one v_pk_add / v_pk_mul.
        // Scaled by 2^-S (S = kPairShift, folded into the GEMM): E' = 2^-S E, d' = 2^-S + E',
        // sigma = 2^-S / d', so d' is in [2^-40, 2^128] and a pair product d0' d1' can overflow
        // only if d1' > 1, i.e. when the partner's sigma is below 2^-40 anyway (unscaled, a logit
        // below -44 next to any moderate one overflowed and silently dropped the partner's sigma;
        // trained models hit that in most tiles).  It never underflows (>= 2^-80).
        constexpr float kOne = 1.0f / 1099511627776.0f;  // 2^-40
        f32x2_t ts2 = {0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < 4 * ng; i += 4) {
          const f32x2_t e02 = {__builtin_amdgcn_exp2f(acc[i]), __builtin_amdgcn_exp2f(acc[i + 2])};
          const f32x2_t e13 = {__builtin_amdgcn_exp2f(acc[i + 1]), __builtin_amdgcn_exp2f(acc[i + 3])};
          const f32x2_t d02 = e02 + kOne, d13 = e13 + kOne;
          const f32x2_t pr = d02 * d13;
          const f32x2_t rc = {fast_rcp(pr.x), fast_rcp(pr.y)};
          ts2 = __builtin_elementwise_fma(d02 + d13, rc, ts2);
        }
        float ts = (ts2.x + ts2.y) * kOne;
        if (__builtin_isnan(ts)) {  // exp2 overflow (logit below ~-116) in this lane: per-element form
          ts = 0.0f;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((i >> 2) < ng) ts += fast_rcp(1.0f + __builtin_amdgcn_exp2f(acc[i] + kPairShift));
        }
        return ts;
      }
    };
    // double-buffered: the MFMA chain of tile t+1 is issued before the epilogue of tile t, so
    // the matrix core works under the (VALU-bound) epilogue
    float fs = 0.0f;
    f32x16_t cur = mfma_tile(0);
#pragma unroll
    for (int t = 0; t < NTB - 1; ++t) {
      const f32x16_t nxt = mfma_tile(t + 1);
      fs += epilogue(cur, std::integral_constant<int, 4>{});
      cur = nxt;
    }
    fs += epilogue(cur, std::integral_constant<int, NGL>{});
    fs += __shfl_xor(fs, 32, kWave);
    if (h == 0) ys[32 * (st - st0) + r] = fs * inv_nb;
  }
  FDX_STAMP(2);
  // f0 (background mean output) and f(x)
  float z0s = 0.0f;
  for (int b = threadIdx.x; b < n_bg; b += kThreads) z0s += LOGITS ? cb[b] : fast_sigmoid(cb[b]);
  z0s = wave_sum(z0s);
  if (lane == 0) red[wv] = z0s;
  float zx = 0.0f;
  if (threadIdx.x < 32) zx = xs[threadIdx.x];  // a o x
  zx = wave_sum(zx);
  if (threadIdx.x == 0) red[4] = zx;
  __syncthreads();
  FDX_STAMP(3);
  float f0l, fxl;
  link_pair(link, (red[0] + red[1] + red[2] + red[3]) * inv_nb, red[4] + bias, f0l, fxl);
  const int s0 = 32 * st0, ns = 32 * (st1 - st0);
  form_y(ys, s0, ns, S, link, f0l);
  __syncthreads();
  FDX_STAMP(4);
  project_part(ys, s0, ns, Amat, S_pad, d, ph);
  FDX_STAMP(5);
  finish(e, p, P, d, ph, Az, fxl - f0l, fxl, f0l, phi, fx_out, f0_out, ws, cnt, &flag);
  FDX_STAMP(6);
  if constexpr (STAMP) {
    if (threadIdx.x == 0 && p == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) stamps[(int64_t)e * 8 + k] = tsv[k];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Linear model, complement-paired design
// ------------------------------------------------------------------------------------------------
// shap's sampler draws coalitions in complement pairs (z, 1 - z), and for the linear model
//   L_b(1 - z) = T_b - L_b(z),   T_b = logit(x) + c_b,
// so one MFMA tile yields the logits of 32 coalitions AND of their 32 complements.  The host
// (ops/kernelshap.py) stores Ppad base coalitions; slot Ppad + p is the complement of base p (a
// base whose complement is not in the design gets a zero A column there).  With
// acc = -log2(e) L_b(z) (shifted by -40 like the unpaired kernel) and tau_b from T_b:
//   sigma(L_b(z)) = 1 / (1 + exp2(acc + 40)),   sigma(L_b(1 - z)) = 1 / (1 + exp2(tau_b - acc + 40)),
// both summed with the unpaired kernel's shifted pair reciprocal: half the MFMA work, U-fragment
// reads and Z traffic of the unpaired kernel for the same evaluations, one extra v_sub per pair.
// Null background rows (past n_bg) have u = 0 and T = 0, i.e. both sigmas are exactly 1/2; that
// constant is subtracted once per coalition.
template <int NTB, int NGL, bool LOGITS>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void kernelshap_paired_kernel(
    const float* __restrict__ X, int d, const float* __restrict__ a, float bias,
    const float* __restrict__ Bg, const float* __restrict__ cb, int n_bg,
    const uint32_t* __restrict__ Zm, int Ppad, int P, const float* __restrict__ Amat,
    const float* __restrict__ Az, int link, float* __restrict__ phi, float* __restrict__ fx_out,
    float* __restrict__ f0_out, float* __restrict__ ws, unsigned* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) float ys[];  // [2][ns]: base, then complements
  __shared__ uint4 Uhi[4 * 2 * 2 * 32], Ulo[4 * 2 * 2 * 32];  // [tile][kstep][half][row]
  // tau_b = -log2(e) T_b in MFMA row order (within 4 rows: 0, 2, 1, 3), one 16-B read per group
  __shared__ float4 Tq[kMaxBg / 4];
  __shared__ f32x2_t rem[kWaves - 1][kWaves][32];  // remainder tiles: per-wave partial sums
  // coalitions travel as 32-bit masks (4 B instead of a 64-B bf16 row per coalition: the next
  // tile's mask is prefetched in one VGPR); a 4-bit slice -> 4 bf16 {0, 1} via a 16-entry LUT
  // (the 256-entry 8-bit table would push the LDS past 4 workgroups per CU)
  __shared__ uint2 zlut[16];
  __shared__ float xs[32];
  __shared__ float red[8];
  __shared__ float ph[32];
  __shared__ int flag;
  const int e = blockIdx.x / P, p = blockIdx.x - e * P;
  const int lane = lane_id(), wv = wave_id();
  const int r = lane & 31, h = lane >> 5;
  const int nst = Ppad >> 5;
  const int st0 = (p * nst) / P, st1 = ((p + 1) * nst) / P;
  const int ns = 32 * (st1 - st0);
  constexpr float kNegLog2e = -1.4426950408889634f;
  if (threadIdx.x < 32) xs[threadIdx.x] = threadIdx.x < d ? a[threadIdx.x] * X[(int64_t)e * d + threadIdx.x] : 0.0f;
  if (threadIdx.x < 16) {
    const unsigned v = threadIdx.x;
    uint32_t w[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      w[j] = (((v >> (2 * j)) & 1u) ? 0x3F80u : 0u) | (((v >> (2 * j + 1)) & 1u) ? 0x3F800000u : 0u);
    zlut[v] = make_uint2(w[0], w[1]);
  }
  __syncthreads();
  const float lx = wave_sum(lane < 32 ? xs[lane] : 0.0f) + bias;  // logit(x), in every wave
  const float us = LOGITS ? 1.0f : kNegLog2e;
  for (int q = threadIdx.x; q < 512; q += kThreads) {
    const int rr = q & 31, hh = (q >> 5) & 1, ks = (q >> 6) & 1, t = q >> 7;
    const int b = 32 * t + rr, k0 = 16 * ks + 8 * hh;
    float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
    const bool okb = b < n_bg;
    if (okb) {
      const float4* wr = reinterpret_cast<const float4*>(Bg + (int64_t)b * kCols + k0);
      w0 = wr[0];
      w1 = wr[1];
    }
    const float wv8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float uu[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)  // column 30: the exp2 shift (-kPairShift, every row, exact in bf16)
        uu[jj] = !LOGITS && k0 + j + jj == kBiasCol ? -kPairShift : okb ? (xs[k0 + j + jj] - wv8[j + jj]) * us : 0.0f;
      const uint16_t h0 = f32_to_bf16(uu[0]), h1 = f32_to_bf16(uu[1]);
      hw[j >> 1] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lw[j >> 1] = pack_bf16x2(uu[0] - bf16_to_f32(h0), uu[1] - bf16_to_f32(h1));
    }
    Uhi[q] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    Ulo[q] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  }
  __syncthreads();
  // T_b from the SAME bf16 hi + lo values the MFMA multiplies (the 30 feature columns plus the
  // intercept column twice: T_b = L_b(1) + c_b; not the shift column), so L_b(1 - z) = T_b - L_b(z)
  // carries exactly the rounding of the terms outside z, as a direct MFMA evaluation of 1 - z
  // would.  (T_b from the fp32 logit instead makes the z and 1 - z errors anti-correlated, and the
  // WLS projection then adds them.)  Stored as tau = T_b - 2 S in accumulator units: with acc =
  // -log2(e) L_b(z) - S, the complement's shifted exponent is tau - acc.
  if (threadIdx.x < kMaxBg) {
    const int b = threadIdx.x, rr = b & 31, t = b >> 5;
    float tsum = 0.0f, c31 = 0.0f;
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {  // e4 = ks * 2 + hh: K columns 8 e4 .. 8 e4 + 7
      const int q = (t * 4 + e4) * 32 + rr;
      const uint4 hv = Uhi[q], lv = Ulo[q];
      const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w}, lw[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if (e4 != 3 || w != 3) tsum += bf16lo(hw[w]) + bf16lo(lw[w]);  // column 30 = the shift
        tsum += bf16hi(hw[w]) + bf16hi(lw[w]);
      }
      if (e4 == 3) c31 = bf16hi(hw[3]) + bf16hi(lw[3]);
    }
    const float tau = (b < n_bg ? tsum + c31 : 0.0f) - (LOGITS ? 0.0f : 2.0f * kPairShift);
    const int q = (b & ~3) | ((b & 1) << 1) | ((b >> 1) & 1);
    reinterpret_cast<float*>(Tq)[q] = tau;
  }
  __syncthreads();
  const float inv_nb = 1.0f / (float)n_bg;
  // null rows evaluated per coalition: each adds exactly 1/2 to both sigma sums
  const float null_half = 0.5f * (float)(32 * (NTB - 1) + 8 * NGL - n_bg);
  float sumT = 0.0f;  // LOGITS: sum_b T_b (complement logit sum = sumT - base logit sum)
  if constexpr (LOGITS) {
    for (int b = lane; b < kMaxBg; b += kWave) sumT += reinterpret_cast<const float*>(Tq)[b];  // nulls: 0
    sumT = wave_sum(sumT);
  }
  // (coalition tile, background tile) -> 32 x 32 logits; zb0/zb1 = the tile's Z fragments
  auto mfma_tile = [&](const bf16x8_t& zb0, const bf16x8_t& zb1, int t, int oz) {
    const int q0 = (t * 2 + 0) * 64 + h * 32 + r + oz, q1 = (t * 2 + 1) * 64 + h * 32 + r + oz;
    f32x16_t acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, Uhi[q0]), zb0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, Ulo[q0]), zb0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, Uhi[q1]), zb1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, Ulo[q1]), zb1, acc, 0, 0, 0);
    return acc;
  };
  // -> (sum of sigma over the lane's rows for z, the same for 1 - z); rows of group j of tile t
  // are 32 t + 8 j + 4 h + {0..3}
  auto epilogue = [&](const f32x16_t& acc, int t, auto ngc) {
    constexpr int ng = decltype(ngc)::value;
    if constexpr (LOGITS) {
      float ts = 0.0f;
#pragma unroll
      for (int i = 0; i < 4 * ng; ++i) ts += acc[i];
      return f32x2_t{ts, 0.0f};
    } else {
      // The unpaired kernel's shifted pair reciprocal, for z and for 1 - z: with shifted
      // exponents E' = exp2(acc) and E'' = exp2(tau - acc) (both 2^-40 times the unshifted ones),
      // d = 2^-40 + E, sigma = 2^-40 / d, rows (0, 1) and (2, 3) share one reciprocal.  A pair
      // product overflows only when the partner's sigma is below 2^-40 and never underflows.
      // (The cheaper complement form E / (E + K_b) has products no shift keeps in range: it
      // dropped sigmas at T_0 + T_1 < -88.)
      constexpr float kOne = 1.0f / 1099511627776.0f;  // 2^-40
      float tb0 = 0.0f, tb1 = 0.0f, tc0 = 0.0f, tc1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 4 * ng; i += 4) {
        const float4 tt = Tq[8 * t + 2 * (i >> 2) + h];
        const float tv[4] = {tt.x, tt.z, tt.y, tt.w};  // rows +0, +1, +2, +3
        float db[4], dc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          db[k] = __builtin_amdgcn_exp2f(acc[i + k]) + kOne;
          dc[k] = __builtin_amdgcn_exp2f(tv[k] - acc[i + k]) + kOne;
        }
        tb0 = fmaf(db[0] + db[1], fast_rcp(db[0] * db[1]), tb0);
        tb1 = fmaf(db[2] + db[3], fast_rcp(db[2] * db[3]), tb1);
        tc0 = fmaf(dc[0] + dc[1], fast_rcp(dc[0] * dc[1]), tc0);
        tc1 = fmaf(dc[2] + dc[3], fast_rcp(dc[2] * dc[3]), tc1);
      }
      f32x2_t out = {(tb0 + tb1) * kOne, (tc0 + tc1) * kOne};
      if (__builtin_isnan(out.x + out.y)) {  // exp2 overflow (a logit below ~-116): per element
        out = f32x2_t{0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < 4 * ng; i += 4) {
          const float4 tt = Tq[8 * t + 2 * (i >> 2) + h];
          const float tv[4] = {tt.x, tt.z, tt.y, tt.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            out.x += fast_rcp(1.0f + __builtin_amdgcn_exp2f(acc[i + k] + kPairShift));
            out.y += fast_rcp(1.0f + __builtin_amdgcn_exp2f(tv[k] - acc[i + k] + kPairShift));
          }
        }
      }
      return out;
    }
  };
  auto store_y = [&](int st, float sb, float sc) {  // per-coalition totals over all background rows
    const float fb = LOGITS ? sb : sb - null_half;
    const float fc = LOGITS ? sumT - sb : sc - null_half;
    ys[32 * (st - st0) + r] = fb * inv_nb;
    ys[ns + 32 * (st - st0) + r] = fc * inv_nb;
  };
  // Whole coalition tiles round-robin over the waves; the remainder (< 4 tiles) is split by
  // background tile so that no SIMD carries an extra tile (wave w of every workgroup sits on SIMD
  // w: 33 tiles as 9 + 8 + 8 + 8 made SIMD 0 the critical path), partials summed in a fixed order.
  const int nfull = (st1 - st0) / kWaves * kWaves;
  auto zfrag = [&](uint32_t m, bf16x8_t& zb0, bf16x8_t& zb1) {  // K columns 8h..8h+7, 16+8h..16+8h+7
    const uint2 a0 = zlut[(m >> (8 * h)) & 0xfu], a1 = zlut[(m >> (8 * h + 4)) & 0xfu];
    const uint2 b0 = zlut[(m >> (16 + 8 * h)) & 0xfu], b1 = zlut[(m >> (20 + 8 * h)) & 0xfu];
    zb0 = __builtin_bit_cast(bf16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
    zb1 = __builtin_bit_cast(bf16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
  };
  uint32_t mnext = st0 + wv < st0 + nfull ? Zm[32 * (st0 + wv) + r] : 0u;
  for (int st = st0 + wv; st < st0 + nfull; st += kWaves) {
    const uint32_t m = mnext;
    if (st + kWaves < st0 + nfull) mnext = Zm[32 * (st + kWaves) + r];
    bf16x8_t zb0, zb1;
    zfrag(m, zb0, zb1);
    // an opaque zero per iteration keeps the U fragment reads inside the loop: hoisted, the 64
    // VGPRs of U plus the two-sum epilogue spill (the LDS re-read is 4 KB per tile per wave)
    int oz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(oz));
    f32x2_t fs = {0.0f, 0.0f};
    f32x16_t cur = mfma_tile(zb0, zb1, 0, oz);
#pragma unroll
    for (int t = 0; t < NTB - 1; ++t) {
      const f32x16_t nxt = mfma_tile(zb0, zb1, t + 1, oz);
      fs += epilogue(cur, t, std::integral_constant<int, 4>{});
      cur = nxt;
    }
    fs += epilogue(cur, NTB - 1, std::integral_constant<int, NGL>{});
    fs.x += __shfl_xor(fs.x, 32, kWave);
    fs.y += __shfl_xor(fs.y, 32, kWave);
    if (h == 0) store_y(st, fs.x, fs.y);
  }
  if (nfull < st1 - st0) {
    for (int st = st0 + nfull; st < st1; ++st) {
      f32x2_t fs = {0.0f, 0.0f};
      if (wv < NTB) {  // wave-uniform
        bf16x8_t zb0, zb1;
        zfrag(Zm[32 * st + r], zb0, zb1);
        const f32x16_t acc = mfma_tile(zb0, zb1, wv, 0);
        fs = wv == NTB - 1 ? epilogue(acc, wv, std::integral_constant<int, NGL>{})
                           : epilogue(acc, wv, std::integral_constant<int, 4>{});
        fs.x += __shfl_xor(fs.x, 32, kWave);
        fs.y += __shfl_xor(fs.y, 32, kWave);
      }
      if (h == 0) rem[st - st0 - nfull][wv][r] = fs;
    }
    __syncthreads();
    if (wv == 0 && h == 0) {
      for (int st = st0 + nfull; st < st1; ++st) {
        f32x2_t tot = rem[st - st0 - nfull][0][r];
        for (int w = 1; w < NTB; ++w) tot += rem[st - st0 - nfull][w][r];  // fixed order
        store_y(st, tot.x, tot.y);
      }
    }
  }
  // f0 (background mean output) and f(x)
  float z0s = 0.0f;
  for (int b = threadIdx.x; b < n_bg; b += kThreads) z0s += LOGITS ? cb[b] : fast_sigmoid(cb[b]);
  z0s = wave_sum(z0s);
  if (lane == 0) red[wv] = z0s;
  __syncthreads();
  float f0l, fxl;
  link_pair(link, (red[0] + red[1] + red[2] + red[3]) * inv_nb, lx, f0l, fxl);
  form_y(ys, 0, 2 * ns, 2 * ns, link, f0l);  // padded slots have zero A columns: no masking
  __syncthreads();
  project_part(ys, 32 * st0, ns, Amat, 2 * Ppad, d, ph, Ppad);
  finish(e, p, P, d, ph, Az, fxl - f0l, fxl, f0l, phi, fx_out, f0_out, ws, cnt, &flag);
}

// ------------------------------------------------------------------------------------------------
// Tree ensemble (depth D <= 5: the 31 internal nodes of a tree fit one 32-bit mask)
// ------------------------------------------------------------------------------------------------
// Walk one tree from the effective direction bits R1 (bit n + 1 = node n goes right; heap 1-based)
template <int D>
__device__ __forceinline__ int walk(uint32_t R1) {
  int node = 1;
#pragma unroll
  for (int l = 0; l < D; ++l) node = (node << 1) | (int)((R1 >> node) & 1u);
  return node - (1 << D);  // leaf index
}

template <int D, bool LOGITS, bool LEAF_LDS>
__global__ __launch_bounds__(kThreads) void kernelshap_tree_kernel(
    const float* __restrict__ Xs, int ldx, int d, const int* __restrict__ feat, const float* __restrict__ thr,
    const float* __restrict__ leaf, int T, float base_margin, const uint32_t* __restrict__ bw, int bw_ld,
    int n_bg, const uint32_t* __restrict__ Zm, int S, int S_pad, int P, const float* __restrict__ Amat,
    const float* __restrict__ Az, int link, float* __restrict__ phi, float* __restrict__ fx_out,
    float* __restrict__ f0_out, float* __restrict__ ws, unsigned* __restrict__ cnt) {
  constexpr int NI = (1 << D) - 1, NL = 1 << D;
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  float* ys = dyn;                          // this part's coalitions
  float* lf = dyn + ((S_pad + 3) & ~3);     // leaves [T][NL] (LEAF_LDS)
  __shared__ float xs[32];
  __shared__ uint32_t xw[kMaxTrees];        // x's direction bits per tree, pre-shifted (bit n + 1)
  __shared__ float red[8];
  __shared__ float ph[32];
  __shared__ int flag;
  const int e = blockIdx.x / P, p = blockIdx.x - e * P;
  const int lane = lane_id(), wv = wave_id();
  const int nst = S_pad >> 5;
  const int st0 = (p * nst) / P, st1 = ((p + 1) * nst) / P;
  const int s0 = 32 * st0, ns = 32 * (st1 - st0);
  if (threadIdx.x < 32) xs[threadIdx.x] = threadIdx.x < d ? Xs[(int64_t)e * ldx + threadIdx.x] : 0.0f;
  if constexpr (LEAF_LDS) {
    for (int i = threadIdx.x; i < T * NL; i += kThreads) lf[i] = leaf[i];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += kThreads) {
    uint32_t m = 0;
    for (int n = 0; n < NI; ++n) {
      const int f = feat[t * NI + n];
      if (f >= 0 && !(xs[f] < thr[t * NI + n])) m |= 2u << n;
    }
    xw[t] = m;
  }
  __syncthreads();
  const float* LF = LEAF_LDS ? lf : leaf;
  const float inv_nb = 1.0f / (float)n_bg;
  // one coalition per lane, 32 background rows per pass (wave-uniform b -> uniform bw / xw loads)
  for (int s = s0 + threadIdx.x; s < s0 + ns; s += kThreads) {
    const uint32_t zmask = Zm[s];
    float fs = 0.0f;
    for (int b0 = 0; b0 < n_bg; b0 += 32) {
      const int nb = min(32, n_bg - b0);  // uniform
      float mg[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) mg[j] = base_margin;
      for (int t = 0; t < T; ++t) {
        const int* ft = feat + t * NI;
        uint32_t Zt = 0;
#pragma unroll
        for (int n = 0; n < NI; ++n) {
          const int f = max(ft[n], 0);  // uniform address: scalar load
          Zt |= ((zmask >> f) & 1u) << (n + 1);
        }
        const uint32_t xt = __builtin_amdgcn_readfirstlane(xw[t]);
        const uint32_t* bt = bw + (int64_t)t * bw_ld + b0;
        const float* lt = LF + t * NL;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          if (j < nb) {
            const uint32_t R1 = (Zt & xt) | (~Zt & bt[j]);
            mg[j] += lt[walk<D>(R1)];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (j < nb) fs += LOGITS ? mg[j] : fast_sigmoid(mg[j]);
    }
    ys[s - s0] = fs * inv_nb;
  }
  // f0 = mean_b link(model(B_b)) and f(x): the same walks with Zt = 0 / all ones
  float z0s = 0.0f;
  for (int b = threadIdx.x; b < n_bg; b += kThreads) {
    float m = base_margin;
    for (int t = 0; t < T; ++t) m += LF[t * NL + walk<D>(bw[(int64_t)t * bw_ld + b])];
    z0s += LOGITS ? m : fast_sigmoid(m);
  }
  z0s = wave_sum(z0s);
  if (lane == 0) red[wv] = z0s;
  if (threadIdx.x == 0) {
    float m = base_margin;
    for (int t = 0; t < T; ++t) m += LF[t * NL + walk<D>(xw[t])];
    red[4] = m;
  }
  __syncthreads();
  float f0l, fxl;
  link_pair(link, (red[0] + red[1] + red[2] + red[3]) * inv_nb, red[4], f0l, fxl);
  form_y(ys, s0, ns, S, link, f0l);
  __syncthreads();
  project_part(ys, s0, ns, Amat, S_pad, d, ph);
  finish(e, p, P, d, ph, Az, fxl - f0l, fxl, f0l, phi, fx_out, f0_out, ws, cnt, &flag);
}

#undef FDX_STAMP

void check_design(int d, int S, int S_pad, int P) {
  if (d < 2 || d > 30) throw std::runtime_error("kernelshap: 2 <= d <= 30");
  if (S < 1 || S_pad % 32 != 0 || S_pad < S || S_pad > kMaxS)
    throw std::runtime_error("kernelshap: S_pad must be a multiple of 32 in [S, 4096]");
  if (P < 1 || P > kMaxParts || P > S_pad / 32) throw std::runtime_error("kernelshap: 1 <= parts <= 8 and <= S_pad/32");
}

size_t part_lds(int S_pad, int P) { return (size_t)(((S_pad / 32 + P - 1) / P) * 32) * sizeof(float); }

}  // namespace

int kernelshap_linear_resident(int S_pad, int P) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernelshap_linear_kernel<4, 4, false, false>, kThreads,
                                                   part_lds(S_pad, P)) != hipSuccess || occ < 1)
    occ = 1;
  return occ * device_cu_count();
}

void launch_kernelshap(const float* X, int n_expl, int d, const float* a, float bias, const float* bg,
                       const float* cb, int n_bg, const uint16_t* Z, int S, int S_pad, int parts,
                       const float* Amat, const float* Az, int link, float* phi, float* fx_out, float* f0_out,
                       float* ws, unsigned* cnt, hipStream_t stream, unsigned long long* stamps) {
  check_design(d, S, S_pad, parts);
  if (n_bg < 1 || n_bg > kMaxBg) throw std::runtime_error("kernelshap: 1 <= n_bg <= 128");
  if (parts > 1 && (ws == nullptr || cnt == nullptr)) throw std::runtime_error("kernelshap: parts > 1 needs ws/cnt");
  if (n_expl <= 0) return;
  const dim3 grid((unsigned)((int64_t)n_expl * parts));
  const size_t lds = part_lds(S_pad, parts);
#define FDX_KS(NT, NG, LG, ST)                                                                     \
  kernelshap_linear_kernel<NT, NG, LG, ST><<<grid, kThreads, lds, stream>>>(                           \
      X, d, a, bias, bg, cb, n_bg, Z, S, S_pad, parts, Amat, Az, link, phi, fx_out, f0_out, ws, cnt, stamps)
#define FDX_KS_NG(NT, LG)                         \
  do {                                            \
    switch (ngl) {                                \
      case 1: FDX_KS(NT, 1, LG, false); break;    \
      case 2: FDX_KS(NT, 2, LG, false); break;    \
      case 3: FDX_KS(NT, 3, LG, false); break;    \
      default: FDX_KS(NT, 4, LG, false); break;   \
    }                                             \
  } while (0)
#define FDX_KS_NT(LG)                           \
  do {                                          \
    switch (ntb) {                              \
      case 1: FDX_KS_NG(1, LG); break;          \
      case 2: FDX_KS_NG(2, LG); break;          \
      case 3: FDX_KS_NG(3, LG); break;          \
      default: FDX_KS_NG(4, LG); break;         \
    }                                           \
  } while (0)
  const bool logits = link == 2;
  const int ntb = (n_bg + 31) >> 5;
  const int ngl = (n_bg - 32 * (ntb - 1) + 7) >> 3;  // groups of 8 rows holding a real row in the last tile
  if (stamps != nullptr) {  // phase stamps: 4 full tiles (padded rows are NULL rows: same result)
    if (logits) FDX_KS(4, 4, true, true); else FDX_KS(4, 4, false, true);
  } else {
    if (logits) FDX_KS_NT(true); else FDX_KS_NT(false);
  }
#undef FDX_KS_NT
#undef FDX_KS_NG
#undef FDX_KS
  check_launch("kernelshap");
}

void launch_kernelshap_paired(const float* X, int n_expl, int d, const float* a, float bias, const float* bg,
                              const float* cb, int n_bg, const uint32_t* Zm, int Ppad, int parts, const float* Amat,
                              const float* Az, int link, float* phi, float* fx_out, float* f0_out, float* ws,
                              unsigned* cnt, hipStream_t stream) {
  check_design(d, 2 * Ppad, 2 * Ppad, 1);
  if (parts < 1 || parts > kMaxParts || parts > Ppad / 32)
    throw std::runtime_error("kernelshap_paired: 1 <= parts <= 8 and <= Ppad/32");
  if (n_bg < 1 || n_bg > kMaxBg) throw std::runtime_error("kernelshap: 1 <= n_bg <= 128");
  if (parts > 1 && (ws == nullptr || cnt == nullptr)) throw std::runtime_error("kernelshap: parts > 1 needs ws/cnt");
  if (n_expl <= 0) return;
  const dim3 grid((unsigned)((int64_t)n_expl * parts));
  const size_t lds = 2 * part_lds(Ppad, parts);
#define FDX_KP(NT, NG, LG)                                                                          \
  kernelshap_paired_kernel<NT, NG, LG><<<grid, kThreads, lds, stream>>>(                             \
      X, d, a, bias, bg, cb, n_bg, Zm, Ppad, parts, Amat, Az, link, phi, fx_out, f0_out, ws, cnt)
#define FDX_KP_NG(NT, LG)                       \
  do {                                          \
    switch (ngl) {                              \
      case 1: FDX_KP(NT, 1, LG); break;         \
      case 2: FDX_KP(NT, 2, LG); break;         \
      case 3: FDX_KP(NT, 3, LG); break;         \
      default: FDX_KP(NT, 4, LG); break;        \
    }                                           \
  } while (0)
#define FDX_KP_NT(LG)                           \
  do {                                          \
    switch (ntb) {                              \
      case 1: FDX_KP_NG(1, LG); break;          \
      case 2: FDX_KP_NG(2, LG); break;          \
      case 3: FDX_KP_NG(3, LG); break;          \
      default: FDX_KP_NG(4, LG); break;         \
    }                                           \
  } while (0)
  const int ntb = (n_bg + 31) >> 5;
  const int ngl = (n_bg - 32 * (ntb - 1) + 7) >> 3;
  if (link == 2) FDX_KP_NT(true); else FDX_KP_NT(false);
#undef FDX_KP_NT
#undef FDX_KP_NG
#undef FDX_KP
  check_launch("kernelshap_paired");
}

void launch_kernelshap_tree(const float* Xs, int ldx, int n_expl, int d, const int* feat, const float* thr,
                            const float* leaf, int ntrees, int depth, float base_margin, const uint32_t* bw,
                            int bw_ld, int n_bg, const uint32_t* Zm, int S, int S_pad, int parts,
                            const float* Amat, const float* Az, int link, float* phi, float* fx_out,
                            float* f0_out, float* ws, unsigned* cnt, hipStream_t stream) {
  check_design(d, S, S_pad, parts);
  if (depth < 1 || depth > 5) throw std::runtime_error("kernelshap_tree: depth must be in [1, 5]");
  if (ntrees < 1 || ntrees > kMaxTrees) throw std::runtime_error("kernelshap_tree: 1 <= trees <= 2048");
  if (n_bg < 1 || bw_ld < n_bg) throw std::runtime_error("kernelshap_tree: bad background");
  if (parts > 1 && (ws == nullptr || cnt == nullptr)) throw std::runtime_error("kernelshap: parts > 1 needs ws/cnt");
  if (n_expl <= 0) return;
  const dim3 grid((unsigned)((int64_t)n_expl * parts));
  const bool lds_leaves = ntrees * (1 << depth) <= kTreeLdsLeaves;
  const size_t lds = ((size_t)((S_pad + 3) & ~3) + (lds_leaves ? (size_t)ntrees << depth : 0)) * sizeof(float);
  const bool logits = link == 2;
#define FDX_KT(D_, LG, LL)                                                                                 \
  kernelshap_tree_kernel<D_, LG, LL><<<grid, kThreads, lds, stream>>>(                                     \
      Xs, ldx, d, feat, thr, leaf, ntrees, base_margin, bw, bw_ld, n_bg, Zm, S, S_pad, parts, Amat, Az, link, \
      phi, fx_out, f0_out, ws, cnt)
#define FDX_KT_D(D_)                                              \
  do {                                                            \
    if (logits) {                                                 \
      if (lds_leaves) FDX_KT(D_, true, true); else FDX_KT(D_, true, false);   \
    } else {                                                      \
      if (lds_leaves) FDX_KT(D_, false, true); else FDX_KT(D_, false, false); \
    }                                                             \
  } while (0)
  switch (depth) {
    case 1: FDX_KT_D(1); break;
    case 2: FDX_KT_D(2); break;
    case 3: FDX_KT_D(3); break;
    case 4: FDX_KT_D(4); break;
    default: FDX_KT_D(5); break;
  }
#undef FDX_KT_D
#undef FDX_KT
  check_launch("kernelshap_tree");
}

}  // namespace fdx
