// K7 kernelshap_coalition_gemm: batched KernelSHAP for the (scaler-folded) logistic model.
//
// Reference: shap.KernelExplainer semantics (BASELINE.json config 4),
// the north-star "coalition-masked batched GEMM" XAI path.  Host side (models/explainers.py):
// coalition design Z [S][M] and the efficiency-constrained WLS operator A [M-1][S] (solved once).
//
// Per explanation e (one workgroup):
//   logit(z_s, b) = sum_k z_sk u_bk + c_b,   u_b = a * x_e - W_b,   W_b = a * B_b,   c_b = a . B_b + bias
// is a (n_bg x 32) x (32 x S) product.  The background intercepts are folded in as K column 31
// (Z[:,31] = 1, U[:,31] = c_b), so the accumulator IS the logit.  v_mfma_f32_32x32x16_bf16 with
// the background row on the M axis and the coalition on the N axis: Z is exactly representable
// in bf16 and u is split into hi + lo bf16 halves (two MFMAs, ~16 mantissa bits per product,
// fp32 accumulation).  The epilogue applies the link (sigmoid for probability space), sums the
// 16 accumulator rows of each lane plus the partner half-wave, i.e. the mean over background
// rows, into LDS f[s].  Then y = link(f) - link(f0) and phi_{<M} = A y - (A z_M) delta,
// phi_M = delta - sum(phi_{<M}), delta = link(f(x)) - link(f0).
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
constexpr int kMaxBg = 128;     // 4 background tiles of 32
constexpr int kMaxS = 4096;     // coalitions per design (LDS f[] capacity)

__device__ __forceinline__ short bf16_bits(float f) { return (short)f32_to_bf16(f); }

// link: 0 = identity on probabilities (shap default), 1 = logit of the mean probability,
//       2 = model log-odds (mean of logits; KernelSHAP == LinearSHAP exactly)
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

template <bool STAMP = false>
__global__ __launch_bounds__(kThreads) void kernelshap_kernel(
    const float* __restrict__ X, int n_expl, int d, const float* __restrict__ a, float bias,
    const float* __restrict__ Bg, const float* __restrict__ cb, int n_bg,
    const uint16_t* __restrict__ Z, int S, int S_pad, const float* __restrict__ Amat,
    const float* __restrict__ Az, int link, float* __restrict__ phi, float* __restrict__ fx_out,
    float* __restrict__ f0_out, unsigned long long* __restrict__ stamps = nullptr) {
  unsigned long long tsv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  FDX_STAMP(0);
  __shared__ __attribute__((aligned(16))) float f[kMaxS];
  __shared__ float xs[32];
  __shared__ float red[8];
  const int e = blockIdx.x;
  const int lane = lane_id(), wv = wave_id();
  const int r = lane & 31, h = lane >> 5;
  // v = a o x (col 31: 0); u_b = v - W_b with W = [a o B_b, 0.., -c_b] precomputed per design
  if (threadIdx.x < 32) xs[threadIdx.x] = threadIdx.x < d ? a[threadIdx.x] * X[(int64_t)e * d + threadIdx.x] : 0.0f;
  __syncthreads();
  const int ntb = (n_bg + 31) >> 5;  // background tiles in use (uniform)
  // sigmoid links: u is pre-scaled by -log2(e), so the accumulator is -z log2(e) and
  // sigma(z) = 1 / (1 + exp2(acc)) needs no multiply per element
  const float us = link == 2 ? 1.0f : -1.4426950408889634f;
  // U fragments (hi / lo) for every background tile and both k-steps: 16 regs x 4 tiles; each
  // lane's 8 W values of a (tile, k-step) are two contiguous float4 loads
  bf16x8_t uhi[4][2], ulo[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int b = 32 * t + r;
    const bool okb = b < n_bg && t < ntb;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int k0 = 16 * ks + 8 * h;
      float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
      if (okb) {
        const float4* wr = reinterpret_cast<const float4*>(Bg + (int64_t)b * kCols + k0);
        w0 = wr[0];
        w1 = wr[1];
      }
      const float wv8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float u = okb ? (xs[k0 + j] - wv8[j]) * us : 0.0f;
        const short hi = bf16_bits(u);
        const float hif = __uint_as_float(((uint32_t)(uint16_t)hi) << 16);
        uhi[t][ks][j] = hi;
        ulo[t][ks][j] = bf16_bits(u - hif);
      }
    }
  }
  FDX_STAMP(1);
  const float inv_nb = 1.0f / (float)n_bg;
  const int nst = S_pad / 32;
  for (int st = wv; st < nst; st += kWaves) {
    const uint4* zr = reinterpret_cast<const uint4*>(Z + (int64_t)(32 * st + r) * kCols);
    const uint4 z0 = zr[h], z1 = zr[2 + h];  // k-step 0: cols 8h..8h+7; k-step 1: 16+8h..
    bf16x8_t zb[2];
    zb[0] = __builtin_bit_cast(bf16x8_t, z0);
    zb[1] = __builtin_bit_cast(bf16x8_t, z1);
    float fs = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= ntb) break;  // uniform
      f32x16_t acc = {};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uhi[t][0], zb[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ulo[t][0], zb[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uhi[t][1], zb[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ulo[t][1], zb[1], acc, 0, 0, 0);
      if (t < ntb - 1 || (n_bg & 31) == 0) {  // full tile (uniform)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          fs += link == 2 ? acc[i] : fast_rcp(1.0f + __builtin_amdgcn_exp2f(acc[i]));
      } else {  // partial last tile: rows past n_bg are skipped (whole-wave skips for i >= 4 at n_bg = 100)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (32 * t + (i & 3) + 8 * (i >> 2) + 4 * h < n_bg)
            fs += link == 2 ? acc[i] : fast_rcp(1.0f + __builtin_amdgcn_exp2f(acc[i]));
        }
      }
    }
    fs += __shfl_xor(fs, 32, kWave);
    if (h == 0) f[32 * st + r] = fs * inv_nb;
  }
  FDX_STAMP(2);
  // f0 (background mean output) and f(x)
  float z0s = 0.0f;
  for (int b = threadIdx.x; b < n_bg; b += kThreads) z0s += link == 2 ? cb[b] : fast_sigmoid(cb[b]);
  z0s = wave_sum(z0s);
  if (lane == 0) red[wv] = z0s;
  float zx = 0.0f;
  if (threadIdx.x < 32) zx = xs[threadIdx.x];  // a o x
  zx = wave_sum(zx);
  if (threadIdx.x == 0) red[4] = zx;
  __syncthreads();
  FDX_STAMP(3);
  const float f0m = (red[0] + red[1] + red[2] + red[3]) * inv_nb;
  const float logit_x = red[4] + bias;
  float f0l, fxl;
  if (link == 2) { f0l = f0m; fxl = logit_x; }
  else if (link == 1) {
    const float p0 = fminf(fmaxf(f0m, 1e-12f), 1.0f - 1e-7f);
    f0l = __logf(p0 / (1.0f - p0));
    fxl = logit_x;
  } else { f0l = f0m; fxl = fast_sigmoid(logit_x); }
  const float delta = fxl - f0l;
  for (int s = threadIdx.x; s < S_pad; s += kThreads) {
    float v = f[s];
    if (link == 1) {
      v = fminf(fmaxf(v, 1e-12f), 1.0f - 1e-7f);
      v = __logf(v / (1.0f - v));
    }
    f[s] = s < S ? v - f0l : 0.0f;  // padded coalitions contribute nothing (A is zero there too)
  }
  __syncthreads();
  FDX_STAMP(4);
  // phi_i = sum_s A[i][s] y_s - Az[i] delta, i < d-1: 8 threads per output, float4 steps of the
  // (S_pad-strided, zero-padded) A row, 4 independent accumulators (4 loads in flight)
  const int i = threadIdx.x >> 3, part = threadIdx.x & 7;
  float acc = 0.0f;
  if (i < d - 1) {
    const float4* Ai = reinterpret_cast<const float4*>(Amat + (int64_t)i * S_pad);
    const float4* fv = reinterpret_cast<const float4*>(f);
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    const int nq = S_pad >> 2;  // float4 columns; S_pad % 32 == 0 -> nq % 8 == 0
    int q = part;
    for (; q + 24 < nq; q += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 av = Ai[q + 8 * u], yv = fv[q + 8 * u];
        a4[u] = fmaf(av.x, yv.x, fmaf(av.y, yv.y, fmaf(av.z, yv.z, fmaf(av.w, yv.w, a4[u]))));
      }
    }
    for (; q < nq; q += 8) {
      const float4 av = Ai[q], yv = fv[q];
      a4[0] = fmaf(av.x, yv.x, fmaf(av.y, yv.y, fmaf(av.z, yv.z, fmaf(av.w, yv.w, a4[0]))));
    }
    acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  }
  acc = group_sum<8>(acc);
  __shared__ float ph[32];
  if (part == 0 && i < d - 1) ph[i] = acc - Az[i] * delta;
  __syncthreads();
  FDX_STAMP(5);
  if (threadIdx.x == 0) {
    float sum = 0.0f;
    for (int k = 0; k < d - 1; ++k) sum += ph[k];
    ph[d - 1] = delta - sum;
    fx_out[e] = fxl;
    f0_out[e] = f0l;
  }
  __syncthreads();
  if (threadIdx.x < d) phi[(int64_t)e * d + threadIdx.x] = ph[threadIdx.x];
  FDX_STAMP(6);
  if constexpr (STAMP) {
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) stamps[(int64_t)e * 8 + k] = tsv[k];
    }
  }
}
#undef FDX_STAMP

}  // namespace

void launch_kernelshap(const float* X, int n_expl, int d, const float* a, float bias, const float* bg,
                       const float* cb, int n_bg, const uint16_t* Z, int S, int S_pad, const float* Amat,
                       const float* Az, int link, float* phi, float* fx_out, float* f0_out,
                       hipStream_t stream, unsigned long long* stamps) {
  if (d < 2 || d > 30) throw std::runtime_error("kernelshap: 2 <= d <= 30");
  if (n_bg < 1 || n_bg > kMaxBg) throw std::runtime_error("kernelshap: 1 <= n_bg <= 128");
  if (S < 1 || S_pad % 32 != 0 || S_pad < S || S_pad > kMaxS)
    throw std::runtime_error("kernelshap: S_pad must be a multiple of 32 in [S, 4096]");
  if (n_expl <= 0) return;
  if (stamps != nullptr)
    kernelshap_kernel<true><<<n_expl, kThreads, 0, stream>>>(X, n_expl, d, a, bias, bg, cb, n_bg, Z, S, S_pad, Amat,
                                                             Az, link, phi, fx_out, f0_out, stamps);
  else
    kernelshap_kernel<false><<<n_expl, kThreads, 0, stream>>>(X, n_expl, d, a, bias, bg, cb, n_bg, Z, S, S_pad, Amat,
                                                              Az, link, phi, fx_out, f0_out);
  check_launch("kernelshap");
}

}  // namespace fdx
