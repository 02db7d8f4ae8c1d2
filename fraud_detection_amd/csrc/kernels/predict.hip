// K5 predict_fused and K6 shap_linear.
//
// Reference behaviour being replaced: LogisticRegression.predict / predict_proba after
// StandardScaler.transform (api/app.py:194-240, predict_single.py:28-32, deploy.py:33-37,
// evaluate_model.py:26-27, xai_tasks.py:95-100) and the linear attribution
// phi_i = w_i (x_i - E[x_i]) of shap.LinearExplainer (explain_model.py:24-27, api/worker.py:75)
// / coef_ * x (xai_tasks.py:103-110).  SURVEY.md §2.3 rows K5, K6.
//
// MI355X mapping: pure HBM streaming.
//   * predict (bf16 rows, 64 B): 4 lanes per row x 16 B, so one wave-instruction reads 16 whole
//     rows = 1 KiB contiguous; 4 row-groups are issued before any is consumed (ILP).  Each lane
//     reduces 8 products, a 4-lane butterfly (DPP-able xor 1/2) finishes the dot, and the 4
//     results land one per quad lane so the 64 output floats of a wave-iteration are written by
//     one store instruction (a 256 B permutation, fully coalesced).
//   * predict (fp8 e4m3 rows, 32 B): 2 lanes per row x 16 B.
//   * predict+SHAP: 8 lanes per row x 4 columns; the SHAP output (30 floats/row) dominates the
//     traffic, so lanes store their 4 attributions directly (16 B stores for padded layouts).
//     Input is either the standardized bf16 training layout or raw fp32 features with the scaler
//     folded into the weights (a_j = w_j / sigma_j, c_j = mu_j + sigma_j * bg_j) so online
//     serving reads each raw byte exactly once.
#include "common.h"
#include "launchers.h"

namespace fdx {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float dot8_bf16(const uint4& v, const float* w) {
  float z = bf16lo(v.x) * w[0];
  z = fmaf(bf16hi(v.x), w[1], z);
  z = fmaf(bf16lo(v.y), w[2], z);
  z = fmaf(bf16hi(v.y), w[3], z);
  z = fmaf(bf16lo(v.z), w[4], z);
  z = fmaf(bf16hi(v.z), w[5], z);
  z = fmaf(bf16lo(v.w), w[6], z);
  z = fmaf(bf16hi(v.w), w[7], z);
  return z;
}

__device__ __forceinline__ float dot16_fp8(const uint4& v, const float* w) {
  const uint32_t words[4] = {v.x, v.y, v.z, v.w};
  float z = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float f[4];
    fp8x4_to_f32(words[k], f);  // hardware OCP e4m3 decode
#pragma unroll
    for (int b = 0; b < 4; ++b) z = fmaf(f[b], w[4 * k + b], z);
  }
  return z;
}

// bf16: LPR = 4 lanes per row (8 elems each); fp8: LPR = 2 (16 elems each).
template <int LPR>
__global__ __launch_bounds__(kThreads) void predict_kernel(const uint4* __restrict__ X, int64_t n,
                                                           const float* __restrict__ w,
                                                           float* __restrict__ prob,
                                                           float* __restrict__ logit) {
  constexpr int EPL = 32 / LPR;            // elements per lane
  constexpr int RPI = kWave / LPR;         // rows per wave-instruction
  constexpr int U = LPR;                   // row groups per iteration (so LPR lanes write U rows)
  const int lane = lane_id();
  const int q = lane & (LPR - 1);
  const int rr = lane / LPR;
  float wl[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int c = q * EPL + j;
    wl[j] = (c == kLabelCol) ? 0.0f : w[c];
  }
  const int64_t step = (int64_t)gridDim.x * (kThreads / kWave) * RPI * U;
  for (int64_t base = ((int64_t)blockIdx.x * (kThreads / kWave) + wave_id()) * RPI * U; base < n;
       base += step) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + u * RPI + rr;
      v[u] = row < n ? X[row * LPR + q] : make_uint4(0, 0, 0, 0);
    }
    float z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float t;
      if constexpr (LPR == 4) t = dot8_bf16(v[u], wl);
      else t = dot16_fp8(v[u], wl);
      z[u] = group_sum<LPR>(t);
    }
    float mine = z[0];
#pragma unroll
    for (int u = 1; u < U; ++u) mine = (q == u) ? z[u] : mine;
    const int64_t row = base + q * RPI + rr;
    if (row < n) {
      if (logit) logit[row] = mine;
      if (prob) prob[row] = fast_sigmoid(mine);
    }
  }
}

// Fused predict + linear SHAP.  8 lanes per row, 4 columns per lane.  OT: the prob / logit
// element type -- float, or double for host-to-host batch scoring (the fp32 result widened on the
// device, so the host receives final fp64 arrays with no conversion pass).
template <int IN, int VEC, typename OT = float>  // IN: 0 = bf16 [n][32], 1 = fp32 [n][ld]
__global__ __launch_bounds__(kThreads) void predict_shap_kernel(
    const void* __restrict__ Xv, int64_t n, int ld, int dz, int dphi, const float* __restrict__ a,
    const float* __restrict__ c, float bias, OT* __restrict__ prob, OT* __restrict__ logit,
    float* __restrict__ phi, int ld_phi) {
  const int lane = lane_id();
  const int c0 = (lane & 7) * 4;
  const int rsub = lane >> 3;
  float al[4], cl[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    al[j] = (c0 + j < dz) ? a[c0 + j] : 0.0f;
    cl[j] = c[c0 + j];
  }
  constexpr int U = 4;
  const int64_t ngroups = (n + 7) >> 3;
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t g = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); g < ngroups;
       g += nwaves * U) {
    float x[U][4];
    int64_t rows[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rows[u] = (g + u * nwaves) * 8 + rsub;
      const bool ok = (g + u * nwaves) < ngroups && rows[u] < n;
      if constexpr (IN == 0) {
        const uint16_t* X = reinterpret_cast<const uint16_t*>(Xv);
        uint2 t = ok ? *reinterpret_cast<const uint2*>(X + rows[u] * kCols + c0) : make_uint2(0, 0);
        x[u][0] = bf16lo(t.x); x[u][1] = bf16hi(t.x); x[u][2] = bf16lo(t.y); x[u][3] = bf16hi(t.y);
      } else {
        const float* X = reinterpret_cast<const float*>(Xv);
        const int dd = dz > dphi ? dz : dphi;
        const float* p = X + rows[u] * (int64_t)ld + c0;
        if (ok) {
          if (VEC == 4 && c0 + 4 <= dd) {
            float4 t = *reinterpret_cast<const float4*>(p);
            x[u][0] = t.x; x[u][1] = t.y; x[u][2] = t.z; x[u][3] = t.w;
          } else if (VEC >= 2 && c0 + 2 <= dd) {
            float2 t = *reinterpret_cast<const float2*>(p);
            x[u][0] = t.x; x[u][1] = t.y;
            if (c0 + 4 <= dd) {
              float2 t2 = *reinterpret_cast<const float2*>(p + 2);
              x[u][2] = t2.x; x[u][3] = t2.y;
            } else {
              x[u][2] = (c0 + 2 < dd) ? p[2] : 0.0f;
              x[u][3] = 0.0f;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[u][j] = (c0 + j < dd) ? p[j] : 0.0f;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) x[u][j] = 0.0f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float z = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) z = fmaf(al[j], x[u][j], z);
      z = group_sum<8>(z) + bias;
      const bool ok = (g + u * nwaves) < ngroups && rows[u] < n;
      if (!ok) continue;
      if (phi) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = al[j] * (x[u][j] - cl[j]);
        float* dst = phi + rows[u] * (int64_t)ld_phi + c0;
        if ((ld_phi & 3) == 0 && c0 + 4 <= dphi) {
          *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
        } else if ((ld_phi & 1) == 0 && c0 + 2 <= dphi) {
          *reinterpret_cast<float2*>(dst) = make_float2(o[0], o[1]);
          if (c0 + 4 <= dphi) *reinterpret_cast<float2*>(dst + 2) = make_float2(o[2], o[3]);
          else if (c0 + 2 < dphi) dst[2] = o[2];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c0 + j < dphi) dst[j] = o[j];
        }
      }
      if ((lane & 7) == 0) {
        if (logit) logit[rows[u]] = (OT)z;
        if (prob) prob[rows[u]] = (OT)fast_sigmoid(z);
      }
    }
  }
}

// Cross-validation scoring (models/cv.py): logits of the raw fp32 rows idx[0..n) under a fit's
// device state -- standardized-space weights w (fp64, w[30] = intercept) and the scaler's mean /
// scale -- folded per block into a = w / scale, bias = w_30 - sum a mean.  The fold's validation
// rows are read in place from the raw table (no gathered copy) and the weights never visit the
// host, so a fold's AUC is enqueued behind its fit with no synchronisation.  8 lanes per row,
// 4 columns per lane (8-byte pieces: raw rows are 120 B, 8-byte aligned).
__global__ __launch_bounds__(kThreads) void predict_gather_logit_kernel(const float* __restrict__ X,
                                                                        const int64_t* __restrict__ idx, int64_t n,
                                                                        int d, const double* __restrict__ w,
                                                                        const double* __restrict__ mean,
                                                                        const double* __restrict__ scale,
                                                                        float* __restrict__ logit) {
  __shared__ float sa[32];
  __shared__ float sb;
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    double a = (t < d) ? w[t] / scale[t] : 0.0;
    double am = (t < d) ? a * mean[t] : 0.0;
    am = wave_sum(am);
    if (t < 32) sa[t] = (float)a;
    if (t == 0) sb = (float)(w[kBiasCol] - am);
  }
  __syncthreads();
  const int lane = lane_id(), c0 = (lane & 7) * 4, rsub = lane >> 3;
  float al[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) al[j] = sa[c0 + j];
  const float bias = sb;
  const int64_t ngroups = (n + 7) >> 3;
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t g = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); g < ngroups; g += nwaves) {
    const int64_t r = g * 8 + rsub;
    float x[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (r < n) {
      const float* p = X + idx[r] * (int64_t)d + c0;
      if (c0 + 2 <= d) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        x[0] = t.x; x[1] = t.y;
      }
      if (c0 + 4 <= d) {
        const float2 t = *reinterpret_cast<const float2*>(p + 2);
        x[2] = t.x; x[3] = t.y;
      }
    }
    float z = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) z = fmaf(al[j], x[j], z);
    z = group_sum<8>(z) + bias;
    if (r < n && (lane & 7) == 0) logit[r] = z;
  }
}

// Persistent serving kernel (launchers.h PersistCtl).  Rows are scored exactly as
// predict_shap_kernel<1, 2> scores them (8 lanes per row, 4 columns per lane, the same fma order
// and DPP row sum, fast_sigmoid), so a request gets the same bits on either path.  Host-memory
// rows are read with system-scope 64-bit atomic loads (never a stale cache line), results are
// stored plainly and published by a system-scope release before `done`.
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(kThreads) void predict_persistent_kernel(PersistCtl* __restrict__ ctl,
                                                                      const float* __restrict__ X, int d, int cap,
                                                                      const float* __restrict__ a,
                                                                      const float* __restrict__ c, float bias,
                                                                      float* __restrict__ prob,
                                                                      float* __restrict__ logit,
                                                                      uint64_t idle_ticks, uint64_t life_ticks) {
  __shared__ uint32_t s_cmd, s_n, s_seq;
  const int tid = threadIdx.x, lane = lane_id();
  const int c0 = (lane & 7) * 4, rsub = lane >> 3;
  float al[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) al[j] = (c0 + j < d) ? a[c0 + j] : 0.0f;
  (void)c;
  uint32_t last = 0, served = 0;
  uint64_t t_start = 0, t_work = 0;
  if (tid == 0) {
    last = ld_sys(&ctl->done);
    t_start = t_work = wall_clock64();
    st_sys(&ctl->served, 0u);
    st_sys(&ctl->state, kPersistRunning);
  }
  for (;;) {
    if (tid == 0) {
      uint32_t cmd = 0, db = 0;
      for (;;) {  // bounded: stop flag, idle timeout, lifetime
        db = ld_sys(&ctl->doorbell);
        if (db != last) { cmd = 1; break; }
        if (ld_sys(&ctl->stop) != 0u) break;
        const uint64_t now = wall_clock64();
        if (now - t_work > idle_ticks || now - t_start > life_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      s_cmd = cmd;
      s_seq = db;
      s_n = cmd == 1 ? min(ld_sys(&ctl->n), (uint32_t)cap) : 0u;
    }
    __syncthreads();
    if (s_cmd != 1) break;
    const int n = (int)s_n;
    // 8 lanes per row, 32 rows per block pass
    for (int r0 = (tid >> 3); r0 < n; r0 += kThreads / 8) {
      float x[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      const float* p = X + (int64_t)r0 * d + c0;
      if (c0 + 4 <= d) {
        const uint64_t u0 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t u1 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p + 2), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        x[0] = __uint_as_float((uint32_t)u0); x[1] = __uint_as_float((uint32_t)(u0 >> 32));
        x[2] = __uint_as_float((uint32_t)u1); x[3] = __uint_as_float((uint32_t)(u1 >> 32));
      } else if (c0 + 2 <= d) {
        const uint64_t u0 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        x[0] = __uint_as_float((uint32_t)u0); x[1] = __uint_as_float((uint32_t)(u0 >> 32));
        if (c0 + 2 < d)
          x[2] = __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p + 2), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c0 + j < d)
            x[j] = __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p + j), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM));
      }
      float z = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) z = fmaf(al[j], x[j], z);
      z = group_sum<8>(z) + bias;
      if ((lane & 7) == 0) {
        logit[r0] = z;
        prob[r0] = fast_sigmoid(z);
      }
    }
    (void)rsub;
    __threadfence_system();
    __syncthreads();
    if (tid == 0) {
      last = s_seq;
      ++served;
      st_sys(&ctl->served, served);
      st_sys(&ctl->done, last);
      t_work = wall_clock64();
    }
  }
  if (tid == 0) st_sys(&ctl->state, kPersistExited);
}

}  // namespace

void launch_predict_bf16(const uint16_t* X, int64_t n, const float* w, float* prob, float* logit,
                         hipStream_t stream) {
  const int grid = stream_grid(n, (kThreads / kWave) * 64, 2048);
  predict_kernel<4><<<grid, kThreads, 0, stream>>>(reinterpret_cast<const uint4*>(X), n, w, prob,
                                                   logit);
  check_launch("predict_bf16");
}

void launch_predict_fp8(const uint8_t* X, int64_t n, const float* w, float* prob, float* logit,
                        hipStream_t stream) {
  const int grid = stream_grid(n, (kThreads / kWave) * 64, 2048);
  predict_kernel<2><<<grid, kThreads, 0, stream>>>(reinterpret_cast<const uint4*>(X), n, w, prob,
                                                   logit);
  check_launch("predict_fp8");
}

void launch_predict_shap(const void* X, int in_kind, int64_t n, int ld, int dz, int dphi,
                         const float* a, const float* c, float bias, float* prob, float* logit,
                         float* phi, int ld_phi, hipStream_t stream) {
  static const int cap01 = resident_cap(predict_shap_kernel<0, 1>, kThreads);
  static const int cap14 = resident_cap(predict_shap_kernel<1, 4>, kThreads);
  static const int cap12 = resident_cap(predict_shap_kernel<1, 2>, kThreads);
  static const int cap11 = resident_cap(predict_shap_kernel<1, 1>, kThreads);
  const int64_t units = (n + 7) / 8, per_block = (kThreads / kWave) * 4;
  int grid = capped_grid(units, per_block, cap01);
  if (in_kind == 0) {
    predict_shap_kernel<0, 1><<<grid, kThreads, 0, stream>>>(X, n, kCols, dz, dphi, a, c, bias,
                                                             prob, logit, phi, ld_phi);
  } else {
    const uintptr_t al = reinterpret_cast<uintptr_t>(X);
    if ((ld % 4) == 0 && (al % 16) == 0)
      predict_shap_kernel<1, 4><<<capped_grid(units, per_block, cap14), kThreads, 0, stream>>>(X, n, ld, dz, dphi, a, c, bias,
                                                               prob, logit, phi, ld_phi);
    else if ((ld % 2) == 0 && (al % 8) == 0)
      predict_shap_kernel<1, 2><<<capped_grid(units, per_block, cap12), kThreads, 0, stream>>>(X, n, ld, dz, dphi, a, c, bias,
                                                               prob, logit, phi, ld_phi);
    else
      predict_shap_kernel<1, 1><<<capped_grid(units, per_block, cap11), kThreads, 0, stream>>>(X, n, ld, dz, dphi, a, c, bias,
                                                               prob, logit, phi, ld_phi);
  }
  check_launch("predict_shap");
}

void launch_predict_raw64(const float* X, int64_t n, int ld, int d, const float* a, float bias, double* prob,
                          double* logit, hipStream_t stream) {
  static const int cap2 = resident_cap(predict_shap_kernel<1, 2, double>, kThreads);
  static const int cap1 = resident_cap(predict_shap_kernel<1, 1, double>, kThreads);
  const int64_t units = (n + 7) / 8, per_block = (kThreads / kWave) * 4;
  // raw fp32 rows of 30 features: 8-byte aligned pairs when ld is even
  if ((ld % 2) == 0 && (reinterpret_cast<uintptr_t>(X) % 8) == 0)
    predict_shap_kernel<1, 2, double><<<capped_grid(units, per_block, cap2), kThreads, 0, stream>>>(
        X, n, ld, d, 0, a, a, bias, prob, logit, nullptr, 0);
  else
    predict_shap_kernel<1, 1, double><<<capped_grid(units, per_block, cap1), kThreads, 0, stream>>>(
        X, n, ld, d, 0, a, a, bias, prob, logit, nullptr, 0);
  check_launch("predict_raw64");
}

void launch_predict_persistent(PersistCtl* ctl, const float* X, int d, int cap, const float* a, const float* c,
                               float bias, float* prob, float* logit, uint64_t idle_ticks, uint64_t life_ticks,
                               hipStream_t stream) {
  if (d < 1 || d > kCols || cap < 1) throw std::runtime_error("predict_persistent: bad shape");
  predict_persistent_kernel<<<1, kThreads, 0, stream>>>(ctl, X, d, cap, a, c, bias, prob, logit, idle_ticks,
                                                        life_ticks);
  check_launch("predict_persistent");
}

}  // namespace fdx

namespace fdx {
void launch_predict_gather_logit(const float* X, const int64_t* idx, int64_t n, int d, const double* w,
                                 const double* mean, const double* scale, float* logit, hipStream_t stream) {
  if (d > 32 || (d & 1) || (reinterpret_cast<uintptr_t>(X) % 8) != 0)
    throw std::invalid_argument("predict_gather_logit: even d <= 32, 8-byte aligned rows");
  if (n <= 0) return;
  const int64_t groups = (n + 7) / 8;
  const int grid = (int)std::min<int64_t>(2048, (groups + 3) / 4);
  predict_gather_logit_kernel<<<grid, kThreads, 0, stream>>>(X, idx, n, d, w, mean, scale, logit);
  check_launch("predict_gather_logit");
}
}  // namespace fdx
