// pybind11 entry points of the native extension `fraud_detection_amd._fdx_native`.
//
// Device pointers and hipStream_t handles cross the boundary as Python integers (taken from
// torch tensors' data_ptr() and torch.cuda.current_stream().cuda_stream).  All operand shape and
// dtype validation happens in fraud_detection_amd/ops/*.py BEFORE a launch (the kernels assume
// padded 32-column rows, 16 B alignment and in-bounds index arrays).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "kernels/launchers.h"
#include "serve/shm_ring.h"

namespace py = pybind11;
using u = uintptr_t;

template <typename T>
static T* P(u p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(u s) { return reinterpret_cast<hipStream_t>(s); }

static py::dict device_info(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) throw std::runtime_error("hipGetDeviceProperties failed");
  py::dict d;
  d["name"] = std::string(prop.name);
  d["gcn_arch"] = std::string(prop.gcnArchName);
  d["cu_count"] = prop.multiProcessorCount;
  d["total_mem"] = (unsigned long long)prop.totalGlobalMem;
  d["lds_per_block"] = (unsigned long long)prop.sharedMemPerBlock;
  d["clock_khz"] = prop.clockRate;
  d["l2_bytes"] = prop.l2CacheSize;
  int rt = 0;
  hipRuntimeGetVersion(&rt);
  d["hip_runtime_version"] = rt;
  return d;
}

static void stream_sync(u stream) {
  hipError_t e = hipStreamSynchronize(S(stream));
  if (e != hipSuccess) throw std::runtime_error(std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Page-lock a caller's host range for the duration of one call (so DMA reads / writes it in
// place: no staging memcpy).  Already-pinned memory (hipHostMalloc, or registered elsewhere) is
// used as it is.
struct HostPin {
  void* p = nullptr;
  explicit HostPin(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return;
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
    if (e == hipSuccess) p = ptr;
    else (void)hipGetLastError();  // hipErrorHostMemoryAlreadyRegistered or unsupported: copy as is
  }
  ~HostPin() {
    if (p) (void)hipHostUnregister(p);
  }
};

// ---- native GPU-owner loop (serve/gpu_owner.py, linear model) ------------------------------
// One C++ thread per owner drains the shared-memory request ring (serve/shm_ring.h) into one of
// two pinned, device-mapped input buffers and runs the fused folded-scaler predict (+ LinearSHAP)
// kernel straight on them, writing the results into mapped pinned output buffers: no copy
// kernels, no Python, no GIL on the serving path.  Batches are pipelined only under load: while a
// batch is on the device, the next is gathered and launched behind it when at least `pipe_rows`
// rows are already queued; otherwise the loop waits for the in-flight batch and then gathers
// everything that queued meanwhile (bigger batches amortise the ~16 us launch + wait).
struct NativeOwner {
  std::unique_ptr<fdx_ring::Ring> ring;
  std::thread th;
  std::atomic<bool> stop{false};
  const float* a = nullptr;
  const float* c = nullptr;
  float bias = 0.f;
  int d = 30;
  uint32_t cap = 0, pipe_rows = 64;
  double window_us = 0.0;
  hipStream_t stream = nullptr;
  float* in_host[2] = {nullptr, nullptr};
  const void* in_dev[2] = {nullptr, nullptr};
  float* out_host[2] = {nullptr, nullptr};
  float* out_dev[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::atomic<uint64_t> errors{0};
  // persistent small-batch path (predict_persistent_kernel): a mailbox in coherent mapped host
  // memory instead of a launch + event per batch
  bool persist = false;
  fdx::PersistCtl* pctl = nullptr;
  fdx::PersistCtl* pctl_dev = nullptr;
  float* p_in = nullptr;
  float* p_in_dev = nullptr;
  float* p_out = nullptr;
  float* p_out_dev = nullptr;
  uint32_t pcap = 0, pseq = 0;
  hipStream_t pstream = nullptr;
  uint64_t idle_ticks = 0, life_ticks = 0;
  std::atomic<uint64_t> p_batches{0}, p_launches{0};

  static uint32_t ld(const uint32_t* q) { return __atomic_load_n(q, __ATOMIC_ACQUIRE); }
  static void st(uint32_t* q, uint32_t v) { __atomic_store_n(q, v, __ATOMIC_RELEASE); }
  static double secs_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  // A running persistent kernel, (re)launched if it exited (idle timeout / lifetime).
  bool ensure_persistent() {
    if (ld(&pctl->state) == fdx::kPersistRunning) return true;
    if (hipStreamSynchronize(pstream) != hipSuccess) return false;  // the exited launch is gone
    st(&pctl->stop, 0u);
    st(&pctl->state, 0u);
    try {
      fdx::launch_predict_persistent(pctl_dev, p_in_dev, d, (int)pcap, a, c, bias, p_out_dev, p_out_dev + pcap,
                                     idle_ticks, life_ticks, pstream);
    } catch (...) {
      return false;
    }
    p_launches.fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    while (ld(&pctl->state) != fdx::kPersistRunning) {
      if (ld(&pctl->state) == fdx::kPersistExited || secs_since(t0) > 5.0) return false;
      __builtin_ia32_pause();
    }
    return true;
  }
  // Post the n rows already in p_in; true once the kernel has written their results to p_out.
  bool serve_persistent(uint32_t n) {
    if (!ensure_persistent()) return false;
    const uint32_t seq = ++pseq;
    st(&pctl->n, n);
    st(&pctl->doorbell, seq);  // release: the rows collect() wrote are visible before the bell
    const auto t0 = std::chrono::steady_clock::now();
    while (ld(&pctl->done) != seq) {
      if (ld(&pctl->state) == fdx::kPersistExited && ld(&pctl->done) != seq) {
        if (!ensure_persistent()) return false;  // exited just before the bell: serve again
      }
      if (secs_since(t0) > 2.0) return false;
      __builtin_ia32_pause();
    }
    return true;
  }

  void launch(int set, uint32_t n, bool explain, const void* in = nullptr) {
    const int dphi = explain ? d : 0;
    float* o = out_dev[set];
    fdx::launch_predict_shap(in ? in : in_dev[set], 1, n, d, d, dphi, a, c, bias, o, o + n,
                             explain ? o + 2 * (size_t)n : nullptr, dphi, stream);
    hip_check(hipEventRecord(ev[set], stream), "hipEventRecord");
  }
  void finish(int set, uint32_t n, bool explain, bool ok) {
    hipError_t e = hipSuccess;
    if (ok) e = hipEventSynchronize(ev[set]);
    const float* o = out_host[set];
    const bool good = ok && e == hipSuccess;
    if (!good) errors.fetch_add(1);
    ring->complete(o, o + n, explain ? o + 2 * (size_t)n : nullptr, explain ? (uint32_t)d : 0u, good, set);
  }
  // Small batch, nothing in flight on the launch path: the persistent kernel (predict) or one
  // synchronous launch from the same staging (explain, or the persistent kernel unavailable).
  void run_small() {
    auto r = ring->collect(p_in, pcap, window_us, 50.0, 0);
    const uint32_t n = r.first;
    if (!n) return;
    const bool explain = r.second == 1;
    if (!explain && serve_persistent(n)) {
      p_batches.fetch_add(1);
      ring->complete(p_out, p_out + pcap, nullptr, 0u, true, 0);
      return;
    }
    try {
      launch(0, n, explain, p_in_dev);
      finish(0, n, explain, true);
    } catch (...) {
      errors.fetch_add(1);
      ring->complete(nullptr, nullptr, nullptr, 0, false, 0);
    }
  }

  void run() {
    int cur = 0, inf_set = -1;
    uint32_t inf_n = 0;
    bool inf_explain = false;
    while (!stop.load(std::memory_order_relaxed) || inf_set >= 0) {
      if (persist && inf_set < 0 && !stop.load(std::memory_order_relaxed) &&
          ring->ready_rows(pcap + 1) <= pcap) {
        run_small();
        continue;
      }
      uint32_t n = 0, op = 0;
      if (!stop.load(std::memory_order_relaxed)) {
        if (inf_set < 0) {
          auto r = ring->collect(in_host[cur], cap, window_us, 50.0, cur);
          n = r.first;
          op = r.second;
        } else if (ring->ready_rows(pipe_rows) >= pipe_rows) {
          auto r = ring->collect(in_host[cur], cap, 0.0, 0.0, cur);
          n = r.first;
          op = r.second;
        }
      }
      bool launched = false;
      if (n) {
        try {
          launch(cur, n, op == 1);
          launched = true;
        } catch (...) {
          errors.fetch_add(1);
          ring->complete(nullptr, nullptr, nullptr, 0, false, cur);
        }
      }
      if (inf_set >= 0) {
        finish(inf_set, inf_n, inf_explain, true);
        inf_set = -1;
      }
      if (launched) {
        inf_set = cur;
        inf_n = n;
        inf_explain = op == 1;
        cur ^= 1;
      }
    }
  }
};

// Host-to-host batch scoring (BASELINE config 2: 1M x 30 raw fp32 rows in host memory -> fp64
// P(fraud) and logits in host memory).  The input is page-locked in place and streamed in chunks:
// H2D of chunk i+1 (DMA engine, stream h2d) overlaps the fused folded-scaler GEMV + sigmoid of
// chunk i (stream comp), whose fp64 results go back on a third stream (the other DMA direction)
// while later chunks upload.  Device buffers hold the whole batch (HBM is not the constraint here),
// so no slot is reused inside a call and only the chunk edges need events.
static void predict_h2h(u x_host, int64_t n, int ld, int d, u a, float bias, u prob_host, u logit_host,
                        u x_dev, u prob_dev, u logit_dev, int64_t chunk, u s_h2d, u s_comp, u s_d2h) {
  if (n <= 0) return;
  chunk = std::max<int64_t>(chunk, 1024);
  const size_t row_b = (size_t)ld * 4;
  HostPin px(P<void>(x_host), (size_t)n * row_b);
  HostPin pp(P<void>(prob_host), (size_t)n * 8);
  HostPin pl(P<void>(logit_host), (size_t)n * 8);
  const int64_t nch = (n + chunk - 1) / chunk;
  std::vector<hipEvent_t> up(nch), done(nch);
  for (int64_t i = 0; i < nch; ++i) {
    hip_check(hipEventCreateWithFlags(&up[i], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&done[i], hipEventDisableTiming), "hipEventCreate");
  }
  for (int64_t i = 0; i < nch; ++i) {
    const int64_t r0 = i * chunk, m = std::min(chunk, n - r0);
    hip_check(hipMemcpyAsync(P<char>(x_dev) + r0 * row_b, P<char>(x_host) + r0 * row_b, (size_t)m * row_b,
                             hipMemcpyHostToDevice, S(s_h2d)), "H2D");
    hip_check(hipEventRecord(up[i], S(s_h2d)), "hipEventRecord");
    hip_check(hipStreamWaitEvent(S(s_comp), up[i], 0), "hipStreamWaitEvent");
    fdx::launch_predict_raw64(P<const float>(x_dev) + r0 * ld, m, ld, d, P<const float>(a), bias,
                              P<double>(prob_dev) + r0, P<double>(logit_dev) + r0, S(s_comp));
    hip_check(hipEventRecord(done[i], S(s_comp)), "hipEventRecord");
    hip_check(hipStreamWaitEvent(S(s_d2h), done[i], 0), "hipStreamWaitEvent");
    if (prob_host)
      hip_check(hipMemcpyAsync(P<double>(prob_host) + r0, P<double>(prob_dev) + r0, (size_t)m * 8,
                               hipMemcpyDeviceToHost, S(s_d2h)), "D2H");
    if (logit_host)
      hip_check(hipMemcpyAsync(P<double>(logit_host) + r0, P<double>(logit_dev) + r0, (size_t)m * 8,
                               hipMemcpyDeviceToHost, S(s_d2h)), "D2H");
  }
  hipError_t e = hipStreamSynchronize(S(s_d2h));
  for (int64_t i = 0; i < nch; ++i) {
    (void)hipEventDestroy(up[i]);
    (void)hipEventDestroy(done[i]);
  }
  hip_check(e, "hipStreamSynchronize");
}

PYBIND11_MODULE(_fdx_native, m) {
  m.doc() = "MI355X (gfx950) HIP kernels for fraud_detection_amd";
  m.attr("ARCH") = "gfx950";
  m.attr("LR_PART_STRIDE") = fdx::kLRPartStride;
  m.def("device_info", &device_info, py::arg("device") = 0);
  // device-side address of a pinned (hipHostMalloc'd) host buffer, 0 if it is not mapped: the
  // small-batch serving path reads requests from / writes results to pinned memory directly
  m.def("host_device_pointer", [](u host_ptr) -> u {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(host_ptr), 0) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return reinterpret_cast<u>(d);
  });
  m.def("stream_sync", &stream_sync, py::call_guard<py::gil_scoped_release>());
  // Native hipGraph capture / launch (runtime/graphs.NativeGraph): stream capture in thread-local
  // mode around launches the caller makes on `stream` (native launchers, RCCL collectives), then
  // one hipGraphLaunch per replay.  torch.cuda.CUDAGraph.replay() waited for the device on this
  // build (a replay call cost the fit's device time, profiles/r6_j): this path does not.
  m.def("graph_begin", [](u stream) {
    hip_check(hipStreamBeginCapture(S(stream), hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  });
  m.def("graph_end", [](u stream) -> u {
    hipGraph_t g = nullptr;
    hip_check(hipStreamEndCapture(S(stream), &g), "hipStreamEndCapture");
    hipGraphExec_t ex = nullptr;
    const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    hip_check(e, "hipGraphInstantiate");
    return reinterpret_cast<u>(ex);
  });
  m.def("graph_launch", [](u exec, u stream) {
    hip_check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), S(stream)), "hipGraphLaunch");
  });
  m.def("graph_destroy", [](u exec) {
    if (exec) (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(exec));
  });
  // raw HIP events for the GPU owner's pipelined batches (wait with the GIL released)
  m.def("event_create", [] {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return reinterpret_cast<u>(e);
  });
  m.def("event_record", [](u e, u stream) {
    hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(e), S(stream)), "hipEventRecord");
  });
  m.def("event_sync", [](u e) {
    hip_check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(e)), "hipEventSynchronize");
  }, py::call_guard<py::gil_scoped_release>());
  m.def("event_destroy", [](u e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); });
  // busy-poll an event (no blocking-wait wake-up latency: for a thread that owns a core)
  m.def("event_spin", [](u e) {
    hipEvent_t ev = reinterpret_cast<hipEvent_t>(e);
    hipError_t r;
    while ((r = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
    hip_check(r, "hipEventQuery");
  }, py::call_guard<py::gil_scoped_release>());
  m.def("predict_h2h", &predict_h2h, py::call_guard<py::gil_scoped_release>());
  m.def("owner_start", [](u ring_base, size_t ring_bytes, u a, u c, float bias, int d, uint32_t cap, double window_us,
                          uint32_t pipe_rows, u stream, u in_host0, u in_host1, u in_dev0, u in_dev1, u out_host0,
                          u out_host1, u out_dev0, u out_dev1, uint32_t persist_rows, double idle_ms,
                          double life_ms) {
    auto* o = new NativeOwner();
    o->ring = std::make_unique<fdx_ring::Ring>(reinterpret_cast<char*>(ring_base), ring_bytes);
    if ((int)o->ring->d_() != d) {
      delete o;
      throw std::runtime_error("owner_start: ring width != model width");
    }
    o->a = P<const float>(a);
    o->c = P<const float>(c);
    o->bias = bias;
    o->d = d;
    o->cap = cap;
    o->window_us = window_us;
    o->pipe_rows = pipe_rows ? pipe_rows : 1;
    o->stream = S(stream);
    o->in_host[0] = P<float>(in_host0);
    o->in_host[1] = P<float>(in_host1);
    o->in_dev[0] = P<const void>(in_dev0);
    o->in_dev[1] = P<const void>(in_dev1);
    o->out_host[0] = P<float>(out_host0);
    o->out_host[1] = P<float>(out_host1);
    o->out_dev[0] = P<float>(out_dev0);
    o->out_dev[1] = P<float>(out_dev1);
    for (int i = 0; i < 2; ++i) hip_check(hipEventCreateWithFlags(&o->ev[i], hipEventDisableTiming), "hipEventCreate");
    if (persist_rows > 0) {
      o->pcap = std::min(persist_rows, cap);
      const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
      void* hp = nullptr;
      hip_check(hipHostMalloc(&hp, sizeof(fdx::PersistCtl), fl), "hipHostMalloc");
      std::memset(hp, 0, sizeof(fdx::PersistCtl));
      o->pctl = static_cast<fdx::PersistCtl*>(hp);
      hip_check(hipHostMalloc(&hp, (size_t)o->pcap * d * sizeof(float), fl), "hipHostMalloc");
      o->p_in = static_cast<float*>(hp);
      hip_check(hipHostMalloc(&hp, (size_t)o->pcap * 2 * sizeof(float), fl), "hipHostMalloc");
      o->p_out = static_cast<float*>(hp);
      void* dp = nullptr;
      hip_check(hipHostGetDevicePointer(&dp, o->pctl, 0), "hipHostGetDevicePointer");
      o->pctl_dev = static_cast<fdx::PersistCtl*>(dp);
      hip_check(hipHostGetDevicePointer(&dp, o->p_in, 0), "hipHostGetDevicePointer");
      o->p_in_dev = static_cast<float*>(dp);
      hip_check(hipHostGetDevicePointer(&dp, o->p_out, 0), "hipHostGetDevicePointer");
      o->p_out_dev = static_cast<float*>(dp);
      hip_check(hipStreamCreateWithFlags(&o->pstream, hipStreamNonBlocking), "hipStreamCreate");
      int dev = 0, khz = 0;
      hip_check(hipGetDevice(&dev), "hipGetDevice");
      if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
      o->idle_ticks = (uint64_t)(idle_ms * khz);
      o->life_ticks = (uint64_t)(life_ms * khz);
      o->persist = true;
    }
    o->th = std::thread([o] { o->run(); });
    return reinterpret_cast<u>(o);
  }, py::arg("ring_base"), py::arg("ring_bytes"), py::arg("a"), py::arg("c"), py::arg("bias"), py::arg("d"),
     py::arg("cap"), py::arg("window_us"), py::arg("pipe_rows"), py::arg("stream"), py::arg("in_host0"),
     py::arg("in_host1"), py::arg("in_dev0"), py::arg("in_dev1"), py::arg("out_host0"), py::arg("out_host1"),
     py::arg("out_dev0"), py::arg("out_dev1"), py::arg("persist_rows") = 0, py::arg("idle_ms") = 200.0,
     py::arg("life_ms") = 10000.0);
  m.def("owner_persistent_stats", [](u h) {
    auto* o = reinterpret_cast<NativeOwner*>(h);
    return py::make_tuple(o->p_batches.load(), o->p_launches.load(), o->persist);
  });
  m.def("owner_stop", [](u h) {
    auto* o = reinterpret_cast<NativeOwner*>(h);
    o->stop.store(true);
    if (o->th.joinable()) o->th.join();
    if (o->persist) {  // tell the kernel to exit, then wait for its launch to finish
      NativeOwner::st(&o->pctl->stop, 1u);
      (void)hipStreamSynchronize(o->pstream);
      (void)hipStreamDestroy(o->pstream);
      (void)hipHostFree(o->pctl);
      (void)hipHostFree(o->p_in);
      (void)hipHostFree(o->p_out);
    }
    const uint64_t err = o->errors.load();
    for (int i = 0; i < 2; ++i) (void)hipEventDestroy(o->ev[i]);
    delete o;
    return err;
  }, py::call_guard<py::gil_scoped_release>());

  // scaler
  m.def("scaler_partial", [](u X, int64_t n, int ld, int d, u pivot, u partial, int nblocks, u s) {
    fdx::launch_scaler_partial(P<const float>(X), n, ld, d, P<const float>(pivot), P<double>(partial), nblocks, S(s));
  });
  m.def("scaler_reduce_scratch_rows", &fdx::scaler_reduce_scratch_rows);
  m.def("scaler_reduce", [](u partial, int nblocks, u sums, u s) {
    fdx::launch_scaler_reduce(P<const double>(partial), nblocks, P<double>(sums), S(s));
  });
  m.def("scaler_reduce_level1", [](u partial, int nblocks, u mid, u s) {
    return fdx::launch_scaler_reduce_level1(P<const double>(partial), nblocks, P<double>(mid), S(s));
  });
  m.def("scaler_finalize", [](u sums, double n, u pivot, int d, u mean64, u var64, u scale64, u mean32, u inv32,
                              u aff, u s, u colscale, int nparts) {
    fdx::launch_scaler_finalize(P<const double>(sums), n, P<const float>(pivot), d, P<double>(mean64), P<double>(var64),
                                P<double>(scale64), P<float>(mean32), P<float>(inv32), P<double>(aff), S(s),
                                P<const float>(colscale), nparts);
  }, py::arg("sums"), py::arg("n"), py::arg("pivot"), py::arg("d"), py::arg("mean64"), py::arg("var64"),
     py::arg("scale64"), py::arg("mean32"), py::arg("inv32"), py::arg("aff"), py::arg("s"), py::arg("colscale"),
     py::arg("nparts") = 1);
  m.def("fp8_hw_check", [](u dec, u vals, int n, u enc, u s) {
    fdx::launch_fp8_hw_check(P<float>(dec), P<const float>(vals), n, P<uint8_t>(enc), S(s));
  });
  m.def("fp8_prescale_blocks", []() { return fdx::fp8_prescale_blocks(); });
  m.def("fp8_prescale", [](u X, int64_t n, int d, int64_t ns, int64_t stride, u partial, u sums, u mu, u k, u s) {
    fdx::launch_fp8_prescale(P<const float>(X), n, d, ns, stride, P<double>(partial), P<double>(sums), P<float>(mu),
                             P<float>(k), S(s));
  });
  m.def("scaler_stats_cast_blocks", [](int fp8) { return fdx::scaler_stats_cast_blocks(fp8); }, py::arg("fp8") = 0);
  m.def("scaler_stats_cast", [](u X, int64_t n, int d, u pivot, u labels, float bias_value, u out, u partial,
                                int nblocks, u s, u colscale, float out_scale, u idx) {
    fdx::launch_scaler_stats_cast(P<const float>(X), n, d, P<const float>(pivot), P<const uint8_t>(labels), bias_value,
                                  P<void>(out), P<double>(partial), nblocks, S(s), P<const float>(colscale), out_scale,
                                  P<const int64_t>(idx));
  }, py::arg("X"), py::arg("n"), py::arg("d"), py::arg("pivot"), py::arg("labels"), py::arg("bias_value"),
     py::arg("out"), py::arg("partial"), py::arg("nblocks"), py::arg("s"), py::arg("colscale") = 0,
     py::arg("out_scale") = 1.0f, py::arg("idx") = 0);
  m.def("scale_cast", [](u X, int64_t n, int ld, int d, u idx, u mean32, u inv32, u labels, float bias_value,
                         float out_scale, int out_kind, u out, u s) {
    fdx::launch_scale_cast(P<const float>(X), n, ld, d, P<const int64_t>(idx), P<const float>(mean32),
                           P<const float>(inv32), P<const uint8_t>(labels), bias_value, out_scale, out_kind,
                           P<void>(out), S(s));
  });
  m.def("compact_count", [](u labels, int64_t n, int target, u counts, int nblocks, u s) {
    fdx::launch_compact_count(P<const uint8_t>(labels), n, target, P<int64_t>(counts), nblocks, S(s));
  });
  m.def("exclusive_scan_small", [](u a, int n, u total, u s, u host_total) {
    fdx::launch_exclusive_scan_small(P<int64_t>(a), n, P<int64_t>(total), S(s), P<int64_t>(host_total));
  }, py::arg("a"), py::arg("n"), py::arg("total"), py::arg("s"), py::arg("host_total") = 0);
  m.def("compact_write", [](u labels, int64_t n, int target, u offsets, u out_idx, int nblocks, u s) {
    fdx::launch_compact_write(P<const uint8_t>(labels), n, target, P<const int64_t>(offsets), P<int64_t>(out_idx),
                              nblocks, S(s));
  });
  m.def("strat_assign", [](u labels, int64_t n, u offsets, u total, uint32_t seed, double test_frac, int k, u out,
                           int nblocks, u s) {
    fdx::launch_strat_assign(P<const uint8_t>(labels), n, P<const int64_t>(offsets), P<const int64_t>(total), seed,
                             test_frac, k, P<uint8_t>(out), nblocks, S(s));
  });

  // predict / linear shap
  m.def("predict_bf16", [](u X, int64_t n, u w, u prob, u logit, u s) {
    fdx::launch_predict_bf16(P<const uint16_t>(X), n, P<const float>(w), P<float>(prob), P<float>(logit), S(s));
  });
  m.def("predict_fp8", [](u X, int64_t n, u w, u prob, u logit, u s) {
    fdx::launch_predict_fp8(P<const uint8_t>(X), n, P<const float>(w), P<float>(prob), P<float>(logit), S(s));
  });
  m.def("predict_shap", [](u X, int in_kind, int64_t n, int ld, int dz, int dphi, u a, u c, float bias, u prob,
                           u logit, u phi, int ld_phi, u s) {
    fdx::launch_predict_shap(P<const void>(X), in_kind, n, ld, dz, dphi, P<const float>(a), P<const float>(c), bias,
                             P<float>(prob), P<float>(logit), P<float>(phi), ld_phi, S(s));
  });
  // GPU-owner batch (serve/gpu_owner.py): launch + wait in one call with the GIL released, so the
  // owner thread never holds the interpreter while the device works
  m.def("predict_shap_sync", [](u X, int in_kind, int64_t n, int ld, int dz, int dphi, u a, u c, float bias, u prob,
                                u logit, u phi, int ld_phi, u s) {
    fdx::launch_predict_shap(P<const void>(X), in_kind, n, ld, dz, dphi, P<const float>(a), P<const float>(c), bias,
                             P<float>(prob), P<float>(logit), P<float>(phi), ld_phi, S(s));
    stream_sync(s);
  }, py::call_guard<py::gil_scoped_release>());

  m.def("predict_gather_logit", [](u X, u idx, int64_t n, int d, u w, u mean, u scale, u logit, u s) {
    fdx::launch_predict_gather_logit(P<const float>(X), P<const int64_t>(idx), n, d, P<const double>(w),
                                     P<const double>(mean), P<const double>(scale), P<float>(logit), S(s));
  });

  // logistic regression
  m.def("logreg_pass_blocks", &fdx::logreg_pass_blocks, py::arg("fmt") = 0);
  auto hole_of = [](int64_t at, int64_t len) {
    fdx::RowHole h;
    h.at = at;
    h.len = len;
    return h;
  };
  // nf (optional): (red, ws, state, w32, done, aff, done_host, C, tol, d, max_iter, fit_intercept,
  // phase_start, seq) -- the pass also reduces and applies the Newton update (launchers.h NewtonFuse)
  auto nf_of = [](const py::object& o, fdx::NewtonFuse& f) -> const fdx::NewtonFuse* {
    if (o.is_none()) return nullptr;
    const py::tuple t = o.cast<py::tuple>();
    if (t.size() != 14) throw std::runtime_error("logreg_pass: nf must have 14 entries");
    f.red = P<double>(t[0].cast<u>());
    f.ws = P<unsigned long long>(t[1].cast<u>());
    f.st = P<double>(t[2].cast<u>());
    f.w32 = P<float>(t[3].cast<u>());
    f.done = P<int>(t[4].cast<u>());
    f.aff = P<const double>(t[5].cast<u>());
    f.done_host = P<int>(t[6].cast<u>());
    f.C = t[7].cast<double>();
    f.tol = t[8].cast<double>();
    f.d = t[9].cast<int>();
    f.max_iter = t[10].cast<int>();
    f.fit_intercept = t[11].cast<int>();
    f.phase_start = t[12].cast<int>();
    f.seq = t[13].cast<int>();
    return &f;
  };
  m.attr("NEWTON_FUSE_WORDS") = fdx::kNewtonFuseWords;
  m.def("logreg_pass", [hole_of, nf_of](u X, int64_t rb, int64_t re, u w, u cw, u done, int hess, int sub, u partial,
                                        int nblocks, u s, int phase, bool fisher, int64_t hole_at, int64_t hole_len,
                                        py::object nf) {
    fdx::NewtonFuse f;
    fdx::launch_logreg_pass(P<const uint16_t>(X), rb, re, P<const float>(w), P<const float>(cw), P<const int>(done),
                            hess, sub, P<float>(partial), nblocks, S(s), nullptr, phase, fisher, hole_of(hole_at, hole_len),
                            nf_of(nf, f));
  }, py::arg("X"), py::arg("rb"), py::arg("re"), py::arg("w"), py::arg("cw"), py::arg("done"), py::arg("hess"),
     py::arg("sub"), py::arg("partial"), py::arg("nblocks"), py::arg("s"), py::arg("phase") = 0,
     py::arg("fisher") = false, py::arg("hole_at") = 0, py::arg("hole_len") = 0, py::arg("nf") = py::none());
  // the same pass over the stored rows [0, n_real) plus virtual SMOTE samples (launchers.h
  // SmoteView); x_scale > 0 selects the fp8 row pass
  m.def("logreg_pass_virtual", [hole_of, nf_of](u X, int64_t rb, int64_t re, u w, u cw, u done, int hess, int sub,
                                                u partial, int nblocks, u s, u parents, u nbr, u lam, u off, u cnt,
                                                int64_t n_real, int64_t q_offset, int mq, int k, float x_scale,
                                                int phase, bool fisher, int64_t hole_at, int64_t hole_len,
                                                py::object nf) {
    fdx::NewtonFuse f;
    const fdx::NewtonFuse* nfp = nf_of(nf, f);
    fdx::SmoteView v;
    v.parents = P<const uint16_t>(parents);
    v.nbr = P<const int>(nbr);
    v.lam = P<const uint16_t>(lam);
    v.off = P<const int>(off);
    v.cnt = P<const int>(cnt);
    v.n_real = n_real;
    v.q_offset = q_offset;
    v.mq = mq;
    v.k = k;
    if (x_scale > 0.0f)
      fdx::launch_logreg_pass_fp8(P<const uint8_t>(X), rb, re, P<const float>(w), P<const float>(cw),
                                  P<const int>(done), hess, sub, x_scale, P<float>(partial), nblocks, S(s), &v, phase,
                                  fisher, hole_of(hole_at, hole_len), nfp);
    else
      fdx::launch_logreg_pass(P<const uint16_t>(X), rb, re, P<const float>(w), P<const float>(cw),
                              P<const int>(done), hess, sub, P<float>(partial), nblocks, S(s), &v, phase, fisher,
                              hole_of(hole_at, hole_len), nfp);
  }, py::arg("X"), py::arg("rb"), py::arg("re"), py::arg("w"), py::arg("cw"), py::arg("done"), py::arg("hess"),
     py::arg("sub"), py::arg("partial"), py::arg("nblocks"), py::arg("s"), py::arg("parents"), py::arg("nbr"),
     py::arg("lam"), py::arg("off"), py::arg("cnt"), py::arg("n_real"), py::arg("q_offset"), py::arg("mq"),
     py::arg("k"), py::arg("x_scale"), py::arg("phase") = 0, py::arg("fisher") = false, py::arg("hole_at") = 0,
     py::arg("hole_len") = 0, py::arg("nf") = py::none());
  m.def("smote_bucket_bins", &fdx::smote_bucket_bins);
  m.def("smote_bucket_blocks", &fdx::smote_bucket_blocks);
  m.def("smote_bucket_max_picks", []() { return (uint64_t)fdx::kSmoteBucketMaxPicks; });
  m.def("smote_bucket_max_samples", &fdx::smote_bucket_max_samples);
  m.def("smote_bucket", [](int stage, int mq, int k, int64_t n_new, int64_t sample_offset, uint64_t seed,
                           uint64_t counter_base, u table, u rec, u tmp, u pstart, u pcnt, u lam, u bump, u s) {
    fdx::launch_smote_bucket(stage, mq, k, n_new, sample_offset, seed, counter_base, P<int>(table),
                             P<uint32_t>(rec), P<uint32_t>(tmp), P<int>(pstart), P<int>(pcnt), P<uint16_t>(lam),
                             P<unsigned long long>(bump), S(s));
  });
  m.def("logreg_pass_fp8", [hole_of, nf_of](u X, int64_t rb, int64_t re, u w, u cw, u done, int hess, int sub,
                                            float xs, u partial, int nblocks, u s, int phase, bool fisher,
                                            int64_t hole_at, int64_t hole_len, py::object nf) {
    fdx::NewtonFuse f;
    fdx::launch_logreg_pass_fp8(P<const uint8_t>(X), rb, re, P<const float>(w), P<const float>(cw),
                                P<const int>(done), hess, sub, xs, P<float>(partial), nblocks, S(s), nullptr, phase,
                                fisher, hole_of(hole_at, hole_len), nf_of(nf, f));
  }, py::arg("X"), py::arg("rb"), py::arg("re"), py::arg("w"), py::arg("cw"), py::arg("done"), py::arg("hess"),
     py::arg("sub"), py::arg("xs"), py::arg("partial"), py::arg("nblocks"), py::arg("s"), py::arg("phase") = 0,
     py::arg("fisher") = false, py::arg("hole_at") = 0, py::arg("hole_len") = 0, py::arg("nf") = py::none());
  m.def("newton_update_stamped", [](u red, u state, u w32, u done, double C, u aff, u stamps, u s) {
    fdx::launch_newton_update_stamped(P<const double>(red), P<double>(state), P<float>(w32), P<int>(done), C,
                                      P<const double>(aff), P<unsigned long long>(stamps), S(s));
  });
  m.def("logreg_reduce", [](u partial, int nblocks, int ncols, u out, u done, u s) {
    fdx::launch_logreg_reduce(P<const float>(partial), nblocks, ncols, P<double>(out), P<const int>(done), S(s));
  });
  m.def("newton_update", [](u red, u state, u w32, u done, int d, double C, double tol, int max_iter, int fi,
                            int phase_start, u aff, u s, u done_host, int seq) {
    fdx::launch_newton_update(P<const double>(red), P<double>(state), P<float>(w32), P<int>(done), d, C, tol,
                              max_iter, fi, phase_start, P<const double>(aff), S(s), P<int>(done_host), seq);
  }, py::arg("red"), py::arg("state"), py::arg("w32"), py::arg("done"), py::arg("d"), py::arg("C"), py::arg("tol"),
     py::arg("max_iter"), py::arg("fi"), py::arg("phase_start"), py::arg("aff"), py::arg("s"), py::arg("done_host") = 0,
     py::arg("seq") = 0);
  m.def("logreg_init", [](u state, u w32, u class_w, u done, std::vector<double> w0, double cw0, double cw1, u aff,
                          u s, u w0_dev, u persist_ws) {
    if (w0.size() != 32) throw std::runtime_error("logreg_init: w0 must have 32 entries");
    fdx::LRInitArgs a;
    for (int j = 0; j < 32; ++j) a.w0[j] = w0[j];
    a.cw0 = (float)cw0;
    a.cw1 = (float)cw1;
    fdx::launch_logreg_init(a, P<double>(state), P<float>(w32), P<float>(class_w), P<int>(done),
                            P<const double>(aff), S(s), P<const double>(w0_dev),
                            P<unsigned long long>(persist_ws));
  }, py::arg("state"), py::arg("w32"), py::arg("class_w"), py::arg("done"), py::arg("w0"), py::arg("cw0"),
     py::arg("cw1"), py::arg("aff"), py::arg("s"), py::arg("w0_dev") = 0, py::arg("persist_ws") = 0);
  m.def("logreg_export", [](u state, u host_dev, u s, long long seq) {
    fdx::launch_logreg_export(P<const double>(state), P<double>(host_dev), S(s), seq);
  }, py::arg("state"), py::arg("host_dev"), py::arg("s"), py::arg("seq") = 0);
  m.def("logreg_fold", [](u state, u aff, u w32, u s) {
    fdx::launch_logreg_fold(P<const double>(state), P<const double>(aff), P<float>(w32), S(s));
  });
  auto sgd_args = [](int d, double C, double c, double mom, int fi, int nb, int avg, int epoch_end, double tol) {
    fdx::SgdArgs a;
    a.d = d; a.C = C; a.c = c; a.momentum = mom; a.fit_intercept = fi; a.nb = nb; a.avg = avg;
    a.epoch_end = epoch_end; a.tol = tol;
    return a;
  };
  m.def("sgd_step", [sgd_args](u partial, int nblocks, u state, u w32, u done, u aff, int d, double C, double c,
                               double mom, int fi, int nb, int avg, int epoch_end, double tol, u s) {
    fdx::launch_sgd_step(P<const float>(partial), nblocks, P<double>(state), P<float>(w32), P<int>(done),
                         P<const double>(aff), sgd_args(d, C, c, mom, fi, nb, avg, epoch_end, tol), S(s));
  });
  // The whole single-process SGD schedule in one call: steps [s0, s1) of epochs x nb minibatches,
  // each one FISH pass (row phase b) + the fused reduce/update -- no Python per step (the host
  // enqueue of two launches per step from Python was ~as long as the device step).
  m.def("sgd_run", [sgd_args](u X, int fp8, float x_scale, int64_t end, u w32, u cw, u done, u partial, int blocks,
                              u s, u parents, u nbr, u lam, u off, u cnt, int64_t n_real, int64_t q_offset, int mq,
                              int k, int64_t hole_at, int64_t hole_len, u state, u aff, int d, double C, double mom,
                              int fi, double tol, int nb, int epochs, int avg_from, std::vector<double> lrs, int s0,
                              int s1, u acc, u ticket, std::vector<int> subs, std::vector<int> nbs) {
    if (nb < 1 || epochs < 1 || (int)lrs.size() < epochs || (int)subs.size() < epochs || (int)nbs.size() < epochs)
      throw std::runtime_error("sgd_run: bad schedule");
    std::vector<int> estart(epochs + 1, 0);  // first step of every epoch (per-epoch minibatch counts)
    for (int e = 0; e < epochs; ++e) {
      if (nbs[e] < 1) throw std::runtime_error("sgd_run: minibatch counts must be >= 1");
      estart[e + 1] = estart[e] + nbs[e];
    }
    if (s0 < 0 || s1 > estart[epochs]) throw std::runtime_error("sgd_run: bad step range");
    fdx::SmoteView v;
    const fdx::SmoteView* vp = nullptr;
    if (parents) {
      v.parents = P<const uint16_t>(parents);
      v.nbr = P<const int>(nbr);
      v.lam = P<const uint16_t>(lam);
      v.off = P<const int>(off);
      v.cnt = P<const int>(cnt);
      v.n_real = n_real;
      v.q_offset = q_offset;
      v.mq = mq;
      v.k = k;
      vp = &v;
    }
    fdx::RowHole h;
    h.at = hole_at;
    h.len = hole_len;
    for (int st = s0; st < s1; ++st) {
      int ep = 0;
      while (ep + 1 < epochs && st >= estart[ep + 1]) ++ep;
      const int nbe = nbs[ep], b = st - estart[ep], sub = subs[ep];
      // sub-sampled epoch: phase b * sub of a grid of nbe * sub minibatches; never decides convergence
      const int rsub = nbe * sub, ph = b * sub;
      const fdx::SgdArgs a = sgd_args(d, C, lrs[ep], mom, fi, rsub, ep >= avg_from, b == nbe - 1,
                                      sub > 1 ? -1.0 : tol);
      if (acc) {  // one launch per step (fixed-point atomics + last-block update)
        fdx::launch_sgd_pass_fused(P<const void>(X), fp8, x_scale, end, P<float>(w32), P<const float>(cw), P<int>(done),
                                   rsub, ph, blocks, vp, h, P<unsigned long long>(acc), P<unsigned int>(ticket),
                                   P<double>(state), P<const double>(aff), a, S(s));
        continue;
      }
      if (fp8)
        fdx::launch_logreg_pass_fp8(P<const uint8_t>(X), 0, end, P<const float>(w32), P<const float>(cw),
                                    P<const int>(done), 0, rsub, x_scale, P<float>(partial), blocks, S(s), vp, ph, true, h);
      else
        fdx::launch_logreg_pass(P<const uint16_t>(X), 0, end, P<const float>(w32), P<const float>(cw),
                                P<const int>(done), 0, rsub, P<float>(partial), blocks, S(s), vp, ph, true, h);
      fdx::launch_sgd_step(P<const float>(partial), blocks, P<double>(state), P<float>(w32), P<int>(done),
                           P<const double>(aff), a, S(s));
    }
  });
  m.def("sgd_update", [sgd_args](u red, u state, u w32, u done, u aff, int d, double C, double c, double mom, int fi,
                                 int nb, int avg, int epoch_end, double tol, u s) {
    fdx::launch_sgd_update(P<const double>(red), P<double>(state), P<float>(w32), P<int>(done), P<const double>(aff),
                           sgd_args(d, C, c, mom, fi, nb, avg, epoch_end, tol), S(s));
  });
  auto smote_view = [](u parents, u nbr, u lam, u off, u cnt, int64_t n_real, int64_t q_offset, int mq, int k) {
    fdx::SmoteView v;
    if (parents) {
      v.parents = P<const uint16_t>(parents);
      v.nbr = P<const int>(nbr);
      v.lam = P<const uint16_t>(lam);
      v.off = P<const int>(off);
      v.cnt = P<const int>(cnt);
      v.n_real = n_real;
      v.q_offset = q_offset;
      v.mq = mq;
      v.k = k;
    }
    return v;
  };
  // One process: steps [s0, s1) of the schedule in ONE persistent launch (logreg.hip
  // sgd_persist_kernel).  Gw: waves of the per-step pass grid (4 x its blocks) -- the minibatch
  // partition.  ws: int64 [kSgdPersistWords] scratch (zeroed by the launcher).
  m.def("sgd_persist", [smote_view](u X, int fp8, float x_scale, int64_t end, u cw, u parents, u nbr, u lam, u off,
                                    u cnt, int64_t n_real, int64_t q_offset, int mq, int k, int64_t hole_at,
                                    int64_t hole_len, u ws, u state, u w32, u done, u aff, int d, double C, double mom,
                                    int fi, double tol, int nb, int epochs, int avg_from, int serpentine,
                                    std::vector<double> lrs, int s0, int s1, int64_t Gw, u s, u stamps,
                                    std::vector<int> subs, std::vector<int> nbs, int fault_test,
                                    unsigned spin_limit, u export_host, int prepped, long long export_seq) -> int {
    if ((int)lrs.size() < epochs || epochs > fdx::kSgdMaxEpochs) throw std::runtime_error("sgd_persist: bad lrs");
    if ((int)subs.size() < epochs) throw std::runtime_error("sgd_persist: one sub-sample factor per epoch");
    if ((int)nbs.size() < epochs) throw std::runtime_error("sgd_persist: one minibatch count per epoch");
    const fdx::SmoteView v = smote_view(parents, nbr, lam, off, cnt, n_real, q_offset, mq, k);
    fdx::RowHole h;
    h.at = hole_at;
    h.len = hole_len;
    fdx::SgdPersistArgs a;
    a.ws = P<unsigned long long>(ws);
    a.st = P<double>(state);
    a.w32 = P<float>(w32);
    a.done = P<int>(done);
    a.aff = P<const double>(aff);
    a.C = C;
    a.momentum = mom;
    a.tol = tol;
    a.estart[0] = 0;
    for (int e = 0; e < epochs; ++e) {
      a.lr[e] = lrs[e];
      if (subs[e] < 1) throw std::runtime_error("sgd_persist: sub-sample factors must be >= 1");
      if (nbs[e] < 1) throw std::runtime_error("sgd_persist: minibatch counts must be >= 1");
      a.sub[e] = subs[e];
      a.nbe[e] = nbs[e];
      a.estart[e + 1] = a.estart[e] + nbs[e];
    }
    a.d = d;
    a.fit_intercept = fi;
    a.nb = nb;
    a.epochs = epochs;
    a.avg_from = avg_from;
    a.serpentine = serpentine;
    a.s0 = s0;
    a.s1 = s1;
    a.Gw = Gw;
    a.stamps = P<unsigned long long>(stamps);
    a.fault_test = fault_test;
    if (spin_limit > 0) a.spin_limit = spin_limit;
    a.export_host = P<double>(export_host);
    a.prepped = prepped;
    a.export_seq = export_seq;
    // 0: enqueued; 1: the cooperative launch refused the grid (the caller launches per step)
    return fdx::launch_sgd_persist(P<const void>(X), fp8, x_scale, end, P<const float>(cw), parents ? &v : nullptr, h,
                                   a, S(s));
  }, py::arg("X"), py::arg("fp8"), py::arg("x_scale"), py::arg("end"), py::arg("cw"), py::arg("parents"),
     py::arg("nbr"), py::arg("lam"), py::arg("off"), py::arg("cnt"), py::arg("n_real"), py::arg("q_offset"),
     py::arg("mq"), py::arg("k"), py::arg("hole_at"), py::arg("hole_len"), py::arg("ws"), py::arg("state"),
     py::arg("w32"), py::arg("done"), py::arg("aff"), py::arg("d"), py::arg("C"), py::arg("mom"), py::arg("fi"),
     py::arg("tol"), py::arg("nb"), py::arg("epochs"), py::arg("avg_from"), py::arg("serpentine"), py::arg("lrs"),
     py::arg("s0"), py::arg("s1"), py::arg("Gw"), py::arg("s"), py::arg("stamps"), py::arg("subs"), py::arg("nbs"),
     py::arg("fault_test") = 0, py::arg("spin_limit") = 0u, py::arg("export_host") = 0, py::arg("prepped") = 0,
     py::arg("export_seq") = 0);
  m.def("sgd_persist_blocks", [](int grid_blocks) { return fdx::sgd_persist_blocks(grid_blocks); });
  m.def("sgd_full_blocks", []() { return fdx::sgd_full_blocks(); });
  m.attr("SGD_PERSIST_WORDS") = fdx::kSgdPersistWords;
  // Data parallel lean step: FISH pass -> fixed-point sums[36] (int64) for the all-reduce, then the
  // update from the reduced sums.
  m.def("sgd_pass_sums", [smote_view](u X, int fp8, float x_scale, int64_t end, u w32, u cw, u done, int nb, int b,
                                      int blocks, u parents, u nbr, u lam, u off, u cnt, int64_t n_real,
                                      int64_t q_offset, int mq, int k, int64_t hole_at, int64_t hole_len, u acc,
                                      u ticket, u sums, u aff, u s) {
    const fdx::SmoteView v = smote_view(parents, nbr, lam, off, cnt, n_real, q_offset, mq, k);
    fdx::RowHole h;
    h.at = hole_at;
    h.len = hole_len;
    fdx::launch_sgd_pass_sums(P<const void>(X), fp8, x_scale, end, P<const float>(w32), P<const float>(cw),
                              P<const int>(done), nb, b, blocks, parents ? &v : nullptr, h,
                              P<unsigned long long>(acc), P<unsigned int>(ticket), P<long long>(sums),
                              P<const double>(aff), S(s));
  });
  m.def("sgd_update_fixed", [sgd_args](u sums, u state, u w32, u done, u aff, int d, double C, double c, double mom,
                                       int fi, int nb, int avg, int epoch_end, double tol, u s) {
    fdx::launch_sgd_update_fixed(P<const long long>(sums), P<double>(state), P<float>(w32), P<int>(done),
                                 P<const double>(aff), sgd_args(d, C, c, mom, fi, nb, avg, epoch_end, tol), S(s));
  });

  // knn / smote
  m.def("knn_prep", [](u X, int m_, int m_pad, int role, u out, u s, u outq, u aff, u parents, u chl, u qhl,
                       u tmax) {
    fdx::launch_knn_prep(P<const float>(X), m_, m_pad, role, P<float>(out), P<float>(outq),
                         P<const double>(aff), P<uint16_t>(parents), S(s), P<void>(chl), P<void>(qhl), P<float>(tmax));
  }, py::arg("X"), py::arg("m"), py::arg("m_pad"), py::arg("role"), py::arg("out"), py::arg("s"),
     py::arg("outq") = 0, py::arg("aff") = 0, py::arg("parents") = 0, py::arg("chl") = 0, py::arg("qhl") = 0,
     py::arg("tmax") = 0);
  m.def("knn_splits", [](int mq_pad, int mc_pad) { return fdx::knn_splits(mq_pad, mc_pad); });
  m.def("knn_lds_splits", [](int mq_pad, int mc_pad) { return fdx::knn_lds_splits(mq_pad, mc_pad); });
  m.def("knn_topk_lds", [](u Q, int mq_pad, int mq, u C, int mc_pad, int mc, int64_t self_off, int k, u oidx,
                           u oscore, u ws_score, u ws_idx, int nsplit, u s) {
    fdx::launch_knn_topk_lds(P<const float>(Q), mq_pad, mq, P<const float>(C), mc_pad, mc, self_off, k, P<int>(oidx),
                             P<float>(oscore), P<float>(ws_score), P<int>(ws_idx), nsplit, S(s));
  });
  m.def("knn3_splits", [](int mq_pad, int mc_pad) { return fdx::knn3_splits(mq_pad, mc_pad); });
  m.def("knn_split", [](u Xp, int m_pad, int role, u hl, u tmax, u s) {
    fdx::launch_knn_split(P<const float>(Xp), m_pad, role, P<uint4>(hl), P<float>(tmax), S(s));
  });
  m.def("knn_topk3", [](u Q, u Qhl, int mq_pad, int mq, u C, u Chl, u tmax, int mc_pad, int mc, int64_t self_off,
                        int k, u oidx, u oscore, u wss, u wsi, int nsplit, u s) {
    fdx::launch_knn_topk3(P<const float>(Q), P<const void>(Qhl), mq_pad, mq, P<const float>(C), P<const void>(Chl),
                          P<const float>(tmax), mc_pad, mc, self_off, k, P<int>(oidx), P<float>(oscore),
                          P<float>(wss), P<int>(wsi), nsplit, S(s));
  });
  m.def("knn_b3top_splits", [](int mq_pad, int mc_pad) { return fdx::knn_b3top_splits(mq_pad, mc_pad); });
  m.def("knn_b3top", [](u Q, u Qhl, int mq_pad, int mq, u C, u Chl, u tmax, int mc_pad, int mc, int64_t self_off,
                        int k, u oidx, u oscore, u wss, u wsi, u wsm, u fail, int nsplit, u s) {
    fdx::launch_knn_b3top(P<const float>(Q), P<const void>(Qhl), mq_pad, mq, P<const float>(C), P<const void>(Chl),
                          P<const float>(tmax), mc_pad, mc, self_off, k, P<int>(oidx), P<float>(oscore),
                          P<float>(wss), P<int>(wsi), P<float>(wsm), P<int>(fail), nsplit, S(s));
  });
  m.def("knn3r_splits", [](int mq_pad, int mc_pad) { return fdx::knn3r_splits(mq_pad, mc_pad); });
  m.attr("KNN3R_LIST_CAP") = fdx::knn3r_list_cap();
  m.def("knn_topk3r", [](u Q, u Qhl, int mq_pad, int mq, u C, u Chl, u tmax, int mc_pad, int mc, int64_t self_off,
                         int k, u oidx, u oscore, u lists, u counts, int nsplit, u s) {
    fdx::launch_knn_topk3r(P<const float>(Q), P<const void>(Qhl), mq_pad, mq, P<const float>(C), P<const void>(Chl),
                           P<const float>(tmax), mc_pad, mc, self_off, k, P<int>(oidx), P<float>(oscore),
                           P<int>(lists), P<int>(counts), nsplit, S(s));
  });
  m.def("knn_topk", [](u Q, int mq_pad, int mq, u C, int mc_pad, int mc, int64_t self_off, int k, u oidx,
                       u oscore, u ws_score, u ws_idx, int nsplit, u s) {
    fdx::launch_knn_topk(P<const float>(Q), mq_pad, mq, P<const float>(C), mc_pad, mc,
                         self_off, k, P<int>(oidx), P<float>(oscore), P<float>(ws_score), P<int>(ws_idx), nsplit,
                         S(s));
  });
  m.def("smote_parents", [](u C, int64_t m_rows, u aff, u out, u s) {
    fdx::launch_smote_parents(P<const float>(C), m_rows, P<const double>(aff), P<uint16_t>(out), S(s));
  });
  m.def("smote_generate", [](u C, int parents_bf16, u nbr, int mq, int k, int64_t q_off, int64_t n_new,
                             int64_t sample_offset, uint64_t seed, uint64_t counter_base, float label, int out_kind,
                             float out_scale, u aff, u out, u s) {
    fdx::launch_smote_generate(P<const void>(C), parents_bf16, P<const int>(nbr), mq, k, q_off, n_new, sample_offset,
                               seed, counter_base, label, out_kind, out_scale, P<const double>(aff), P<void>(out), S(s));
  });

  // kernelshap
  m.def("kernelshap", [](u X, int E, int d, u a, float bias, u bg, u cb, int nbg, u Z, int nS, int S_pad, int parts,
                         u A, u Az, int link, u phi, u fx, u f0, u ws, u cnt, u s, u stamps) {
    fdx::launch_kernelshap(P<const float>(X), E, d, P<const float>(a), bias, P<const float>(bg), P<const float>(cb),
                           nbg, P<const uint16_t>(Z), nS, S_pad, parts, P<const float>(A), P<const float>(Az), link,
                           P<float>(phi), P<float>(fx), P<float>(f0), P<float>(ws), P<unsigned>(cnt), S(s),
                           P<unsigned long long>(stamps));
  });
  m.def("kernelshap_paired", [](u X, int E, int d, u a, float bias, u bg, u cb, int nbg, u Z, int Ppad, int parts,
                                u A, u Az, int link, u phi, u fx, u f0, u ws, u cnt, u s) {
    fdx::launch_kernelshap_paired(P<const float>(X), E, d, P<const float>(a), bias, P<const float>(bg),
                                  P<const float>(cb), nbg, P<const uint32_t>(Z), Ppad, parts, P<const float>(A),
                                  P<const float>(Az), link, P<float>(phi), P<float>(fx), P<float>(f0), P<float>(ws),
                                  P<unsigned>(cnt), S(s));
  });
  m.def("kernelshap_linear_resident", [](int S_pad, int parts) { return fdx::kernelshap_linear_resident(S_pad, parts); });
  m.def("treeshap", [](u Xs, int ldx, int E, int d, u feat, u thr, u leaf, int T, int depth, float base, u bw,
                       int bw_ld, int n_bg, float f0, u phi, u fx, u f0o, u s) {
    fdx::launch_treeshap(P<const float>(Xs), ldx, E, d, P<const int>(feat), P<const float>(thr), P<const float>(leaf),
                         T, depth, base, P<const uint32_t>(bw), bw_ld, n_bg, f0, P<float>(phi), P<float>(fx),
                         P<float>(f0o), S(s));
  });
  m.def("kernelshap_tree", [](u Xs, int ldx, int E, int d, u feat, u thr, u leaf, int T, int depth, float base, u bw,
                              int bw_ld, int nbg, u Zm, int nS, int S_pad, int parts, u A, u Az, int link, u phi,
                              u fx, u f0, u ws, u cnt, u s) {
    fdx::launch_kernelshap_tree(P<const float>(Xs), ldx, E, d, P<const int>(feat), P<const float>(thr),
                                P<const float>(leaf), T, depth, base, P<const uint32_t>(bw), bw_ld, nbg,
                                P<const uint32_t>(Zm), nS, S_pad, parts, P<const float>(A), P<const float>(Az), link,
                                P<float>(phi), P<float>(fx), P<float>(f0), P<float>(ws), P<unsigned>(cnt), S(s));
  });

  // gbdt (K11)
  m.def("gbdt_bin", [](u X, int64_t n, int ld, int d, u cuts, u nbins, u bins, u s) {
    fdx::launch_gbdt_bin(P<const float>(X), n, ld, d, P<const float>(cuts), P<const int>(nbins), P<uint8_t>(bins), S(s));
  });
  m.def("gbdt_grad", [](u margin, u label, int64_t n, float spw, float gscale, float hscale, u gh, u s) {
    fdx::launch_gbdt_grad(P<const float>(margin), P<const uint8_t>(label), n, spw, gscale, hscale, P<uint32_t>(gh), S(s));
  });
  m.def("gbdt_hist_blocks", [] { return fdx::gbdt_hist_blocks(); });
  m.def("quantile_select_ws_bytes", [](int64_t m, int d) { return fdx::quantile_select_ws_bytes(m, d); });
  m.def("quantile_select", [](u X, int64_t m, int64_t stride, int ld, int d, int max_bin, u ws, u out, u s) {
    fdx::launch_quantile_select(P<const float>(X), m, stride, ld, d, max_bin, P<void>(ws), P<float>(out), S(s));
  });
  m.def("gbdt_hist_slot_words", [] { return fdx::gbdt_hist_slot_words(); });
  m.def("set_gbdt_hist_variant", [](int v) { fdx::set_gbdt_hist_variant(v); });
  m.def("gbdt_hist", [](u bins, u gh, u ridx, u seg, u gcnt, int level, int d, u hist, u slots, u s,
                        int64_t flush_rows, int64_t hole_at, int64_t hole_len) {
    fdx::launch_gbdt_hist(P<const uint8_t>(bins), P<const uint32_t>(gh), P<const int>(ridx), P<const int64_t>(seg),
                          P<const int64_t>(gcnt), level, d, P<unsigned long long>(hist), P<long long>(slots), S(s),
                          flush_rows, hole_at, hole_len);
  }, py::arg("bins"), py::arg("gh"), py::arg("ridx"), py::arg("seg"), py::arg("gcnt"), py::arg("level"),
     py::arg("d"), py::arg("hist"), py::arg("slots"), py::arg("s"), py::arg("flush_rows") = 0,
     py::arg("hole_at") = 0, py::arg("hole_len") = 0);
  m.def("gbdt_hist_l0_fused", [](u bins, u gh, u seg, u gcnt, int d, u hist, u slots, u s, int64_t flush_rows,
                                 int64_t hole_at, int64_t hole_len, u feat, u bin, u leaf, int depth, u margin,
                                 u label, float spw, float gscale, float hscale) {
    fdx::launch_gbdt_hist_l0_fused(P<const uint8_t>(bins), P<uint32_t>(gh), P<const int64_t>(seg),
                                   P<const int64_t>(gcnt), d, P<unsigned long long>(hist), P<long long>(slots), S(s),
                                   flush_rows, hole_at, hole_len, P<const int>(feat), P<const int>(bin),
                                   P<const float>(leaf), depth, P<float>(margin), P<const uint8_t>(label), spw, gscale,
                                   hscale);
  });
  m.def("gbdt_split", [](u hist, u gcnt, int level, int d, u nbins, u cuts, double ginv, double hinv, double lam,
                         double mcw, double gamma, u feat, u bin, u thr, u gain, u ng, u nh, u s) {
    fdx::launch_gbdt_split(P<unsigned long long>(hist), P<const int64_t>(gcnt), level, d, P<const int>(nbins),
                           P<const float>(cuts), ginv, hinv, lam, mcw, gamma, P<int>(feat), P<int>(bin), P<float>(thr),
                           P<double>(gain), P<long long>(ng), P<long long>(nh), S(s));
  });
  m.def("gbdt_transpose", [](u bins, int64_t n, int d, u binsT, int64_t ldt, u s) {
    fdx::launch_gbdt_transpose(P<const uint8_t>(bins), n, d, P<uint8_t>(binsT), ldt, S(s));
  });
  m.def("gbdt_partition", [](u binsT, int64_t ldt, u ridx, u nid, int64_t n, u feat, u bin, int level, u flag, u counts,
                             int nblocks, u seg, u node_r, u ridx_out, u nid_out, u s, u gcnt, int64_t hole_at,
                             int64_t hole_len) {
    fdx::launch_gbdt_partition(P<const uint8_t>(binsT), ldt, P<const int>(ridx), P<const uint8_t>(nid), n, P<const int>(feat),
                               P<const int>(bin), level, P<uint8_t>(flag), P<int64_t>(counts), nblocks, P<int64_t>(seg),
                               P<int64_t>(node_r), P<int>(ridx_out), P<uint8_t>(nid_out), S(s), P<int64_t>(gcnt),
                               hole_at, hole_len);
  }, py::arg("binsT"), py::arg("ldt"), py::arg("ridx"), py::arg("nid"), py::arg("n"), py::arg("feat"), py::arg("bin"),
     py::arg("level"), py::arg("flag"), py::arg("counts"), py::arg("nblocks"), py::arg("seg"), py::arg("node_r"),
     py::arg("ridx_out"), py::arg("nid_out"), py::arg("s"), py::arg("gcnt") = 0, py::arg("hole_at") = 0,
     py::arg("hole_len") = 0);
  m.def("gbdt_round_init", [](u hist, int64_t hist_words, u seg, u gcnt, int64_t n, int64_t n_global, u s,
                              u node_r, int n_nodes) {
    fdx::launch_gbdt_round_init(P<unsigned long long>(hist), hist_words, P<int64_t>(seg), P<int64_t>(gcnt), n,
                                n_global, S(s), P<int64_t>(node_r), n_nodes);
  });
  m.def("gbdt_leaf", [](u ng, u nh, int depth, double ginv, double hinv, double lam, double mcw, double eta, u leaf,
                        u s) {
    fdx::launch_gbdt_leaf(P<const long long>(ng), P<const long long>(nh), depth, ginv, hinv, lam, mcw, eta,
                          P<float>(leaf), S(s));
  });
  m.def("gbdt_margin", [](u binsT, int64_t ldt, int64_t n, u feat, u bin, u leaf, int depth, u margin, u label,
                          float spw, float gscale, float hscale, u gh, u s) {
    fdx::launch_gbdt_margin(P<const uint8_t>(binsT), ldt, n, P<const int>(feat), P<const int>(bin),
                            P<const float>(leaf), depth, P<float>(margin), P<const uint8_t>(label), spw, gscale,
                            hscale, P<uint32_t>(gh), S(s));
  });
  m.def("gbdt_predict", [](u X, int64_t n, int ld, int d, u feat, u thr, u leaf, int ntrees, int depth, float base,
                           u out, u s) {
    fdx::launch_gbdt_predict(P<const float>(X), n, ld, d, P<const int>(feat), P<const float>(thr), P<const float>(leaf),
                             ntrees, depth, base, P<float>(out), S(s));
  });

  // auc / confusion
  m.def("auc_hist", [](u scores, u labels, int64_t n, int bits, u hist, u s) {
    fdx::launch_auc_hist(P<const float>(scores), P<const uint8_t>(labels), n, bits, P<unsigned>(hist), S(s));
  });
  m.def("auc_hist_reduce", [](u hist, int bits, u out, u s) {
    fdx::launch_auc_hist_reduce(P<const unsigned>(hist), bits, P<unsigned long long>(out), S(s));
  });
  m.def("auc_compact", [](u scores, u labels, int64_t n, u pos, u counter, u s) {
    fdx::launch_auc_compact(P<const float>(scores), P<const uint8_t>(labels), n, P<float>(pos),
                            P<unsigned long long>(counter), S(s));
  });
  m.def("sort_chunks", [](u pos, int64_t cap, u counter, int chunk, int nchunks, u s) {
    fdx::launch_sort_chunks(P<float>(pos), cap, P<const unsigned long long>(counter), chunk, nchunks, S(s));
  });
  m.def("auc_count", [](u scores, u labels, int64_t n, u pos, u counter, int chunk, int nchunks, u out, u s) {
    fdx::launch_auc_count(P<const float>(scores), P<const uint8_t>(labels), n, P<const float>(pos),
                          P<const unsigned long long>(counter), chunk, nchunks, P<unsigned long long>(out), S(s));
  });
  m.def("auc_radix_workspace_bytes", &fdx::auc_radix_workspace_bytes);
  m.def("auc_radix_layout", [](int64_t n) {
    size_t off[8];
    fdx::auc_radix_layout(n, off);
    return std::vector<size_t>(off, off + 8);
  });
  m.def("auc_radix", [](u scores, u labels, int64_t n, u ws, u res, u auc, u s) {
    fdx::launch_auc_radix(P<const float>(scores), P<const uint8_t>(labels), n, P<void>(ws), P<int64_t>(res),
                          P<double>(auc), S(s));
  });
  m.def("confusion", [](u scores, u labels, int64_t n, float thr, u out4, u s) {
    fdx::launch_confusion(P<const float>(scores), P<const uint8_t>(labels), n, thr, P<unsigned long long>(out4), S(s));
  });
}
