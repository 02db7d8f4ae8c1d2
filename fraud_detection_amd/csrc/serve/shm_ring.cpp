// pybind11 module of the shared-memory request ring (the protocol lives in shm_ring.h, shared with
// the native GPU-owner loop in csrc/bindings.cpp).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <chrono>
#include <thread>

#include "shm_ring.h"

namespace py = pybind11;
using fdx_ring::Ring;
using fdx_ring::OWNER_READY;
using fdx_ring::OWNER_STARTING;
using fdx_ring::OWNER_STOPPED;

namespace {
template <class T>
T* data_of(py::array& a, const char* what) {
  if (!(a.flags() & py::array::c_style)) throw std::runtime_error(std::string(what) + " must be C-contiguous");
  return static_cast<T*>(a.mutable_data());
}

}  // namespace

PYBIND11_MODULE(_fdx_ring, m) {
  m.doc() = "shared-memory request ring: serving front-ends -> the GPU-owner process";
  py::class_<Ring>(m, "Ring")
      .def(py::init<const std::string&, uint32_t, uint32_t, uint32_t, uint32_t>(), py::arg("path"),
           py::arg("nslots"), py::arg("d"), py::arg("slot_rows"), py::arg("out_w"))
      .def(py::init<const std::string&>(), py::arg("path"))
      .def_property_readonly("d", &Ring::d)
      .def_property_readonly("out_w", &Ring::out_w)
      .def_property_readonly("slot_rows", &Ring::slot_rows)
      .def_property_readonly("nslots", &Ring::nslots)
      .def_property_readonly("owner_pid", &Ring::owner_pid)
      .def_property("owner_state", &Ring::owner_state, &Ring::set_owner_state)
      .def_property("host_max_rows", &Ring::host_max_rows, &Ring::set_host_max_rows)
      .def("stats", [](const Ring& r) {
        auto s = r.stats();
        py::dict o;
        o["batches"] = s.batches;
        o["rows"] = s.rows;
        o["slots"] = s.slots;
        o["queued_tickets"] = s.queued;
        o["cancelled"] = s.cancelled;
        o["reclaimed"] = s.reclaimed;
        return o;
      })
      .def_property("reclaim_ms", &Ring::reclaim_ms, &Ring::set_reclaim_ms,
                    "how long a tail ticket may stay unpublished / unfreed before the owner reclaims it")
      .def("ready_rows", &Ring::ready_rows, py::arg("limit") = 1u << 30)
      .def_property_readonly("base_address", [](const Ring& r) { return reinterpret_cast<uintptr_t>(r.base_address()); })
      .def_property_readonly("total_bytes", &Ring::total_bytes)
      .def("request",
           [](Ring& r, py::array_t<float, py::array::c_style | py::array::forcecast> X, uint32_t op, double timeout_ms) {
             if (X.ndim() != 2 || (uint32_t)X.shape(1) != r.d()) throw std::runtime_error("ring: X must be [n, d]");
             uint32_t n = (uint32_t)X.shape(0);
             py::array_t<float> out({(py::ssize_t)n, (py::ssize_t)r.out_w()});
             const float* xp = X.data();
             float* op_ = out.mutable_data();
             if (n) {
               py::gil_scoped_release nogil;
               r.request(xp, op_, n, op, timeout_ms);
             }
             return out;
           },
           py::arg("X"), py::arg("op") = 0, py::arg("timeout_ms") = 10000.0)
      .def("collect",
           [](Ring& r, uintptr_t dst, uint32_t max_rows, double window_us, double timeout_ms, int set) {
             py::gil_scoped_release nogil;
             auto res = r.collect(reinterpret_cast<float*>(dst), max_rows, window_us, timeout_ms, set);
             return std::make_tuple(res.first, res.second);
           },
           py::arg("dst"), py::arg("max_rows"), py::arg("window_us") = 0.0, py::arg("timeout_ms") = 50.0,
           py::arg("set") = 0, "gather READY rows into the float32 buffer at address dst as batch `set`; -> (rows, op)")
      .def("complete",
           [](Ring& r, uintptr_t prob, uintptr_t logit, uintptr_t phi, uint32_t dphi, bool ok, int set) {
             py::gil_scoped_release nogil;
             r.complete(reinterpret_cast<const float*>(prob), reinterpret_cast<const float*>(logit),
                        reinterpret_cast<const float*>(phi), dphi, ok, set);
           },
           py::arg("prob"), py::arg("logit"), py::arg("phi") = 0, py::arg("dphi") = 0, py::arg("ok") = true,
           py::arg("set") = 0)
      .def("pending_slots", &Ring::pending_slots)
      .def("debug_tags", [](const Ring& r) {
        py::list o;
        for (uint64_t v : r.debug_tags()) o.append(v);
        return o;
      })
      .def("debug_take_tickets", &Ring::debug_take_tickets, py::arg("n"),
           "take n tickets without publishing them (simulates a producer that died mid-request)")
      .def("debug_publish",
           [](Ring& r, py::array_t<float, py::array::c_style | py::array::forcecast> X, uint32_t op) {
             if (X.ndim() != 2 || (uint32_t)X.shape(1) != r.d()) throw std::runtime_error("ring: X must be [n, d]");
             return r.debug_publish(X.data(), (uint32_t)X.shape(0), op);
           },
           py::arg("X"), py::arg("op") = 0,
           "publish rows and never consume the results (simulates a producer killed while waiting)");
  // Native load generator (tools/serve_latency.py): `threads` C++ producer threads, each issuing
  // `per_thread` synchronous requests of `rows` rows -- the owner's capacity without a Python
  // producer's interpreter in the measurement.  -> (elapsed seconds, per-request latencies in us)
  m.def("loadgen", [](const std::string& path, int threads, int per_thread, int rows, double timeout_ms) {
    Ring r(path);
    const uint32_t d = r.d(), W = r.out_w();
    std::vector<std::vector<float>> lat(threads);
    std::vector<int> failures(threads, 0);
    double elapsed = 0.0;
    {
      py::gil_scoped_release nogil;
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int k = 0; k < threads; ++k) {
        th.emplace_back([&, k] {
          std::vector<float> X((size_t)rows * d), out((size_t)rows * W);
          for (size_t i = 0; i < X.size(); ++i) X[i] = (float)((i * 2654435761u + k) % 1000) * 1e-3f - 0.5f;
          lat[k].reserve(per_thread);
          for (int i = 0; i < per_thread; ++i) {
            auto a = std::chrono::steady_clock::now();
            try {
              r.request(X.data(), out.data(), (uint32_t)rows, 0, timeout_ms);
            } catch (...) {
              ++failures[k];
            }
            auto b = std::chrono::steady_clock::now();
            lat[k].push_back((float)std::chrono::duration<double, std::micro>(b - a).count());
          }
        });
      }
      for (auto& t : th) t.join();
      elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    size_t total = 0;
    for (auto& v : lat) total += v.size();
    py::array_t<float> L(total);
    float* o = L.mutable_data();
    for (auto& v : lat) o = std::copy(v.begin(), v.end(), o);
    int fails = 0;
    for (int f : failures) fails += f;
    return py::make_tuple(elapsed, L, fails);
  }, py::arg("path"), py::arg("threads"), py::arg("per_thread"), py::arg("rows") = 1, py::arg("timeout_ms") = 10000.0);
  m.attr("OWNER_STARTING") = (int)OWNER_STARTING;
  m.attr("OWNER_READY") = (int)OWNER_READY;
  m.attr("OWNER_STOPPED") = (int)OWNER_STOPPED;
}
