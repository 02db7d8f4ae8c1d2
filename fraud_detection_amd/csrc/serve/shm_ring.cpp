// pybind11 module of the shared-memory request ring (the protocol lives in shm_ring.h, shared with
// the native GPU-owner loop in csrc/bindings.cpp).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

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
        return o;
      })
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
      .def("pending_slots", &Ring::pending_slots);
  m.attr("OWNER_STARTING") = (int)OWNER_STARTING;
  m.attr("OWNER_READY") = (int)OWNER_READY;
  m.attr("OWNER_STOPPED") = (int)OWNER_STOPPED;
}
