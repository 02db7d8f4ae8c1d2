// Native RCCL communicator: one process per GPU, ncclCommInitRank on a unique id
// exchanged through the torch.distributed TCPStore, collectives enqueued directly on the caller's
// hipStream_t (the compute stream) -- no ProcessGroup work objects, no cross-stream events, and
// capturable into hipGraphs.  The payloads of this framework are latency-bound (the Newton
// gradient+Hessian vector is 8.5 KB), so removing per-call host overhead is the lever; RCCL itself
// picks the xGMI transport between the GPUs of one node.
//
// Linked against librccl.so.1: torch already loaded the same SONAME, so the process holds a single
// RCCL instance.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t dtype_of(int k) {
  switch (k) {
    case 0: return ncclFloat32;
    case 1: return ncclFloat64;
    case 2: return ncclInt64;
    case 3: return ncclUint8;
    case 4: return ncclInt32;
    case 5: return ncclBfloat16;
    default: throw std::runtime_error("rccl: unsupported dtype code");
  }
}

ncclRedOp_t op_of(int k) {
  switch (k) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    default: throw std::runtime_error("rccl: unsupported reduction op");
  }
}

inline ncclComm_t C(uintptr_t h) { return reinterpret_cast<ncclComm_t>(h); }
inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

PYBIND11_MODULE(_fdx_comm, m) {
  m.doc() = "native RCCL communicator for fraud_detection_amd data parallelism";
  m.def("version", [] {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  m.def("unique_id", [] {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "GetUniqueId");
    return py::bytes(id.internal, sizeof(id.internal));
  });
  m.def("init_rank", [](py::bytes uid, int nranks, int rank) {
    std::string s = uid;
    ncclUniqueId id;
    if (s.size() != sizeof(id.internal)) throw std::runtime_error("rccl: bad unique id size");
    std::memcpy(id.internal, s.data(), sizeof(id.internal));
    ncclComm_t comm;
    {
      py::gil_scoped_release nogil;
      check(ncclCommInitRank(&comm, nranks, id, rank), "CommInitRank");
    }
    return reinterpret_cast<uintptr_t>(comm);
  });
  m.def("all_reduce", [](uintptr_t comm, uintptr_t sendbuf, uintptr_t recvbuf, size_t count, int dtype, int op,
                         uintptr_t stream) {
    check(ncclAllReduce(reinterpret_cast<const void*>(sendbuf), reinterpret_cast<void*>(recvbuf), count,
                        dtype_of(dtype), op_of(op), C(comm), S(stream)),
          "AllReduce");
  });
  m.def("all_gather", [](uintptr_t comm, uintptr_t sendbuf, uintptr_t recvbuf, size_t count, int dtype,
                         uintptr_t stream) {
    check(ncclAllGather(reinterpret_cast<const void*>(sendbuf), reinterpret_cast<void*>(recvbuf), count,
                        dtype_of(dtype), C(comm), S(stream)),
          "AllGather");
  });
  m.def("broadcast", [](uintptr_t comm, uintptr_t buf, size_t count, int dtype, int root, uintptr_t stream) {
    check(ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), count, dtype_of(dtype),
                        root, C(comm), S(stream)),
          "Broadcast");
  });
  m.def("destroy", [](uintptr_t comm) { check(ncclCommDestroy(C(comm)), "CommDestroy"); });
}
