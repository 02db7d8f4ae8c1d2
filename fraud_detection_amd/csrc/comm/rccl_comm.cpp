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
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

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

size_t size_of(int k) {
  switch (k) {
    case 0: return 4;
    case 1: return 8;
    case 2: return 8;
    case 3: return 1;
    case 4: return 4;
    case 5: return 2;
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
  // Variable-count all-gather (collective C3: SMOTE minority rows, k-NN neighbour lists, test
  // scores): every rank sends its rows straight to every peer over its own xGMI link (grouped
  // point-to-point -- on a fully connected 8-GPU node each pair has a direct link, so the payload
  // is not relayed around a ring) and receives each peer's rows at that peer's displacement of
  // the compact output; its own rows are a local D2D copy.  No padding to the largest count and no
  // concatenation afterwards.  counts / displs are in elements.
  m.def("all_gatherv", [](uintptr_t comm, uintptr_t send, size_t send_count, uintptr_t recv,
                          std::vector<size_t> counts, std::vector<size_t> displs, int dtype, int rank,
                          uintptr_t stream) {
    const size_t es = size_of(dtype);
    const int nranks = (int)counts.size();
    if ((int)displs.size() != nranks || rank < 0 || rank >= nranks || counts[rank] != send_count)
      throw std::runtime_error("rccl all_gatherv: inconsistent counts");
    ncclDataType_t dt = dtype_of(dtype);
    char* out = reinterpret_cast<char*>(recv);
    check(ncclGroupStart(), "GroupStart");
    for (int p = 0; p < nranks; ++p) {
      if (p == rank) continue;
      if (send_count) check(ncclSend(reinterpret_cast<const void*>(send), send_count, dt, p, C(comm), S(stream)), "Send");
      if (counts[p]) check(ncclRecv(out + displs[p] * es, counts[p], dt, p, C(comm), S(stream)), "Recv");
    }
    check(ncclGroupEnd(), "GroupEnd");
    if (send_count && out + displs[rank] * es != reinterpret_cast<char*>(send)) {
      hipError_t e = hipMemcpyAsync(out + displs[rank] * es, reinterpret_cast<const void*>(send), send_count * es,
                                    hipMemcpyDeviceToDevice, S(stream));
      if (e != hipSuccess) throw std::runtime_error(std::string("all_gatherv local copy: ") + hipGetErrorString(e));
    }
  });
  m.def("broadcast", [](uintptr_t comm, uintptr_t buf, size_t count, int dtype, int root, uintptr_t stream) {
    check(ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), count, dtype_of(dtype),
                        root, C(comm), S(stream)),
          "Broadcast");
  });
  m.def("destroy", [](uintptr_t comm) { check(ncclCommDestroy(C(comm)), "CommDestroy"); });
}
