// Native RCCL communicator for the tensor-parallel data plane (part of module llmss_amd._C).
//
// Reference: every collective of the reference goes through torch.distributed's NCCL process group
// (utils/dist.py:40-77 creates it with is_high_priority_stream; layers.py:125,133,178,213 call
// all_reduce / all_gather on it). Here the row-parallel all-reduces, the vocab-parallel gathers and
// the step broadcasts are plain RCCL calls on a communicator this module owns, enqueued on whatever
// HIP stream the caller passes (the compute stream inside a captured decode graph, a priority -1 comm
// stream for the overlapped prefill buckets):
//   * no per-collective torch Work object, CUDA event or watchdog entry (a HIP-graph capture can not
//     race a watchdog thread polling events of earlier collectives - the hazard the torch process
//     group path had to sleep around);
//   * one host call per collective (pybind11 -> ncclAllReduce), i.e. a few microseconds of launch cost
//     on the eager prefill path instead of c10d's dispatch + bookkeeping.
// The bootstrap (unique-id exchange) rides on the CPU (gloo) process group; see parallel/dist.py.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t rccl_dtype(int code) {
  if (code < 0 || code >= (int)ncclNumTypes) throw std::invalid_argument("RCCL: bad dtype code " + std::to_string(code));
  return (ncclDataType_t)code;
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

class RcclComm {
 public:
  RcclComm(const std::string& uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id has the wrong size");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RcclComm: bad rank / size");
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RcclComm: hipSetDevice failed");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    rccl_check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
  }
  ~RcclComm() {
    if (comm_ != nullptr) ncclCommDestroy(comm_);
  }

  void all_reduce(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    rccl_check(ncclAllReduce(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                             rccl_dtype(dtype), ncclSum, comm_, as_stream(stream)),
               "ncclAllReduce");
  }
  // dst holds nranks * count elements, rank r's block at offset r * count
  void all_gather(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    rccl_check(ncclAllGather(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                             rccl_dtype(dtype), comm_, as_stream(stream)),
               "ncclAllGather");
  }
  // src holds nranks * count elements; dst receives the sum of every rank's block `rank`
  void reduce_scatter(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    rccl_check(ncclReduceScatter(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                                 rccl_dtype(dtype), ncclSum, comm_, as_stream(stream)),
               "ncclReduceScatter");
  }
  void broadcast(uintptr_t buf, int64_t count, int dtype, int root, uintptr_t stream) {
    live();
    rccl_check(ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), (size_t)count,
                             rccl_dtype(dtype), root, comm_, as_stream(stream)),
               "ncclBroadcast");
  }
  // Tear down without waiting for peers (a dead or hung rank): pending collectives are cancelled.
  void abort() {
    if (comm_ != nullptr) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  void destroy() {
    if (comm_ != nullptr) {
      rccl_check(ncclCommDestroy(comm_), "ncclCommDestroy");
      comm_ = nullptr;
    }
  }
  std::string async_error() {
    if (comm_ == nullptr) return "destroyed";
    ncclResult_t e = ncclSuccess;
    rccl_check(ncclCommGetAsyncError(comm_, &e), "ncclCommGetAsyncError");
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }

 private:
  void live() const {
    if (comm_ == nullptr) throw std::runtime_error("RcclComm: communicator was destroyed / aborted");
  }
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_;
};

}  // namespace

void register_comm(py::module_& m) {
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  });
  m.def("rccl_version", []() {
    int v = 0;
    rccl_check(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  py::dict codes;
  codes["int8"] = (int)ncclInt8;
  codes["uint8"] = (int)ncclUint8;
  codes["int32"] = (int)ncclInt32;
  codes["int64"] = (int)ncclInt64;
  codes["float16"] = (int)ncclFloat16;
  codes["float32"] = (int)ncclFloat32;
  codes["float64"] = (int)ncclFloat64;
  codes["bfloat16"] = (int)ncclBfloat16;
  m.attr("rccl_dtypes") = codes;
  // init, destroy and a collective's first call (lazy peer connection) block on the peers: release the GIL so
  // other Python threads (the serving heartbeat) keep running
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::call_guard<py::gil_scoped_release>())
      .def("all_reduce", &RcclComm::all_reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device);
}
