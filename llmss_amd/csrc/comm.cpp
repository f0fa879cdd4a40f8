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

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

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

// Bounded communicator set-up (reference: the NCCL process group's 60 s timeout, utils/dist.py:54,71). The
// communicator is created non-blocking (ncclConfig_t.blocking = 0): ncclCommInitRankConfig returns at once and
// its state is polled with ncclCommGetAsyncError against a deadline; a peer that never joins (died, hung, or
// failed before its own init) makes this rank abort the half-built communicator and raise instead of blocking
// in the init forever. The same poll bounds every later call that reports ncclInProgress (a non-blocking
// communicator's first collective builds its peer connections asynchronously); collectives whose connections
// exist return ncclSuccess at once, so captured decode graphs are unaffected.
class RcclComm {
 public:
  RcclComm(const std::string& uid, int nranks, int rank, int device, double timeout_s)
      : nranks_(nranks), rank_(rank), device_(device), timeout_s_(timeout_s) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id has the wrong size");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RcclComm: bad rank / size");
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RcclComm: hipSetDevice failed");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const auto t0 = std::chrono::steady_clock::now();
    const ncclResult_t r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_ != nullptr) ncclCommAbort(comm_);
      comm_ = nullptr;
      rccl_check(r, "ncclCommInitRankConfig");
    }
    settle("ncclCommInitRankConfig", timeout_s);
    init_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  ~RcclComm() {
    if (comm_ != nullptr) ncclCommDestroy(comm_);
  }

  void all_reduce(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    done(ncclAllReduce(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                       rccl_dtype(dtype), ncclSum, comm_, as_stream(stream)),
         "ncclAllReduce");
  }
  // dst holds nranks * count elements, rank r's block at offset r * count
  void all_gather(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    done(ncclAllGather(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                       rccl_dtype(dtype), comm_, as_stream(stream)),
         "ncclAllGather");
  }
  // src holds nranks * count elements; dst receives the sum of every rank's block `rank`
  void reduce_scatter(uintptr_t src, uintptr_t dst, int64_t count, int dtype, uintptr_t stream) {
    live();
    done(ncclReduceScatter(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), (size_t)count,
                           rccl_dtype(dtype), ncclSum, comm_, as_stream(stream)),
         "ncclReduceScatter");
  }
  void broadcast(uintptr_t buf, int64_t count, int dtype, int root, uintptr_t stream) {
    live();
    done(ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), (size_t)count,
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
      // non-blocking communicator: flush (finalize, bounded poll), then free
      const ncclResult_t r = ncclCommFinalize(comm_);
      if (r != ncclSuccess && r != ncclInProgress) {
        abort();
        rccl_check(r, "ncclCommFinalize");
      }
      settle("ncclCommFinalize", timeout_s_);
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
  double init_seconds() const { return init_s_; }

 private:
  void live() const {
    if (comm_ == nullptr) throw std::runtime_error("RcclComm: communicator was destroyed / aborted");
  }
  // poll the communicator's state until it leaves ncclInProgress; past the deadline (or on an error) abort it
  // and raise, so the caller's agreement step (parallel/dist.py) sees a failure instead of a hang
  void settle(const char* what, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0;; ++it) {
      ncclResult_t st = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
      if (q != ncclSuccess) st = q;
      if (st == ncclSuccess) return;
      if (st != ncclInProgress) {
        abort();
        throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(st));
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (timeout_s > 0 && el > timeout_s) {
        abort();
        throw std::runtime_error(std::string("RCCL ") + what + ": timed out after " + std::to_string(timeout_s) +
                                 " s waiting for the peer ranks (communicator aborted)");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(it < 100 ? 20 : 1000));
    }
  }
  void done(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) settle(what, timeout_s_);
    else rccl_check(r, what);
  }
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_;
  double timeout_s_ = 0, init_s_ = 0;
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
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("uid"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"), py::arg("timeout_s") = 120.0, py::call_guard<py::gil_scoped_release>())
      .def("all_reduce", &RcclComm::all_reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("init_seconds", &RcclComm::init_seconds);
}
