// _dgcomm: a thin native RCCL communicator for the data-parallel training step.
//
// Why native instead of torch.distributed's ProcessGroupNCCL for the gradient path:
//   * the collectives are issued on OUR comm stream with plain ncclAllReduce calls, so they
//     can be captured INSIDE the step's hipGraph (forked from the compute stream by an event
//     after each weight-gradient group, joined before the optimizer) — one graph launch per
//     step, no host round trip and no graph-to-graph boundary per bucket;
//   * no per-call Work objects, tensor-liveness bookkeeping or watchdog threads on the hot
//     path; failure detection is explicit: async_error() polls ncclCommGetAsyncError and
//     abort() tears the communicator down (faults.py CommWatchdog).
// torch.distributed is still used for rendezvous (the unique id travels through its store),
// validation scalars and barriers.
//
// The process loads ONE librccl.so.1: torch's bundled copy (same SONAME) is already mapped
// when this module is imported (ops/native.py imports torch first).
//
// Reference: the single-process DataParallelTable gradient reduce + parameter broadcast of
// makeDataParallel (/root/reference/experiments.lua:155-168).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t dtype_of(const std::string& d) {
  if (d == "fp32") return ncclFloat32;
  if (d == "bf16") return ncclBfloat16;
  if (d == "fp16") return ncclFloat16;
  if (d == "fp64") return ncclFloat64;
  if (d == "i32") return ncclInt32;
  if (d == "i64") return ncclInt64;
  throw std::invalid_argument("dgcomm: unsupported dtype " + d);
}

ncclRedOp_t op_of(const std::string& o) {
  if (o == "sum") return ncclSum;
  if (o == "max") return ncclMax;
  if (o == "min") return ncclMin;
  if (o == "avg") return ncclAvg;
  throw std::invalid_argument("dgcomm: unsupported op " + o);
}

class Comm {
 public:
  Comm(py::bytes uid, int world, int rank, int device) : world_(world), rank_(rank) {
    std::string s = uid;
    if (s.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("dgcomm: bad unique id");
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("dgcomm: rank/world");
    ncclUniqueId id;
    memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("dgcomm: hipSetDevice");
    {
      py::gil_scoped_release nogil;  // init rendezvous blocks until every rank arrives
      check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
    }
  }
  ~Comm() {
    if (comm_) ncclCommDestroy(comm_);
  }

  // in place when src == dst; count in elements; stream = hipStream_t as an integer
  void all_reduce(uintptr_t src, uintptr_t dst, size_t count, const std::string& dt,
                  const std::string& op, uintptr_t stream) {
    live();
    check(ncclAllReduce((const void*)src, (void*)dst, count, dtype_of(dt), op_of(op), comm_,
                        (hipStream_t)stream),
          "ncclAllReduce");
  }
  void broadcast(uintptr_t buf, size_t count, const std::string& dt, int root, uintptr_t stream) {
    live();
    check(ncclBroadcast((const void*)buf, (void*)buf, count, dtype_of(dt), root, comm_,
                        (hipStream_t)stream),
          "ncclBroadcast");
  }
  void reduce_scatter(uintptr_t src, uintptr_t dst, size_t recv_count, const std::string& dt,
                      const std::string& op, uintptr_t stream) {
    live();
    check(ncclReduceScatter((const void*)src, (void*)dst, recv_count, dtype_of(dt), op_of(op),
                            comm_, (hipStream_t)stream),
          "ncclReduceScatter");
  }
  void all_gather(uintptr_t src, uintptr_t dst, size_t send_count, const std::string& dt,
                  uintptr_t stream) {
    live();
    check(ncclAllGather((const void*)src, (void*)dst, send_count, dtype_of(dt), comm_,
                        (hipStream_t)stream),
          "ncclAllGather");
  }
  void group_start() { check(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() { check(ncclGroupEnd(), "ncclGroupEnd"); }

  // "" when healthy, else the error string (ncclCommGetAsyncError: a peer died, a network
  // or xGMI transport error, or an abort)
  std::string async_error() {
    if (!comm_) return "destroyed";
    ncclResult_t st = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(comm_, &st);
    if (r != ncclSuccess) return std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(r);
    if (st == ncclSuccess || st == ncclInProgress) return "";
    return ncclGetErrorString(st);
  }
  // unblocks any collective waiting on a dead peer; the communicator is unusable afterwards
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  void destroy() {
    if (comm_) {
      py::gil_scoped_release nogil;
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }
  int world() const { return world_; }
  int rank() const { return rank_; }
  // what the communicator itself reports (ncclCommCount / UserRank / CuDevice): the
  // bench's "ranks_seen", checked against WORLD_SIZE
  int count() const {
    live();
    int n = 0;
    check(ncclCommCount(comm_, &n), "ncclCommCount");
    return n;
  }
  int user_rank() const {
    live();
    int r = -1;
    check(ncclCommUserRank(comm_, &r), "ncclCommUserRank");
    return r;
  }
  int device() const {
    live();
    int d = -1;
    check(ncclCommCuDevice(comm_, &d), "ncclCommCuDevice");
    return d;
  }

 private:
  void live() const {
    if (!comm_) throw std::runtime_error("dgcomm: communicator destroyed or aborted");
  }
  ncclComm_t comm_ = nullptr;
  int world_, rank_;
};

}  // namespace

PYBIND11_MODULE(_dgcomm, m) {
  m.doc() = "native RCCL communicator (deep_go_amd data parallelism)";
  m.def("unique_id", []() {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  });
  m.def("version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<Comm>(m, "Comm")
      .def(py::init<py::bytes, int, int, int>(), py::arg("uid"), py::arg("world"),
           py::arg("rank"), py::arg("device"))
      .def("all_reduce", &Comm::all_reduce, py::arg("src"), py::arg("dst"), py::arg("count"),
           py::arg("dtype"), py::arg("op"), py::arg("stream"))
      .def("broadcast", &Comm::broadcast, py::arg("buf"), py::arg("count"), py::arg("dtype"),
           py::arg("root"), py::arg("stream"))
      .def("reduce_scatter", &Comm::reduce_scatter)
      .def("all_gather", &Comm::all_gather)
      .def("group_start", &Comm::group_start)
      .def("group_end", &Comm::group_end)
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def("destroy", &Comm::destroy)
      .def("count", &Comm::count)
      .def("user_rank", &Comm::user_rank)
      .def("device", &Comm::device)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("rank", &Comm::rank);
}
