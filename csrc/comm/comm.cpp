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
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

// oneshot.hip
namespace dgipc {
constexpr int MAXW = 8;
struct OneShotArgs {
  const void* src;
  void* dst;
  long long nvec;
  int dtype;
  int rank, world;
  char* bufs[MAXW];
  unsigned* flags[MAXW];
  long long half_bytes;
  unsigned* state;
  long long timeout_ticks;
};
}  // namespace dgipc
extern "C" hipError_t dg_oneshot_allreduce(const dgipc::OneShotArgs* a, int blocks,
                                           hipStream_t stream);

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

void hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("dgcomm ") + what + ": " + hipGetErrorString(e));
}

// The one-shot IPC all-reduce of small buckets (oneshot.hip): this rank's uncached staging
// buffer (2 halves of `capacity` bytes) and flag array, exported as IPC handles; open_peers
// maps every other rank's pair (handles exchanged by the caller, e.g. through the c10d store).
class IpcOneShot {
 public:
  IpcOneShot(int world, int rank, int device, long long capacity, double timeout_s)
      : world_(world), rank_(rank), cap_((capacity + 15) / 16 * 16) {
    if (world < 1 || world > dgipc::MAXW || rank < 0 || rank >= world || capacity <= 0)
      throw std::invalid_argument("dgcomm ipc: world 1..8, 0 <= rank < world, capacity > 0");
    hcheck(hipSetDevice(device), "hipSetDevice");
    hcheck(hipExtMallocWithFlags((void**)&buf_, 2 * cap_, hipDeviceMallocUncached),
           "staging alloc");
    hcheck(hipExtMallocWithFlags((void**)&flags_, dgipc::MAXW * sizeof(unsigned),
                                 hipDeviceMallocUncached),
           "flag alloc");
    hcheck(hipMemset(flags_, 0, dgipc::MAXW * sizeof(unsigned)), "flag init");
    hcheck(hipMalloc((void**)&state_, 4 * sizeof(unsigned)), "state alloc");
    hcheck(hipMemset(state_, 0, 4 * sizeof(unsigned)), "state init");
    hcheck(hipDeviceSynchronize(), "init sync");
    a_ = dgipc::OneShotArgs{};
    a_.rank = rank;
    a_.world = world;
    a_.half_bytes = cap_;
    a_.state = state_;
    a_.timeout_ticks = (long long)(timeout_s * 1e8);
    a_.bufs[rank] = buf_;
    a_.flags[rank] = flags_;
  }
  ~IpcOneShot() { close(); }

  py::bytes handle_buf() const { return handle(buf_); }
  py::bytes handle_flags() const { return handle(flags_); }

  // handles[j] = (staging handle, flag handle) of rank j (this rank's own entry is ignored)
  void open_peers(const std::vector<std::pair<py::bytes, py::bytes>>& handles) {
    if ((int)handles.size() != world_) throw std::invalid_argument("dgcomm ipc: one pair per rank");
    for (int j = 0; j < world_; ++j) {
      if (j == rank_) continue;
      a_.bufs[j] = (char*)open(handles[j].first);
      a_.flags[j] = (unsigned*)open(handles[j].second);
      opened_.push_back(a_.bufs[j]);
      opened_.push_back(a_.flags[j]);
    }
  }
  // count elements of dtype ("fp32" | "bf16"), a multiple of 16 bytes (the kernel moves
  // 16-byte vectors; the flat gradient's layer ranges are aligned)
  void all_reduce(uintptr_t src, uintptr_t dst, size_t count, const std::string& dt,
                  int blocks, uintptr_t stream) {
    const int es = dt == "fp32" ? 4 : dt == "bf16" ? 2 : 0;
    if (!es) throw std::invalid_argument("dgcomm ipc: fp32 | bf16");
    const long long nbytes = (long long)count * es;
    if (nbytes > cap_) throw std::invalid_argument("dgcomm ipc: bucket larger than capacity");
    if (nbytes % 16 != 0) throw std::invalid_argument("dgcomm ipc: bucket not a multiple of 16 B");
    for (int j = 0; j < world_; ++j)
      if (!a_.bufs[j]) throw std::runtime_error("dgcomm ipc: peers not opened");
    dgipc::OneShotArgs a = a_;
    a.src = (const void*)src;
    a.dst = (void*)dst;
    a.nvec = nbytes / 16;
    a.dtype = es == 4 ? 0 : 1;
    hcheck(dg_oneshot_allreduce(&a, blocks, (hipStream_t)stream), "oneshot all-reduce");
  }
  // non-zero once a call timed out waiting for a peer (its result is garbage)
  unsigned error() const {
    unsigned v[4];
    hcheck(hipMemcpy(v, state_, sizeof(v), hipMemcpyDeviceToHost), "state read");
    return v[3];
  }
  unsigned calls() const {
    unsigned v[4];
    hcheck(hipMemcpy(v, state_, sizeof(v), hipMemcpyDeviceToHost), "state read");
    return v[0];
  }
  long long capacity() const { return cap_; }
  void close() {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    if (buf_) (void)hipFree(buf_);
    if (flags_) (void)hipFree(flags_);
    if (state_) (void)hipFree(state_);
    buf_ = nullptr;
    flags_ = nullptr;
    state_ = nullptr;
  }

 private:
  static py::bytes handle(void* p) {
    hipIpcMemHandle_t h;
    hcheck(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
    return py::bytes((const char*)&h, sizeof(h));
  }
  static void* open(const py::bytes& b) {
    const std::string s = b;
    hipIpcMemHandle_t h;
    if (s.size() != sizeof(h)) throw std::invalid_argument("dgcomm ipc: bad handle");
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hcheck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return p;
  }
  int world_, rank_;
  long long cap_;
  char* buf_ = nullptr;
  unsigned* flags_ = nullptr;
  unsigned* state_ = nullptr;
  dgipc::OneShotArgs a_;
  std::vector<void*> opened_;
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
  py::class_<IpcOneShot>(m, "IpcOneShot")
      .def(py::init<int, int, int, long long, double>(), py::arg("world"), py::arg("rank"),
           py::arg("device"), py::arg("capacity"), py::arg("timeout_s") = 10.0)
      .def("handle_buf", &IpcOneShot::handle_buf)
      .def("handle_flags", &IpcOneShot::handle_flags)
      .def("open_peers", &IpcOneShot::open_peers)
      .def("all_reduce", &IpcOneShot::all_reduce, py::arg("src"), py::arg("dst"),
           py::arg("count"), py::arg("dtype"), py::arg("blocks"), py::arg("stream"))
      .def("error", &IpcOneShot::error)
      .def("calls", &IpcOneShot::calls)
      .def("capacity", &IpcOneShot::capacity)
      .def("close", &IpcOneShot::close);
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
