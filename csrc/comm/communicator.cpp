// Native RCCL communicator (the reference reaches NCCL through
// `init_process_group(backend="nccl")`, `02 DDP基本概念/ddp_gpus.py:20-22`, and torch's ProcessGroupNCCL).
//
// One communicator = one ncclComm_t over a group of ranks (one process per GPU) + one
// HIP stream of its own.  Every collective is enqueued on that stream after an event-wait on the
// streams that produced its input, and returns a Work handle: an event recorded behind the collective,
// which a consumer stream waits on (hipStreamWaitEvent, no host blocking) or the host polls.  So
// gradient buckets are reduced on the comm stream while backward kernels keep running on the compute
// and weight-gradient streams, and the compute stream only waits where it consumes the result.
//
// Bootstrap: rank 0 of the group creates the ncclUniqueId, the ranks exchange it through the
// framework's key-value store (Python side, pytorchdistributed_amd/comm.py), then ncclCommInitRank.
// Failure handling: every live communicator is registered with the process-wide abort hook that the
// native collective watchdog (csrc/runtime/watchdog.cpp) runs on a timeout, so a hung collective is
// ncclCommAbort-ed (its kernels exit, the waiting streams are released) before the watchdog acts.
//
// librccl is torch's own copy (linked from torch/lib, so this and ProcessGroupNCCL share one RCCL).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "runtime.h"

namespace pda_comm {

namespace {

void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
}

bool comm_nonblocking() {
  // PDA_COMM_NONBLOCKING=0: the blocking communicator (ncclCommInitRank) as before round 5
  const char* v = std::getenv("PDA_COMM_NONBLOCKING");
  return !(v && v[0] == '0');
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// PDA_COMM_CUS: CUs the comm stream may use (0 = all, no mask)
int comm_cu_budget() { return env_int("PDA_COMM_CUS", 0); }

// PDA_COMM_MAX_CTAS: RCCL blocks per collective (default: the CU budget when one is set, else RCCL's own)
int comm_max_ctas(int cu_budget) { return env_int("PDA_COMM_MAX_CTAS", cu_budget > 0 ? cu_budget : 0); }

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + " failed: " + hipGetErrorString(e));
}

// framework dtype ids (pytorchdistributed_amd/comm.py:_DTYPE)
ncclDataType_t to_nccl_dtype(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    case 4: return ncclInt64;
    case 5: return ncclInt32;
    case 6: return ncclUint8;
    case 7: return ncclInt8;
    default: throw std::invalid_argument("communicator: unsupported dtype id " + std::to_string(d));
  }
}

ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclProd;
    default: throw std::invalid_argument("communicator: unsupported reduce op " + std::to_string(op));
  }
}

// current-device guard
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    check_hip(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) check_hip(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

// Recycled completion events (one hipEventCreate per collective showed up as host time on the
// launch path); shared by a communicator and its outstanding Work handles.
class EventPool {
 public:
  explicit EventPool(int device) : device_(device) {}
  ~EventPool() {
    for (hipEvent_t e : free_) (void)hipEventDestroy(e);
  }
  hipEvent_t get() {
    {
      std::lock_guard<std::mutex> l(mu_);
      if (!free_.empty()) {
        hipEvent_t e = free_.back();
        free_.pop_back();
        return e;
      }
    }
    DeviceGuard g(device_);
    hipEvent_t e = nullptr;
    check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  void put(hipEvent_t e) {
    std::lock_guard<std::mutex> l(mu_);
    free_.push_back(e);
  }

 private:
  int device_;
  std::mutex mu_;
  std::vector<hipEvent_t> free_;
};

// Completion handle of one enqueued collective (or of a group of point-to-point ops).
class Work {
 public:
  Work(int device, hipStream_t s, std::shared_ptr<EventPool> pool) : device_(device), pool_(std::move(pool)) {
    DeviceGuard g(device_);
    ev_ = pool_->get();
    check_hip(hipEventRecord(ev_, s), "hipEventRecord");
  }
  ~Work() {
    // a re-record of a recycled event only moves its completion point forward, so handing it out
    // while the GPU has not reached it yet is harmless: nothing waits on this handle any more
    if (ev_) pool_->put(ev_);
  }
  Work(const Work&) = delete;
  Work& operator=(const Work&) = delete;
  // order `stream` after the collective (no host wait)
  void wait(uintptr_t stream) {
    DeviceGuard g(device_);
    check_hip(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev_, 0), "hipStreamWaitEvent");
  }
  bool is_completed() {
    const hipError_t e = hipEventQuery(ev_);
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    check_hip(e, "hipEventQuery");
    return false;
  }
  void synchronize() { check_hip(hipEventSynchronize(ev_), "hipEventSynchronize"); }
  uintptr_t event() const { return reinterpret_cast<uintptr_t>(ev_); }

 private:
  int device_;
  std::shared_ptr<EventPool> pool_;
  hipEvent_t ev_ = nullptr;
};

class Communicator;

namespace {
std::mutex g_live_mu;
std::set<Communicator*> g_live;
}  // namespace

class Communicator {
 public:
  Communicator(const std::string& uid, int nranks, int rank, int device, bool high_priority)
      : nranks_(nranks), rank_(rank), device_(device), pool_(std::make_shared<EventPool>(device)) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("communicator: bad unique id size");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("communicator: bad rank / size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    DeviceGuard g(device_);
    // CU budget (PDA_COMM_CUS = n > 0): the comm stream's hardware queue may only dispatch to n CUs,
    // spread evenly over the 8 XCDs, and RCCL launches at most n blocks (ncclConfig_t.maxCTAs), so
    // collective kernels — and the D2D blits of a one-rank group — never take more than n of the 256
    // CUs from the compute streams' one-workgroup-per-CU GEMM tiles.  n = 0: an unmasked stream.
    cu_budget_ = comm_cu_budget();
    if (cu_budget_ > 0) {
      int ncu = 0;
      check_hip(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_), "hipDeviceGetAttribute");
      if (ncu <= 0) ncu = 256;
      if (cu_budget_ > ncu) cu_budget_ = ncu;
      std::vector<uint32_t> mask = pda_rt::cu_mask_spread(cu_budget_, ncu);
      check_hip(hipExtStreamCreateWithCUMask(&stream_, (uint32_t)mask.size(), mask.data()),
                "hipExtStreamCreateWithCUMask");
    } else {
      int lo = 0, hi = 0;
      check_hip(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
      check_hip(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo),
                "hipStreamCreateWithPriority");
    }
    check_hip(hipEventCreateWithFlags(&dep_, hipEventDisableTiming), "hipEventCreate");
    nonblocking_ = comm_nonblocking();
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    const int max_ctas = comm_max_ctas(cu_budget_);
    if (max_ctas > 0) {
      cfg.maxCTAs = max_ctas;
      cfg.minCTAs = 1;
    }
    if (!nonblocking_) {
      cfg.blocking = 1;
      check_nccl(ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg), "ncclCommInitRankConfig");
      inited_.store(true);
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live.insert(this);
      return;
    }
    // Non-blocking init (ncclConfig_t.blocking = 0): the communicator is visible to the abort hook
    // BEFORE it has connected, and this thread polls its state instead of blocking inside RCCL, so a
    // peer that never joins ends in a watchdog abort that releases the init
    // instead of a SIGABRT while stuck in ncclCommInitRank.
    cfg.blocking = 0;
    check_nccl(ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg), "ncclCommInitRankConfig");
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live.insert(this);
    }
    ncclResult_t st = ncclInProgress;
    while (true) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
      if (st != ncclInProgress || aborted_.load()) break;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (st == ncclSuccess && !aborted_.load()) {
      inited_.store(true);
      if (!aborted_.load()) return;  // abort() raced in after the check: release the comm below
    }
    do_abort();
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live.erase(this);
    }
    (void)hipEventDestroy(dep_);
    throw std::runtime_error(std::string("RCCL communicator init ") +
                             (aborted_.load() ? "aborted" : std::string("failed: ") + ncclGetErrorString(st)));
  }

  ~Communicator() {
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live.erase(this);
    }
    DeviceGuard g(device_);
    release();
    if (dep_) (void)hipEventDestroy(dep_);
    // stream_ is deliberately NOT destroyed: tensors the collectives used were record_stream()-ed on it
    // (comm.py _hold), and the caching allocator records an event on that stream when such a tensor
    // is freed — possibly after the communicator is gone (destroy_process_group, then the tensors go
    // out of scope).  An event record on a destroyed stream is a use-after-free; one idle stream per
    // communicator ever created is the price.
  }

  // explicit teardown (destroy_process_group): drain the stream, then ncclCommDestroy,
  // while the peers and the store still exist; later calls on this communicator raise
  void close() {
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live.erase(this);
    }
    DeviceGuard g(device_);
    release();
  }

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(stream_); }
  bool aborted() const { return aborted_.load(); }
  bool closed() const { return closed_.load(); }
  bool nonblocking() const { return nonblocking_; }
  int cu_budget() const { return cu_budget_; }

  // the comm stream waits for everything queued so far on `s` (the producers of the next input)
  void wait_stream(uintptr_t s) {
    DeviceGuard g(device_);
    check_hip(hipEventRecord(dep_, reinterpret_cast<hipStream_t>(s)), "hipEventRecord");
    check_hip(hipStreamWaitEvent(stream_, dep_, 0), "hipStreamWaitEvent");
  }

  // the comm stream waits for a recorded event (cross-communicator ordering, comm.py:_order)
  void wait_event(uintptr_t ev) {
    DeviceGuard g(device_);
    check_hip(hipStreamWaitEvent(stream_, reinterpret_cast<hipEvent_t>(ev), 0), "hipStreamWaitEvent");
  }

  std::shared_ptr<Work> all_reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclAllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), (size_t)count,
                             to_nccl_dtype(dtype), to_nccl_op(op), comm_, stream_),
               "ncclAllReduce");
    settle("ncclAllReduce");
    return done();
  }

  // recv[recvcount] = op over ranks of send[rank * recvcount : (rank + 1) * recvcount]
  std::shared_ptr<Work> reduce_scatter(uintptr_t send, uintptr_t recv, int64_t recvcount, int dtype, int op) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                                 (size_t)recvcount, to_nccl_dtype(dtype), to_nccl_op(op), comm_, stream_),
               "ncclReduceScatter");
    settle("ncclReduceScatter");
    return done();
  }

  // recv[r * sendcount : (r + 1) * sendcount] = send of rank r
  std::shared_ptr<Work> all_gather(uintptr_t send, uintptr_t recv, int64_t sendcount, int dtype) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), (size_t)sendcount,
                             to_nccl_dtype(dtype), comm_, stream_),
               "ncclAllGather");
    settle("ncclAllGather");
    return done();
  }

  // recv (root only) = op over ranks of send; parameter-server gradients (parallel/param_server.py)
  std::shared_ptr<Work> reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, int root) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), (size_t)count,
                          to_nccl_dtype(dtype), to_nccl_op(op), root, comm_, stream_),
               "ncclReduce");
    settle("ncclReduce");
    return done();
  }

  std::shared_ptr<Work> broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclBroadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), (size_t)count,
                             to_nccl_dtype(dtype), root, comm_, stream_),
               "ncclBroadcast");
    settle("ncclBroadcast");
    return done();
  }

  // point-to-point: inside group_start / group_end they are fused into one launch (returns None then)
  std::shared_ptr<Work> send(uintptr_t buf, int64_t count, int dtype, int peer) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclSend(reinterpret_cast<const void*>(buf), (size_t)count, to_nccl_dtype(dtype), peer, comm_, stream_),
               "ncclSend");
    if (!group_depth_) settle("ncclSend");
    return group_depth_ ? nullptr : done();
  }

  std::shared_ptr<Work> recv(uintptr_t buf, int64_t count, int dtype, int peer) {
    std::lock_guard<std::timed_mutex> l(op_mu_);
    live();
    DeviceGuard g(device_);
    check_nccl(ncclRecv(reinterpret_cast<void*>(buf), (size_t)count, to_nccl_dtype(dtype), peer, comm_, stream_),
               "ncclRecv");
    if (!group_depth_) settle("ncclRecv");
    return group_depth_ ? nullptr : done();
  }

  void group_start() {
    live();
    check_nccl(ncclGroupStart(), "ncclGroupStart");
    ++group_depth_;
  }

  std::shared_ptr<Work> group_end() {
    if (group_depth_ == 0) throw std::runtime_error("communicator: group_end without group_start");
    std::lock_guard<std::timed_mutex> l(op_mu_);
    DeviceGuard g(device_);
    // RCCL group state is thread-local: close the group even after an abort (ignoring its result),
    // or every later NCCL call of this thread — c10d's included — would be deferred into it and hang
    const ncclResult_t r = ncclGroupEnd();
    --group_depth_;
    live();
    check_nccl(r, "ncclGroupEnd");
    if (!group_depth_) settle("ncclGroupEnd");
    return group_depth_ ? nullptr : done();
  }

  // abort: in-flight collectives exit, further calls raise (used by the watchdog hook, which runs on
  // its own thread).  The flag is atomic and set first, so no enqueue starts after it; an enqueue
  // already past its check holds op_mu_, which abort waits for (bounded: an enqueue blocked inside
  // RCCL, e.g. on a peer that never connects, is exactly what ncclCommAbort must release).  comm_
  // itself never changes after construction, so no thread ever reads a nulled handle.  During a
  // non-blocking init only the flag is set: the initialising thread sees it and aborts the comm itself
  // (no second thread touches a half-built communicator).
  void abort() {
    aborted_.store(true);
    if (!inited_.load()) return;
    do_abort();
  }

  std::string async_error() {
    if (aborted_.load()) return "aborted";
    if (!comm_) return "";
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
    return r == ncclSuccess || r == ncclInProgress ? "" : ncclGetErrorString(r);
  }

  static int abort_all() {
    std::lock_guard<std::mutex> l(g_live_mu);
    int n = 0;
    for (Communicator* c : g_live) {
      if (!c->aborted_.load()) {
        c->abort();
        ++n;
      }
    }
    return n;
  }

 private:
  void live() const {
    if (aborted_.load()) throw std::runtime_error("communicator was aborted (collective timeout / abort())");
    if (closed_.load()) throw std::runtime_error("communicator was closed (destroy_process_group)");
  }

  void do_abort() {
    bool expected = false;
    if (!comm_ || !abort_done_.compare_exchange_strong(expected, true)) return;
    std::unique_lock<std::timed_mutex> l(op_mu_, std::defer_lock);
    (void)l.try_lock_for(std::chrono::seconds(2));
    (void)ncclCommAbort(comm_);
  }

  // non-blocking communicator: an enqueue may return ncclInProgress; RCCL needs the state to reach
  // ncclSuccess before the next call on the comm (polled; an abort ends the wait)
  void settle(const char* what) {
    if (!nonblocking_) return;
    ncclResult_t st = ncclInProgress;
    while (true) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
      if (st != ncclInProgress) break;
      if (aborted_.load()) throw std::runtime_error(std::string(what) + ": communicator aborted");
      std::this_thread::yield();
    }
    check_nccl(st, what);
  }

  // ncclCommDestroy once (close() or the destructor); an aborted comm was released by ncclCommAbort
  void release() {
    bool expected = false;
    if (!comm_ || !closed_.compare_exchange_strong(expected, true)) return;
    if (aborted_.load() || !inited_.load()) return;
    std::lock_guard<std::timed_mutex> l(op_mu_);
    (void)hipStreamSynchronize(stream_);
    if (nonblocking_) {
      ncclResult_t st = ncclCommFinalize(comm_);
      // bounded (~20 s): a finalize only waits for work already in flight
      for (int i = 0; st == ncclInProgress && i < 200000; ++i) {
        std::this_thread::sleep_for(std::chrono::microseconds(100));
        if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) st = ncclInternalError;
      }
      if (st == ncclInProgress) {
        (void)ncclCommAbort(comm_);
        return;
      }
    }
    (void)ncclCommDestroy(comm_);
  }
  std::shared_ptr<Work> done() { return std::make_shared<Work>(device_, stream_, pool_); }

  int nranks_, rank_, device_;
  std::shared_ptr<EventPool> pool_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t dep_ = nullptr;
  int group_depth_ = 0;
  int cu_budget_ = 0;
  bool nonblocking_ = false;
  std::atomic<bool> inited_{false}, abort_done_{false}, closed_{false};
  std::atomic<bool> aborted_{false};
  std::timed_mutex op_mu_;  // held across the aborted check + enqueue of every RCCL call
};

void bind_comm(pybind11::module& m) {
  namespace py = pybind11;
  m.def("rccl_unique_id", [] {
    ncclUniqueId id;
    check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("rccl_version", [] {
    int v = 0;
    check_nccl(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  m.def("rccl_abort_all", &Communicator::abort_all, "ncclCommAbort every live communicator of this process");
  m.def("cu_mask_spread", &pda_rt::cu_mask_spread, py::arg("n"), py::arg("ncu"), py::arg("invert") = false,
        "CU mask words: n of ncu CUs spread over the XCDs (the comm stream's budget; invert = the rest)");
  py::class_<Work, std::shared_ptr<Work>>(m, "RcclWork")
      .def("wait", &Work::wait, py::arg("stream"))
      .def("is_completed", &Work::is_completed)
      .def_property_readonly("event", &Work::event)
      .def("synchronize", &Work::synchronize, py::call_guard<py::gil_scoped_release>());
  py::class_<Communicator>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int nranks, int rank, int device, bool high_priority) {
             std::string u = uid;
             py::gil_scoped_release nogil;  // ncclCommInitRank blocks until every rank joined
             return new Communicator(u, nranks, rank, device, high_priority);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("high_priority") = true)
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("size", &Communicator::size)
      .def_property_readonly("device", &Communicator::device)
      .def_property_readonly("stream", &Communicator::stream)
      .def_property_readonly("aborted", &Communicator::aborted)
      .def_property_readonly("closed", &Communicator::closed)
      .def_property_readonly("nonblocking", &Communicator::nonblocking)
      .def_property_readonly("cu_budget", &Communicator::cu_budget)
      .def("close", &Communicator::close, py::call_guard<py::gil_scoped_release>())
      .def("wait_stream", &Communicator::wait_stream)
      .def("wait_event", &Communicator::wait_event)
      .def("all_reduce", &Communicator::all_reduce)
      .def("reduce_scatter", &Communicator::reduce_scatter)
      .def("all_gather", &Communicator::all_gather)
      .def("broadcast", &Communicator::broadcast)
      .def("reduce", &Communicator::reduce)
      .def("send", &Communicator::send)
      .def("recv", &Communicator::recv)
      .def("group_start", &Communicator::group_start)
      .def("group_end", &Communicator::group_end)
      .def("abort", &Communicator::abort)
      .def("async_error", &Communicator::async_error);
  // the watchdog aborts every communicator before it acts on a timed-out collective
  pda_rt::set_abort_hook([] { Communicator::abort_all(); });
  // event-backed watchdog tickets (DDP / FSDP / pipeline collectives) retire on completion; each
  // ticket records and owns its own event on the collective's stream
  pda_rt::EventOps ops;
  ops.record = [](uintptr_t stream) -> uintptr_t {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int dev = -1;
    if (hipStreamGetDevice(s, &dev) != hipSuccess) return 0;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
    hipEvent_t e = nullptr;
    uintptr_t out = 0;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
      if (hipEventRecord(e, s) == hipSuccess) out = reinterpret_cast<uintptr_t>(e);
      else (void)hipEventDestroy(e);
    }
    if (prev != dev && prev >= 0) (void)hipSetDevice(prev);
    return out;
  };
  ops.query = [](uintptr_t ev) -> int {
    const hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(ev));
    return e == hipSuccess ? 1 : (e == hipErrorNotReady ? 0 : -1);
  };
  ops.destroy = [](uintptr_t ev) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)); };
  pda_rt::set_event_ops(ops);
}

}  // namespace pda_comm
