// Native host runtime of pytorchdistributed_amd (SURVEY §2.3 N02 TCPStore/rendezvous, N03 DDP
// Reducer, §5.8 host ring transport, §5.3 watchdog).  Plain C++17 + POSIX: no HIP, torch or Python
// dependency (bindings live in bind_runtime.cpp), so it builds into the sanitizer self-test.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pda_rt {

// ------------------------------------------------------------------ CU masks
// n of ncu CU bits (the hipExtStreamCreateWithCUMask word array), spread so that they land evenly on the 8
// XCDs whether the logical CU ids run XCD-major (CU i on XCD i / (ncu / 8)) or round-robin (CU i on XCD
// i % 8): bit k sits in block k % 8 of ncu / 8 CUs at offset (k % 8 + 8 j + j / 4) mod (ncu / 8), j = k / 8.
// invert: the complement (the CUs a mask of n leaves to everything else).
inline std::vector<uint32_t> cu_mask_spread(int n, int ncu, bool invert = false) {
  std::vector<uint32_t> m((ncu + 31) / 32, 0u);
  const int blk = ncu / 8 > 0 ? ncu / 8 : 1;
  int placed = 0;
  for (int k = 0; placed < n && k < 64 * ncu; ++k) {
    const int r = k % 8, j = k / 8;
    const int bit = (r * blk + (r + 8 * j + j / 4) % blk) % ncu;
    if (m[bit / 32] & (1u << (bit % 32))) continue;
    m[bit / 32] |= 1u << (bit % 32);
    ++placed;
  }
  if (invert) {
    for (int b = 0; b < ncu; ++b) m[b / 32] ^= 1u << (b % 32);
  }
  return m;
}

// ------------------------------------------------------------------ sockets
int tcp_listen(const std::string& host, int port, int* bound_port);
int tcp_connect(const std::string& host, int port, double timeout_s);
void send_all(int fd, const void* buf, size_t n);
void recv_all(int fd, void* buf, size_t n);

// ------------------------------------------------------------------ TCP key-value store
// Rendezvous store with torch c10d Store semantics (set/get/add/wait/check/delete/compare_set).
// Rank 0 (or the launcher) hosts the server; every rank owns one client connection.
class StoreServer {
 public:
  StoreServer(const std::string& host, int port);
  ~StoreServer();
  int port() const { return port_; }
  void stop();

 private:
  void loop();
  int listen_fd_ = -1, port_ = 0;
  int wake_[2] = {-1, -1};
  std::thread thread_;
  std::atomic<bool> stop_{false};
};

class StoreClient {
 public:
  StoreClient(const std::string& host, int port, double timeout_s);
  ~StoreClient();
  void set(const std::string& key, const std::string& value);
  std::string get(const std::string& key);
  int64_t add(const std::string& key, int64_t delta);
  bool check(const std::vector<std::string>& keys);
  void wait(const std::vector<std::string>& keys, double timeout_s);
  bool delete_key(const std::string& key);
  int64_t num_keys();
  std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired);
  void set_timeout(double t) { timeout_s_ = t; }
  double timeout() const { return timeout_s_; }

 private:
  std::string request(const std::string& msg, double timeout_s);
  int fd_ = -1;
  double timeout_s_;
  std::mutex mu_;
};

// ------------------------------------------------------------------ DDP bucket reducer
// Assigns parameters to gradient buckets (reverse registration order ~ backward order, a small first
// bucket so communication starts early, per-dtype buckets, cap in bytes) and tracks readiness.
// Buckets are released strictly in index order so every rank issues collectives in the same order.
class BucketReducer {
 public:
  BucketReducer(const std::vector<int64_t>& numels, const std::vector<int64_t>& elem_sizes,
                const std::vector<int>& dtype_ids, int64_t bucket_cap_bytes, int64_t first_bucket_bytes,
                int64_t align_elems, const std::vector<int64_t>& order);
  int num_buckets() const { return (int)buckets_.size(); }
  std::vector<int64_t> bucket_params(int b) const { return buckets_.at(b).params; }
  std::vector<int64_t> bucket_offsets(int b) const { return buckets_.at(b).offsets; }
  int64_t bucket_numel(int b) const { return buckets_.at(b).numel; }
  int bucket_dtype(int b) const { return buckets_.at(b).dtype; }
  int param_bucket(int64_t p) const { return param_bucket_.at(p); }
  void prepare();
  std::vector<int> mark_ready(int64_t p);
  std::vector<int> flush_unready();  // mark every unready parameter ready (unused params), return buckets
  bool all_launched() const { return next_launch_ == (int)buckets_.size(); }
  bool any_marked() const { return !ready_order_.empty(); }
  std::vector<int64_t> unready_params() const;
  std::vector<int64_t> ready_order() const { return ready_order_; }

 private:
  struct Bucket {
    std::vector<int64_t> params, offsets;
    int64_t numel = 0;
    int dtype = 0;
    int pending = 0;
  };
  std::vector<Bucket> buckets_;
  std::vector<int> param_bucket_;
  std::vector<char> ready_;
  std::vector<int64_t> ready_order_;
  int next_launch_ = 0;
};

// ------------------------------------------------------------------ host ring transport
// The ring algorithm of the reference's DDP chapter (`02 DDP基本概念/02_ddp.ipynb` raw lines
// 33-47: N-1 scatter-reduce steps then N-1 all-gather steps), executable over TCP for CPU tensors.
class HostRing {
 public:
  HostRing(int rank, int world);
  ~HostRing();
  std::string listen(const std::string& host);
  void connect(const std::string& right_host, int right_port, double timeout_s);
  void allreduce_f32(uintptr_t data, int64_t n);
  void allreduce_f64(uintptr_t data, int64_t n);
  void broadcast(uintptr_t data, int64_t bytes, int root);
  void allgather(uintptr_t in, uintptr_t out, int64_t bytes);
  void barrier();
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  template <typename T>
  void allreduce(T* data, int64_t n);
  void sendrecv(const void* sbuf, size_t sn, void* rbuf, size_t rn);
  int rank_, world_;
  int listen_fd_ = -1, right_fd_ = -1, left_fd_ = -1;
};

// ------------------------------------------------------------------ collective watchdog
// Per-process native thread (no GIL) that enforces a deadline on every armed collective; on expiry it
// reports all pending operations and aborts / exits the rank (see watchdog.cpp).
// Process-wide hook run by the watchdog before it acts on a timed-out collective (the RCCL communicators
// register ncclCommAbort of every live communicator here: csrc/comm/communicator.cpp).
void set_abort_hook(void (*hook)());
void run_abort_hook();
// GPU event operations for event-backed tickets (registered by the HIP side, csrc/comm/communicator.cpp):
//   record(stream) -> a NEW event recorded on `stream`, owned by the ticket (0 on failure);
//   query(event)   -> 1 when the event has completed, 0 when not yet, -1 on error;
//   destroy(event) -> releases an event that record() returned.
// A ticket owns its event, so it never queries a handle whose owner (a Python work object, a DDP
// module) was garbage-collected while the ticket was still armed.
struct EventOps {
  uintptr_t (*record)(uintptr_t stream) = nullptr;
  int (*query)(uintptr_t event) = nullptr;
  void (*destroy)(uintptr_t event) = nullptr;
};
void set_event_ops(const EventOps& ops);

class Watchdog {
 public:
  Watchdog(double timeout_s, int rank, const std::string& action, int exit_code, double poll_s);
  ~Watchdog();
  int64_t arm(const std::string& desc, double timeout_s);
  bool disarm(int64_t id);
  // attach the completion point of the armed collective: an event owned by the ticket is recorded on
  // `stream` right behind the collective, and the watchdog thread disarms the ticket by itself once
  // that event has completed.  Returns false when the ticket is gone or no event ops are registered.
  bool attach_stream(int64_t id, uintptr_t stream);
  size_t armed() const;
  std::vector<std::string> pending() const;
  std::vector<std::string> expired() const;
  int64_t armed_total() const;
  double timeout() const { return timeout_s_; }
  void stop();

 private:
  struct Ticket {
    std::string desc;
    double start = 0, deadline = 0;
    bool reported = false;
    uintptr_t event = 0;  // owned: destroyed when the ticket is erased
  };
  void erase_locked(std::map<int64_t, Ticket>::iterator it);
  void loop();
  double timeout_s_;
  int rank_;
  std::string action_;
  int exit_code_;
  double poll_s_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<int64_t, Ticket> tickets_;
  std::vector<std::string> expired_;
  int64_t next_id_ = 1, armed_total_ = 0;
  bool stop_ = false;
  std::thread thread_;
};


}  // namespace pda_rt
