// Collective watchdog (SURVEY §5.3 "a communicator watchdog thread per process enforces a timeout
// per outstanding collective").  The reference has no timeouts at all (torchrun defaults, `NB02:287`);
// a rank that stops participating leaves every other rank blocked inside RCCL forever.
//
// The watchdog is a native thread that never takes the Python GIL, so it keeps running while the
// main thread is blocked in a collective wait.  Callers arm a ticket (description + deadline) when
// they launch a collective and disarm it when the collective completed.  When a ticket outlives its
// deadline the thread prints every pending ticket of this rank to stderr and then either
//   * raises SIGABRT (default: Python's faulthandler, enabled by the framework, dumps every thread's
//     stack, the launcher sees the abnormal exit and tears the job down), or
//   * _exit(code), or
//   * only records the expiry (report mode, used by tests and by callers that poll `expired()`).
#include <atomic>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <stdexcept>
#include <unistd.h>

#include "runtime.h"

namespace pda_rt {

namespace {
std::atomic<void (*)()> g_abort_hook{nullptr};
std::mutex g_ops_mu;
EventOps g_ops;  // set once at module load, read under g_ops_mu

EventOps event_ops() {
  std::lock_guard<std::mutex> g(g_ops_mu);
  return g_ops;
}
}  // namespace

void set_abort_hook(void (*hook)()) { g_abort_hook.store(hook); }
void set_event_ops(const EventOps& ops) {
  std::lock_guard<std::mutex> g(g_ops_mu);
  g_ops = ops;
}

void run_abort_hook() {
  if (auto h = g_abort_hook.load()) h();
}

namespace {
double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}
}  // namespace

Watchdog::Watchdog(double timeout_s, int rank, const std::string& action, int exit_code, double poll_s)
    : timeout_s_(timeout_s), rank_(rank), action_(action), exit_code_(exit_code), poll_s_(poll_s) {
  if (action_ != "abort" && action_ != "exit" && action_ != "report")
    throw std::invalid_argument("Watchdog action must be abort | exit | report");
  thread_ = std::thread([this] { loop(); });
}

Watchdog::~Watchdog() { stop(); }

void Watchdog::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

int64_t Watchdog::arm(const std::string& desc, double timeout_s) {
  std::lock_guard<std::mutex> g(mu_);
  const int64_t id = next_id_++;
  const double t = timeout_s > 0 ? timeout_s : timeout_s_;
  tickets_[id] = Ticket{desc, now_s(), now_s() + t};
  ++armed_total_;
  return id;
}

void Watchdog::erase_locked(std::map<int64_t, Ticket>::iterator it) {
  if (it->second.event) {
    const EventOps ops = event_ops();
    if (ops.destroy) ops.destroy(it->second.event);
  }
  tickets_.erase(it);
}

bool Watchdog::disarm(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = tickets_.find(id);
  if (it == tickets_.end()) return false;
  erase_locked(it);
  return true;
}

bool Watchdog::attach_stream(int64_t id, uintptr_t stream) {
  const EventOps ops = event_ops();
  if (!ops.record || !ops.query || !ops.destroy) return false;
  const uintptr_t ev = ops.record(stream);  // outside the lock: a HIP call
  if (!ev) return false;
  std::lock_guard<std::mutex> g(mu_);
  auto it = tickets_.find(id);
  if (it == tickets_.end() || it->second.event) {
    ops.destroy(ev);
    return false;
  }
  it->second.event = ev;
  return true;
}

size_t Watchdog::armed() const {
  std::lock_guard<std::mutex> g(mu_);
  return tickets_.size();
}

std::vector<std::string> Watchdog::pending() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  const double t = now_s();
  for (auto& kv : tickets_) {
    char buf[64];
    snprintf(buf, sizeof(buf), " (%.1fs)", t - kv.second.start);
    out.push_back(kv.second.desc + buf);
  }
  return out;
}

std::vector<std::string> Watchdog::expired() const {
  std::lock_guard<std::mutex> g(mu_);
  return expired_;
}

int64_t Watchdog::armed_total() const {
  std::lock_guard<std::mutex> g(mu_);
  return armed_total_;
}

void Watchdog::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    // system_clock: wait_for(steady) lowers to pthread_cond_clockwait, which GCC 11's ThreadSanitizer
    // does not intercept (false "double lock" reports); the poll period does not need a steady clock
    cv_.wait_until(lk, std::chrono::system_clock::now() +
                           std::chrono::duration_cast<std::chrono::system_clock::duration>(
                               std::chrono::duration<double>(poll_s_)));
    if (stop_) break;
    // event-backed tickets retire themselves: a collective whose completion event has fired is done
    // whether or not its owner ever gets back to disarm it (e.g. a DDP stage driven by a pipeline
    // schedule, whose forward never runs the owner's sweep)
    if (auto q = event_ops().query) {
      for (auto it = tickets_.begin(); it != tickets_.end();) {
        auto cur = it++;
        if (cur->second.event && !cur->second.reported && q(cur->second.event) == 1) erase_locked(cur);
      }
    }
    const double t = now_s();
    bool fire = false;
    for (auto& kv : tickets_) {
      if (t > kv.second.deadline && !kv.second.reported) {
        kv.second.reported = true;
        expired_.push_back(kv.second.desc);
        fire = true;
      }
    }
    if (!fire) continue;
    fprintf(stderr, "[pda watchdog] rank %d: collective timeout; %zu pending operation(s):\n", rank_,
            tickets_.size());
    for (auto& kv : tickets_)
      fprintf(stderr, "[pda watchdog] rank %d:   #%lld %s pending %.1fs (deadline %.1fs)\n", rank_,
              (long long)kv.first, kv.second.desc.c_str(), t - kv.second.start, kv.second.deadline - kv.second.start);
    fflush(stderr);
    if (action_ == "report") continue;
    // release every RCCL communicator first: their in-flight kernels exit and the streams waiting on
    // them drain, so the abort / exit below does not leave the GPU with a stuck collective
    lk.unlock();
    run_abort_hook();
    lk.lock();
    if (action_ == "exit") {
      fprintf(stderr, "[pda watchdog] rank %d: exiting with code %d\n", rank_, exit_code_);
      fflush(stderr);
      _exit(exit_code_);
    }
    fprintf(stderr, "[pda watchdog] rank %d: aborting (SIGABRT)\n", rank_);
    fflush(stderr);
    lk.unlock();
    std::raise(SIGABRT);
    lk.lock();
  }
}

}  // namespace pda_rt
