// Native runtime self-test, built with AddressSanitizer + UndefinedBehaviorSanitizer and, separately,
// ThreadSanitizer (SURVEY §5.2 race detection — host code only; GPU sanitizers are not used on this
// pool).  It drives the rendezvous store, the bucket reducer, the host ring transport and the
// collective watchdog from many threads at once, the way ranks and the autograd engine do.
//
//   tools/sanitize.sh            (or tests/test_sanitizers_cpu.py) builds and runs both flavours
#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

using namespace pda_rt;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static void test_store(int nthreads) {
  StoreServer srv("127.0.0.1", 0);
  std::vector<std::thread> ts;
  std::atomic<int> ok{0};
  for (int t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      StoreClient c("127.0.0.1", srv.port(), 30.0);
      // every client publishes, then blocks on every other client's key (a barrier over the store)
      c.set("k" + std::to_string(t), std::string(100 + t, 'a' + t % 26));
      std::vector<std::string> keys;
      for (int u = 0; u < nthreads; ++u) keys.push_back("k" + std::to_string(u));
      c.wait(keys, 30.0);
      for (int u = 0; u < nthreads; ++u) CHECK(c.get("k" + std::to_string(u)).size() == (size_t)(100 + u));
      for (int i = 0; i < 50; ++i) c.add("ctr", 1);
      c.compare_set("leader", "", std::to_string(t));
      ok++;
    });
  }
  for (auto& th : ts) th.join();
  CHECK(ok == nthreads);
  StoreClient c("127.0.0.1", srv.port(), 5.0);
  CHECK(c.add("ctr", 0) == 50 * nthreads);
  const std::string leader = c.get("leader");
  CHECK(!leader.empty() && std::stoi(leader) < nthreads);
  CHECK(c.delete_key("leader") && !c.check({"leader"}));
  bool timed_out = false;
  try {
    StoreClient d("127.0.0.1", srv.port(), 0.2);
    d.get("never-set");
  } catch (const std::exception&) {
    timed_out = true;
  }
  CHECK(timed_out);
  srv.stop();
  printf("store: %d concurrent clients ok\n", nthreads);
}

static void test_reducer() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 20; ++trial) {
    const int P = 1 + rng() % 60;
    std::vector<int64_t> numels, es;
    std::vector<int> dts;
    for (int i = 0; i < P; ++i) {
      numels.push_back(1 + rng() % 5000);
      es.push_back(rng() % 2 ? 2 : 4);
      dts.push_back(es.back() == 2 ? 1 : 0);
    }
    BucketReducer r(numels, es, dts, 16 << 10, 2 << 10, 8, {});
    std::vector<int> seen(P, 0);
    for (int b = 0; b < r.num_buckets(); ++b)
      for (auto p : r.bucket_params(b)) seen[p]++;
    for (int i = 0; i < P; ++i) CHECK(seen[i] == 1);
    for (int iter = 0; iter < 3; ++iter) {
      r.prepare();
      std::vector<int> order(P);
      for (int i = 0; i < P; ++i) order[i] = i;
      std::shuffle(order.begin(), order.end(), rng);
      std::vector<int> launched;
      for (int p : order)
        for (int b : r.mark_ready(p)) launched.push_back(b);
      CHECK(r.all_launched());
      for (size_t i = 0; i < launched.size(); ++i) CHECK(launched[i] == (int)i);
    }
  }
  printf("reducer: randomized ready orders ok\n");
}

static void test_ring(int W) {
  std::vector<std::unique_ptr<HostRing>> rings;
  std::vector<int> ports;
  for (int r = 0; r < W; ++r) {
    rings.emplace_back(new HostRing(r, W));
    const std::string a = rings[r]->listen("127.0.0.1");
    ports.push_back(std::stoi(a.substr(a.find(':') + 1)));
  }
  std::vector<std::thread> ts;
  std::atomic<int> ok{0};
  for (int r = 0; r < W; ++r) {
    ts.emplace_back([&, r] {
      HostRing& ring = *rings[r];
      ring.connect("127.0.0.1", ports[(r + 1) % W], 10.0);
      for (int n : {1, 7, 1000, 100003}) {
        std::vector<float> v(n);
        for (int i = 0; i < n; ++i) v[i] = (float)(r + 1) * (float)(i % 13);
        ring.allreduce_f32((uintptr_t)v.data(), n);
        const float tot = W * (W + 1) / 2.0f;
        for (int i = 0; i < n; ++i) CHECK(std::fabs(v[i] - tot * (float)(i % 13)) < 1e-3f);
      }
      std::vector<double> b(33, r == 1 % W ? 3.5 : 0.0);
      ring.broadcast((uintptr_t)b.data(), 33 * sizeof(double), 1 % W);
      for (double x : b) CHECK(x == 3.5);
      std::vector<int> mine(4, r), all(4 * W, -1);
      ring.allgather((uintptr_t)mine.data(), (uintptr_t)all.data(), 4 * sizeof(int));
      for (int q = 0; q < W; ++q)
        for (int j = 0; j < 4; ++j) CHECK(all[q * 4 + j] == q);
      ring.barrier();
      ok++;
    });
  }
  for (auto& th : ts) th.join();
  CHECK(ok == W);
  printf("host ring: world %d ok\n", W);
}

static void test_watchdog() {
  Watchdog wd(0.15, 0, "report", 17, 0.02);
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) {
    ts.emplace_back([&, t] {
      for (int i = 0; i < 200; ++i) {
        const int64_t id = wd.arm("op " + std::to_string(t) + "/" + std::to_string(i), 10.0);
        CHECK(wd.disarm(id));
      }
    });
  }
  for (auto& th : ts) th.join();
  const int64_t stuck = wd.arm("stuck all_reduce", -1.0);
  std::this_thread::sleep_for(std::chrono::milliseconds(400));
  CHECK(wd.expired().size() == 1 && wd.expired()[0] == "stuck all_reduce");
  CHECK(wd.armed_total() == 8 * 200 + 1);
  CHECK(wd.disarm(stuck));
  wd.stop();
  printf("watchdog: concurrent arm/disarm + expiry ok\n");
}

int main() {
  test_store(16);
  test_reducer();
  test_ring(2);
  test_ring(5);
  test_watchdog();
  printf("runtime self-test passed\n");
  return 0;
}
