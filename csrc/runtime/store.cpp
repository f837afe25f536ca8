// TCP rendezvous key-value store (reference rendezvous `PY1:18-22`
// MASTER_ADDR/MASTER_PORT + init_process_group, torchrun env:// `PY2:14-18`).
//
// Wire format, client -> server:  u8 op | fields ; strings are u32 length + bytes.
// The server is one poll() event loop: blocking requests (GET on a missing key, WAIT) are parked
// and answered when a SET / ADD / CAS creates the key, so a slow rank never blocks the others.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <deque>
#include <set>
#include <stdexcept>
#include <unordered_map>

#include "runtime.h"

namespace pda_rt {

enum Op : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, WAIT = 5, DEL = 6, NUMKEYS = 7, CAS = 8 };

// ------------------------------------------------------------------ socket helpers
static void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int tcp_listen(const std::string& host, int port, int* bound_port) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  const std::string p = std::to_string(port);
  const char* h = host.empty() ? nullptr : host.c_str();
  if (getaddrinfo(h, p.c_str(), &hints, &res) != 0 || !res) throw std::runtime_error("getaddrinfo failed for " + host);
  int fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (bind(fd, res->ai_addr, res->ai_addrlen) != 0) {
    freeaddrinfo(res);
    close(fd);
    throw std::runtime_error("bind failed on " + host + ":" + p + ": " + strerror(errno));
  }
  freeaddrinfo(res);
  if (::listen(fd, 1024) != 0) {
    close(fd);
    throw std::runtime_error(std::string("listen failed: ") + strerror(errno));
  }
  sockaddr_in sa{};
  socklen_t len = sizeof(sa);
  getsockname(fd, (sockaddr*)&sa, &len);
  if (bound_port) *bound_port = ntohs(sa.sin_port);
  return fd;
}

int tcp_connect(const std::string& host, int port, double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  std::string last_err;
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        set_nodelay(fd);
        return fd;
      }
      last_err = strerror(errno);
      close(fd);
      freeaddrinfo(res);
    } else {
      last_err = "getaddrinfo failed";
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("connect to " + host + ":" + std::to_string(port) + " timed out: " + last_err);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

void send_all(int fd, const void* buf, size_t n) {
  const char* p = (const char*)buf;
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      throw std::runtime_error(std::string("send failed: ") + strerror(errno));
    }
    p += k;
    n -= (size_t)k;
  }
}

void recv_all(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) throw std::runtime_error("peer closed the connection");
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) throw std::runtime_error("socket receive timed out");
      throw std::runtime_error(std::string("recv failed: ") + strerror(errno));
    }
    p += k;
    n -= (size_t)k;
  }
}

// ------------------------------------------------------------------ message encoding
static void put_u32(std::string& s, uint32_t v) { s.append((const char*)&v, 4); }
static void put_i64(std::string& s, int64_t v) { s.append((const char*)&v, 8); }
static void put_str(std::string& s, const std::string& v) {
  put_u32(s, (uint32_t)v.size());
  s.append(v);
}

struct Reader {  // incremental parser over a connection buffer
  const std::string& b;
  size_t pos = 0;
  bool ok = true;
  explicit Reader(const std::string& buf) : b(buf) {}
  bool need(size_t n) {
    if (pos + n > b.size()) ok = false;
    return ok;
  }
  uint8_t u8() {
    if (!need(1)) return 0;
    return (uint8_t)b[pos++];
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t v;
    memcpy(&v, b.data() + pos, 4);
    pos += 4;
    return v;
  }
  int64_t i64() {
    if (!need(8)) return 0;
    int64_t v;
    memcpy(&v, b.data() + pos, 8);
    pos += 8;
    return v;
  }
  std::string str() {
    const uint32_t n = u32();
    if (!ok || !need(n)) return std::string();
    std::string s = b.substr(pos, n);
    pos += n;
    return s;
  }
};

// ------------------------------------------------------------------ server
namespace {
struct Conn {
  int fd;
  std::string in;
};
struct Waiter {
  int fd;
  uint8_t op;                     // GET or WAIT
  std::vector<std::string> keys;  // keys to wait for
};
}  // namespace

StoreServer::StoreServer(const std::string& host, int port) {
  listen_fd_ = tcp_listen(host, port, &port_);
  if (pipe(wake_) != 0) throw std::runtime_error("pipe failed");
  thread_ = std::thread([this] { loop(); });
}

StoreServer::~StoreServer() { stop(); }

void StoreServer::stop() {
  if (stop_.exchange(true)) return;
  char c = 1;
  if (wake_[1] >= 0) (void)!write(wake_[1], &c, 1);
  if (thread_.joinable()) thread_.join();
  if (listen_fd_ >= 0) close(listen_fd_);
  if (wake_[0] >= 0) close(wake_[0]);
  if (wake_[1] >= 0) close(wake_[1]);
  listen_fd_ = wake_[0] = wake_[1] = -1;
}

void StoreServer::loop() {
  std::unordered_map<std::string, std::string> kv;
  std::unordered_map<int, Conn> conns;
  std::deque<Waiter> waiters;

  auto reply = [&](int fd, const std::string& payload) {
    std::string msg;
    put_u32(msg, (uint32_t)payload.size());
    msg += payload;
    try {
      send_all(fd, msg.data(), msg.size());
    } catch (...) {
    }
  };
  auto all_present = [&](const std::vector<std::string>& keys) {
    for (auto& k : keys)
      if (!kv.count(k)) return false;
    return true;
  };
  auto answer_waiter = [&](const Waiter& w) {
    if (w.op == GET) reply(w.fd, kv[w.keys[0]]);
    else reply(w.fd, std::string(1, '\1'));
  };
  auto wake_waiters = [&]() {
    for (auto it = waiters.begin(); it != waiters.end();) {
      if (conns.count(it->fd) && all_present(it->keys)) {
        answer_waiter(*it);
        it = waiters.erase(it);
      } else {
        ++it;
      }
    }
  };

  // Handle one complete request at the head of c.in; returns bytes consumed (0 = incomplete).
  auto handle = [&](Conn& c) -> size_t {
    Reader r(c.in);
    const uint8_t op = r.u8();
    if (!r.ok) return 0;
    switch (op) {
      case SET: {
        std::string k = r.str(), v = r.str();
        if (!r.ok) return 0;
        kv[k] = v;
        reply(c.fd, std::string(1, '\1'));
        wake_waiters();
        break;
      }
      case GET: {
        std::string k = r.str();
        if (!r.ok) return 0;
        if (kv.count(k)) reply(c.fd, kv[k]);
        else waiters.push_back(Waiter{c.fd, GET, {k}});
        break;
      }
      case ADD: {
        std::string k = r.str();
        int64_t d = r.i64();
        if (!r.ok) return 0;
        int64_t v = 0;
        auto it = kv.find(k);
        if (it != kv.end() && !it->second.empty()) v = std::stoll(it->second);
        v += d;
        kv[k] = std::to_string(v);
        std::string out;
        put_i64(out, v);
        reply(c.fd, out);
        wake_waiters();
        break;
      }
      case CHECK:
      case WAIT: {
        const uint32_t n = r.u32();
        std::vector<std::string> keys;
        for (uint32_t i = 0; i < n && r.ok; ++i) keys.push_back(r.str());
        if (!r.ok) return 0;
        if (op == CHECK) reply(c.fd, std::string(1, all_present(keys) ? '\1' : '\0'));
        else if (all_present(keys)) reply(c.fd, std::string(1, '\1'));
        else waiters.push_back(Waiter{c.fd, WAIT, keys});
        break;
      }
      case DEL: {
        std::string k = r.str();
        if (!r.ok) return 0;
        reply(c.fd, std::string(1, kv.erase(k) ? '\1' : '\0'));
        break;
      }
      case NUMKEYS: {
        std::string out;
        put_i64(out, (int64_t)kv.size());
        reply(c.fd, out);
        break;
      }
      case CAS: {
        std::string k = r.str(), expected = r.str(), desired = r.str();
        if (!r.ok) return 0;
        auto it = kv.find(k);
        if (it == kv.end()) {
          if (expected.empty()) kv[k] = desired;
        } else if (it->second == expected) {
          it->second = desired;
        }
        auto now = kv.find(k);
        reply(c.fd, now == kv.end() ? expected : now->second);
        wake_waiters();
        break;
      }
      default:
        return c.in.size();  // protocol error: drop the buffer
    }
    return r.pos;
  };

  while (!stop_) {
    std::vector<pollfd> fds;
    fds.push_back({listen_fd_, POLLIN, 0});
    fds.push_back({wake_[0], POLLIN, 0});
    for (auto& kvp : conns) fds.push_back({kvp.first, POLLIN, 0});
    if (poll(fds.data(), fds.size(), 1000) < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (fds[1].revents) break;
    if (fds[0].revents & POLLIN) {
      int cfd = accept(listen_fd_, nullptr, nullptr);
      if (cfd >= 0) {
        set_nodelay(cfd);
        conns[cfd] = Conn{cfd, std::string()};
      }
    }
    for (size_t i = 2; i < fds.size(); ++i) {
      if (!fds[i].revents) continue;
      const int fd = fds[i].fd;
      char buf[65536];
      ssize_t k = recv(fd, buf, sizeof(buf), 0);
      if (k <= 0) {
        close(fd);
        conns.erase(fd);
        for (auto it = waiters.begin(); it != waiters.end();) it = (it->fd == fd) ? waiters.erase(it) : it + 1;
        continue;
      }
      Conn& c = conns[fd];
      c.in.append(buf, (size_t)k);
      while (!c.in.empty()) {
        const size_t used = handle(c);
        if (used == 0) break;
        c.in.erase(0, used);
      }
    }
  }
  for (auto& kvp : conns) close(kvp.first);
}

// ------------------------------------------------------------------ client
StoreClient::StoreClient(const std::string& host, int port, double timeout_s) : timeout_s_(timeout_s) {
  fd_ = tcp_connect(host, port, timeout_s);
}

StoreClient::~StoreClient() {
  if (fd_ >= 0) close(fd_);
}

std::string StoreClient::request(const std::string& msg, double timeout_s) {
  std::lock_guard<std::mutex> lk(mu_);
  timeval tv{};
  if (timeout_s > 0) {
    tv.tv_sec = (long)timeout_s;
    tv.tv_usec = (long)((timeout_s - (double)tv.tv_sec) * 1e6);
  }
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  send_all(fd_, msg.data(), msg.size());
  uint32_t n;
  recv_all(fd_, &n, 4);
  std::string out(n, '\0');
  if (n) recv_all(fd_, &out[0], n);
  return out;
}

void StoreClient::set(const std::string& key, const std::string& value) {
  std::string m(1, (char)SET);
  put_str(m, key);
  put_str(m, value);
  request(m, timeout_s_);
}

std::string StoreClient::get(const std::string& key) {
  std::string m(1, (char)GET);
  put_str(m, key);
  return request(m, timeout_s_);
}

int64_t StoreClient::add(const std::string& key, int64_t delta) {
  std::string m(1, (char)ADD);
  put_str(m, key);
  put_i64(m, delta);
  const std::string r = request(m, timeout_s_);
  int64_t v;
  memcpy(&v, r.data(), 8);
  return v;
}

bool StoreClient::check(const std::vector<std::string>& keys) {
  std::string m(1, (char)CHECK);
  put_u32(m, (uint32_t)keys.size());
  for (auto& k : keys) put_str(m, k);
  return request(m, timeout_s_)[0] == '\1';
}

void StoreClient::wait(const std::vector<std::string>& keys, double timeout_s) {
  std::string m(1, (char)WAIT);
  put_u32(m, (uint32_t)keys.size());
  for (auto& k : keys) put_str(m, k);
  request(m, timeout_s > 0 ? timeout_s : timeout_s_);
}

bool StoreClient::delete_key(const std::string& key) {
  std::string m(1, (char)DEL);
  put_str(m, key);
  return request(m, timeout_s_)[0] == '\1';
}

int64_t StoreClient::num_keys() {
  std::string m(1, (char)NUMKEYS);
  const std::string r = request(m, timeout_s_);
  int64_t v;
  memcpy(&v, r.data(), 8);
  return v;
}

std::string StoreClient::compare_set(const std::string& key, const std::string& expected,
                                     const std::string& desired) {
  std::string m(1, (char)CAS);
  put_str(m, key);
  put_str(m, expected);
  put_str(m, desired);
  return request(m, timeout_s_);
}

}  // namespace pda_rt
