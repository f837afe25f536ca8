// Host ring transport: the reference's ring all-reduce concept (`NB02:33-47`:
// scatter-reduce of N chunks over N-1 neighbour steps, then an N-1 step all-gather) made executable
// over TCP for CPU tensors.  Used by the CPU plumbing config (BASELINE config 1) and as a
// correctness cross-check of the device collectives.  Each step sends to the right neighbour while
// receiving from the left one (non-blocking poll loop, so neither side can deadlock on full buffers).
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace pda_rt {

HostRing::HostRing(int rank, int world) : rank_(rank), world_(world) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("HostRing: bad rank/world");
}

HostRing::~HostRing() {
  for (int fd : {listen_fd_, right_fd_, left_fd_})
    if (fd >= 0) close(fd);
}

std::string HostRing::listen(const std::string& host) {
  int port = 0;
  listen_fd_ = tcp_listen(host, 0, &port);
  return host + ":" + std::to_string(port);
}

void HostRing::connect(const std::string& right_host, int right_port, double timeout_s) {
  if (world_ == 1) return;
  // Connect to the right neighbour first, then accept the left one: the listen backlog makes
  // the order deadlock-free.
  right_fd_ = tcp_connect(right_host, right_port, timeout_s);
  left_fd_ = accept(listen_fd_, nullptr, nullptr);
  if (left_fd_ < 0) throw std::runtime_error(std::string("HostRing accept failed: ") + strerror(errno));
  int32_t hello = rank_, got = -1;
  send_all(right_fd_, &hello, 4);
  recv_all(left_fd_, &got, 4);
  if (got != (rank_ + world_ - 1) % world_) throw std::runtime_error("HostRing: unexpected left neighbour");
}

void HostRing::sendrecv(const void* sbuf, size_t sn, void* rbuf, size_t rn) {
  const char* sp = (const char*)sbuf;
  char* rp = (char*)rbuf;
  fcntl(right_fd_, F_SETFL, fcntl(right_fd_, F_GETFL) | O_NONBLOCK);
  fcntl(left_fd_, F_SETFL, fcntl(left_fd_, F_GETFL) | O_NONBLOCK);
  while (sn || rn) {
    pollfd fds[2];
    int nf = 0;
    if (sn) fds[nf++] = {right_fd_, POLLOUT, 0};
    if (rn) fds[nf++] = {left_fd_, POLLIN, 0};
    if (poll(fds, nf, 60000) <= 0) throw std::runtime_error("HostRing: poll timeout / error");
    for (int i = 0; i < nf; ++i) {
      if (!fds[i].revents) continue;
      if (fds[i].fd == right_fd_ && sn) {
        ssize_t k = ::send(right_fd_, sp, sn, MSG_NOSIGNAL);
        if (k < 0 && errno != EAGAIN && errno != EINTR) throw std::runtime_error("HostRing send failed");
        if (k > 0) {
          sp += k;
          sn -= (size_t)k;
        }
      } else if (fds[i].fd == left_fd_ && rn) {
        ssize_t k = ::recv(left_fd_, rp, rn, 0);
        if (k == 0) throw std::runtime_error("HostRing: left neighbour closed");
        if (k < 0 && errno != EAGAIN && errno != EINTR) throw std::runtime_error("HostRing recv failed");
        if (k > 0) {
          rp += k;
          rn -= (size_t)k;
        }
      }
    }
  }
}

template <typename T>
void HostRing::allreduce(T* data, int64_t n) {
  const int W = world_;
  if (W == 1 || n == 0) return;
  std::vector<int64_t> off(W + 1);
  for (int i = 0; i <= W; ++i) off[i] = n * i / W;
  const int64_t maxc = (n + W - 1) / W;
  std::vector<T> tmp(maxc);
  // reduce-scatter: after W-1 steps rank r owns the full sum of chunk (r + 1) % W
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ - s) % W + W) % W, rc = ((rank_ - s - 1) % W + W) % W;
    sendrecv(data + off[sc], (off[sc + 1] - off[sc]) * sizeof(T), tmp.data(), (off[rc + 1] - off[rc]) * sizeof(T));
    T* dst = data + off[rc];
    for (int64_t i = 0; i < off[rc + 1] - off[rc]; ++i) dst[i] += tmp[i];
  }
  // all-gather: circulate the reduced chunks
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ + 1 - s) % W + W) % W, rc = ((rank_ - s) % W + W) % W;
    sendrecv(data + off[sc], (off[sc + 1] - off[sc]) * sizeof(T), data + off[rc],
             (off[rc + 1] - off[rc]) * sizeof(T));
  }
}

void HostRing::allreduce_f32(uintptr_t data, int64_t n) {
  allreduce<float>((float*)data, n);
}
void HostRing::allreduce_f64(uintptr_t data, int64_t n) {
  allreduce<double>((double*)data, n);
}

void HostRing::broadcast(uintptr_t data, int64_t bytes, int root) {
  if (world_ == 1) return;
  // pass along the ring from root; the rank just before root does not forward
  char* p = (char*)data;
  const int dist = ((rank_ - root) % world_ + world_) % world_;
  if (dist != 0) {
    fcntl(left_fd_, F_SETFL, fcntl(left_fd_, F_GETFL) & ~O_NONBLOCK);
    recv_all(left_fd_, p, (size_t)bytes);
  }
  if (dist != world_ - 1) {
    fcntl(right_fd_, F_SETFL, fcntl(right_fd_, F_GETFL) & ~O_NONBLOCK);
    send_all(right_fd_, p, (size_t)bytes);
  }
}

void HostRing::allgather(uintptr_t in, uintptr_t out, int64_t bytes) {
  char* o = (char*)out;
  memcpy(o + rank_ * bytes, (const void*)in, (size_t)bytes);
  for (int s = 0; s < world_ - 1; ++s) {
    const int sc = ((rank_ - s) % world_ + world_) % world_, rc = ((rank_ - s - 1) % world_ + world_) % world_;
    sendrecv(o + sc * bytes, (size_t)bytes, o + rc * bytes, (size_t)bytes);
  }
}

void HostRing::barrier() {
  float x = 0.f;
  allreduce_f32((uintptr_t)&x, 1);
}

// ------------------------------------------------------------------ bindings
}  // namespace pda_rt
