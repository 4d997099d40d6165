// HostTransport: the CPU data plane (host memory + a full TCP mesh).
//
// Exists so the complete engine (schedules, grouped send/recv semantics,
// timing, verification, reports) runs and is tested without a GPU, and as the
// native counterpart of the gloo plumbing config in BASELINE.json
// ("2-rank CPU/gloo send/recv of a 4 KiB buffer").  A group is executed at
// group_end() by a non-blocking progress loop over all of its ops, so the
// symmetric send+recv groups of bi-directional / ring / all-pairs phases
// cannot deadlock on socket buffers — the same guarantee ncclGroupEnd gives.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <thread>
#include <vector>

#include "bootstrap.hpp"
#include "common.hpp"
#include "transport.hpp"

namespace p2p {

void host_fill(void* p, size_t bytes, uint64_t seed) {
  auto* b = static_cast<uint8_t*>(p);
  size_t nw = bytes / 4;
  for (size_t i = 0; i < nw; ++i) {
    const uint32_t w = prng_word(seed, i);
    std::memcpy(b + 4 * i, &w, 4);  // any alignment
  }
  for (size_t i = nw * 4; i < bytes; ++i) b[i] = prng_byte(seed, i);
}

VerifyResult host_verify(const void* p, size_t bytes, uint64_t seed) {
  VerifyResult r;
  const auto* b = static_cast<const uint8_t*>(p);
  size_t nw = bytes / 4;
  for (size_t i = 0; i < nw; ++i) {
    uint32_t got;
    std::memcpy(&got, b + 4 * i, 4);
    r.checksum += got;
    if (got != prng_word(seed, i)) {
      if (!r.mismatches) r.first_bad = 4 * i;
      ++r.mismatches;
    }
  }
  size_t tail = bytes - nw * 4;
  if (tail) {
    uint32_t got = 0, want = prng_word(seed, nw);
    std::memcpy(&got, b + 4 * nw, tail);
    uint32_t mask = (1u << (8 * tail)) - 1u;
    r.checksum += got;
    if ((got & mask) != (want & mask)) {
      if (!r.mismatches) r.first_bad = 4 * nw;
      ++r.mismatches;
    }
  }
  return r;
}

namespace {

void sockopts(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void blocking_io(int fd, void* buf, size_t n, bool is_send, double timeout_s) {
  char* p = static_cast<char*>(buf);
  double deadline = now_seconds() + timeout_s;
  while (n) {
    ssize_t k = is_send ? ::send(fd, p, n, MSG_NOSIGNAL) : ::recv(fd, p, n, 0);
    if (k > 0) {
      p += k;
      n -= static_cast<size_t>(k);
    } else if (k == 0) {
      P2P_FATAL("host transport: peer closed connection");
    } else if (errno != EINTR && errno != EAGAIN) {
      P2P_FATAL(strfmt("host transport io: %s", std::strerror(errno)));
    }
    if (now_seconds() > deadline) P2P_FATAL("host transport: handshake timeout");
  }
}

struct Endpoint {
  char host[64];
  int32_t port;
  uint64_t host_hash;
};

class HostTransport final : public Transport {
 public:
  HostTransport(Bootstrap& boot, const TransportOptions& opt) : rank_(boot.rank()), n_(boot.size()), timeout_(opt.timeout_s) {
    fds_.assign(static_cast<size_t>(n_), -1);
    TcpListener listener(0);
    Endpoint me{};
    std::string hn = real_hostname();  // routable name, not the P2P_HOSTNAME test override
    std::snprintf(me.host, sizeof(me.host), "%s", hn.c_str());
    me.port = listener.port();
    me.host_hash = host_hash(hn);
    auto eps = boot.allgather_value(me);
    int lfd = listener.release();
    // Rank i connects to every j < i; j accepts.
    for (int j = 0; j < rank_; ++j) {
      std::string host = eps[j].host_hash == me.host_hash ? "127.0.0.1" : std::string(eps[j].host);
      fds_[j] = connect_to(host, eps[j].port);
      int32_t id = rank_;
      blocking_io(fds_[j], &id, sizeof(id), true, timeout_);
    }
    for (int got = 0; got < n_ - 1 - rank_; ++got) {
      pollfd p{lfd, POLLIN, 0};
      int rc = ::poll(&p, 1, static_cast<int>(timeout_ * 1000));
      P2P_CHECK(rc > 0, "host transport: timed out waiting for mesh connections");
      int fd = ::accept(lfd, nullptr, nullptr);
      P2P_CHECK(fd >= 0, "accept failed");
      sockopts(fd);
      int32_t id = -1;
      blocking_io(fd, &id, sizeof(id), false, timeout_);
      P2P_CHECK(id > rank_ && id < n_ && fds_[id] < 0, strfmt("bad mesh peer id %d", id));
      fds_[id] = fd;
    }
    ::close(lfd);
    boot.barrier();
  }

  ~HostTransport() override {
    release_discard_sink();
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
  }

  void set_timeout(double seconds) override { timeout_ = seconds; }
  // A CPU transport moves data inside group_end(), so there is no stream to
  // hold.  P2P_TEST_FAKE_GATE=1 (host unit tests) accepts the gate anyway, so
  // run_latency's batched pre-posted path runs on the CPU.
  bool gate_arm(double) override {
    const char* f = std::getenv("P2P_TEST_FAKE_GATE");
    return f && std::atoi(f) != 0;
  }
  std::string name() const override { return "host"; }
  int rank() const override { return rank_; }
  int nranks() const override { return n_; }
  std::string device_desc() const override { return "cpu:" + short_hostname(); }

  void* alloc(size_t bytes) override {
    void* p = nullptr;
    P2P_CHECK(posix_memalign(&p, 256, std::max<size_t>(bytes, 1)) == 0, "host alloc failed");
    return p;
  }
  void release(void* p) override { std::free(p); }
  void fill(void* p, size_t bytes, uint64_t seed) override { host_fill(p, bytes, seed); }
  void zero(void* p, size_t bytes) override { std::memset(p, 0, bytes); }
  VerifyResult verify(const void* p, size_t bytes, uint64_t seed) override { return host_verify(p, bytes, seed); }

  void group_begin() override {
    P2P_CHECK(!in_group_, "nested group");
    in_group_ = true;
    ops_.clear();
  }
  void send(const void* p, size_t bytes, int peer) override {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    ops_.push_back({true, peer, const_cast<char*>(static_cast<const char*>(p)), bytes});
    if (!in_group_) run_ops();
  }
  void recv(void* p, size_t bytes, int peer) override {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    // Injected skip fault: the bytes are read off the wire into a sink.
    ops_.push_back({false, peer, static_cast<char*>(discarding() ? discard_sink(bytes) : p), bytes});
    if (!in_group_) run_ops();
  }
  void group_end() override {
    P2P_CHECK(in_group_, "group_end without group_begin");
    in_group_ = false;
    std::vector<size_t> sent(static_cast<size_t>(n_), 0);
    for (const auto& op : ops_)
      if (op.is_send) sent[static_cast<size_t>(op.peer)] += op.bytes;
    emulate_link_delay(sent, rank_);
    run_ops();
  }

  int mark() override {
    marks_.push_back(now_seconds());
    return static_cast<int>(marks_.size()) - 1;
  }
  double elapsed_ms(int a, int b) override { return (marks_.at(b) - marks_.at(a)) * 1e3; }
  void clear_marks() override { marks_.clear(); }
  void sync() override {}

 private:
  struct Op {
    bool is_send;
    int peer;
    char* buf;
    size_t bytes;
    size_t done = 0;
  };

  int connect_to(const std::string& host, int port) {
    double deadline = now_seconds() + timeout_;
    while (now_seconds() < deadline) {
      addrinfo hints{};
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      addrinfo* res = nullptr;
      if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0) {
        for (addrinfo* ai = res; ai; ai = ai->ai_next) {
          int fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
          if (fd < 0) continue;
          if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
            freeaddrinfo(res);
            sockopts(fd);
            return fd;
          }
          ::close(fd);
        }
        freeaddrinfo(res);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    P2P_FATAL(strfmt("host transport: cannot connect to %s:%d", host.c_str(), port));
  }

  // Progress every op of the group; per peer, sends complete in posting order
  // and receives complete in posting order (NCCL's matching rule).
  void run_ops() {
    std::vector<std::deque<Op*>> sendq(static_cast<size_t>(n_)), recvq(static_cast<size_t>(n_));
    for (auto& op : ops_) (op.is_send ? sendq : recvq)[static_cast<size_t>(op.peer)].push_back(&op);
    // Self transfers: the k-th send to self matches the k-th recv from self.
    auto& ss = sendq[static_cast<size_t>(rank_)];
    auto& rs = recvq[static_cast<size_t>(rank_)];
    P2P_CHECK(ss.size() == rs.size() || !in_group_, "unmatched self send/recv in group");
    while (!ss.empty() && !rs.empty()) {
      P2P_CHECK(ss.front()->bytes == rs.front()->bytes, "self send/recv size mismatch");
      std::memcpy(rs.front()->buf, ss.front()->buf, ss.front()->bytes);
      ss.pop_front();
      rs.pop_front();
    }
    P2P_CHECK(ss.empty() && rs.empty(), "self send without matching recv");
    double deadline = now_seconds() + timeout_;
    for (;;) {
      std::vector<pollfd> pfds;
      for (int p = 0; p < n_; ++p) {
        if (p == rank_) continue;
        short ev = 0;
        if (!sendq[p].empty()) ev |= POLLOUT;
        if (!recvq[p].empty()) ev |= POLLIN;
        if (ev) pfds.push_back({fds_[p], ev, 0});
      }
      if (pfds.empty()) break;
      int rc = ::poll(pfds.data(), pfds.size(), 100);
      if (rc < 0 && errno == EINTR) continue;
      P2P_CHECK(rc >= 0, "poll failed");
      if (rc == 0) {
        if (now_seconds() > deadline) P2P_FATAL("host transport: group timed out (peer hung or dead)");
        if (abort_requested()) abort_wait("host transport");
        continue;
      }
      for (auto& pf : pfds) {
        int peer = static_cast<int>(std::find(fds_.begin(), fds_.end(), pf.fd) - fds_.begin());
        if (pf.revents & (POLLERR | POLLNVAL)) P2P_FATAL(strfmt("host transport: socket error with peer %d", peer));
        if ((pf.revents & POLLOUT) && !sendq[peer].empty()) {
          Op* op = sendq[peer].front();
          ssize_t k = ::send(pf.fd, op->buf + op->done, op->bytes - op->done, MSG_NOSIGNAL | MSG_DONTWAIT);
          if (k > 0) op->done += static_cast<size_t>(k);
          else if (k < 0 && errno != EAGAIN && errno != EINTR)
            P2P_FATAL(strfmt("host transport send to %d: %s", peer, std::strerror(errno)));
          if (op->done == op->bytes) sendq[peer].pop_front();
        }
        if ((pf.revents & (POLLIN | POLLHUP)) && !recvq[peer].empty()) {
          Op* op = recvq[peer].front();
          ssize_t k = ::recv(pf.fd, op->buf + op->done, op->bytes - op->done, MSG_DONTWAIT);
          // Re-arm quick ACKs: a delayed ACK stalls a sender whose message is
          // larger than its current send window.
          int one = 1;
          setsockopt(pf.fd, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof(one));
          if (k > 0) op->done += static_cast<size_t>(k);
          else if (k == 0) P2P_FATAL(strfmt("host transport: peer %d closed the connection", peer));
          else if (errno != EAGAIN && errno != EINTR)
            P2P_FATAL(strfmt("host transport recv from %d: %s", peer, std::strerror(errno)));
          if (op->done == op->bytes) recvq[peer].pop_front();
        }
      }
    }
    ops_.clear();
  }

  int rank_, n_;
  double timeout_;
  std::vector<int> fds_;
  bool in_group_ = false;
  std::vector<Op> ops_;
  std::vector<double> marks_;
};

}  // namespace

std::unique_ptr<Transport> make_host_transport(Bootstrap& boot, const TransportOptions& opt) {
  return std::make_unique<HostTransport>(boot, opt);
}

}  // namespace p2p
