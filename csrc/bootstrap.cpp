// LocalBootstrap, TcpBootstrap, bootstrap selection and host placement.
#include "bootstrap.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <set>
#include <thread>

#include "common.hpp"

namespace p2p {

double Bootstrap::allreduce_max(double v) {
  auto all = allgather_value(v);
  return *std::max_element(all.begin(), all.end());
}

double Bootstrap::allreduce_sum(double v) {
  double s = 0;
  for (double x : allgather_value(v)) s += x;
  return s;
}

uint64_t Bootstrap::allreduce_sum_u64(uint64_t v) {
  uint64_t s = 0;
  for (uint64_t x : allgather_value(v)) s += x;
  return s;
}

// ---------------------------------------------------------------- local ----

namespace {

class LocalBootstrap final : public Bootstrap {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  void allgather(const void* mine, void* all, size_t bytes) override {
    if (bytes) std::memcpy(all, mine, bytes);
  }
  void bcast(void*, size_t, int root) override { P2P_CHECK(root == 0, "bad root"); }
  void barrier() override {}
  void abort(int) override {}
  std::string name() const override { return "local"; }
};

// ------------------------------------------------------------------ tcp ----

void set_sockopts(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// Waits until fd is readable/writable or the deadline passes.  A requested
// abort (bench.py's deadline watchdog) ends the wait too, so the thread leaves
// the engine and the watchdog can abort the communicators (abort_if_idle).
void wait_fd(int fd, short events, double deadline, const char* what) {
  for (;;) {
    double left = deadline - now_seconds();
    if (left <= 0) P2P_FATAL(strfmt("bootstrap timeout while %s", what));
    if (abort_requested()) P2P_FATAL(strfmt("bootstrap wait aborted while %s (the run's deadline passed)", what));
    pollfd p{fd, events, 0};
    int ms = static_cast<int>(std::min(left, 1.0) * 1000) + 1;
    int rc = ::poll(&p, 1, ms);
    if (rc < 0 && errno == EINTR) continue;
    if (rc < 0) P2P_FATAL(strfmt("poll failed while %s: %s", what, std::strerror(errno)));
    if (rc > 0) {
      if (p.revents & (POLLERR | POLLNVAL)) P2P_FATAL(strfmt("socket error while %s", what));
      return;
    }
  }
}

void send_all(int fd, const void* buf, size_t n, double timeout_s) {
  const char* p = static_cast<const char*>(buf);
  double deadline = now_seconds() + timeout_s;
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (k > 0) {
      p += k;
      n -= static_cast<size_t>(k);
      continue;
    }
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) {
      wait_fd(fd, POLLOUT, deadline, "sending");
      continue;
    }
    P2P_FATAL(strfmt("bootstrap send failed (peer gone?): %s", k < 0 ? std::strerror(errno) : "closed"));
  }
}

void recv_all(int fd, void* buf, size_t n, double timeout_s) {
  char* p = static_cast<char*>(buf);
  double deadline = now_seconds() + timeout_s;
  while (n) {
    ssize_t k = ::recv(fd, p, n, MSG_DONTWAIT);
    if (k > 0) {
      p += k;
      n -= static_cast<size_t>(k);
      continue;
    }
    if (k == 0) P2P_FATAL("bootstrap peer closed the connection (a rank died or aborted)");
    if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) {
      wait_fd(fd, POLLIN, deadline, "receiving");
      continue;
    }
    P2P_FATAL(strfmt("bootstrap recv failed: %s", std::strerror(errno)));
  }
}

int connect_with_retry(const std::string& host, int port, double timeout_s) {
  double deadline = now_seconds() + timeout_s;
  std::string last_err = "no attempt";
  int backoff_ms = 10;
  while (now_seconds() < deadline) {
    addrinfo hints{};
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    int gai = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (gai != 0) {
      last_err = gai_strerror(gai);
    } else {
      for (addrinfo* ai = res; ai; ai = ai->ai_next) {
        int fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
        if (fd < 0) continue;
        if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
          freeaddrinfo(res);
          set_sockopts(fd);
          return fd;
        }
        last_err = std::strerror(errno);
        ::close(fd);
      }
      freeaddrinfo(res);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(backoff_ms));
    backoff_ms = std::min(backoff_ms * 2, 500);
  }
  P2P_FATAL(strfmt("could not connect to bootstrap root %s:%d: %s", host.c_str(), port, last_err.c_str()));
}

class TcpBootstrap final : public Bootstrap {
 public:
  TcpBootstrap(int rank, int size, const std::string& host, int port, double timeout_s, TcpListener* listener)
      : rank_(rank), size_(size), timeout_(timeout_s) {
    P2P_CHECK(size >= 1 && rank >= 0 && rank < size, strfmt("bad rank %d / size %d", rank, size));
    if (size == 1) return;
    if (rank == 0) {
      int lfd;
      if (listener) {
        lfd = listener->release();
      } else {
        TcpListener l(port);
        lfd = l.release();
      }
      peers_.assign(static_cast<size_t>(size), -1);
      double deadline = now_seconds() + timeout_s;
      for (int got = 0; got < size - 1;) {
        wait_fd(lfd, POLLIN, deadline, "accepting bootstrap peers");
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) {
          if (errno == EINTR || errno == EAGAIN) continue;
          P2P_FATAL(strfmt("accept failed: %s", std::strerror(errno)));
        }
        set_sockopts(fd);
        int32_t hello[2];
        recv_all(fd, hello, sizeof(hello), timeout_s);
        P2P_CHECK(hello[1] == size, strfmt("peer reports world size %d, expected %d", hello[1], size));
        P2P_CHECK(hello[0] > 0 && hello[0] < size && peers_[hello[0]] < 0, strfmt("bad/duplicate rank %d", hello[0]));
        peers_[static_cast<size_t>(hello[0])] = fd;
        ++got;
      }
      ::close(lfd);
    } else {
      root_ = connect_with_retry(host, port, timeout_s);
      int32_t hello[2] = {rank, size};
      send_all(root_, hello, sizeof(hello), timeout_s);
    }
    P2P_DEBUG("tcp bootstrap up: rank %d/%d", rank, size);
  }

  ~TcpBootstrap() override { close_all(); }

  void set_timeout(double seconds) override { timeout_ = seconds; }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return "tcp"; }

  void allgather(const void* mine, void* all, size_t bytes) override {
    char* out = static_cast<char*>(all);
    if (bytes) std::memcpy(out + static_cast<size_t>(rank_) * bytes, mine, bytes);
    if (size_ == 1) return;
    if (rank_ == 0) {
      for (int r = 1; r < size_; ++r) recv_all(peers_[r], out + static_cast<size_t>(r) * bytes, bytes, timeout_);
      for (int r = 1; r < size_; ++r) send_all(peers_[r], out, bytes * static_cast<size_t>(size_), timeout_);
    } else {
      send_all(root_, mine, bytes, timeout_);
      recv_all(root_, out, bytes * static_cast<size_t>(size_), timeout_);
    }
  }

  void bcast(void* buf, size_t bytes, int root) override {
    if (size_ == 1) return;
    if (root != 0) {  // route through rank 0
      if (rank_ == root) send_all(root_, buf, bytes, timeout_);
      if (rank_ == 0) recv_all(peers_[root], buf, bytes, timeout_);
    }
    if (rank_ == 0) {
      for (int r = 1; r < size_; ++r)
        if (r != root) send_all(peers_[r], buf, bytes, timeout_);
    } else if (rank_ != root) {
      recv_all(root_, buf, bytes, timeout_);
    }
  }

  void barrier() override {
    char c = 0;
    std::vector<char> all(static_cast<size_t>(size_));
    allgather(&c, all.data(), 1);
  }

  void abort(int) override { close_all(); }

 private:
  void close_all() {
    for (int& fd : peers_)
      if (fd >= 0) {
        ::close(fd);
        fd = -1;
      }
    if (root_ >= 0) {
      ::close(root_);
      root_ = -1;
    }
  }

  int rank_, size_;
  double timeout_;
  int root_ = -1;
  std::vector<int> peers_;
};

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

}  // namespace

TcpListener::TcpListener(int port, const std::string& bind_addr) {
  fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  P2P_CHECK(fd_ >= 0, "socket() failed");
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  P2P_CHECK(inet_pton(AF_INET, bind_addr.c_str(), &addr.sin_addr) == 1, "bad bind address " + bind_addr);
  if (::bind(fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
    P2P_FATAL(strfmt("bootstrap bind to port %d failed: %s", port, std::strerror(errno)));
  P2P_CHECK(::listen(fd_, 1024) == 0, "listen() failed");
  socklen_t len = sizeof(addr);
  getsockname(fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
}

TcpListener::~TcpListener() {
  if (fd_ >= 0) ::close(fd_);
}

int TcpListener::release() {
  int fd = fd_;
  fd_ = -1;
  P2P_CHECK(fd >= 0, "listener already released");
  return fd;
}

std::unique_ptr<Bootstrap> make_local_bootstrap() { return std::make_unique<LocalBootstrap>(); }

std::unique_ptr<Bootstrap> make_tcp_bootstrap(int rank, int size, const std::string& host, int port, double timeout_s,
                                              TcpListener* listener) {
  return std::make_unique<TcpBootstrap>(rank, size, host, port, timeout_s, listener);
}

namespace {
MpiFactory g_mpi_factory = nullptr;
}

void register_mpi_factory(MpiFactory f) { g_mpi_factory = f; }
bool mpi_available() { return g_mpi_factory != nullptr; }

bool mpi_launch_detected() {
  for (const char* v : {"PMI_RANK", "PMI_SIZE", "OMPI_COMM_WORLD_RANK", "PMIX_RANK", "MPI_LOCALRANKID"})
    if (std::getenv(v)) return true;
  return false;
}

std::unique_ptr<Bootstrap> make_bootstrap(const std::string& kind, int* argc, char*** argv) {
  std::string k = kind;
  if (k == "auto") {
    if (mpi_launch_detected())
      k = "mpi";
    else if (std::getenv("RANK") && std::getenv("WORLD_SIZE"))
      k = "env";
    else
      k = "local";
  }
  if (k == "mpi") {
    if (!g_mpi_factory) P2P_FATAL("this binary has no MPI support (the Python extension uses the TCP bootstrap)");
    return g_mpi_factory(argc, argv);
  }
  if (k == "env") {
    int rank = env_int("RANK", 0), size = env_int("WORLD_SIZE", 1);
    const char* addr = std::getenv("MASTER_ADDR");
    int port = env_int("P2P_BOOTSTRAP_PORT", env_int("MASTER_PORT", 29500) + 1);
    double timeout = env_int("P2P_BOOTSTRAP_TIMEOUT", 600);
    return make_tcp_bootstrap(rank, size, addr ? addr : "127.0.0.1", port, timeout);
  }
  if (k == "local") return make_local_bootstrap();
  P2P_FATAL("unknown bootstrap '" + kind + "' (auto|mpi|env|local)");
}

// ------------------------------------------------------------ placement ----

uint64_t host_hash(const std::string& s) {
  // Same recurrence as getHostHash (p2p_matrix.cc:44-51): h = (h*33) ^ c,
  // seeded with 5381; chars are sign-extended like the reference's `char`.
  uint64_t h = 5381;
  for (char c : s) h = ((h << 5) + h) ^ static_cast<uint64_t>(static_cast<int64_t>(static_cast<signed char>(c)));
  return h;
}

std::string short_hostname() {
  // P2P_HOSTNAME overrides gethostname(): lets the placement tests emulate a
  // multi-host job on one machine.
  if (const char* o = std::getenv("P2P_HOSTNAME")) return o;
  char buf[1024] = {0};
  if (gethostname(buf, sizeof(buf) - 1) != 0) return "unknown";
  std::string h(buf);
  auto dot = h.find('.');
  if (dot != std::string::npos) h.resize(dot);
  return h;
}

std::string real_hostname() {
  char buf[1024] = {0};
  if (gethostname(buf, sizeof(buf) - 1) != 0) return "localhost";
  return buf;
}

Placement compute_placement(const std::vector<uint64_t>& hashes, int rank) {
  Placement p;
  int size = static_cast<int>(hashes.size());
  std::set<uint64_t> uniq(hashes.begin(), hashes.end());
  p.num_hosts = static_cast<int>(uniq.size());
  if (size == 0 || p.num_hosts == 0) {
    p.error = "empty job";
    return p;
  }
  if (size % p.num_hosts != 0) {
    p.error = strfmt("%d ranks cannot be split evenly over %d hosts", size, p.num_hosts);
    return p;
  }
  p.ranks_per_host = size / p.num_hosts;
  for (int h = 0; h < p.num_hosts; ++h) {
    for (int i = 1; i < p.ranks_per_host; ++i) {
      if (hashes[h * p.ranks_per_host + i] != hashes[h * p.ranks_per_host]) {
        // The reference's message says "round-robin" (p2p_matrix.cc:96) but the
        // rule it enforces is block placement; say so.
        p.error = strfmt(
            "ranks must be placed in contiguous blocks of %d per host (block placement); rank %d is not on the "
            "same host as rank %d",
            p.ranks_per_host, h * p.ranks_per_host + i, h * p.ranks_per_host);
        return p;
      }
    }
  }
  p.host_index = rank / p.ranks_per_host;
  p.local_rank = rank % p.ranks_per_host;
  p.ok = true;
  return p;
}

Placement check_placement(Bootstrap& boot) {
  uint64_t mine = host_hash(short_hostname());
  auto all = boot.allgather_value(mine);
  return compute_placement(all, boot.rank());
}

}  // namespace p2p
