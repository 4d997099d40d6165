// ShmTransport: the CPU data plane over POSIX shared memory (one host).
//
// The host transport (transport_host.cpp) moves bytes through TCP loopback
// sockets; every message pays two syscalls and the kernel's socket copy, so a
// 4 KiB one-way message costs 6.7-8.5 us (CPU plumbing config:
// "2-rank CPU/gloo send/recv of a 4 KiB buffer"; gloo itself: 36-65 us).
// Here every ordered pair (a -> b) owns a single-producer / single-consumer
// byte ring in one shared segment:
//
//   [ head | pad ][ tail | pad ][ ring of R bytes ]   per channel, 64-B lines
//
// The sender copies into the ring at head % R and publishes head with a
// release store; the receiver sees it with an acquire load, copies out and
// publishes tail.  No syscall, no lock: a 4 KiB message is two memcpys and two
// cache-line handoffs.  Group semantics are those of the host transport: a
// group runs at group_end() as one non-blocking progress loop over all of its
// ops (per peer, sends and receives complete in posting order), so the
// symmetric send+recv groups of bi / ring / all-pairs phases cannot deadlock
// on a full ring.
//
// The segment is created by rank 0 (shm_open + ftruncate), its name travels
// over the bootstrap, every rank maps it, and rank 0 unlinks it as soon as all
// ranks have mapped it, so nothing is left in /dev/shm even if a rank dies.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <thread>
#include <vector>

#include "bootstrap.hpp"
#include "common.hpp"
#include "transport.hpp"
#include "units.hpp"

namespace p2p {
namespace {

constexpr size_t kLine = 64;

struct ChannelHeader {
  alignas(kLine) std::atomic<uint64_t> head;  // bytes written by the sender
  alignas(kLine) std::atomic<uint64_t> tail;  // bytes consumed by the receiver
};
static_assert(sizeof(ChannelHeader) == 2 * kLine, "channel header is two cache lines");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory rings need lock-free 64-bit atomics");

struct SegmentName {
  char name[64];
  uint64_t host_hash;
  uint64_t ring_bytes;
};

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

class ShmTransport final : public Transport {
 public:
  ShmTransport(Bootstrap& boot, const TransportOptions& opt) : rank_(boot.rank()), n_(boot.size()), timeout_(opt.timeout_s) {
    // 1 MiB per ordered pair, shrunk so the segment stays within 256 MiB
    // (n^2 rings) for large jobs; P2P_SHM_RING overrides.
    const size_t pairs = static_cast<size_t>(n_) * static_cast<size_t>(n_);
    ring_ = std::max<size_t>(size_t{64} << 10, std::min<size_t>(size_t{1} << 20, (size_t{256} << 20) / pairs) / kLine * kLine);
    if (const char* r = std::getenv("P2P_SHM_RING")) ring_ = parse_size(r);
    P2P_CHECK(ring_ >= 4096 && ring_ % kLine == 0, "P2P_SHM_RING must be a multiple of 64 bytes, at least 4 KiB");
    const uint64_t my_hash = host_hash(real_hostname());
    SegmentName seg{};
    if (rank_ == 0) {
      std::snprintf(seg.name, sizeof(seg.name), "/p2p_shm_%d_%llx", static_cast<int>(getpid()),
                    static_cast<unsigned long long>(now_seconds() * 1e9) & 0xffffffffull);
      seg.host_hash = my_hash;
      seg.ring_bytes = ring_;
    }
    boot.bcast(&seg, sizeof(seg), 0);
    P2P_CHECK(seg.host_hash == my_hash, strfmt("shm transport is single-host only: rank %d is not on rank 0's host", rank_));
    ring_ = seg.ring_bytes;
    stride_ = sizeof(ChannelHeader) + ring_;
    bytes_ = stride_ * static_cast<size_t>(n_) * static_cast<size_t>(n_);
    if (rank_ == 0) {
      int fd = ::shm_open(seg.name, O_CREAT | O_EXCL | O_RDWR, 0600);
      P2P_CHECK(fd >= 0, strfmt("shm_open(%s): %s", seg.name, std::strerror(errno)));
      if (::ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
        ::close(fd);
        ::shm_unlink(seg.name);
        P2P_FATAL(strfmt("ftruncate of the %zu-byte shm segment: %s", bytes_, std::strerror(errno)));
      }
      map(fd);
      for (int a = 0; a < n_; ++a)
        for (int b = 0; b < n_; ++b) {
          ChannelHeader* h = header(a, b);
          new (h) ChannelHeader();
          h->head.store(0, std::memory_order_relaxed);
          h->tail.store(0, std::memory_order_relaxed);
        }
      std::atomic_thread_fence(std::memory_order_release);
    }
    boot.barrier();  // the segment exists and is initialised
    if (rank_ != 0) {
      int fd = ::shm_open(seg.name, O_RDWR, 0600);
      P2P_CHECK(fd >= 0, strfmt("shm_open(%s) on rank %d: %s", seg.name, rank_, std::strerror(errno)));
      map(fd);
    }
    boot.barrier();  // every rank has mapped it
    if (rank_ == 0) ::shm_unlink(seg.name);
  }

  ~ShmTransport() override {
    release_discard_sink();
    if (base_) ::munmap(base_, bytes_);
  }

  void set_timeout(double seconds) override { timeout_ = seconds; }
  std::string name() const override { return "shm"; }
  int rank() const override { return rank_; }
  int nranks() const override { return n_; }
  std::string device_desc() const override { return "cpu:" + short_hostname() + " shm"; }

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

  void map(int fd) {
    void* p = ::mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    P2P_CHECK(p != MAP_FAILED, strfmt("mmap of the shm segment: %s", std::strerror(errno)));
    base_ = static_cast<char*>(p);
  }
  ChannelHeader* header(int from, int to) const {
    return reinterpret_cast<ChannelHeader*>(base_ + stride_ * (static_cast<size_t>(from) * n_ + static_cast<size_t>(to)));
  }
  char* ring(int from, int to) const { return reinterpret_cast<char*>(header(from, to)) + sizeof(ChannelHeader); }

  // Moves as much of a send as the ring has room for; returns bytes moved.
  size_t push(Op* op) {
    ChannelHeader* h = header(rank_, op->peer);
    const uint64_t head = h->head.load(std::memory_order_relaxed);
    const uint64_t tail = h->tail.load(std::memory_order_acquire);
    size_t n = std::min<size_t>(ring_ - static_cast<size_t>(head - tail), op->bytes - op->done);
    if (n == 0) return 0;
    char* r = ring(rank_, op->peer);
    const size_t at = static_cast<size_t>(head % ring_);
    const size_t first = std::min(n, ring_ - at);
    std::memcpy(r + at, op->buf + op->done, first);
    if (n > first) std::memcpy(r, op->buf + op->done + first, n - first);
    h->head.store(head + n, std::memory_order_release);
    op->done += n;
    return n;
  }
  // Moves as much of a receive as the ring holds; returns bytes moved.
  size_t pull(Op* op) {
    ChannelHeader* h = header(op->peer, rank_);
    const uint64_t tail = h->tail.load(std::memory_order_relaxed);
    const uint64_t head = h->head.load(std::memory_order_acquire);
    size_t n = std::min<size_t>(static_cast<size_t>(head - tail), op->bytes - op->done);
    if (n == 0) return 0;
    const char* r = ring(op->peer, rank_);
    const size_t at = static_cast<size_t>(tail % ring_);
    const size_t first = std::min(n, ring_ - at);
    std::memcpy(op->buf + op->done, r + at, first);
    if (n > first) std::memcpy(op->buf + op->done + first, r, n - first);
    h->tail.store(tail + n, std::memory_order_release);
    op->done += n;
    return n;
  }

  // Progress every op of the group; per peer, sends complete in posting order
  // and receives complete in posting order (NCCL's matching rule).  Spins
  // (with pause) while the peers make progress, yields after a while, and
  // gives up at the transport's timeout.
  void run_ops() {
    if (ops_.size() == 1 && ops_[0].peer != rank_) {
      // One message (ping-pong, pair cells): spin on it alone, no queues.
      Op& op = ops_[0];
      double deadline = 0;
      for (long idle = 0; op.done < op.bytes;) {
        if ((op.is_send ? push(&op) : pull(&op)) > 0) {
          idle = 0;
          deadline = 0;
        } else if (++idle >= 4096) {
          const double now = now_seconds();
          if (deadline == 0) deadline = now + timeout_;
          if (now > deadline) P2P_FATAL("shm transport: message timed out (peer hung or dead)");
          if (abort_requested()) abort_wait("shm transport");
          std::this_thread::yield();
        } else {
          cpu_relax();
        }
      }
      ops_.clear();
      return;
    }
    std::vector<std::deque<Op*>> sendq(static_cast<size_t>(n_)), recvq(static_cast<size_t>(n_));
    for (auto& op : ops_) (op.is_send ? sendq : recvq)[static_cast<size_t>(op.peer)].push_back(&op);
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
    size_t pending = 0;
    for (int p = 0; p < n_; ++p) pending += sendq[static_cast<size_t>(p)].size() + recvq[static_cast<size_t>(p)].size();
    double deadline = 0;
    for (long idle = 0; pending;) {
      bool moved = false;
      for (int p = 0; p < n_; ++p) {
        auto& sq = sendq[static_cast<size_t>(p)];
        while (!sq.empty() && (push(sq.front()) > 0 || sq.front()->done == sq.front()->bytes)) {
          moved = true;
          if (sq.front()->done < sq.front()->bytes) break;
          sq.pop_front();
          --pending;
        }
        auto& rq = recvq[static_cast<size_t>(p)];
        while (!rq.empty() && (pull(rq.front()) > 0 || rq.front()->done == rq.front()->bytes)) {
          moved = true;
          if (rq.front()->done < rq.front()->bytes) break;
          rq.pop_front();
          --pending;
        }
      }
      if (moved) {
        idle = 0;
        deadline = 0;
        continue;
      }
      if (++idle < 4096) {
        cpu_relax();
        continue;
      }
      const double now = now_seconds();
      if (deadline == 0) deadline = now + timeout_;
      if (now > deadline) P2P_FATAL("shm transport: group timed out (peer hung or dead)");
      if (abort_requested()) abort_wait("shm transport");
      std::this_thread::yield();
    }
    ops_.clear();
  }

  int rank_, n_;
  double timeout_;
  size_t ring_ = 0, stride_ = 0, bytes_ = 0;
  char* base_ = nullptr;
  bool in_group_ = false;
  std::vector<Op> ops_;
  std::vector<double> marks_;
};

}  // namespace

std::unique_ptr<Transport> make_shm_transport(Bootstrap& boot, const TransportOptions& opt) {
  return std::make_unique<ShmTransport>(boot, opt);
}

}  // namespace p2p
