// Data plane abstraction: buffers, grouped point-to-point ops, timestamps.
//
// The measurement engine (runner.cpp) is written against this interface only.
// Implementations:
//   * RcclTransport (transport_rccl.cpp, HIP + RCCL): MI355X device buffers in
//     HBM3E, ncclSend/ncclRecv over xGMI inside ncclGroupStart/End (reference
//     call sites p2p_matrix.cc:156-169, 211-249), hipEvent timestamps on the
//     comm stream, hand-written gfx950 fill/verify kernels.
//   * IpcTransport (transport_ipc.cpp, HIP): one-sided pulls from hipIpc-mapped
//     peer send buffers by the gfx950 multi-copy kernel (or SDMA) — the
//     hand-written data plane, and the multi-rank path on one GPU.
//   * HostTransport (transport_host.cpp): host memory over a TCP mesh, steady
//     clock timestamps.  Same schedule, same runner, same report — it is the
//     CPU plumbing path (BASELINE.json config 1) and what the CPU test tier
//     drives, so the whole engine is exercised without a GPU.
//   * ShmTransport (transport_shm.cpp): host memory over lock-free rings in
//     one POSIX shared-memory segment; the single-host CPU path without
//     syscalls per message.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "prng.hpp"

namespace p2p {

class Bootstrap;

class Transport {
 public:
  virtual ~Transport() = default;
  virtual std::string name() const = 0;
  virtual int rank() const = 0;
  virtual int nranks() const = 0;
  virtual std::string device_desc() const { return ""; }
  // Names the memory this rank allocates from: ranks with the same non-empty
  // key share one GPU's HBM (host name + PCI bus id); "" for host memory.
  virtual std::string device_key() const { return ""; }

  // ---- memory ----
  // Free / total device memory, when the transport knows it (sizing checks).
  virtual bool mem_info(size_t* /*free_bytes*/, size_t* /*total_bytes*/) { return false; }
  virtual void* alloc(size_t bytes) = 0;
  virtual void release(void* p) = 0;
  // Stream-ordered fill of `bytes` with the PRNG stream `seed`.
  virtual void fill(void* p, size_t bytes, uint64_t seed) = 0;
  // Stream-ordered zeroing (used to poison receive buffers before a cell).
  virtual void zero(void* p, size_t bytes) = 0;
  // Blocking: compares `bytes` at p against the PRNG stream `seed`.
  virtual VerifyResult verify(const void* p, size_t bytes, uint64_t seed) = 0;
  // Blocking: result i == verify(jobs[i]).  GPU transports check the whole
  // list in batched launches with one readback and one sync (the post-timing
  // check of many receive slots); the default checks one buffer at a time.
  struct VerifyJob {
    const void* p = nullptr;
    size_t bytes = 0;
    uint64_t seed = 0;
  };
  virtual std::vector<VerifyResult> verify_many(const std::vector<VerifyJob>& jobs) {
    std::vector<VerifyResult> out;
    out.reserve(jobs.size());
    for (const auto& j : jobs) out.push_back(verify(j.p, j.bytes, j.seed));
    return out;
  }

  // ---- data plane: one group == one fused launch ----
  virtual void group_begin() = 0;
  virtual void send(const void* p, size_t bytes, int peer) = 0;
  virtual void recv(void* p, size_t bytes, int peer) = 0;
  virtual void group_end() = 0;
  // A receive of the message the peer sends from `src_offset` bytes into its
  // registered send buffer (the step driver gives every message of a step its
  // own region there, so each carries its own payload).  One-sided pull
  // transports read from that offset; two-sided ones match by order and
  // ignore it.
  virtual void recv_from(void* p, size_t bytes, int peer, size_t /*src_offset*/) { recv(p, bytes, peer); }
  // A send whose payload lands in receive slot `remote_slot` of the peer's
  // buffer set (the receiver's index of this sender in its recv list).  Push
  // transports need it to address the peer's memory; the rest ignore it.
  virtual void send_to_slot(const void* p, size_t bytes, int peer, int /*remote_slot*/) { send(p, bytes, peer); }
  // Multi-path transports (IPC relay engine) move parts of a message through
  // ranks that are neither its sender nor its receiver, so every rank must
  // know every flow of a group.  When wants_group_flows() is true the runner
  // posts every group on EVERY rank (also ranks without sends or receives of
  // their own) and calls group_flows() right after group_begin(), once per
  // message of each flow, with the identical list on every rank;
  // `set_send` names the buffer set (its send buffer on this rank).  The
  // endpoints then post their send / recv calls as usual.
  struct GroupFlow {
    int src = -1;
    int dst = -1;
    int slot = 0;           // receive slot of the flow on dst
    size_t src_offset = 0;  // where the message starts in src's send buffer
  };
  virtual bool wants_group_flows() const { return false; }
  virtual void group_flows(const void* /*set_send*/, const std::vector<GroupFlow>& /*flows*/, size_t /*bytes*/) {}

  // ---- timing ----
  // Enqueue a timestamp behind all work posted so far; returns its id.
  virtual int mark() = 0;
  // Milliseconds between two marks; only valid after sync().
  virtual double elapsed_ms(int from, int to) = 0;
  virtual void clear_marks() = 0;
  // Consecutive messages that may run side by side on independent streams
  // (RCCL with K communicators: K).  Marks then record completion frontiers
  // of overlapping messages, so per-message samples are taken over rounds of
  // this many marks (run_phase).
  virtual int concurrency() const { return 1; }
  // Wait for all posted work (bounded by the transport's watchdog timeout).
  virtual void sync() = 0;
  // Teardown's wait (destructors of buffers and drivers): like sync() but
  // never throws.  False when the work did not finish; the caller then
  // leaks rather than free memory under running kernels.  RCCL aborts its
  // communicators past the timeout (or on an abort request) first.
  virtual bool drain_quietly() {
    try {
      sync();
      return true;
    } catch (const std::exception&) {
      return false;
    }
  }

  // A buffer set: one send buffer plus `nslots` receive slots of
  // `slot_bytes`, `stride` bytes apart in one receive arena (slot i at
  // recv + i * stride).  The number of slots may differ between ranks.
  struct BufferSet {
    void* send = nullptr;
    size_t send_bytes = 0;
    void* recv = nullptr;
    size_t stride = 0;
    size_t slot_bytes = 0;
    int nslots = 0;
  };
  // Collective: called by every rank, in the same order, right after it
  // allocated a buffer set (Buffers' constructor / destructor).  One-sided
  // transports map the peers' send buffers (and, when they write remotely,
  // receive arenas) here and route a receive into a slot of the set to the
  // same set's send buffer on the peer; two-sided ones (RCCL, host) ignore it.
  virtual void register_buffers(const BufferSet& /*set*/) {}
  virtual void unregister_buffers(void* /*send*/) {}

  // ---- graphs: record posted work once, replay it with one launch ----
  // Between capture_begin() and capture_end() nothing executes; the returned
  // handle replays the recorded groups with graph_launch().  Transports that
  // cannot capture return false from supports_graphs().
  virtual bool supports_graphs() const { return false; }
  virtual void capture_begin() {}
  virtual int capture_end() { return -1; }
  virtual void graph_launch(int /*handle*/) {}
  // Frees a captured graph (its handle must not be launched again); after a
  // drain of the stream that replays it.
  virtual void graph_release(int /*handle*/) {}

  // ---- device-initiated ping-pong (one-sided transports) ----
  // pingpong_setup() is collective (every rank, same order).  Then both
  // partners call device_pingpong(peer = each other, same bytes / iters), or
  // one rank calls it with peer == rank() for the self path.  Blocking;
  // returns the leader's (lower rank's) per-iteration one-way times in
  // microseconds (half of each device-timed round trip), empty on the
  // follower.
  virtual bool supports_device_pingpong() const { return false; }
  virtual void pingpong_setup() {}
  virtual std::vector<double> device_pingpong(int /*peer*/, size_t /*bytes*/, int /*iters*/) { return {}; }
  // Ring token chain on the device (after pingpong_setup()): every rank
  // calls it with its predecessor and successor; rank `leader` injects the
  // token and returns the `laps` lap times in microseconds (empty elsewhere).
  // Each hop forwards only after the token arrived: a dependent chain.
  virtual std::vector<double> device_ring_token(int /*pred*/, int /*succ*/, bool /*leader*/, size_t /*bytes*/,
                                                int /*laps*/) {
    return {};
  }

  // ---- stream gate (pre-posted latency, run_latency with preposted > 0) ----
  // gate_arm() enqueues a one-wave kernel that holds the stream carrying
  // small messages until gate_release() (or `timeout_s`); what is posted in
  // between then runs back to back on the GPU with no host in the loop, so
  // per-message marks time the operation itself, not the host's posting rate.
  // Returns false where there is nothing to gate (CPU transports).
  // gate_timed_out() (after sync) reports a gate that expired instead.
  virtual bool gate_arm(double /*timeout_s*/) { return false; }
  virtual void gate_release() {}
  virtual bool gate_timed_out() { return false; }

  // ---- message chunking (RCCL) ----
  // Largest single op a message to a peer is posted as (0 = unsplit): the
  // limit the transport derived for that peer, capped by set_chunk_cap(cap)
  // (0 lifts the cap).  Both ends of a message must split it alike, so callers
  // set the cap collectively.  false / 0 where nothing is split.
  virtual bool set_chunk_cap(size_t /*bytes*/) { return false; }
  virtual size_t chunk_cap() const { return 0; }
  virtual size_t max_chunk(int /*peer*/) const { return 0; }
  // Collective (every rank, same order): re-derive the per-peer op limits
  // from what the data plane connected (RCCL: its connection lines, which
  // exist only after the lazy connects of a warm-up).  True on every rank when
  // any rank's limits changed: graphs that recorded ops must be captured
  // again.  Transports without per-peer limits return false.
  virtual bool refine_op_limits(Bootstrap& /*boot*/) { return false; }

  // What the data plane set up towards each peer, as a JSON object (RCCL: the
  // p2p channels its INFO log reports per communicator, the transport each
  // peer connection uses, the op limit derived from them); "" where there is
  // nothing to report.  Local (not collective); call it after the runs, once
  // the lazy connections exist.
  virtual std::string link_report() { return ""; }
  // Per peer, the class of transport the data plane reaches it through
  // ("P2P", "SHM", "NET", "self"; "" unknown or not connected); empty where
  // the transport has no such notion.
  virtual std::vector<std::string> peer_transports() { return {}; }

  // ---- health ----
  // Non-empty when the transport saw an asynchronous error (e.g. a peer died).
  virtual std::string async_error() { return ""; }
  // Seconds any one wait (sync, rendezvous, init) may take before the
  // transport aborts; callers shrink it as a global deadline approaches.
  virtual void set_timeout(double /*seconds*/) {}

  // ---- fault injection (P2P_INJECT_FAULT=skip@<rank>) ----
  // While set, this rank's transfers still run their protocol (so no peer
  // hangs) but move no payload into the receive slots they name: receives
  // land in a private sink, one-sided writers skip their copies.  It
  // emulates a data plane that silently drops timed transfers; verification
  // after timing must catch it.
  void set_discard(bool on) { discard_ = on; }
  bool discarding() const { return discard_; }

 protected:
  // Scratch of at least `bytes` that discarded receives land in (allocated
  // with alloc(); the transport frees it in its destructor through
  // release_discard_sink()).
  void* discard_sink(size_t bytes) {
    if (bytes > sink_bytes_) {
      if (sink_) release(sink_);
      sink_ = alloc(bytes);
      sink_bytes_ = bytes;
    }
    return sink_;
  }
  void release_discard_sink() {
    if (sink_) release(sink_);
    sink_ = nullptr;
    sink_bytes_ = 0;
  }

 private:
  bool discard_ = false;
  void* sink_ = nullptr;
  size_t sink_bytes_ = 0;
};

struct TransportOptions {
  int device = -1;                 // -1: local rank from placement
  double timeout_s = 300.0;        // watchdog for init / sync
  bool nonblocking_init = true;    // RCCL: ncclCommInitRankConfig(blocking=0) + polling
  int verify_impl = 0;             // dev::VerifyImpl: 0 auto (= 1), 1 LDS-DMA staged (lds8), 2 register staged (stride)
  // IPC transport: kernel (gfx950 pull kernel) | sdma | push (rendezvous +
  // remote writes) | relay (push over the direct link plus two-hop relays
  // through the other GPUs, routing.hpp)
  std::string ipc_engine = "kernel";
  bool two_streams = false;        // RCCL: receives on a second stream (reference layout)
  int rccl_comms = 1;              // RCCL: communicators per rank, messages spread over them (P2P_RCCL_COMMS)
  bool rccl_stock = false;         // RCCL: leave its kernel unroll alone (--reference)
};

// HIP + RCCL on the local MI355X.  Defined in transport_rccl.cpp (hipcc).
std::unique_ptr<Transport> make_rccl_transport(Bootstrap& boot, const TransportOptions& opt);
bool rccl_transport_available();

// One-sided pulls through hipIpc-mapped peer send buffers, moved by the
// gfx950 multi-copy kernel (or the SDMA engines).  Defined in
// transport_ipc.cpp.  Intra-node only; several ranks may share one GPU.
std::unique_ptr<Transport> make_ipc_transport(Bootstrap& boot, const TransportOptions& opt);

// Host memory over TCP sockets.  Defined in transport_host.cpp.
std::unique_ptr<Transport> make_host_transport(Bootstrap& boot, const TransportOptions& opt);

// Host memory over single-producer / single-consumer rings in one POSIX
// shared-memory segment (all ranks on one host).  Defined in transport_shm.cpp.
std::unique_ptr<Transport> make_shm_transport(Bootstrap& boot, const TransportOptions& opt);

// CPU reference of the verify kernel, bit-compatible with it (tests and the
// host transport use it).
VerifyResult host_verify(const void* p, size_t bytes, uint64_t seed);
void host_fill(void* p, size_t bytes, uint64_t seed);

}  // namespace p2p
