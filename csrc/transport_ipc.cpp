// IpcTransport: one-sided point-to-point over xGMI without RCCL.
//
// Every rank exports its send buffer with hipIpcGetMemHandle when the
// buffers are created (register_buffers, collective); every peer maps it
// with hipIpcOpenMemHandle.  A receive is then a *pull*: the receiver's GPU
// reads the sender's send buffer directly over the xGMI link into its own
// receive buffer.  A send moves nothing (the receiver does the work), which
// is valid for this benchmark because a phase's payload is written once
// (fill + sync + barrier) before any timed receive reads it.
//
// Data movers (TransportOptions::ipc_engine):
//   kernel — one launch of the gfx950 multi-source copy kernel per group
//            (kernels.hip: all receives of the group in one grid, workgroups
//            split by size, 4 x 16 B remote loads in flight per lane);
//   sdma   — hipMemcpyAsync per receive, forked onto one stream per receive
//            slot so the copies of an all-pairs group run concurrently.
//   push   — two-sided rendezvous with remote writes: a receive posts a
//            "ready" flag into the sender's signal page, the sender's stream
//            waits for it (one-wave signal kernel), the multi-copy kernel
//            writes the payload straight into the receiver's slot over xGMI,
//            and a second signal kernel releases it and raises "done" on the
//            receiver, whose stream waits for that.  Real send/recv semantics
//            (a send never overwrites a slot the receiver has not posted) on
//            the direction xGMI handles best (remote stores).
//   relay  — push, multi-path: each message is split into stripes
//            (routing.hpp plan_routes), one over the direct link, written by
//            the sender, and one per two-hop path s -> k -> d through a GPU k
//            whose links s->k and k->d carry no direct flow of the group.
//            k's copy kernel loads its stripe from s's hipIpc-mapped send
//            buffer and stores it into d's mapped receive slot, so the bytes
//            cross s->k and k->d and never touch k's HBM.  Every writer
//            (sender or relay) waits for the receiver's ready flag and raises
//            its done flag, exactly as in push.  The runner posts every group
//            on every rank and passes the group's global flows
//            (Transport::group_flows), so a relay knows what to move.  A
//            single pair of an 8-GPU node can then use up to 7 links; RCCL's
//            ncclSend/ncclRecv (and the reference's NCCL p2p) only ever use
//            the direct one.
//
// Why it exists: it is the hand-written CDNA4 data plane to compare RCCL's
// ncclSend/ncclRecv against on the same links, and, because IPC mappings
// also work between processes on ONE GPU, it lets the complete multi-rank GPU
// engine (events, kernels, verification, every schedule) run on a single
// MI355X, where RCCL refuses duplicate-GPU ranks.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>
#include <vector>

#include "batch_verify.hpp"
#include "bootstrap.hpp"
#include "common.hpp"
#include "hip_check.hpp"
#include "kernels.hpp"
#include "provenance.hpp"
#include "routing.hpp"
#include "stream_gate.hpp"
#include "transport.hpp"
#include "units.hpp"

namespace p2p {
namespace {

struct Export {
  hipIpcMemHandle_t handle;
  uint64_t bytes;
  uint64_t host_hash;
  int32_t device;
  int32_t pid;
};

class IpcTransport final : public Transport {
 public:
  IpcTransport(Bootstrap& boot, const TransportOptions& opt)
      : boot_(boot), rank_(boot.rank()), n_(boot.size()), timeout_(opt.timeout_s), engine_(opt.ipc_engine),
        relay_(engine_ == "relay"), push_(engine_ == "push" || relay_) {
    P2P_CHECK(engine_ == "kernel" || engine_ == "sdma" || engine_ == "push" || relay_,
              "ipc engine must be 'kernel', 'sdma', 'push' or 'relay'");
    if (relay_) route_opt_ = route_options_from_env();
    verify_impl_ = static_cast<dev::VerifyImpl>(opt.verify_impl);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) P2P_FATAL("ipc transport: no HIP device visible");
    device_ = opt.device >= 0 ? opt.device : 0;
    P2P_CHECK(device_ < ndev, strfmt("rank %d wants GPU %d but only %d are visible", rank_, device_, ndev));
    HIPCHECK(hipSetDevice(device_));
    HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&acc_, dev::verify_accum_bytes()));
    HIPCHECK(hipHostMalloc(&acc_host_, sizeof(dev::VerifyAccum), hipHostMallocDefault));
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device_));
    desc_ = strfmt("hip:%d %s (%s, %d CUs) ipc-%s", device_, prop.name, prop.gcnArchName, prop.multiProcessorCount,
                   engine_.c_str());
    int khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_));
    P2P_CHECK(khz > 0, "device reports no wall clock rate");
    tick_hz_ = khz * 1e3;
    if (const char* pc = std::getenv("P2P_IPC_POOL")) pool_cap_ = std::strcmp(pc, "0") ? parse_size(pc) : 0;
    if (const char* ir = std::getenv("P2P_INJECT_EXPORT_REFUSALS")) inject_refusals_ = std::atoi(ir);
    // HIP 7.0's hipIpcOpenMemHandle never returns for a block whose size mod
    // 4 GiB is 2 GiB or more (scripts/ipc_open_probe.hip: 2 and 3.75 and 7 GiB
    // hang, 2 GiB - 2 MiB, 4, 4 GiB + 2 MiB and 5 GiB open in 0.1 s; HIP 7.2
    // opens them all).  Exported blocks are sized around it on such runtimes.
    int hip_rt = 0;
    if (hipRuntimeGetVersion(&hip_rt) != hipSuccess) hip_rt = 0;
    size_fix_ = hip_rt < 70200000;
    if (const char* sf = std::getenv("P2P_IPC_SIZE_FIX")) size_fix_ = std::atoi(sf) != 0;
    if (push_) setup_sync_pages();
  }

  ~IpcTransport() override {
    (void)hipStreamSynchronize(stream_);
    if (relay_ && std::getenv("P2P_RELAY_STATS"))
      std::fprintf(stderr, "p2p_matrix: rank %d relayed %llu bytes in %llu stripes\n", rank_, relayed_bytes_,
                   relayed_stripes_);
    for (auto& r : regs_) close_registration(r);
    regs_.clear();
    release_pingpong();
    release_sync_pages();
    drain_pool();
    for (auto ex : execs_)
      if (ex) (void)hipGraphExecDestroy(ex);
    for (auto s : side_) (void)hipStreamDestroy(s);
    for (auto e : side_done_) (void)hipEventDestroy(e);
    if (fork_) (void)hipEventDestroy(fork_);
    for (auto ev : events_) (void)hipEventDestroy(ev);
    if (acc_) (void)hipFree(acc_);
    if (acc_host_) (void)hipHostFree(acc_host_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  std::string name() const override { return "ipc"; }
  int rank() const override { return rank_; }
  int nranks() const override { return n_; }
  std::string device_desc() const override { return desc_; }
  std::string device_key() const override { return gpu_memory_key(device_); }

  bool mem_info(size_t* free_b, size_t* total_b) override {
    if (hipMemGetInfo(free_b, total_b) != hipSuccess) return false;
    *free_b += pool_bytes_;  // pooled blocks are handed back on demand
    return true;
  }
  // At least 2 MiB, rounded to 2 MiB, so every exported buffer is an
  // allocation of its own.  Each block is exported once, when it is created
  // (see exportable()), and keeps its handle.
  //
  // Released buffers are kept for reuse (up to pool_cap_, 32 GiB, or
  // P2P_IPC_POOL bytes -- lower it when many ranks share one GPU): a buffer
  // set is created per run, and reusing the same exported blocks avoids
  // allocation churn between runs.
  void* alloc(size_t bytes) override {
    constexpr size_t kGrain = size_t{2} << 20;
    size_t size = (std::max<size_t>(bytes, 1) + kGrain - 1) / kGrain * kGrain;
    constexpr size_t k4G = size_t{4} << 30;
    if (size_fix_ && size % k4G >= k4G / 2) size = (size / k4G + 1) * k4G;  // see size_fix_
    for (auto it = pool_.begin(); it != pool_.end(); ++it)
      if (it->second.size == size) {
        void* p = it->first;
        pool_bytes_ -= size;
        blocks_[p] = it->second;
        pool_.erase(it);
        return p;
      }
    Block b;
    b.size = size;
    void* p = exportable(size, &b.handle, [&](void** q) {
      hipError_t e = hipMalloc(q, size);
      if (e != hipSuccess && !pool_.empty()) {  // give the pool back and retry once
        (void)hipGetLastError();
        drain_pool();
        e = hipMalloc(q, size);
      }
      return e;
    });
    blocks_[p] = b;
    return p;
  }
  void release(void* p) override {
    if (!p) return;
    auto it = blocks_.find(p);
    P2P_CHECK(it != blocks_.end(), "release of a buffer this transport did not allocate");
    const Block b = it->second;
    blocks_.erase(it);
    if (pool_bytes_ + b.size <= pool_cap_) {
      pool_.emplace_back(p, b);
      pool_bytes_ += b.size;
    } else {
      HIPCHECK(hipFree(p));
    }
  }
  void fill(void* p, size_t bytes, uint64_t seed) override { dev::launch_fill(p, bytes, seed, stream_); }
  void zero(void* p, size_t bytes) override { HIPCHECK(hipMemsetAsync(p, 0, bytes, stream_)); }

  VerifyResult verify(const void* p, size_t bytes, uint64_t seed) override {
    dev::launch_verify_reset(acc_, stream_);
    dev::launch_verify(p, bytes, seed, acc_, verify_impl_, true, stream_);
    HIPCHECK(hipMemcpyAsync(acc_host_, acc_, sizeof(dev::VerifyAccum), hipMemcpyDeviceToHost, stream_));
    sync();
    VerifyResult r;
    r.mismatches = acc_host_->mismatches;
    r.checksum = acc_host_->checksum;
    r.first_bad = acc_host_->first_bad;
    return r;
  }
  std::vector<VerifyResult> verify_many(const std::vector<VerifyJob>& jobs) override {
    if (jobs.empty()) return {};
    if ((verify_impl_ != dev::VerifyImpl::Auto && verify_impl_ != dev::VerifyImpl::Lds8) || !batch_verify_enabled())
      return Transport::verify_many(jobs);
    return batch_verify(batch_, jobs, stream_, [this] { sync(); });
  }

  // Buffer sets are registered collectively in the same order on every rank,
  // so "the same set" on a peer is the one with the same position.  A receive
  // into one of a set's receive slots pulls from that set's send buffer on the
  // peer (at the message's offset).  Push / relay also map every peer's
  // receive arena: one export per set, slot i at base + i * stride.
  void register_buffers(const BufferSet& set) override {
    if (debug_)
      std::fprintf(stderr, "ipc rank %d: register send %zu B, arena %d x %zu B\n", rank_, set.send_bytes, set.nslots,
                   set.stride);
    Export me{};
    me.handle = handle_of(set.send);
    me.bytes = set.send_bytes;
    me.host_hash = host_hash(real_hostname());
    me.device = device_;
    me.pid = static_cast<int32_t>(getpid());
    auto all = boot_.allgather_value(me);
    Registration reg;
    reg.send = set.send;
    reg.send_bytes = set.send_bytes;
    reg.recv = set.recv;
    reg.stride = set.stride;
    reg.slot_bytes = set.slot_bytes;
    reg.nslots = set.nslots;
    reg.peer_send.assign(static_cast<size_t>(n_), nullptr);
    for (int r = 0; r < n_; ++r) {
      if (r == rank_) {
        reg.peer_send[static_cast<size_t>(r)] = set.send;
        continue;
      }
      P2P_CHECK(all[static_cast<size_t>(r)].host_hash == me.host_hash,
                strfmt("ipc transport is intra-node only: rank %d is on another host", r));
      P2P_CHECK(all[static_cast<size_t>(r)].bytes == set.send_bytes,
                "ipc transport: send buffers differ in size across ranks");
      void* mapped = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&mapped, all[static_cast<size_t>(r)].handle, hipIpcMemLazyEnablePeerAccess));
      reg.peer_send[static_cast<size_t>(r)] = mapped;
      if (debug_) std::fprintf(stderr, "ipc rank %d: mapped send buffer of rank %d\n", rank_, r);
    }
    if (push_) {
      // The sender (or a relay) writes into the receiver's slot: map every
      // peer's receive arena.  Slot counts may differ between ranks.
      ArenaExport a{};
      a.handle = handle_of(set.recv);
      a.stride = set.stride;
      a.nslots = set.nslots;
      auto arenas = boot_.allgather_value(a);
      reg.peer_recv.assign(static_cast<size_t>(n_), nullptr);
      reg.peer_nslots.assign(static_cast<size_t>(n_), 0);
      for (int r = 0; r < n_; ++r) {
        P2P_CHECK(arenas[static_cast<size_t>(r)].stride == set.stride, "ipc transport: receive slots differ in size");
        void* mapped = set.recv;
        if (r != rank_)
          HIPCHECK(hipIpcOpenMemHandle(&mapped, arenas[static_cast<size_t>(r)].handle, hipIpcMemLazyEnablePeerAccess));
        reg.peer_recv[static_cast<size_t>(r)] = mapped;
        reg.peer_nslots[static_cast<size_t>(r)] = arenas[static_cast<size_t>(r)].nslots;
        if (debug_) std::fprintf(stderr, "ipc rank %d: mapped receive arena of rank %d\n", rank_, r);
      }
    }
    regs_.push_back(std::move(reg));
    boot_.barrier();
  }

  void unregister_buffers(void* send) override {
    auto it = std::find_if(regs_.begin(), regs_.end(), [&](const Registration& r) { return r.send == send; });
    if (it == regs_.end()) return;
    sync();
    // Every rank stops moving data before any mapping goes, and every rank
    // has closed its mappings of a buffer before its owner releases it.
    boot_.barrier();
    close_registration(*it);
    regs_.erase(it);
    boot_.barrier();
  }

  void group_begin() override {
    P2P_CHECK(!in_group_, "nested group");
    in_group_ = true;
    ops_.clear();
    covered_.clear();
  }

  bool wants_group_flows() const override { return relay_; }

  // Relay engine: plans every flow of the group (identically on every rank)
  // and posts this rank's part of each: the direct stripe as its sender, the
  // stripes routed through it as a relay, the flags as the receiver.  The
  // endpoints' own send / recv calls for these flows are then checks only.
  void group_flows(const void* set_send, const std::vector<GroupFlow>& flows, size_t bytes) override {
    if (!relay_) return;
    P2P_CHECK(in_group_, "group_flows outside a group");
    const Registration* reg = nullptr;
    for (const auto& r : regs_)
      if (r.send == set_send) reg = &r;
    P2P_CHECK(reg && bytes <= reg->slot_bytes, "ipc relay: flows of an unregistered buffer set");
    std::vector<std::pair<int, int>> pairs;
    pairs.reserve(flows.size());
    for (const auto& f : flows) pairs.emplace_back(f.src, f.dst);
    const auto plan = plan_routes(n_, pairs, bytes, route_opt_);
    for (size_t i = 0; i < flows.size(); ++i) {
      const GroupFlow& f = flows[i];
      if (f.src == f.dst) continue;  // self flows: the endpoint's send / recv copy locally
      P2P_CHECK(f.src_offset + bytes <= reg->send_bytes, "ipc relay: message outside the send buffer");
      char* slot = remote_slot_ptr(*reg, f.dst, f.slot);
      for (const Stripe& st : plan[i]) {
        const int writer = st.via < 0 ? f.src : st.via;
        if (rank_ == writer) {
          const char* src = static_cast<const char*>(reg->peer_send[static_cast<size_t>(f.src)]) + f.src_offset;
          if (!discarding()) ops_.push_back({src + st.offset, slot + st.offset, st.bytes, true});
          push_sends_.push_back(f.dst);  // wait for its ready, raise its done
          if (st.via >= 0) {
            relayed_bytes_ += st.bytes;
            ++relayed_stripes_;
          }
        }
        if (rank_ == f.dst) push_recvs_.push_back(writer);  // post ready, wait for done
      }
      if (rank_ == f.src || rank_ == f.dst) covered_.push_back({f.src, f.dst, f.slot});
    }
  }

  void send(const void* p, size_t bytes, int peer) override { send_to_slot(p, bytes, peer, 0); }
  void send_to_slot(const void* p, size_t bytes, int peer, int slot) override {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    const Registration* reg = nullptr;
    for (const auto& r : regs_)
      if (p >= r.send && static_cast<const char*>(p) + bytes <= static_cast<const char*>(r.send) + r.send_bytes &&
          bytes <= r.slot_bytes)
        reg = &r;
    P2P_CHECK(reg, "ipc transport sends only from a registered send buffer");
    if (!push_) return;  // nothing to move: the receiver pulls
    if (take_covered(rank_, peer, slot)) return;  // posted by group_flows
    char* dst = remote_slot_ptr(*reg, peer, slot);
    // Injected skip fault: the rendezvous runs, the payload stays behind.
    if (!discarding()) ops_.push_back({p, dst, bytes, peer != rank_});
    if (peer != rank_) push_sends_.push_back(peer);
    if (!in_group_) flush();
  }
  void recv(void* p, size_t bytes, int peer) override { recv_from(p, bytes, peer, 0); }
  void recv_from(void* p, size_t bytes, int peer, size_t src_offset) override {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    const Registration* reg = nullptr;
    int slot = -1;
    for (const auto& r : regs_) {
      const int s = slot_of(r, p);
      if (s >= 0 && bytes <= r.slot_bytes) {
        reg = &r;
        slot = s;
      }
    }
    P2P_CHECK(reg, "ipc transport receives only into a registered receive slot");
    if (push_) {
      if (take_covered(peer, rank_, slot)) return;  // posted by group_flows
      if (peer != rank_) push_recvs_.push_back(peer);  // a self receive is the self send's copy
      if (!in_group_) flush();
      return;
    }
    P2P_CHECK(src_offset + bytes <= reg->send_bytes, "ipc transport: receive beyond the peer's send buffer");
    // Injected skip fault: the pull is not issued.
    if (!discarding())
      ops_.push_back({static_cast<const char*>(reg->peer_send[static_cast<size_t>(peer)]) + src_offset, p, bytes,
                      peer != rank_});
    if (!in_group_) flush();
  }
  void group_end() override {
    P2P_CHECK(in_group_, "group_end without group_begin");
    in_group_ = false;
    P2P_CHECK(covered_.empty(), "ipc relay: group_flows named a flow this rank did not post");
    flush();
  }

  int mark() override {
    if (next_event_ == static_cast<int>(events_.size())) {
      hipEvent_t ev;
      HIPCHECK(hipEventCreateWithFlags(&ev, timing_event_flags()));
      events_.push_back(ev);
    }
    HIPCHECK(hipEventRecord(events_[static_cast<size_t>(next_event_)], stream_));
    return next_event_++;
  }
  double elapsed_ms(int a, int b) override {
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, events_.at(static_cast<size_t>(a)), events_.at(static_cast<size_t>(b))));
    return ms;
  }
  void clear_marks() override { next_event_ = 0; }

  // Push / relay: the flag values are baked into each launch, so a replay
  // would wait for flags that were already consumed; no graphs there.
  bool supports_graphs() const override { return engine_ == "kernel"; }
  void capture_begin() override { HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal)); }
  int capture_end() override {
    hipGraph_t g = nullptr;
    HIPCHECK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t ex = nullptr;
    HIPCHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    HIPCHECK(hipGraphDestroy(g));
    execs_.push_back(ex);
    return static_cast<int>(execs_.size()) - 1;
  }
  void graph_launch(int h) override {
    hipGraphExec_t ex = execs_.at(static_cast<size_t>(h));
    P2P_CHECK(ex != nullptr, "graph_launch: the graph was released");
    HIPCHECK(hipGraphLaunch(ex, stream_));
  }
  void graph_release(int h) override {
    hipGraphExec_t& ex = execs_.at(static_cast<size_t>(h));
    if (ex) HIPCHECK(hipGraphExecDestroy(ex));
    ex = nullptr;
  }

  // Signal pages: every rank owns one page of n + 1 inbox slots (slot r =
  // messages from rank r, slot n = replies of the self path), exported over
  // hipIpc so peers write into it directly.  Uncached device memory when the
  // runtime allows it, so the spinning wave reads HBM, not a stale line.
  bool gate_arm(double timeout_s) override {
    gate_.arm(stream_, timeout_s);
    return true;
  }
  void gate_release() override { gate_.release(); }
  bool gate_timed_out() override { return gate_.timed_out(); }
  bool supports_device_pingpong() const override { return true; }
  void pingpong_setup() override {
    if (ping_ready_) return;  // same state on every rank: they all set up together
    // Set only once everything below completed: a setup that
    // failed half way (the bounded sync() timed out or was aborted) leaves no
    // page_ behind that a later call would take for a finished setup.
    try {
      pingpong_setup_once();
    } catch (...) {
      release_pingpong();
      throw;
    }
    ping_ready_ = true;
  }

  void release_pingpong() {
    for (size_t r = 0; r < peer_pages_.size(); ++r)
      if (peer_pages_[r] && static_cast<int>(r) != rank_) (void)hipIpcCloseMemHandle(peer_pages_[r]);
    peer_pages_.clear();
    if (page_) (void)hipFree(page_);
    if (ping_scratch_) (void)hipFree(ping_scratch_);
    if (ping_host_) (void)hipHostFree(ping_host_);
    page_ = ping_scratch_ = nullptr;
    ping_host_ = nullptr;
    sent_.clear();
    recvd_.clear();
    ping_ready_ = false;
  }

  void pingpong_setup_once() {
    const size_t bytes = kPingSlot * static_cast<size_t>(n_ + 1);
    Export me{};
    page_ = exportable(bytes, &me.handle, [&](void** q) { return alloc_signal_page(q, bytes); });
    // Stream-ordered and waited for with the bounded sync(): a device-wide
    // synchronize would also wait, unbounded, for any other session's work.
    HIPCHECK(hipMemsetAsync(page_, 0, bytes, stream_));
    sync();
    me.bytes = bytes;
    me.host_hash = host_hash(real_hostname());
    me.device = device_;
    me.pid = static_cast<int32_t>(getpid());
    auto all = boot_.allgather_value(me);
    peer_pages_.assign(static_cast<size_t>(n_), nullptr);
    for (int r = 0; r < n_; ++r) {
      if (r == rank_) {
        peer_pages_[static_cast<size_t>(r)] = page_;
        continue;
      }
      P2P_CHECK(all[static_cast<size_t>(r)].host_hash == me.host_hash,
                strfmt("device ping-pong is intra-node only: rank %d is on another host", r));
      void* mapped = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&mapped, all[static_cast<size_t>(r)].handle, hipIpcMemLazyEnablePeerAccess));
      peer_pages_[static_cast<size_t>(r)] = mapped;
    }
    sent_.assign(static_cast<size_t>(n_), 0);
    recvd_.assign(static_cast<size_t>(n_), 0);
    HIPCHECK(hipMalloc(&ping_scratch_, kPingScratch));
    HIPCHECK(hipHostMalloc(&ping_host_, kPingScratch, hipHostMallocDefault));
    boot_.barrier();
  }

  std::vector<double> device_pingpong(int peer, size_t bytes, int iters) override {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    const bool self = peer == rank_;
    dev::PingRole a = ping_role(bytes, iters);
    a.leader = (self || rank_ < peer) ? 1 : 0;
    if (self) {
      // Both waves on this GPU: a writes slot `rank`, the reply wave slot n.
      a.base = a.in_base = sent_[static_cast<size_t>(rank_)];
      a.out_flag = reinterpret_cast<unsigned long long*>(ping_slot(page_, rank_));
      a.out_payload = ping_slot(page_, rank_) + kPingHeader;
      a.in_flag = reinterpret_cast<const unsigned long long*>(ping_slot(page_, n_));
      a.in_payload = ping_slot(page_, n_) + kPingHeader;
      dev::PingRole b = a;  // the reply wave: mirror image through slot n
      b.leader = 0;
      b.out_flag = const_cast<unsigned long long*>(a.in_flag);
      b.out_payload = const_cast<unsigned char*>(a.in_payload);
      b.in_flag = a.out_flag;
      b.in_payload = a.out_payload;
      dev::launch_pingpong(a, &b, stream_);
      sent_[static_cast<size_t>(rank_)] += static_cast<unsigned long long>(iters);
    } else {
      set_links(&a, peer, peer);
      dev::launch_pingpong(a, nullptr, stream_);
      sent_[static_cast<size_t>(peer)] += static_cast<unsigned long long>(iters);
      recvd_[static_cast<size_t>(peer)] += static_cast<unsigned long long>(iters);
    }
    return finish_ping(a.leader != 0, iters, 2.0, strfmt("device ping-pong with rank %d", peer));
  }

  std::vector<double> device_ring_token(int pred, int succ, bool leader, size_t bytes, int laps) override {
    P2P_CHECK(pred >= 0 && pred < n_ && succ >= 0 && succ < n_ && pred != rank_ && succ != rank_,
              "ring token: predecessor and successor must be other ranks");
    dev::PingRole a = ping_role(bytes, laps);
    a.leader = leader ? 1 : 0;
    set_links(&a, pred, succ);
    dev::launch_pingpong(a, nullptr, stream_);
    sent_[static_cast<size_t>(succ)] += static_cast<unsigned long long>(laps);
    recvd_[static_cast<size_t>(pred)] += static_cast<unsigned long long>(laps);
    return finish_ping(leader, laps, 1.0, strfmt("ring token (from %d, to %d)", pred, succ));
  }

  void set_timeout(double seconds) override { timeout_ = seconds; }

  void sync() override {
    double deadline = now_seconds() + timeout_;
    double t0 = now_seconds();
    for (long it = 0;; ++it) {
      hipError_t e = hipStreamQuery(stream_);
      if (e == hipSuccess) {
        if (sig_status_ && (*sig_status_ & 1u))
          P2P_FATAL(strfmt("rank %d: ipc push rendezvous timed out (a peer never posted its side)", rank_));
        return;
      }
      if (e != hipErrorNotReady) P2P_FATAL(strfmt("stream error: %s", hipGetErrorString(e)));
      if ((it & 255) == 0) {
        if (abort_requested()) {
          note_abort_done();
          P2P_FATAL(strfmt("rank %d: aborted while waiting (the run's deadline passed)", rank_));
        }
        double now = now_seconds();
        if (now > deadline) P2P_FATAL(strfmt("rank %d: ipc stream did not finish within %.0f s", rank_, timeout_));
        if (now - t0 > 20e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }

 private:
  struct Registration {
    void* send = nullptr;
    size_t send_bytes = 0;
    void* recv = nullptr;  // receive arena: slot i at recv + i * stride
    size_t stride = 0;
    size_t slot_bytes = 0;
    int nslots = 0;
    std::vector<void*> peer_send;  // mapped send buffer of every rank (own one for self)
    std::vector<void*> peer_recv;  // push / relay: mapped receive arena of every rank
    std::vector<int> peer_nslots;  // push / relay: slots in each rank's arena
  };
  struct ArenaExport {
    hipIpcMemHandle_t handle;
    uint64_t stride;
    int32_t nslots;
  };

  // Slot index of receive pointer p in reg's arena, -1 if it is not one.
  static int slot_of(const Registration& reg, const void* p) {
    const char* base = static_cast<const char*>(reg.recv);
    const char* q = static_cast<const char*>(p);
    if (q < base || reg.stride == 0) return -1;
    const size_t off = static_cast<size_t>(q - base);
    if (off % reg.stride || off / reg.stride >= static_cast<size_t>(reg.nslots)) return -1;
    return static_cast<int>(off / reg.stride);
  }
  char* remote_slot_ptr(const Registration& reg, int peer, int slot) const {
    P2P_CHECK(static_cast<size_t>(peer) < reg.peer_recv.size(), "ipc push: receive arenas are not mapped");
    P2P_CHECK(slot >= 0 && slot < reg.peer_nslots[static_cast<size_t>(peer)],
              strfmt("bad remote slot %d (rank %d has %d)", slot, peer, reg.peer_nslots[static_cast<size_t>(peer)]));
    return static_cast<char*>(reg.peer_recv[static_cast<size_t>(peer)]) + reg.stride * static_cast<size_t>(slot);
  }

  // ---- device ping-pong / ring token helpers ----
  unsigned char* ping_slot(void* page, int k) const {
    return static_cast<unsigned char*>(page) + kPingSlot * static_cast<size_t>(k);
  }
  // A role with its timing buffers and bounds set; links and bases follow.
  dev::PingRole ping_role(size_t bytes, int iters) {
    P2P_CHECK(ping_ready_, "pingpong_setup() first");
    P2P_CHECK(iters >= 1 && iters <= kPingMaxIters, strfmt("device ping-pong: 1..%d iterations", kPingMaxIters));
    P2P_CHECK(bytes <= kPingMaxBytes, strfmt("device ping-pong payload is at most %zu bytes", kPingMaxBytes));
    auto* stamps = static_cast<unsigned long long*>(ping_scratch_);
    auto* status = reinterpret_cast<unsigned int*>(stamps + kPingMaxIters + 1);
    HIPCHECK(hipMemsetAsync(status, 0, 2 * sizeof(unsigned int), stream_));
    dev::PingRole a{};
    a.bytes = std::max<size_t>(16, (bytes + 15) / 16 * 16);
    a.iters = iters;
    a.stamps = stamps;
    a.status = status;
    a.timeout_ticks = static_cast<unsigned long long>(std::min(timeout_, 30.0) * tick_hz_);
    return a;
  }
  // Writes go to `to`'s inbox slot for this rank; waits read the slot `from`
  // writes here.  Sequence bases: what this rank has written to `to` and
  // read from `from` so far (flags are monotonic, never reset).
  void set_links(dev::PingRole* a, int from, int to) {
    unsigned char* out = ping_slot(peer_pages_[static_cast<size_t>(to)], rank_);
    unsigned char* in = ping_slot(page_, from);
    a->base = sent_[static_cast<size_t>(to)];
    a->in_base = recvd_[static_cast<size_t>(from)];
    a->out_flag = reinterpret_cast<unsigned long long*>(out);
    a->out_payload = out + kPingHeader;
    a->in_flag = reinterpret_cast<const unsigned long long*>(in);
    a->in_payload = in + kPingHeader;
  }
  // Waits for the kernel, checks its status words, and returns the leader's
  // per-iteration times in microseconds divided by `div` (empty elsewhere).
  std::vector<double> finish_ping(bool leader, int iters, double div, const std::string& what) {
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(ping_host_, ping_scratch_, kPingScratch, hipMemcpyDeviceToHost, stream_));
    sync();
    const auto* host = static_cast<const unsigned long long*>(ping_host_);
    const auto* st = reinterpret_cast<const unsigned int*>(host + kPingMaxIters + 1);
    if (st[0] & 1u) P2P_FATAL(strfmt("rank %d: %s timed out (partner kernel never answered)", rank_, what.c_str()));
    if (st[1]) P2P_FATAL(strfmt("rank %d: %s: %u payloads arrived before their data", rank_, what.c_str(), st[1]));
    std::vector<double> us;
    if (leader)
      for (int i = 0; i < iters; ++i)
        us.push_back(static_cast<double>(host[static_cast<size_t>(i) + 1] - host[static_cast<size_t>(i)]) / tick_hz_ * 1e6 /
                     div);
    return us;
  }

  void close_registration(Registration& reg) {
    for (int r = 0; r < n_; ++r) {
      void*& m = reg.peer_send[static_cast<size_t>(r)];
      if (m && r != rank_) (void)hipIpcCloseMemHandle(m);
      m = nullptr;
      if (static_cast<size_t>(r) < reg.peer_recv.size()) {
        void*& a = reg.peer_recv[static_cast<size_t>(r)];
        if (a && r != rank_) (void)hipIpcCloseMemHandle(a);
        a = nullptr;
      }
    }
  }

  // A flow (src, dst, slot) that group_flows already posted for this rank;
  // consumed by the endpoint's matching send / recv call.
  bool take_covered(int src, int dst, int slot) {
    const std::array<int, 3> key{src, dst, slot};
    auto it = std::find(covered_.begin(), covered_.end(), key);
    if (it == covered_.end()) return false;
    covered_.erase(it);
    return true;
  }

  // Push group: readies out / readies in, the copies, then done out / done in.
  void flush_push() {
    dev::SignalArgs pre{}, post{};
    for (int p : push_recvs_) add_post(&pre, p, kReady, ++ready_posted_[static_cast<size_t>(p)]);
    for (int q : push_sends_) add_wait(&pre, q, kReady, ++ready_seen_[static_cast<size_t>(q)]);
    if (debug_) {
      std::string msg = strfmt("[ipc %d] group %ld sends-to:", rank_, groups_);
      for (int q : push_sends_) msg += strfmt(" %d", q);
      msg += " recvs-from:";
      for (int p : push_recvs_) msg += strfmt(" %d", p);
      msg += " ready_posted:";
      for (auto v : ready_posted_) msg += strfmt(" %llu", v);
      msg += " ready_seen:";
      for (auto v : ready_seen_) msg += strfmt(" %llu", v);
      std::fprintf(stderr, "%s ops %zu\n", msg.c_str(), ops_.size());
    }
    ++groups_;
    launch_signals(pre, false);
    if (!ops_.empty()) dev::launch_multi_copy(ops_.data(), static_cast<int>(ops_.size()), stream_);
    for (int q : push_sends_) add_post(&post, q, kDone, ++done_posted_[static_cast<size_t>(q)]);
    for (int p : push_recvs_) add_wait(&post, p, kDone, ++done_seen_[static_cast<size_t>(p)]);
    launch_signals(post, true);
    ops_.clear();
    push_sends_.clear();
    push_recvs_.clear();
  }

  // Signal page line of kind k (ready / done) that rank `from` writes.
  unsigned long long* sync_line(void* page, int kind, int from) const {
    return reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(page) +
                                                 kSyncLine * (static_cast<size_t>(kind) * n_ + static_cast<size_t>(from)));
  }
  // Several messages to one peer in a group share its flag: keep one entry
  // per flag with the highest value (lanes storing to one address at once
  // would leave an arbitrary one of the values).
  void add_post(dev::SignalArgs* a, int peer, int kind, unsigned long long v) {
    unsigned long long* f = sync_line(sync_peer_[static_cast<size_t>(peer)], kind, rank_);
    for (int i = 0; i < a->nposts; ++i)
      if (a->post_flag[i] == f) {
        a->post_value[i] = std::max(a->post_value[i], v);
        return;
      }
    if (a->nposts == dev::kMaxSignals) launch_signals(*a, false), *a = dev::SignalArgs{};
    a->post_flag[a->nposts] = f;
    a->post_value[a->nposts++] = v;
  }
  void add_wait(dev::SignalArgs* a, int peer, int kind, unsigned long long v) {
    const unsigned long long* f = sync_line(sync_page_, kind, peer);
    for (int i = 0; i < a->nwaits; ++i)
      if (a->wait_flag[i] == f) {
        a->wait_value[i] = std::max(a->wait_value[i], v);
        return;
      }
    if (a->nwaits == dev::kMaxSignals) launch_signals(*a, false), *a = dev::SignalArgs{};
    a->wait_flag[a->nwaits] = f;
    a->wait_value[a->nwaits++] = v;
  }
  void launch_signals(dev::SignalArgs a, bool release_first) {
    if (a.nposts == 0 && a.nwaits == 0) return;
    a.release_first = release_first ? 1 : 0;
    a.status = sig_status_;
    a.timeout_ticks = static_cast<unsigned long long>(timeout_ * tick_hz_);
    dev::launch_signal(a, stream_);
  }

  // Collective (constructor): one signal page per rank, 2 x n flag lines
  // (ready / done from every peer), exported to every peer.  A setup that
  // fails half way releases what it made (the constructor throws, so the
  // destructor does not run).
  void setup_sync_pages() {
    try {
      setup_sync_pages_once();
    } catch (...) {
      release_sync_pages();
      throw;
    }
  }

  void release_sync_pages() {
    for (size_t r = 0; r < sync_peer_.size(); ++r)
      if (sync_peer_[r] && static_cast<int>(r) != rank_) (void)hipIpcCloseMemHandle(sync_peer_[r]);
    sync_peer_.clear();
    if (sync_page_) (void)hipFree(sync_page_);
    if (sig_status_) (void)hipHostFree(sig_status_);
    sync_page_ = nullptr;
    sig_status_ = nullptr;
  }

  void setup_sync_pages_once() {
    const size_t bytes = kSyncLine * 2 * static_cast<size_t>(n_);
    Export me{};
    sync_page_ = exportable(bytes, &me.handle, [&](void** q) { return alloc_signal_page(q, bytes); });
    HIPCHECK(hipMemsetAsync(sync_page_, 0, bytes, stream_));
    sync();  // bounded (see pingpong_setup)
    HIPCHECK(hipHostMalloc(&sig_status_, 64, hipHostMallocMapped));
    *sig_status_ = 0;
    me.host_hash = host_hash(real_hostname());
    auto all = boot_.allgather_value(me);
    sync_peer_.assign(static_cast<size_t>(n_), nullptr);
    for (int r = 0; r < n_; ++r) {
      if (r == rank_) {
        sync_peer_[static_cast<size_t>(r)] = sync_page_;
        continue;
      }
      P2P_CHECK(all[static_cast<size_t>(r)].host_hash == me.host_hash,
                strfmt("ipc transport is intra-node only: rank %d is on another host", r));
      void* mapped = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&mapped, all[static_cast<size_t>(r)].handle, hipIpcMemLazyEnablePeerAccess));
      sync_peer_[static_cast<size_t>(r)] = mapped;
    }
    for (auto* v : {&ready_posted_, &ready_seen_, &done_posted_, &done_seen_}) v->assign(static_cast<size_t>(n_), 0);
    boot_.barrier();
  }

  void flush() {
    if (push_) {
      flush_push();
      return;
    }
    if (ops_.empty()) return;
    if (engine_ == "kernel") {
      dev::launch_multi_copy(ops_.data(), static_cast<int>(ops_.size()), stream_);
    } else if (ops_.size() == 1) {
      HIPCHECK(hipMemcpyAsync(ops_[0].dst, ops_[0].src, ops_[0].bytes, hipMemcpyDeviceToDevice, stream_));
    } else {
      // Fork: the receives round-robin over a few side streams so the copy
      // engines overlap, then join back into the main stream.  A small pool
      // (P2P_SDMA_STREAMS, default 4) rather than a stream per receive: more
      // streams than the process's hardware queues only share queues, and
      // every extra queue is one more for the GPU's scheduler to map.
      const size_t k = std::min(ops_.size(), sdma_streams());
      ensure_side_streams(k);
      HIPCHECK(hipEventRecord(fork_, stream_));
      for (size_t j = 0; j < k; ++j) HIPCHECK(hipStreamWaitEvent(side_[j], fork_, 0));
      for (size_t i = 0; i < ops_.size(); ++i)
        HIPCHECK(hipMemcpyAsync(ops_[i].dst, ops_[i].src, ops_[i].bytes, hipMemcpyDeviceToDevice, side_[i % k]));
      for (size_t j = 0; j < k; ++j) {
        HIPCHECK(hipEventRecord(side_done_[j], side_[j]));
        HIPCHECK(hipStreamWaitEvent(stream_, side_done_[j], 0));
      }
    }
    ops_.clear();
  }

  static size_t sdma_streams() {
    static const size_t k = [] {
      const char* e = std::getenv("P2P_SDMA_STREAMS");
      const int v = e ? std::atoi(e) : 4;
      return static_cast<size_t>(std::max(1, std::min(64, v)));
    }();
    return k;
  }

  void ensure_side_streams(size_t n) {
    if (!fork_) HIPCHECK(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
    while (side_.size() < n) {
      hipStream_t s;
      HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      side_.push_back(s);
      hipEvent_t e;
      HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      side_done_.push_back(e);
    }
  }

  Bootstrap& boot_;
  int rank_, n_;
  double timeout_;
  std::string engine_;
  bool relay_;  // multi-path push (engine "relay")
  bool push_;   // rendezvous + remote writes (engines "push" and "relay")
  RouteOptions route_opt_;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  StreamGate gate_;
  std::vector<hipEvent_t> events_;
  int next_event_ = 0;
  std::vector<hipGraphExec_t> execs_;
  std::vector<hipStream_t> side_;
  std::vector<hipEvent_t> side_done_;
  hipEvent_t fork_ = nullptr;
  dev::VerifyAccum* acc_ = nullptr;
  dev::VerifyAccum* acc_host_ = nullptr;
  dev::BatchVerifier batch_;
  dev::VerifyImpl verify_impl_ = dev::VerifyImpl::Auto;
  std::string desc_;
  std::vector<Registration> regs_;
  bool in_group_ = false;
  std::vector<dev::CopyOp> ops_;
  std::vector<std::array<int, 3>> covered_;  // relay: (src, dst, slot) posted by group_flows
  unsigned long long relayed_bytes_ = 0, relayed_stripes_ = 0;  // moved by this rank as a relay (P2P_RELAY_STATS)
  bool debug_ = std::getenv("P2P_IPC_DEBUG") != nullptr;     // per-group flag bookkeeping on stderr
  long groups_ = 0;

  struct Block {
    size_t size = 0;
    hipIpcMemHandle_t handle{};
  };

  // A new device allocation whose IPC export works, with its handle.  On
  // this stack hipIpcGetMemHandle now and then refuses a fresh block
  // ("invalid argument", seen with 8 processes allocating on one GPU); such a
  // block is held (so the allocator cannot hand it straight back) until a
  // good one is found, then freed, and the retry is reported on stderr.
  template <class AllocFn>
  void* exportable(size_t size, hipIpcMemHandle_t* handle, AllocFn&& alloc_fn) {
    std::vector<void*> refused;
    void* p = nullptr;
    for (int attempt = 0;; ++attempt) {
      hipError_t e = alloc_fn(&p);
      if (e != hipSuccess) {
        for (void* r : refused) (void)hipFree(r);
        P2P_FATAL(strfmt("device allocation of %zu bytes failed: %s", size, hipGetErrorString(e)));
      }
      e = hipIpcGetMemHandle(handle, p);
      if (e == hipSuccess && inject_refusals_ > 0) {  // test hook: P2P_INJECT_EXPORT_REFUSALS=<n>
        --inject_refusals_;
        e = hipErrorInvalidValue;
      }
      if (e == hipSuccess) break;
      (void)hipGetLastError();
      refused.push_back(p);
      if (attempt == 7) {
        for (void* r : refused) (void)hipFree(r);
        P2P_FATAL(strfmt("hipIpcGetMemHandle refused 8 fresh %zu-byte blocks: %s", size, hipGetErrorString(e)));
      }
    }
    if (!refused.empty())
      std::fprintf(stderr, "p2p_matrix: rank %d: hipIpcGetMemHandle refused %zu fresh %zu-byte block(s); reallocated\n",
                   rank_, refused.size(), size);
    for (void* r : refused) (void)hipFree(r);
    return p;
  }
  const hipIpcMemHandle_t& handle_of(void* p) const {
    auto it = blocks_.find(p);
    P2P_CHECK(it != blocks_.end(), "ipc transport exports only buffers it allocated");
    return it->second.handle;
  }
  // Uncached device memory when the runtime allows it, so a spinning wave
  // reads HBM rather than a stale line.
  static hipError_t alloc_signal_page(void** q, size_t bytes) {
    if (hipExtMallocWithFlags(q, bytes, hipDeviceMallocUncached) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    return hipMalloc(q, bytes);
  }
  void drain_pool() {
    for (auto& b : pool_) (void)hipFree(b.first);
    pool_.clear();
    pool_bytes_ = 0;
  }
  size_t pool_cap_ = size_t{32} << 30;
  bool size_fix_ = true;  // round exported blocks so size mod 4 GiB < 2 GiB (HIP < 7.2 IPC import hang)
  int inject_refusals_ = 0;
  std::vector<std::pair<void*, Block>> pool_;  // released, kept for reuse
  size_t pool_bytes_ = 0;
  std::map<void*, Block> blocks_;              // live allocations

  // Push / relay engine state.
  static constexpr size_t kSyncLine = 128;
  static constexpr int kReady = 0, kDone = 1;
  void* sync_page_ = nullptr;
  std::vector<void*> sync_peer_;
  unsigned int* sig_status_ = nullptr;  // host-mapped; bit 0 = a signal wait timed out
  std::vector<unsigned long long> ready_posted_, ready_seen_, done_posted_, done_seen_;
  std::vector<int> push_sends_, push_recvs_;  // peers this rank writes to / receives from in the group

  static constexpr size_t kPingHeader = 256;            // flag + padding (own cache lines)
  static constexpr size_t kPingMaxBytes = 64u << 10;
  static constexpr size_t kPingSlot = kPingHeader + kPingMaxBytes;
  static constexpr int kPingMaxIters = 100000;
  void* page_ = nullptr;
  bool ping_ready_ = false;  // pingpong_setup completed
  std::vector<void*> peer_pages_;
  std::vector<unsigned long long> sent_, recvd_;  // ping messages written to / read from each rank
  double tick_hz_ = 1e8;
  static constexpr size_t kPingScratch = sizeof(unsigned long long) * (kPingMaxIters + 1) + 64;
  void* ping_scratch_ = nullptr;  // device: stamps[kPingMaxIters + 1], status[2]
  void* ping_host_ = nullptr;     // pinned copy of it
};

}  // namespace

std::unique_ptr<Transport> make_ipc_transport(Bootstrap& boot, const TransportOptions& opt) {
  return std::make_unique<IpcTransport>(boot, opt);
}

}  // namespace p2p
