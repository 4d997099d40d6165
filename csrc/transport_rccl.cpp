// RcclTransport: MI355X device buffers + RCCL point-to-point over xGMI.
//
// Reference call sites replaced here (/root/reference/p2p_matrix.cc):
//   ncclGetUniqueId + MPI_Bcast + cudaSetDevice + ncclCommInitRank  :111-120
//   cudaStreamCreateWithFlags(cudaStreamNonBlocking) x2               :121-122
//   cudaMalloc + cudaMemset                                           :124-130
//   ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd               :156-169, 211-249
//   cudaStreamSynchronize                                             :162, :170, :229-251
//   ncclCommDestroy                                                   :270
// Differences by design:
//   * ncclGetUniqueId and every RCCL call are checked (the reference leaves
//     :116 and :270 unchecked); the unique id travels over the Bootstrap.
//   * The communicator is created non-blocking (ncclCommInitRankConfig with
//     blocking = 0) and polled with a deadline, and every sync is a bounded
//     poll of hipStreamQuery + ncclCommGetAsyncError: a dead peer becomes
//     ncclCommAbort + a fatal error on every rank instead of a silent hang.
//   * One non-blocking stream by default: the reference's second stream for
//     the bi direction is joined by the group anyway; --two-streams (implied
//     by --reference) restores its s_0 / s_1 layout.
//   * Optionally K communicators (--comms K, TransportOptions::rccl_comms):
//     the i-th message of at least 1 MiB from a to b goes to communicator
//     (i + a + b) mod K on both ends (a running count per peer and direction,
//     so every send meets its receive whatever the group structure; smaller
//     messages stay on the first), each communicator on its own stream.
//     Streams are synchronised only where data requires it: a side stream
//     waits for the main stream after the main stream wrote or read payload
//     buffers (fill, zero, verify), and the main stream waits for the side
//     streams before such buffer work and at sync().  A mark is an event on
//     every stream that ran work since the previous mark, so back-to-back
//     steps flow on all K streams without any per-step barrier.  One
//     RCCL send/recv kernel uses at most 32 channels (workgroups); several
//     communicators run several kernels side by side, so the messages of a
//     group are moved by K x 32 workgroups.
//     The ops of a group are handed to RCCL sorted by communicator (stable,
//     so each communicator's per-peer order is kept), which makes every rank
//     launch its kernels in the same (group, communicator) order.  HIP maps
//     more streams than GPU_MAX_HW_QUEUES (4 on the box) onto shared hardware
//     queues that run in order; were rank a to launch communicator 1 before 0
//     on a queue where rank b launches 0 before 1, each would wait for a
//     kernel the other has queued behind its own: a cross-rank deadlock (ring
//     bi and all-pairs groups start on different communicators per rank).
//     With one global launch order the earliest unfinished kernel on every
//     rank has only finished work ahead of it in any queue.
//   * hipEvents on the stream give GPU-timeline timestamps.
//   * Payloads are written / checked by the gfx950 kernels in kernels.hip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <strings.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <sstream>
#include <thread>
#include <vector>

#include "batch_verify.hpp"
#include "bootstrap.hpp"
#include "common.hpp"
#include "hip_check.hpp"
#include "kernels.hpp"
#include "provenance.hpp"
#include "rccl_log.hpp"
#include "report.hpp"
#include "stream_gate.hpp"
#include "topology.hpp"
#include "transport.hpp"
#include "units.hpp"

namespace p2p {
namespace {

class RcclTransport final : public Transport {
 public:
  RcclTransport(Bootstrap& boot, const TransportOptions& opt)
      : rank_(boot.rank()), n_(boot.size()), timeout_(opt.timeout_s) {
    verify_impl_ = static_cast<dev::VerifyImpl>(opt.verify_impl);
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0)
      P2P_FATAL(strfmt("rank %d: no HIP device visible (%s)", rank_, e == hipSuccess ? "0 devices" : hipGetErrorString(e)));
    device_ = opt.device >= 0 ? opt.device : 0;
    // The reference never checks this and lets cudaSetDevice fail.
    if (device_ >= ndev)
      P2P_FATAL(strfmt("rank %d wants GPU %d but only %d are visible: more ranks per host than GPUs", rank_, device_, ndev));
    int ncomms = opt.rccl_comms;
    if (const char* kc = std::getenv("P2P_RCCL_COMMS")) ncomms = std::atoi(kc);
    P2P_CHECK(ncomms >= 1 && ncomms <= kMaxComms, strfmt("rccl communicators per rank: 1..%d", kMaxComms));
    P2P_CHECK(ncomms == 1 || !opt.two_streams, "--two-streams (the reference layout) uses one communicator");
    HIPCHECK(hipSetDevice(device_));
    open_streams(opt, ncomms);
    stale_.assign(static_cast<size_t>(ncomms), true);
    pending_.assign(static_cast<size_t>(ncomms), false);
    unjoined_.assign(static_cast<size_t>(ncomms), false);
    send_seq_.assign(static_cast<size_t>(n_), 0);
    recv_seq_.assign(static_cast<size_t>(n_), 0);
    touched_.assign(static_cast<size_t>(n_), 0);
    HIPCHECK(hipMalloc(&acc_, dev::verify_accum_bytes()));
    HIPCHECK(hipHostMalloc(&acc_host_, sizeof(dev::VerifyAccum), hipHostMallocDefault));
    open_communicators(boot, opt, ncomms);
    describe(ncomms);
  }

  ~RcclTransport() override {
    remove_abort_hook(hook_);
    if (!drain_quietly()) {
      // Kernels still run after the abort: free nothing under them (process
      // exit tears the queues down).
      std::fprintf(stderr, "p2p WARN rank %d: RCCL streams still busy after the abort; leaving them to exit\n",
                   rank_);
      return;
    }
    // Graphs that captured RCCL work hold references to the communicator's
    // persistent resources: release them before the communicator, or
    // ncclCommDestroy waits for them forever.
    for (auto ex : execs_)
      if (ex) (void)hipGraphExecDestroy(ex);
    for (auto g : graphs_)
      if (g) (void)hipGraphDestroy(g);
    execs_.clear();
    graphs_.clear();
    // An aborted communicator took its registrations with it.
    for (auto& r : reg_sets_)
      for (auto& ch : r.handles)
        if (live(ch.first)) ncclCommDeregister(ch.first, ch.second);
    reg_sets_.clear();
    try {
      release_discard_sink();
    } catch (const std::exception&) {
    }
    for (void* p : nccl_alloc_) ncclMemFree(p);
    nccl_alloc_.clear();
    for (auto& c : comms_)
      if (c) {
        // Destroy (unlike the unchecked p2p_matrix.cc:270 we drained first).
        ncclCommDestroy(c);
        c = nullptr;
      }
    for (auto ev : events_) (void)hipEventDestroy(ev);
    for (auto& v : side_ev_)
      for (auto ev : v)
        if (ev) (void)hipEventDestroy(ev);
    for (auto ev : cjoin_)
      if (ev) (void)hipEventDestroy(ev);
    if (fork_) (void)hipEventDestroy(fork_);
    if (acc_) (void)hipFree(acc_);
    if (acc_host_) (void)hipHostFree(acc_host_);
    if (recv_stream_) (void)hipStreamDestroy(recv_stream_);
    if (join_) (void)hipEventDestroy(join_);
    for (auto cs : cstreams_)
      if (cs != stream_) (void)hipStreamDestroy(cs);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  std::string name() const override { return "rccl"; }
  int rank() const override { return rank_; }
  int nranks() const override { return n_; }
  std::string device_desc() const override { return desc_; }
  std::string device_key() const override { return gpu_memory_key(device_); }

  bool mem_info(size_t* free_b, size_t* total_b) override { return hipMemGetInfo(free_b, total_b) == hipSuccess; }
  void* alloc(size_t bytes) override {
    void* p = nullptr;
    if (register_ == 2) {  // RCCL's own allocator (P2P_RCCL_REGISTER=2)
      nccl_ok(ncclMemAlloc(&p, std::max<size_t>(bytes, 256)), "ncclMemAlloc");
      nccl_alloc_.push_back(p);
      return p;
    }
    hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 256));
    if (e != hipSuccess) P2P_FATAL(strfmt("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e)));
    return p;
  }
  void release(void* p) override {
    if (!p) return;
    auto it = std::find(nccl_alloc_.begin(), nccl_alloc_.end(), p);
    if (it != nccl_alloc_.end()) {
      nccl_alloc_.erase(it);
      nccl_ok(ncclMemFree(p), "ncclMemFree");
      return;
    }
    HIPCHECK(hipFree(p));
  }

  // P2P_RCCL_REGISTER=1|2: every buffer of a set is registered with every
  // communicator (ncclCommRegister), which lets RCCL move point-to-point
  // messages between registered user buffers without its staging FIFOs
  // where it supports that.  An experiment knob (profiles/r1_comms/).
  void register_buffers(const BufferSet& set) override {
    if (!register_) return;
    RegSet r;
    r.send = set.send;
    const std::pair<void*, size_t> all[2] = {{set.send, set.send_bytes},
                                             {set.recv, set.stride * static_cast<size_t>(set.nslots)}};
    for (auto c : comms_)
      for (const auto& pb : all) {
        void* h = nullptr;
        nccl_ok(ncclCommRegister(c, pb.first, pb.second, &h), "ncclCommRegister");
        r.handles.emplace_back(c, h);
      }
    reg_sets_.push_back(std::move(r));
  }
  void unregister_buffers(void* send) override {
    auto it = std::find_if(reg_sets_.begin(), reg_sets_.end(), [&](const RegSet& r) { return r.send == send; });
    if (it == reg_sets_.end()) return;
    sync();
    for (auto& ch : it->handles)
      if (live(ch.first)) nccl_ok(ncclCommDeregister(ch.first, ch.second), "ncclCommDeregister");
    reg_sets_.erase(it);
  }
  // Not aborted (abort_all clears the communicator's slot).
  bool live(ncclComm_t c) const { return c && std::find(comms_.begin(), comms_.end(), c) != comms_.end(); }
  void fill(void* p, size_t bytes, uint64_t seed) override {
    buffer_work();
    dev::launch_fill(p, bytes, seed, stream_);
  }
  void zero(void* p, size_t bytes) override {
    buffer_work();
    HIPCHECK(hipMemsetAsync(p, 0, bytes, stream_));
  }

  VerifyResult verify(const void* p, size_t bytes, uint64_t seed) override {
    buffer_work();
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
    // The batched kernel is the default LDS8 verify; another --verify-impl
    // keeps the one-buffer path.
    if ((verify_impl_ != dev::VerifyImpl::Auto && verify_impl_ != dev::VerifyImpl::Lds8) || !batch_verify_enabled())
      return Transport::verify_many(jobs);
    buffer_work();
    return batch_verify(batch_, jobs, stream_, [this] { sync(); });
  }

  void group_begin() override {
    check_live("group_begin");
    nccl_ok(ncclGroupStart(), "ncclGroupStart");
    in_group_ = true;
    sent_in_group_ = false;
    if (cstreams_.size() > 1) {
      std::fill(used_.begin(), used_.end(), false);
      used_.resize(cstreams_.size(), false);
    }
  }
  // Messages above the peer's op limit are posted as several back-to-back
  // ops of at most that many bytes inside the same group (matched in order
  // on both sides): RCCL 2.26 / 2.27 on MI355X deliver only the first half of
  // an op whose share of one p2p channel exceeds 16 MiB
  // (scripts/rccl_half_repro.cpp, profiles/r3_rccl_half_repro/), so the
  // limit is 16 MiB x the channels RCCL splits an op to that peer over
  // (derive_op_limits).
  void send(const void* p, size_t bytes, int peer) override {
    check_live("send");
    const int j = pick(&send_seq_, peer, bytes);
    touched_[static_cast<size_t>(peer)] = 1;
    sent_in_group_ = true;
    const char* c = static_cast<const char*>(p);
    do {
      size_t n = chunk_of(bytes, peer);
      issue({j, true, const_cast<char*>(c), n, peer, cstreams_[static_cast<size_t>(j)]});
      c += n;
      bytes -= n;
    } while (bytes);
  }
  void recv(void* p, size_t bytes, int peer) override {
    check_live("recv");
    const int j = pick(&recv_seq_, peer, bytes);
    touched_[static_cast<size_t>(peer)] = 1;
    // Reference two-stream layout: the bi loop receives on s_1 next to its
    // send on s_0 (p2p_matrix.cc:214-225, sends are posted first), the uni
    // loop receives alone on s_0 (:163-168).
    const bool side = j == 0 && recv_stream_ && sent_in_group_;
    hipStream_t s = side ? recv_stream_ : cstreams_[static_cast<size_t>(j)];
    // Injected skip fault: the receive completes into a private sink.
    char* c = static_cast<char*>(discarding() ? discard_sink(bytes) : p);
    do {
      size_t n = chunk_of(bytes, peer);
      issue({j, false, c, n, peer, s});
      c += n;
      bytes -= n;
    } while (bytes);
    recv_on_side_ = recv_on_side_ || side;
  }
  void group_end() override {
    in_group_ = false;
    std::stable_sort(deferred_.begin(), deferred_.end(), [](const Op& a, const Op& b) { return a.comm < b.comm; });
    for (const Op& o : deferred_) post(o);
    // Non-blocking comm: the ops are only enqueued once the comm leaves
    // ncclInProgress, so wait before any event is recorded behind them.
    wait_ready(ncclGroupEnd(), "ncclGroupEnd");
    deferred_.clear();
    if (recv_on_side_) {
      // Reference two-stream layout (sends on s_0, receives on s_1,
      // p2p_matrix.cc:214-225): join s_1 back so marks and syncs on the main
      // stream cover the receives too.
      HIPCHECK(hipEventRecord(join_, recv_stream_));
      HIPCHECK(hipStreamWaitEvent(stream_, join_, 0));
      recv_on_side_ = false;
    }
    // Side streams are not joined here: each keeps running its
    // communicator's groups back to back.  A mark records on every stream
    // used since the previous one; the main stream waits for them only
    // before it touches buffers and at sync() (join_all).
    for (size_t j = 0; j < used_.size(); ++j)
      if (used_[j]) {
        pending_[j] = true;
        unjoined_[j] = true;
        used_[j] = false;
      }
  }

  // A mark is an event on the main stream plus one on every side stream
  // that ran work since the previous mark; a side stream that did not stands
  // for itself by its latest earlier event (nothing ran on it since).  The
  // mark completes when all of them have.  elapsed_ms(a, b) = (latest event
  // of b) - (latest event of a): the time between the completions of all
  // work up to a and all work up to b, so back-to-back intervals add up to
  // the whole run even when side streams finish a step after the main one.
  int mark() override {
    const size_t m = static_cast<size_t>(next_event_);
    if (m == events_.size()) {
      hipEvent_t ev;
      HIPCHECK(hipEventCreateWithFlags(&ev, timing_event_flags()));
      events_.push_back(ev);
      side_ev_.emplace_back(cstreams_.size(), nullptr);
      side_rec_.emplace_back(cstreams_.size(), 0);
      side_ref_.emplace_back(cstreams_.size(), -1);
    }
    last_side_.resize(cstreams_.size(), -1);
    HIPCHECK(hipEventRecord(events_[m], stream_));
    for (size_t j = 0; j < cstreams_.size(); ++j) {
      side_rec_[m][j] = 0;
      if (j < pending_.size() && pending_[j]) {
        if (!side_ev_[m][j]) HIPCHECK(hipEventCreateWithFlags(&side_ev_[m][j], timing_event_flags()));
        HIPCHECK(hipEventRecord(side_ev_[m][j], cstreams_[j]));
        side_rec_[m][j] = 1;
        pending_[j] = false;
        last_side_[j] = static_cast<int>(m);
      }
      side_ref_[m][j] = last_side_[j];
    }
    return next_event_++;
  }
  double elapsed_ms(int a, int b) override {
    const size_t ia = static_cast<size_t>(a), ib = static_cast<size_t>(b);
    hipEvent_t ref = events_.at(ia);
    auto since_ref = [&](hipEvent_t e) {
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, ref, e));
      return static_cast<double>(ms);
    };
    double start = 0, end = since_ref(events_.at(ib));
    for (size_t j = 0; j < cstreams_.size(); ++j) {
      const int ra = side_ref_[ia][j], rb = side_ref_[ib][j];
      if (ra >= 0) start = std::max(start, since_ref(side_ev_[static_cast<size_t>(ra)][j]));
      if (rb >= 0) end = std::max(end, since_ref(side_ev_[static_cast<size_t>(rb)][j]));
    }
    return end - start;
  }
  // Reused event slots must not stand in for a stream's latest work, so the
  // references are dropped: the first mark after a clear covers the main
  // stream and the side streams that ran since their last mark (callers
  // clear between runs, with the streams drained or about to be).
  void clear_marks() override {
    next_event_ = 0;
    std::fill(last_side_.begin(), last_side_.end(), -1);
  }

  // hipGraph capture of grouped ncclSend/ncclRecv: a step's back-to-back
  // groups become one graph launch, removing the per-group host launch cost
  // (microarch price list: ~3.3-3.8 us host launch per kernel eager).  One
  // communicator only: capturing the fork / join of several communicators'
  // streams crashed inside RCCL 2.26 on MI355X (scripts/comms_probe.py
  // --graph 1, profiles/r1_comms/).
  bool supports_graphs() const override { return comms_.size() == 1; }
  void capture_begin() override { HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal)); }
  int capture_end() override {
    hipGraph_t g = nullptr;
    HIPCHECK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t ex = nullptr;
    HIPCHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    graphs_.push_back(g);
    execs_.push_back(ex);
    return static_cast<int>(execs_.size()) - 1;
  }
  void graph_launch(int h) override {
    hipGraphExec_t ex = execs_.at(static_cast<size_t>(h));
    P2P_CHECK(ex != nullptr, "graph_launch: the graph was released");
    HIPCHECK(hipGraphLaunch(ex, stream_));
  }
  // The executable graph and the graph that captured RCCL work (both hold
  // references to the communicator's resources, see the destructor).
  void graph_release(int h) override {
    hipGraphExec_t& ex = execs_.at(static_cast<size_t>(h));
    hipGraph_t& g = graphs_.at(static_cast<size_t>(h));
    if (ex) HIPCHECK(hipGraphExecDestroy(ex));
    if (g) HIPCHECK(hipGraphDestroy(g));
    ex = nullptr;
    g = nullptr;
  }

  void sync() override {
    // Bounded poll instead of hipStreamSynchronize: spins for the first 20 ms
    // (so per-message syncs in wallclock mode are not inflated by sleeps),
    // then backs off; checks RCCL's async error so a failed peer aborts.
    check_live("sync");
    join_all();
    double t0 = now_seconds();
    double deadline = t0 + timeout_;
    for (long it = 0;; ++it) {
      hipError_t e = hipStreamQuery(stream_);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) P2P_FATAL(strfmt("stream error: %s", hipGetErrorString(e)));
      if ((it & 255) == 0) {
        if (abort_requested()) {
          abort_all();
          note_abort_done();
          P2P_FATAL(strfmt("rank %d: aborted while waiting (the run's deadline passed)", rank_));
        }
        // Either way the communicators are aborted first: RCCL's kernels poll
        // the abort flag and exit, so the streams (and any hardware queue they
        // share with another session's streams) drain instead of staying
        // stuck behind a transfer that will never complete.
        std::string err = async_error();
        if (!err.empty()) {
          abort_all();
          P2P_FATAL("RCCL asynchronous error while waiting: " + err);
        }
        double now = now_seconds();
        if (now > deadline) {
          abort_all();
          P2P_FATAL(strfmt("rank %d: stream did not finish within %.0f s (peer hung or dead?); aborting", rank_, timeout_));
        }
        if (now - t0 > 20e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }

  // Every stream idle, bounded like sync() but without throwing: past the
  // timeout, or when the run's deadline asks for an abort, the communicators
  // are aborted (RCCL's kernels poll the abort flag and exit) and the streams
  // get 10 s more.  A destructor that waited unbounded here -- with the GIL
  // held under the Python bindings -- could keep bench.py's deadline watchdog
  // from ever printing its line.
  bool drain_quietly() override {
    double deadline = now_seconds() + timeout_;
    bool aborted = false;
    for (long it = 0;; ++it) {
      bool busy = false;
      for (hipStream_t s : {stream_, recv_stream_})
        if (s && hipStreamQuery(s) == hipErrorNotReady) busy = true;
      for (auto cs : cstreams_)
        if (hipStreamQuery(cs) == hipErrorNotReady) busy = true;
      if (!busy) return true;
      const double now = now_seconds();
      // RCCL's async error, as sync() checks it: work pending on
      // a dead peer aborts now, not at the end of the session's timeout.
      const bool failed = !aborted && (it & 255) == 0 && !async_error().empty();
      if (!aborted && (failed || now > deadline || abort_requested())) {
        const bool requested = abort_requested();
        abort_all();
        if (requested) note_abort_done();
        aborted = true;
        deadline = now + 10.0;
      } else if (aborted && now > deadline) {
        return false;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }

  int concurrency() const override { return static_cast<int>(comms_.size()); }
  bool set_chunk_cap(size_t bytes) override {
    cap_ = bytes;
    return true;
  }
  size_t chunk_cap() const override { return cap_; }
  std::string link_report() override { return peers_json(); }
  std::vector<std::string> peer_transports() override {
    std::vector<std::string> out;
    for (const auto& l : our_links()) out.push_back(l.transport);
    return out;
  }
  size_t max_chunk(int peer) const override { return chunk_for(peer); }

  bool gate_arm(double timeout_s) override {
    gate_.arm(stream_, timeout_s);
    return true;
  }
  void gate_release() override { gate_.release(); }
  bool gate_timed_out() override { return gate_.timed_out(); }
  void set_timeout(double seconds) override { timeout_ = seconds; }

  std::string async_error() override {
    for (auto c : comms_) {
      if (!c) return "communicator aborted";
      ncclResult_t st = ncclSuccess;
      ncclResult_t r = ncclCommGetAsyncError(c, &st);
      if (r != ncclSuccess) return ncclGetErrorString(r);
      if (st != ncclSuccess && st != ncclInProgress) return ncclGetErrorString(st);
    }
    return "";
  }

 private:
  // Main stream (fill / verify; communicator 0's too), the optional
  // reference receive stream, and one stream + join event per further
  // communicator.  (Round 5 removed the experiments that gave communicator 0
  // a stream of its own or each communicator a CU mask, P2P_RCCL_MAIN_IDLE /
  // P2P_RCCL_CU_MASK: neutral or slower, profiles/r2_cu_mask/.)
  void open_streams(const TransportOptions& opt, int ncomms) {
    HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (opt.two_streams) {
      HIPCHECK(hipStreamCreateWithFlags(&recv_stream_, hipStreamNonBlocking));
      HIPCHECK(hipEventCreateWithFlags(&join_, hipEventDisableTiming));
    }
    for (int j = 0; j < ncomms; ++j) {
      hipStream_t s = stream_;
      if (j > 0) HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      cstreams_.push_back(s);
      hipEvent_t ev = nullptr;
      if (ncomms > 1) HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      cjoin_.push_back(ev);
    }
    if (ncomms > 1) HIPCHECK(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
  }

  // ncclUniqueIds from rank 0 through the bootstrap, then the communicators.
  void open_communicators(Bootstrap& boot, const TransportOptions& opt, int ncomms) {
    // Before anything of RCCL's runs in this process (ncclGetUniqueId
    // initialises its logging too): point its INFO log at our file, and pick
    // the kernels' unroll factor.
    rccl_log_file();
    if (!opt.rccl_stock) rccl_unroll_setup();
    // P2P_RCCL_DISTINCT_HOSTS=1 (tests on one GPU): every rank tells RCCL it
    // is on a host of its own (NCCL_HOSTID, read when RCCL first hashes the
    // host), so several ranks may share one GPU -- RCCL refuses duplicate GPUs
    // on one host -- and talk over its network transport (sockets, e.g.
    // NCCL_SOCKET_IFNAME=lo).  Not xGMI: this exercises the multi-rank RCCL
    // paths (communicators, schedules, ordering across K communicators) where
    // only one GPU is available.
    if (const char* dh = std::getenv("P2P_RCCL_DISTINCT_HOSTS"); dh && std::atoi(dh) != 0)
      setenv("NCCL_HOSTID", strfmt("p2p-emulated-host-%d", rank_).c_str(), 1);
    // RCCL prints a version banner to stdout on first use; send it to stderr
    // so stdout keeps the reference's output (P2P_RCCL_BANNER=1 keeps it).
    const char* banner = std::getenv("P2P_RCCL_BANNER");
    StdoutToStderr quiet(!(banner && std::atoi(banner)));
    std::vector<ncclUniqueId> ids(static_cast<size_t>(ncomms));
    std::memset(ids.data(), 0, sizeof(ncclUniqueId) * ids.size());
    if (rank_ == 0)
      for (auto& id : ids) nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
    boot.bcast(ids.data(), sizeof(ncclUniqueId) * ids.size(), 0);

    if (const char* sm = std::getenv("P2P_RCCL_SPLIT_MIN")) split_min_ = parse_size(sm);
    if (const char* rg = std::getenv("P2P_RCCL_REGISTER")) register_ = std::atoi(rg);
    const char* blk = std::getenv("P2P_RCCL_BLOCKING");
    nonblocking_ = opt.nonblocking_init && !(blk && std::atoi(blk));
    comms_.assign(static_cast<size_t>(ncomms), nullptr);
    hook_ = push_abort_hook([this](int) { abort_all(); });
    log_start_ = rccl_log_size();
    // One communicator after the other, in the same order on every rank.
    for (int j = 0; j < ncomms; ++j) {
      const size_t before = rccl_log_size();
      if (nonblocking_) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r = ncclCommInitRankConfig(&comms_[static_cast<size_t>(j)], n_, ids[static_cast<size_t>(j)], rank_, &cfg);
        wait_ready(r, "ncclCommInitRankConfig");
      } else {
        nccl_ok(ncclCommInitRank(&comms_[static_cast<size_t>(j)], n_, ids[static_cast<size_t>(j)], rank_), "ncclCommInitRank");
      }
      comm_info_.push_back(parse_rccl_init(rccl_log_since(before)));
    }
    derive_op_limits(boot);
  }

  // Largest op per peer: RCCL delivers only the first half of an op whose
  // share of one p2p channel exceeds 16 MiB (scripts/rccl_half_repro.cpp,
  // both RCCLs of the image), so ops stay at 16 MiB x the channels an op to
  // that peer is split over.  From RCCL's init line: min(p2p channels, p2p
  // channels per peer) of every communicator, and at most
  // NCCL_NCHANNELS_PER_NET_PEER (2) for a peer on another host.  That rule is
  // pinned on the self path only (profiles/r3_rccl_half_repro/), so a remote
  // peer on this host starts at 2 channels (32 MiB) until refine_op_limits()
  // has read the channels RCCL connected to it (its lazy connection lines,
  // ADVICE r3).  Both ends must split a message alike, so the ranks agree on
  // min(a's view of b, b's view of a).  Without the log (the user set
  // NCCL_DEBUG, or RCCL was initialised before), round 2's guess stands: 64
  // channels to itself, 2 to others, fewer under the NCCL channel knobs.
  // P2P_RCCL_MAX_CHUNK=<bytes> sets every peer's limit, 0 disables splitting.
  static constexpr int kUnconnectedPeerChannels = 2;
  void derive_op_limits(Bootstrap& boot) {
    char host[128] = {0};
    std::snprintf(host, sizeof(host), "%s", rccl_host_id().c_str());
    std::vector<char> hosts(static_cast<size_t>(n_) * sizeof(host));
    boot.allgather(host, hosts.data(), sizeof(host));
    net_peer_.assign(static_cast<size_t>(n_), 0);
    for (int p = 0; p < n_; ++p)
      net_peer_[static_cast<size_t>(p)] = std::strcmp(&hosts[static_cast<size_t>(p) * sizeof(host)], host) != 0;
    int net_per_peer = 2;
    if (const char* v = std::getenv("NCCL_NCHANNELS_PER_NET_PEER"))
      if (std::atoi(v) > 0) net_per_peer = std::atoi(v);
    // The channel counts are the communicator's, the same on every rank; a
    // rank whose log lacks them (no private log, or RCCL printed the line
    // elsewhere) takes them from the lowest rank that has them.
    std::vector<int> triples;
    for (const auto& ci : comm_info_) triples.insert(triples.end(), {ci.p2p_channels, ci.p2p_per_peer, ci.nnodes});
    const std::vector<int> every = boot.allgather_vector(triples);
    for (size_t j = 0; j < comm_info_.size(); ++j) {
      if (comm_info_[j].found()) continue;
      for (int r = 0; r < n_; ++r) {
        const int* t = &every[static_cast<size_t>(r) * triples.size() + 3 * j];
        if (t[0] > 0 && t[1] > 0) {
          comm_info_[j].p2p_channels = t[0];
          comm_info_[j].p2p_per_peer = t[1];
          comm_info_[j].nnodes = t[2];
          comm_info_[j].from_rank = r;
          break;
        }
      }
    }
    bool logged = !comm_info_.empty();
    for (const auto& ci : comm_info_) logged = logged && ci.found();
    std::vector<int> mine(static_cast<size_t>(n_), 0);
    init_channels_.assign(static_cast<size_t>(n_), 0);
    for (int p = 0; p < n_; ++p) {
      const bool net = net_peer_[static_cast<size_t>(p)] != 0;
      int c = 0;
      if (logged) {
        for (const auto& ci : comm_info_) {
          const int x = rccl_op_channels(ci, net, net_per_peer);
          c = c == 0 ? x : std::min(c, x);
        }
        if (p != rank_) init_channels_[static_cast<size_t>(p)] = c;
        if (p != rank_ && !net) c = std::min(c, kUnconnectedPeerChannels);
      } else {
        c = p2p_channel_limit(p == rank_ ? 64 : 2);
      }
      mine[static_cast<size_t>(p)] = c;
    }
    const std::vector<int> all = boot.allgather_vector(mine);
    op_channels_.assign(static_cast<size_t>(n_), 0);
    peer_limit_.assign(static_cast<size_t>(n_), 0);
    peer_source_.assign(static_cast<size_t>(n_), "");
    for (int p = 0; p < n_; ++p) {
      const int c = std::min(all[static_cast<size_t>(rank_) * n_ + p], all[static_cast<size_t>(p) * n_ + rank_]);
      op_channels_[static_cast<size_t>(p)] = c;
      peer_limit_[static_cast<size_t>(p)] = kRcclBytesPerChannel * static_cast<size_t>(std::max(c, 1));
      peer_source_[static_cast<size_t>(p)] = !logged ? "default"
                                             : p == rank_ ? "init line"
                                             : net_peer_[static_cast<size_t>(p)] ? "init line (net peer)"
                                                                                 : "unconnected (2 channels)";
    }
    limit_source_ = logged ? "rccl INFO log: 16M x min(p2p channels, per peer[, net per peer]); remote peers "
                             "2 channels until their connection lines"
                           : "default (no RCCL INFO log): 16M x 64 self / 2 peers";
    if (const char* mc = std::getenv("P2P_RCCL_MAX_CHUNK")) {
      const size_t v = std::strcmp(mc, "0") ? parse_size(mc) : 0;
      std::fill(peer_limit_.begin(), peer_limit_.end(), v);
      limit_source_ = strfmt("P2P_RCCL_MAX_CHUNK=%s", mc);
      std::fill(peer_source_.begin(), peer_source_.end(), "P2P_RCCL_MAX_CHUNK");
    }
  }

  // The connection lines of this transport's communicators only (another
  // transport of the process may log into the same file meanwhile).
  std::vector<RcclPeerLink> our_links() const {
    std::vector<std::string> ours;
    for (auto c : comms_) ours.push_back(strfmt("%p", static_cast<void*>(c)));
    return rccl_peer_links(connections_of(parse_rccl_connections(rccl_log_since(log_start_)), ours), rank_, n_);
  }

 public:
  // After the warm-up connected every peer: each remote peer's op channels
  // become min(init-line channels, channels RCCL connected to it), agreed by
  // both ends (rccl_log.hpp proposed_op_channels / agree_op_channels).  Peers
  // without connection lines keep their limit.
  bool refine_op_limits(Bootstrap& boot) override {
    std::vector<int> prop(static_cast<size_t>(n_), 0);
    const bool forced = std::getenv("P2P_RCCL_MAX_CHUNK") != nullptr;
    if (!forced && !init_channels_.empty()) prop = proposed_op_channels(init_channels_, our_links(), rank_);
    const std::vector<int> all = boot.allgather_vector(prop);
    const std::vector<int> agreed = agree_op_channels(all, n_, rank_, op_channels_, &peer_source_);
    bool changed = false;
    for (int p = 0; p < n_; ++p) {
      const size_t i = static_cast<size_t>(p);
      if (agreed[i] == op_channels_[i]) continue;
      changed = true;
      op_channels_[i] = agreed[i];
      peer_limit_[i] = kRcclBytesPerChannel * static_cast<size_t>(std::max(agreed[i], 1));
    }
    ++refinements_;
    find_unparsed_peers(forced);
    return boot.allreduce_max(changed ? 1.0 : 0.0) > 0.0;
  }

 private:
  // A same-host peer this rank has exchanged messages with but whose
  // connection lines the parser found none of: RCCL's format changed under
  // us, and that peer's ops stay at the 2-channel default (VERDICT r4 item
  // 5).  Recorded with its raw lines in link_report (unparsed_peers) and
  // named once on stderr.
  void find_unparsed_peers(bool forced) {
    if (forced || rccl_log_file().path.empty() || init_channels_.empty()) return;
    unparsed_ = rccl_unparsed_peers(rccl_log_since(log_start_), our_links(), net_peer_, touched_, rank_);
    if (unparsed_.empty() || warned_unparsed_) return;
    warned_unparsed_ = true;
    std::string peers;
    for (const auto& u : unparsed_) peers += strfmt("%s%d", peers.empty() ? "" : ",", u.peer);
    std::fprintf(stderr,
                 "p2p WARN rank %d: RCCL connected peer(s) %s but none of its connection lines parsed; their ops "
                 "stay at the unconnected 2-channel limit (raw lines: link_report unparsed_peers)\n",
                 rank_, peers.c_str());
  }

 public:

 private:
  // link_report(): the communicators' channel counts, and per peer the
  // transport and channels RCCL's connection lines show, next to the op
  // limit in use.
  std::string peers_json() const {
    const auto links = our_links();
    std::string o = strfmt("{\"rank\":%d,\"log\":%s,\"op_limit_source\":\"%s\",\"refinements\":%d,\"comms\":[",
                           rank_, rccl_log_file().path.empty() ? "null" : "true", json_escape(limit_source_).c_str(),
                           refinements_);
    for (size_t j = 0; j < comm_info_.size(); ++j)
      o += strfmt("%s{\"p2p_channels\":%d,\"p2p_channels_per_peer\":%d,\"nnodes\":%d,\"from_rank\":%d,\"unroll\":%d}",
                  j ? "," : "", comm_info_[j].p2p_channels, comm_info_[j].p2p_per_peer, comm_info_[j].nnodes,
                  comm_info_[j].from_rank < 0 ? rank_ : comm_info_[j].from_rank, comm_info_[j].unroll);
    o += "],\"log_sample\":[";
    // (From the start of the process's log: rank 0's ncclGetUniqueId prints
    // RCCL's version before this transport's part begins.)
    const auto sample = rccl_log_sample(rccl_log_since(0));
    for (size_t k = 0; k < sample.size(); ++k) o += strfmt("%s\"%s\"", k ? "," : "", json_escape(sample[k]).c_str());
    o += "],\"unparsed_peers\":[";
    for (size_t i = 0; i < unparsed_.size(); ++i) {
      o += strfmt("%s{\"peer\":%d,\"lines\":[", i ? "," : "", unparsed_[i].peer);
      for (size_t k = 0; k < unparsed_[i].lines.size(); ++k)
        o += strfmt("%s\"%s\"", k ? "," : "", json_escape(unparsed_[i].lines[k]).c_str());
      o += "]}";
    }
    o += "],\"peers\":[";
    for (int p = 0; p < n_; ++p) {
      const auto& l = links[static_cast<size_t>(p)];
      o += strfmt("%s{\"peer\":%d,\"transport\":\"%s\",\"via\":\"%s\",\"channels_connected\":%d,\"op_channels\":%d,"
                  "\"op_limit\":%zu,\"op_limit_source\":\"%s\",\"net\":%s}",
                  p ? "," : "", p, json_escape(l.transport).c_str(), json_escape(l.via).c_str(), l.channels_connected,
                  op_channels_.empty() ? 0 : op_channels_[static_cast<size_t>(p)], chunk_for(p),
                  peer_source_.empty() ? "" : json_escape(peer_source_[static_cast<size_t>(p)]).c_str(),
                  !net_peer_.empty() && net_peer_[static_cast<size_t>(p)] ? "true" : "false");
    }
    return o + "]}";
  }

  void describe(int ncomms) {
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device_));
    char pci[64] = {0};
    if (hipDeviceGetPCIBusId(pci, sizeof(pci), device_) != hipSuccess) pci[0] = 0;
    int ver = 0;
    ncclGetVersion(&ver);
    desc_ = strfmt("hip:%d %s (%s, %d CUs, %.0f GiB, pci %s) rccl %d", device_, prop.name, prop.gcnArchName,
                   prop.multiProcessorCount, static_cast<double>(prop.totalGlobalMem) / (1ull << 30), pci, ver);
    if (ncomms > 1) desc_ += strfmt(" x%d comms", ncomms);
  }

  static constexpr int kMaxComms = 16;

  // The main stream is about to touch payload buffers: side streams must wait
  // for it before their next transfer.
  void buffer_work() {
    join_all();
    forked_ = false;
    std::fill(stale_.begin(), stale_.end(), true);
  }

  // The main stream waits for every side stream that ran work since the
  // last join.
  void join_all() {
    for (size_t j = 0; j < unjoined_.size(); ++j)
      if (unjoined_[j]) {
        HIPCHECK(hipEventRecord(cjoin_[j], cstreams_[j]));
        HIPCHECK(hipStreamWaitEvent(stream_, cjoin_[j], 0));
        unjoined_[j] = false;
      }
  }

  // Communicator of the next message to / from `peer`.  Messages below
  // split_min_ stay on communicator 0 and do not advance the count (both ends
  // see the same sizes, so they still agree): a small message gains nothing
  // from a side stream and would pay the fork / join.
  int pick(std::vector<unsigned long long>* seq, int peer, size_t bytes) {
    P2P_CHECK(peer >= 0 && peer < n_, "bad peer");
    if (comms_.size() == 1) return 0;
    int j = 0;
    if (bytes >= split_min_) {
      // (count + sender + receiver): both ends know all three, and the
      // messages of an all-pairs group spread over the communicators too.
      const unsigned long long key = (*seq)[static_cast<size_t>(peer)]++ + static_cast<unsigned long long>(rank_ + peer);
      j = static_cast<int>(key % comms_.size());
    }
    if (cstreams_[static_cast<size_t>(j)] != stream_ && !used_[static_cast<size_t>(j)]) {
      if (stale_[static_cast<size_t>(j)]) {
        // The main stream wrote payload / receive buffers (fill, zero) or read
        // them (verify) since this side stream last waited for it.  The fork
        // is recorded at the group's first such message: nothing of the group
        // is on the main stream before ncclGroupEnd.  Between steps that only
        // move data no fork is needed, so the side streams run back to back
        // and only the main stream waits for them (its join per group).
        if (!forked_) {
          HIPCHECK(hipEventRecord(fork_, stream_));
          forked_ = true;
        }
        HIPCHECK(hipStreamWaitEvent(cstreams_[static_cast<size_t>(j)], fork_, 0));
        stale_[static_cast<size_t>(j)] = false;
      }
      used_[static_cast<size_t>(j)] = true;
    }
    return j;
  }

  struct Op {
    int comm;
    bool send;
    char* p;
    size_t n;
    int peer;
    hipStream_t stream;
  };
  void post(const Op& o) {
    ncclComm_t c = comms_[static_cast<size_t>(o.comm)];
    if (o.send)
      nccl_ok(ncclSend(o.p, o.n, ncclUint8, o.peer, c, o.stream), "ncclSend");
    else
      nccl_ok(ncclRecv(o.p, o.n, ncclUint8, o.peer, c, o.stream), "ncclRecv");
  }
  // Several communicators: a group's ops are posted at group_end, sorted by
  // communicator (header comment).  One communicator: posted right away.
  void issue(const Op& o) {
    if (in_group_ && comms_.size() > 1)
      deferred_.push_back(o);
    else
      post(o);
  }

  void abort_all() {
    aborted_.store(true, std::memory_order_release);
    for (auto& c : comms_)
      if (c) {
        ncclCommAbort(c);
        c = nullptr;
      }
  }

  // Every entry point that would post work first: once the
  // communicators are aborted -- a wait that timed out, an RCCL error, the
  // run's deadline, a driver's teardown drain -- a session that outlives its
  // driver fails with this, not with an invalid-argument error from RCCL on a
  // null communicator.
  void check_live(const char* what) const {
    if (aborted_.load(std::memory_order_acquire))
      P2P_FATAL(strfmt("rank %d: %s on an aborted session: its RCCL communicators were aborted earlier (a wait that "
                       "timed out, an RCCL error or the run's deadline); open a new session",
                       rank_, what));
  }

  void nccl_ok(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return;
    if (r == ncclInProgress && nonblocking_ && !comms_.empty()) {
      wait_ready(r, what);
      return;
    }
    ncclComm_t c = comms_.empty() ? nullptr : comms_[0];
    std::string msg = strfmt("rank %d: %s failed: %s (%s)", rank_, what, ncclGetErrorString(r), c ? ncclGetLastError(c) : "") +
                      rccl_log_warnings(log_start_);
    abort_all();  // a communicator that returned an error is not used again
    P2P_FATAL(msg);
  }

  // Polls every communicator created so far until none is in progress.
  void wait_ready(ncclResult_t r, const char* what) {
    double deadline = now_seconds() + timeout_;
    while (r == ncclInProgress) {
      if (abort_requested()) {
        abort_all();
        note_abort_done();
        P2P_FATAL(strfmt("rank %d: %s aborted (the run's deadline passed)", rank_, what));
      }
      if (now_seconds() > deadline) {
        abort_all();
        P2P_FATAL(strfmt("rank %d: %s did not complete within %.0f s (peer missing?)", rank_, what, timeout_));
      }
      std::this_thread::yield();
      r = ncclSuccess;
      for (auto c : comms_) {
        if (!c) continue;
        ncclResult_t st = ncclSuccess;
        ncclResult_t q = ncclCommGetAsyncError(c, &st);
        if (q != ncclSuccess) {
          r = q;
          break;
        }
        if (st != ncclSuccess) {
          r = st;
          if (st != ncclInProgress) break;
        }
      }
    }
    if (r != ncclSuccess) {
      abort_all();
      P2P_FATAL(strfmt("rank %d: %s failed: %s", rank_, what, ncclGetErrorString(r)) + rccl_log_warnings(log_start_));
    }
  }

  int rank_, n_;
  double timeout_;
  int device_ = 0;
  bool nonblocking_ = true;
  hipStream_t stream_ = nullptr;
  hipStream_t recv_stream_ = nullptr;  // two-stream (reference) layout only
  hipEvent_t join_ = nullptr;
  bool recv_on_side_ = false;
  bool sent_in_group_ = false;  // this group posted a send (two-stream layout)
  // Message chunking (see send()): at most kRcclBytesPerChannel per p2p
  // channel of the peer (derive_op_limits), capped by set_chunk_cap().
  std::vector<size_t> peer_limit_;       // per peer; 0 = unsplit
  std::vector<int> op_channels_;         // per peer: channels an op is split over (0 unknown)
  std::vector<char> net_peer_;           // per peer: RCCL reaches it through its network transport
  std::vector<RcclInitInfo> comm_info_;  // per communicator, from RCCL's INFO log
  std::string limit_source_;             // how peer_limit_ was set
  std::vector<int> init_channels_;       // per remote peer: channels from the init line (before refinement)
  std::vector<std::string> peer_source_; // per peer: what set its limit
  int refinements_ = 0;                  // refine_op_limits() calls
  size_t cap_ = 0;                       // set_chunk_cap (0: none)
  size_t log_start_ = 0;                 // this transport's part of the RCCL log
  // `fallback` channels, or fewer where NCCL_MAX_P2P_NCHANNELS /
  // NCCL_NCHANNELS_PER_PEER ask RCCL for fewer.
  static int p2p_channel_limit(int fallback) {
    int c = fallback;
    for (const char* k : {"NCCL_MAX_P2P_NCHANNELS", "NCCL_NCHANNELS_PER_PEER"})
      if (const char* v = std::getenv(k))
        if (const int x = std::atoi(v); x > 0) c = std::min(c, x);
    return c;
  }
  size_t chunk_for(int peer) const {
    const size_t lim = peer_limit_.empty() ? 0 : peer_limit_[static_cast<size_t>(peer)];
    if (cap_ == 0) return lim;
    return lim == 0 ? cap_ : std::min(lim, cap_);
  }
  size_t chunk_of(size_t bytes, int peer) const {
    const size_t c = chunk_for(peer);
    return (c && bytes > c) ? c : bytes;
  }
  std::vector<ncclComm_t> comms_;      // comms_[0] on stream_
  std::vector<hipStream_t> cstreams_;  // stream of each communicator (cstreams_[0] == stream_)
  std::vector<hipEvent_t> cjoin_;      // per communicator with a side stream: joins it into stream_
  hipEvent_t fork_ = nullptr;          // recorded on stream_ when a stale side stream is first used
  bool forked_ = false;                // fork_ covers the main stream's latest buffer work
  std::vector<bool> stale_;            // side stream j has not waited for the latest buffer work
  size_t split_min_ = size_t{1} << 20;  // smaller messages stay on communicator 0 (P2P_RCCL_SPLIT_MIN)
  std::vector<bool> used_;             // side communicators used by the open group
  bool in_group_ = false;              // between group_begin and group_end
  std::vector<Op> deferred_;           // the open group's ops (several communicators)
  std::vector<unsigned long long> send_seq_, recv_seq_;  // messages posted to / from each peer
  std::vector<char> touched_;                            // per peer: any message posted to / from it
  std::vector<RcclUnparsedPeer> unparsed_;               // find_unparsed_peers
  bool warned_unparsed_ = false;
  struct RegSet {
    void* send = nullptr;
    std::vector<std::pair<ncclComm_t, void*>> handles;
  };
  int register_ = 0;                 // P2P_RCCL_REGISTER: 0 off, 1 ncclCommRegister, 2 + ncclMemAlloc
  std::vector<RegSet> reg_sets_;
  std::vector<void*> nccl_alloc_;    // buffers from ncclMemAlloc
  std::vector<hipEvent_t> events_;                 // per mark: on the main stream
  std::vector<std::vector<hipEvent_t>> side_ev_;   // per mark: on each side stream (lazily created)
  std::vector<std::vector<char>> side_rec_;        // per mark: side event j recorded by that mark
  std::vector<std::vector<int>> side_ref_;         // per mark: the mark whose side event j stands for stream j (-1 none)
  std::vector<int> last_side_;                     // latest mark that recorded on side stream j
  std::vector<bool> pending_;                      // side stream ran work since the last mark
  std::vector<bool> unjoined_;                     // side stream ran work since the last join
  std::vector<hipGraph_t> graphs_;
  std::vector<hipGraphExec_t> execs_;
  int next_event_ = 0;
  dev::VerifyAccum* acc_ = nullptr;
  dev::VerifyAccum* acc_host_ = nullptr;
  dev::BatchVerifier batch_;
  dev::VerifyImpl verify_impl_ = dev::VerifyImpl::Auto;
  std::string desc_;
  int hook_ = 0;
  std::atomic<bool> aborted_{false};  // abort_all ran: check_live refuses new work
  StreamGate gate_;
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(Bootstrap& boot, const TransportOptions& opt) {
  return std::make_unique<RcclTransport>(boot, opt);
}

std::string rccl_runtime_json() {
  int ver = 0;
  if (ncclGetVersion(&ver) != ncclSuccess) ver = -1;
  // The RCCL that runs is the one the loader resolved, which inside a torch
  // process is torch's own (Makefile RUNTIME): name it by path.
  return strfmt("{\"version\":%d,\"version_string\":\"%d.%d.%d\",\"library\":\"%s\"}", ver, ver / 10000,
                (ver / 100) % 100, ver % 100, json_escape(library_of(reinterpret_cast<const void*>(&ncclGetVersion))).c_str());
}

bool rccl_transport_available() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

}  // namespace p2p
