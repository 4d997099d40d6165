#include "runner.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <thread>

#include "bootstrap.hpp"
#include "common.hpp"
#include "runner_detail.hpp"
#include "units.hpp"

namespace p2p {

using detail::fault_applies;
using detail::flow_slots;
using detail::posts_phase;
using detail::slot_stride;

const char* timing_name(Timing t) { return t == Timing::Events ? "events" : "wallclock"; }

Timing parse_timing(const std::string& s) {
  if (s == "events" || s == "event" || s == "hipevents") return Timing::Events;
  if (s == "wallclock" || s == "wall" || s == "reference") return Timing::Wallclock;
  P2P_FATAL("unknown timing '" + s + "' (events|wallclock)");
}

// ------------------------------------------------------------- Buffers ----

namespace detail {
size_t slot_stride(size_t bytes) { return (std::max<size_t>(bytes, 16) + 4095) / 4096 * 4096; }
}  // namespace detail

Buffers::Buffers(Transport& t, size_t slot_bytes, int recv_slots, size_t send_bytes)
    : t_(t), cap_(std::max<size_t>(slot_bytes, 16)), send_cap_(std::max(send_bytes, cap_)), stride_(slot_stride(cap_)),
      nslots_(std::max(recv_slots, 1)) {
  // One send buffer + one receive arena: check against free HBM up front so a
  // 288 GB sweep fails with an explanation instead of a hipMalloc error mid-run.
  size_t free_b = 0, total_b = 0;
  const double arena = static_cast<double>(stride_) * static_cast<double>(nslots_);
  const double need = static_cast<double>(send_cap_) + arena;
  if (t_.mem_info(&free_b, &total_b) && need > 0.98 * static_cast<double>(free_b))
    P2P_FATAL(strfmt("buffers need %.2f GiB (send %s + %d receive slots of %s) but only %.2f of %.2f GiB are free on "
                     "this GPU; use a smaller --size/--sizes maximum or a mode with fewer concurrent peers",
                     need / (1ull << 30), format_size(send_cap_).c_str(), nslots_, format_size(cap_).c_str(),
                     static_cast<double>(free_b) / (1ull << 30), static_cast<double>(total_b) / (1ull << 30)));
  send_ = t_.alloc(send_cap_);
  recv_ = t_.alloc(stride_ * static_cast<size_t>(nslots_));
  Transport::BufferSet set;
  set.send = send_;
  set.send_bytes = send_cap_;
  set.recv = recv_;
  set.stride = stride_;
  set.slot_bytes = cap_;
  set.nslots = nslots_;
  t_.register_buffers(set);
}

Buffers::~Buffers() {
  // A destructor must not throw (the Python bindings turn fatal errors into
  // exceptions): when tearing down after an error fails too, say so and go
  // on, so the first error is the one that surfaces.
  try {
    t_.unregister_buffers(send_);
    if (recv_) t_.release(recv_);
    if (send_) t_.release(send_);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "p2p_matrix: buffer teardown failed: %s\n", e.what());
  }
}

void* Buffers::recv_buf(int slot) const {
  P2P_CHECK(slot >= 0 && slot < nslots_, strfmt("receive slot %d of %d", slot, nslots_));
  return static_cast<char*>(recv_) + stride_ * static_cast<size_t>(slot);
}

// -------------------------------------------------------------- helpers ----

int remote_slot(const Phase& phase, int me, int peer) {
  const auto& from = phase.ranks[static_cast<size_t>(peer)].recv_from;
  auto it = std::find(from.begin(), from.end(), me);
  P2P_CHECK(it != from.end(), strfmt("rank %d sends to %d, which does not receive from it", me, peer));
  return static_cast<int>(it - from.begin());
}

std::vector<int> remote_slots(const Phase& phase, int me) {
  const auto& to = phase.ranks[static_cast<size_t>(me)].send_to;
  std::vector<int> out;
  out.reserve(to.size());
  for (size_t j = 0; j < to.size(); ++j) {
    const int peer = to[j];
    const int kth = static_cast<int>(std::count(to.begin(), to.begin() + static_cast<long>(j), peer));
    const auto& from = phase.ranks[static_cast<size_t>(peer)].recv_from;
    int seen = 0, slot = -1;
    for (size_t i = 0; i < from.size() && slot < 0; ++i)
      if (from[i] == me && seen++ == kth) slot = static_cast<int>(i);
    P2P_CHECK(slot >= 0, strfmt("rank %d sends to %d, which does not receive from it", me, peer));
    out.push_back(slot);
  }
  return out;
}

namespace detail {

std::vector<int> flow_slots(const Phase& phase) {
  std::vector<int> slots;
  std::vector<int> seen(phase.ranks.size(), 0);
  for (const auto& f : phase.flows) slots.push_back(seen[static_cast<size_t>(f.dst)]++);
  return slots;
}

bool posts_phase(const Transport& t, const Phase& phase, int r) {
  return !phase.idle && (phase.participates(r) || t.wants_group_flows());
}

}  // namespace detail

namespace {

// Every flow of one iteration of a phase (Transport::group_flows).
std::vector<Transport::GroupFlow> group_flow_list(const Phase& phase) {
  const auto slots = flow_slots(phase);
  std::vector<Transport::GroupFlow> out(phase.flows.size());
  for (size_t i = 0; i < phase.flows.size(); ++i) {
    out[i].src = phase.flows[i].src;
    out[i].dst = phase.flows[i].dst;
    out[i].slot = slots[i];
  }
  return out;
}

}  // namespace

void post_phase_iteration(Transport& t, const Phase& phase, size_t bytes, Buffers& bufs, int gen) {
  const RankOps& ops = phase.ranks[static_cast<size_t>(t.rank())];
  const std::vector<int> rs = remote_slots(phase, t.rank());
  const int base = gen * std::max(1, phase.max_recv_slots());
  const size_t off = slot_stride(bytes) * static_cast<size_t>(gen);
  t.group_begin();
  if (t.wants_group_flows()) {
    std::vector<Transport::GroupFlow> flows = group_flow_list(phase);
    for (auto& f : flows) {
      f.slot += base;
      f.src_offset = off;
    }
    t.group_flows(bufs.send_buf(), flows, bytes);
  }
  for (size_t j = 0; j < ops.send_to.size(); ++j) t.send_to_slot(bufs.send_at(off), bytes, ops.send_to[j], base + rs[j]);
  for (size_t i = 0; i < ops.recv_from.size(); ++i)
    t.recv_from(bufs.recv_buf(base + static_cast<int>(i)), bytes, ops.recv_from[i], off);
  t.group_end();
}

size_t slot_stride_bytes(size_t bytes) { return slot_stride(bytes); }

uint64_t generation_seed(int src, size_t bytes, uint64_t salt, int gen) {
  return payload_seed(src, bytes, gen == 0 ? salt : salt ^ (static_cast<uint64_t>(gen) << 40));
}

size_t shared_free_budget(Transport& t, Bootstrap& boot, size_t fallback, size_t cap) {
  t.sync();
  boot.barrier();
  size_t free_b = 0, total_b = 0;
  size_t budget = t.mem_info(&free_b, &total_b) ? std::min(free_b / 4, cap) : fallback;
  const std::string key = t.device_key();
  int sharing = 0;
  for (const auto& k : boot.allgather_string(key)) sharing += !key.empty() && k == key;
  budget /= static_cast<size_t>(std::max(1, sharing));
  boot.barrier();  // every rank has read before any rank allocates
  return budget;
}

int verify_generations(Transport& t, Bootstrap& boot, size_t max_bytes, int slots, int iters) {
  // One generation = a send region + `slots` receive slots.
  const size_t per_gen = slot_stride(max_bytes) * static_cast<size_t>(std::max(1, slots) + 1);
  size_t budget = shared_free_budget(t, boot, size_t{256} << 20, size_t{32} << 30);
  if (const char* b = std::getenv("P2P_VERIFY_BUDGET")) budget = parse_size(b);
  long g = std::max(1, iters);
  g = std::min<long>(g, std::max<long>(1, static_cast<long>(budget / per_gen)));
  return static_cast<int>(-boot.allreduce_max(-static_cast<double>(g)));
}

namespace {

// Generations a phase of `cfg` uses in `bufs`: cfg.gens, capped by the
// iterations and by the send regions and receive slots the buffers hold (the
// same on every rank: every rank allocates the same buffers).
int phase_generations(const Phase& phase, const RunConfig& cfg, const Buffers& bufs) {
  if (!cfg.verify) return 1;
  const long per = std::max(1, phase.max_recv_slots());
  long g = std::min<long>(std::max(1, cfg.gens), std::max(cfg.iters, cfg.warmup));
  g = std::min<long>(g, bufs.slots() / per);
  g = std::min<long>(g, static_cast<long>(bufs.send_capacity() / slot_stride(cfg.bytes)));
  return static_cast<int>(std::max<long>(1, g));
}

// Slots g * per + i of generations [0, gens) are contiguous in the receive
// arena: one zeroing launch covers them all (and the padding between them),
// not one memset per slot.
void zero_slots(Transport& t, const Phase& phase, const RunConfig& cfg, Buffers& bufs, int gens) {
  const RankOps& ops = phase.ranks[static_cast<size_t>(t.rank())];
  if (ops.recv_from.empty()) return;
  const int per = std::max(1, phase.max_recv_slots());
  const int last = (gens - 1) * per + static_cast<int>(ops.recv_from.size()) - 1;
  char* first = static_cast<char*>(bufs.recv_buf(0));
  t.zero(first, static_cast<size_t>(static_cast<char*>(bufs.recv_buf(last)) - first) + cfg.bytes);
}

void prepare_payload(Transport& t, const Phase& phase, const RunConfig& cfg, Buffers& bufs, int gens) {
  const RankOps& ops = phase.ranks[static_cast<size_t>(t.rank())];
  P2P_CHECK(cfg.bytes <= bufs.capacity(), "message larger than buffers");
  P2P_CHECK(static_cast<int>(ops.recv_from.size()) <= bufs.slots(), "not enough receive slots");
  if (!ops.send_to.empty())
    for (int g = 0; g < gens; ++g)
      t.fill(bufs.send_at(slot_stride(cfg.bytes) * static_cast<size_t>(g)), cfg.bytes,
             generation_seed(t.rank(), cfg.bytes, cfg.salt, g));
  if (cfg.verify) zero_slots(t, phase, cfg, bufs, gens);
}

// Wrong words in this rank's receive slots of generations [0, gens).
uint64_t check_slots(Transport& t, const Phase& phase, const RunConfig& cfg, Buffers& bufs, int gens,
                     std::vector<uint64_t>* per_slot = nullptr) {
  const RankOps& ops = phase.ranks[static_cast<size_t>(t.rank())];
  const int per = std::max(1, phase.max_recv_slots());
  std::vector<Transport::VerifyJob> jobs;
  for (int g = 0; g < gens; ++g)
    for (size_t i = 0; i < ops.recv_from.size(); ++i)
      jobs.push_back({bufs.recv_buf(g * per + static_cast<int>(i)), cfg.bytes,
                      generation_seed(ops.recv_from[i], cfg.bytes, cfg.salt, g)});
  const std::vector<VerifyResult> res = t.verify_many(jobs);  // one batched check
  uint64_t bad = 0;
  for (int g = 0, k = 0; g < gens; ++g)
    for (size_t i = 0; i < ops.recv_from.size(); ++i, ++k) {
      const VerifyResult& v = res[static_cast<size_t>(k)];
      bad += v.mismatches;
      if (per_slot) {
        (*per_slot)[2 * i] += v.mismatches;
        if (g == 0) (*per_slot)[2 * i + 1] = v.checksum;
      }
    }
  return bad;
}

// Fault injection for the failure-detection tests: P2P_INJECT_FAULT =
// "<kind>@<rank>[:<phase>]" with kind one of
//   corrupt — zero the first 64 B of receive slot 0 after the timed loop
//             (verification must report it, exit code 2),
//   skip    — the rank's transport silently moves no payload during the
//             timed iterations (Transport::set_discard; the protocol still
//             runs, so nothing hangs): verification must report it, exit 2,
//   skip-some — the same for every other timed iteration (the even ones):
//             caught only because every iteration has its own receive
//             generation (RunConfig::gens),
//   exit    — the rank dies abruptly (peers must fail, not hang),
//   hang    — the rank stops responding (peers' watchdogs must fire).
struct FaultSpec {
  std::string kind;
  int rank = -1;
  long phase = -1;
};

const FaultSpec& fault_spec() {
  static FaultSpec spec = [] {
    FaultSpec s;
    const char* e = std::getenv("P2P_INJECT_FAULT");
    if (!e || !*e) return s;
    std::string v(e);
    auto at = v.find('@');
    if (at == std::string::npos) return s;
    s.kind = v.substr(0, at);
    std::string rest = v.substr(at + 1);
    auto colon = rest.find(':');
    s.rank = std::atoi(rest.substr(0, colon).c_str());
    if (colon != std::string::npos) s.phase = std::atol(rest.substr(colon + 1).c_str());
    return s;
  }();
  return spec;
}


}  // namespace

namespace detail {
bool fault_applies(const char* kind, int rank, long phase_index) {
  const FaultSpec& f = fault_spec();
  if (f.kind != kind || f.rank != rank) return false;
  return f.phase < 0 || f.phase == phase_index;
}
}  // namespace detail

namespace {

void maybe_inject_fault(Transport& t, Buffers& bufs, int rank, size_t phase_index, size_t bytes) {
  const FaultSpec& f = fault_spec();
  if (f.kind.empty() || f.kind == "skip" || f.kind == "skip-some" || f.rank != rank) return;
  if (f.phase >= 0 && static_cast<size_t>(f.phase) != phase_index) return;
  if (f.kind == "corrupt") {
    if (bufs.slots() > 0) {
      t.zero(bufs.recv_buf(0), std::min<size_t>(bytes, 64));
      t.sync();
    }
  } else if (f.kind == "exit") {
    std::fprintf(stderr, "[p2p] injected fault: rank %d exits\n", rank);
    std::fflush(stderr);
    std::_Exit(17);
  } else if (f.kind == "hang") {
    std::fprintf(stderr, "[p2p] injected fault: rank %d hangs\n", rank);
    std::fflush(stderr);
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
  }
}

}  // namespace

// ------------------------------------------------------------ run_phase ----

namespace {

// RCCL 2.26 delivers exactly half of an op whose share of one p2p channel
// exceeds 16 MiB and reports no error; the RCCL transport sizes its ops from
// the channels RCCL set up for each peer (transport_rccl.cpp).  With --verify
// the warmup's deliveries are checked as a second line of defence: should any
// rank see a wrong word, every rank caps its ops at 16, 4, then 1 MiB (the
// same on all: chunking must match on both ends of a message), re-poisons its
// slots once every rank has drained, and warms up again, until the warmup
// verifies.  The cap lasts for this phase only (run_phase lifts it) and the
// phase record keeps what happened (warmup_mismatches, rechunked_to).
// Transports that split nothing (set_chunk_cap false) are left as they are.
void rechunk_until_warmup_verifies(Transport& t, Bootstrap& boot, const Phase& phase, const RunConfig& cfg,
                                   Buffers& bufs, bool active, int gens, PhaseResult* res) {
  const int me = t.rank();
  const int warm_gens = std::min(gens, cfg.warmup);
  auto local_mismatches = [&]() -> uint64_t { return active ? check_slots(t, phase, cfg, bufs, warm_gens) : 0; };
  uint64_t bad = boot.allreduce_sum_u64(local_mismatches());
  res->warmup_mismatches = bad;
  if (!cfg.rechunk) return;
  for (const size_t c : {size_t{16} << 20, size_t{4} << 20, size_t{1} << 20}) {
    if (bad == 0) return;
    // Agreed on every rank: each posts the same groups, so each must take the
    // same branch.
    const size_t cur = static_cast<size_t>(boot.allreduce_max(static_cast<double>(res->op_bytes ? res->op_bytes : cfg.bytes)));
    if (c >= cur) continue;
    if (!t.set_chunk_cap(c)) return;
    res->rechunked_to.push_back(c);
    res->op_bytes = c;
    if (me == 0)
      std::fprintf(stderr, "[p2p] %s: %llu wrong words in the warmup; messages now posted as ops of <= %zu MiB\n",
                   phase.label.c_str(), static_cast<unsigned long long>(bad), c >> 20);
    boot.barrier();  // every rank drained its warmup (push writers too)
    if (active) {
      zero_slots(t, phase, cfg, bufs, gens);
      t.sync();
    }
    boot.barrier();
    if (active) {
      for (int i = 0; i < cfg.warmup; ++i) post_phase_iteration(t, phase, cfg.bytes, bufs, i % gens);
      t.sync();
    }
    bad = boot.allreduce_sum_u64(local_mismatches());
  }
  res->warmup_residual = bad;
  if (bad && me == 0 && !res->rechunked_to.empty())
    std::fprintf(stderr,
                 "[p2p] %s: still %llu wrong words in the warmup with ops of <= %zu KiB: the loss does not follow "
                 "the op size (RCCL channel knobs? e.g. NCCL_NCHANNELS_PER_PEER above the p2p channel count lost half "
                 "of every message over RCCL's socket transport, profiles/r4_node_rehearsal/)\n",
                 phase.label.c_str(), static_cast<unsigned long long>(bad), res->rechunked_to.back() >> 10);
}

// Largest op this rank posts for the phase's messages (0: one op each).
size_t phase_op_bytes(const Transport& t, const Phase& phase, size_t bytes) {
  const RankOps& ops = phase.ranks[static_cast<size_t>(t.rank())];
  size_t most = 0;
  bool split = false;
  auto see = [&](int peer) {
    const size_t c = t.max_chunk(peer);
    if (c && bytes > c) {
      split = true;
      most = std::max(most, c);
    }
  };
  for (int p : ops.send_to) see(p);
  for (int p : ops.recv_from) see(p);
  return split ? most : 0;
}

}  // namespace

PhaseResult run_phase(Transport& t, Bootstrap& boot, const Phase& phase, size_t phase_index, const RunConfig& cfg,
                      Buffers& bufs) {
  const int n = boot.size();
  const int me = boot.rank();
  PhaseResult res;
  res.index = phase_index;
  res.label = phase.label;
  res.row = phase.row;
  res.col = phase.col;
  res.idle = phase.idle;
  res.bytes = cfg.bytes;
  res.iters = cfg.iters;
  res.rank_seconds.assign(static_cast<size_t>(n), 0.0);

  if (phase.idle) {
    // p2p_matrix.cc:146-152: every rank takes the barrier, then the diagonal
    // is reported as 0.00 without moving data.
    boot.barrier();
    return res;
  }
  P2P_CHECK(cfg.iters >= 1, "iters must be >= 1");
  // Relay ranks of a multi-path transport post (and time) the phase too; a
  // flow is still charged by its two endpoints only.
  const bool active = posts_phase(t, phase, me);
  const int gens = phase_generations(phase, cfg, bufs);
  res.generations = gens;
  res.op_bytes = phase_op_bytes(t, phase, cfg.bytes);
  // The ops a phase's messages are posted as: what the transport derived, or
  // less after a warmup that did not verify (this phase only).
  struct ChunkCap {
    Transport& t;
    size_t before;  // a cap set by the caller (e.g. bench.py's warmup check) stays after the phase
    bool set = false;
    ~ChunkCap() {
      if (set) t.set_chunk_cap(before);
    }
  } cap{t, t.chunk_cap()};

  if (active) {
    prepare_payload(t, phase, cfg, bufs, gens);
    for (int i = 0; i < cfg.warmup; ++i) post_phase_iteration(t, phase, cfg.bytes, bufs, i % gens);
    t.sync();
  }
  if (cfg.verify && cfg.warmup > 0) {
    rechunk_until_warmup_verifies(t, boot, phase, cfg, bufs, active, gens, &res);
    cap.set = !res.rechunked_to.empty();
    // The warmup delivered the payload already: poison the slots again (after
    // every rank drained its warmup), so the check after timing passes only
    // for data the timed iterations delivered.
    boot.barrier();
    if (active) {
      zero_slots(t, phase, cfg, bufs, gens);
      t.sync();
    }
  }
  const bool skip = active && fault_applies("skip", me, static_cast<long>(phase_index));
  const bool skip_some = active && fault_applies("skip-some", me, static_cast<long>(phase_index));
  if (skip) {
    std::fprintf(stderr, "[p2p] injected fault: rank %d moves no payload in the timed iterations\n", me);
    t.set_discard(true);
  }
  if (skip_some)
    std::fprintf(stderr, "[p2p] injected fault: rank %d moves no payload in every other timed iteration\n", me);
  // Iteration i posts generation i mod gens; skip-some drops the even ones.
  auto post = [&](int i) {
    if (skip_some) t.set_discard(i % 2 == 0);
    post_phase_iteration(t, phase, cfg.bytes, bufs, i % gens);
  };

  double my_seconds = 0;
  std::vector<double> iter_samples;
  boot.barrier();
  TraceRange trace_range(phase.label.c_str());
  const double w0 = now_seconds();
  if (cfg.timing == Timing::Wallclock) {
    // Reference semantics: a host stream-sync after every message
    // (p2p_matrix.cc:162, :170, :229-230, :250-251) and a barrier-bracketed
    // host clock (:153, :173-176).
    if (active) {
      iter_samples.reserve(static_cast<size_t>(cfg.iters));
      for (int i = 0; i < cfg.iters; ++i) {
        double a = now_seconds();
        post(i);
        t.sync();
        iter_samples.push_back((now_seconds() - a) * 1e6);
      }
    }
    boot.barrier();
    my_seconds = now_seconds() - w0;
  } else {
    if (active) {
      t.clear_marks();
      int m0 = t.mark();
      std::vector<int> marks;
      marks.reserve(static_cast<size_t>(cfg.iters));
      for (int i = 0; i < cfg.iters; ++i) {
        post(i);
        if (cfg.samples || i + 1 == cfg.iters) marks.push_back(t.mark());
      }
      t.sync();
      my_seconds = t.elapsed_ms(m0, marks.back()) / 1e3;
      if (cfg.samples) {
        // With K messages in flight on K streams (t.concurrency()), one mark
        // to the next is a completion frontier, often 0 when a later message
        // finished first: a sample then spans K marks and is divided by K
        // (per-message time over a round of one message per stream).
        const size_t k = static_cast<size_t>(std::max(1, t.concurrency()));
        if (marks.size() < k) {
          iter_samples.push_back(t.elapsed_ms(m0, marks.back()) * 1e3 / static_cast<double>(marks.size()));
        } else {
          int prev = m0;
          for (size_t i = k - 1; i < marks.size(); i += k) {
            iter_samples.push_back(t.elapsed_ms(prev, marks[i]) * 1e3 / static_cast<double>(k));
            prev = marks[i];
          }
        }
      }
    }
    boot.barrier();
  }
  const double w1 = now_seconds();
  res.wall_seconds = w1 - w0;
  if (skip || skip_some) t.set_discard(false);

  if (active) maybe_inject_fault(t, bufs, me, phase_index, cfg.bytes);

  std::string err = t.async_error();
  if (!err.empty()) P2P_FATAL("transport reported an asynchronous error: " + err);

  // Verification of every receive slot of every generation on this rank:
  // per slot, the wrong words summed over generations and generation 0's
  // checksum.
  const int maxslots = std::max(1, phase.max_recv_slots());
  std::vector<uint64_t> vr(static_cast<size_t>(maxslots) * 2, 0);
  const int timed_gens = std::min(gens, cfg.iters);
  uint64_t cover[2] = {0, 0};  // timed deliveries, verified deliveries (this rank)
  if (active) {
    const uint64_t nrecv = phase.ranks[static_cast<size_t>(me)].recv_from.size();
    cover[0] = nrecv * static_cast<uint64_t>(cfg.iters);
    if (cfg.verify) {
      check_slots(t, phase, cfg, bufs, timed_gens, &vr);
      cover[1] = nrecv * static_cast<uint64_t>(timed_gens);
    }
  }
  res.timed_msgs = boot.allreduce_sum_u64(cover[0]);
  res.verified_msgs = boot.allreduce_sum_u64(cover[1]);

  res.rank_seconds = boot.allgather_value(my_seconds);
  const double span[2] = {w0, w1};
  std::vector<double> spans(static_cast<size_t>(2 * n));
  boot.allgather(span, spans.data(), sizeof(span));
  for (int r = 0; r < n; ++r) {
    res.host_begin.push_back(spans[static_cast<size_t>(2 * r)]);
    res.host_end.push_back(spans[static_cast<size_t>(2 * r + 1)]);
  }
  Summary mine = summarize(iter_samples);
  auto summaries = boot.allgather_value(mine);
  auto all_vr = boot.allgather_vector(vr);

  double phase_s = 0;
  for (int r = 0; r < n; ++r)
    if (cfg.timing == Timing::Wallclock || phase.participates(r)) phase_s = std::max(phase_s, res.rank_seconds[static_cast<size_t>(r)]);
  res.seconds_per_iter = phase_s / cfg.iters;
  res.bytes_per_iter = static_cast<double>(cfg.bytes) * static_cast<double>(phase.flows.size());
  res.agg_gbs = gbytes_per_s(res.bytes_per_iter, res.seconds_per_iter);

  auto slots = flow_slots(phase);
  for (size_t fi = 0; fi < phase.flows.size(); ++fi) {
    const Flow& f = phase.flows[fi];
    FlowResult fr;
    fr.flow = f;
    double s = cfg.timing == Timing::Wallclock
                   ? phase_s
                   : std::max(res.rank_seconds[static_cast<size_t>(f.src)], res.rank_seconds[static_cast<size_t>(f.dst)]);
    fr.seconds = s / cfg.iters;
    fr.gbps = gbps(static_cast<double>(cfg.bytes), fr.seconds);
    fr.gbs = gbytes_per_s(static_cast<double>(cfg.bytes), fr.seconds);
    fr.iter_us = summaries[static_cast<size_t>(f.dst)];
    if (cfg.verify) {
      size_t base = static_cast<size_t>(f.dst) * vr.size() + 2 * static_cast<size_t>(slots[fi]);
      fr.verified = true;
      fr.mismatches = all_vr[base];
      fr.checksum = all_vr[base + 1];
      res.total_mismatches += fr.mismatches;
    }
    res.flows.push_back(fr);
  }
  return res;
}

std::vector<PhaseResult> run_schedule(Transport& t, Bootstrap& boot, const Schedule& s, const RunConfig& cfg, Buffers& bufs,
                                      const PhaseCallback& on_phase) {
  std::string bad = validate(s);
  P2P_CHECK(bad.empty(), "invalid schedule: " + bad);
  std::vector<PhaseResult> out;
  out.reserve(s.phases.size());
  for (size_t i = 0; i < s.phases.size(); ++i) {
    out.push_back(run_phase(t, boot, s.phases[i], i, cfg, bufs));
    if (on_phase) on_phase(out.back());
  }
  return out;
}

void warm_connections(Transport& t, Bootstrap& boot, const Schedule& s, Buffers& bufs, size_t bytes) {
  bytes = std::min(bytes, bufs.capacity());
  for (const Phase& p : s.phases) {
    if (!posts_phase(t, p, t.rank())) continue;
    post_phase_iteration(t, p, bytes, bufs);
    t.sync();
  }
  boot.barrier();
}

// -------------------------------------------------------------- latency ----

std::vector<LatencyResult> run_latency(Transport& t, Bootstrap& boot, size_t bytes, int iters, int warmup, Buffers& bufs,
                                       int preposted) {
  const int n = boot.size(), me = boot.rank();
  P2P_CHECK(bytes <= bufs.capacity() && bufs.slots() >= 1, "latency buffers too small");
  P2P_CHECK(iters >= 1, "latency iters must be >= 1");
  std::vector<LatencyResult> out;
  // A transport without a gate (CPU) says so on its first arm: probe once,
  // collectively, and fall back to host-posted samples everywhere.
  bool gated = false;
  if (preposted > 0) {
    gated = t.gate_arm(1.0);
    if (gated) {
      t.gate_release();
      t.sync();
    }
    gated = boot.allreduce_max(gated ? 0.0 : 1.0) == 0.0;
  }
  constexpr double kGateTimeoutS = 5.0;  // a gate opens by itself after this (never a hung stream)

  auto run_round = [&](int partner) -> Summary {
    const bool self = (partner == me);
    const bool lead = self || (partner >= 0 && me < partner);
    auto exchange = [&]() {
      if (self) {
        t.group_begin();
        t.send(bufs.send_buf(), bytes, me);
        t.recv(bufs.recv_buf(0), bytes, me);
        t.group_end();
      } else if (lead) {
        t.group_begin(); t.send(bufs.send_buf(), bytes, partner); t.group_end();
        t.group_begin(); t.recv(bufs.recv_buf(0), bytes, partner); t.group_end();
      } else {
        t.group_begin(); t.recv(bufs.recv_buf(0), bytes, partner); t.group_end();
        t.group_begin(); t.send(bufs.send_buf(), bytes, partner); t.group_end();
      }
    };
    if (partner >= 0) {
      for (int i = 0; i < warmup; ++i) exchange();
      t.sync();
    }
    boot.barrier();
    std::vector<double> samples;
    auto sample = [&](const std::vector<int>& marks, size_t from) {
      if (!lead) return;
      for (size_t i = from; i < marks.size(); ++i) {
        double us = t.elapsed_ms(marks[i - 1], marks[i]) * 1e3;
        samples.push_back(self ? us : us / 2.0);
      }
    };
    if (gated) {
      // Batches of `batch` exchanges behind a gate on every rank; all ranks
      // have posted theirs before any gate opens (barrier), so the batch runs
      // with no host in the loop.  Every rank runs the same batches, active
      // or not, so the barriers match.
      const int batch = std::max(2, preposted);
      for (int done = 0; done < iters; done += batch - 1) {
        const int k = std::min(batch, iters - done + 1);
        std::vector<int> marks;
        if (partner >= 0) {
          t.clear_marks();
          P2P_CHECK(t.gate_arm(kGateTimeoutS), "stream gate unavailable");
          marks.push_back(t.mark());
          for (int i = 0; i < k; ++i) {
            exchange();
            marks.push_back(t.mark());
          }
        }
        boot.barrier();  // every rank's batch is posted
        if (partner >= 0) {
          t.gate_release();
          t.sync();
          P2P_CHECK(!t.gate_timed_out(), "stream gate expired before its release (host stalled?)");
          sample(marks, 2);  // marks[1]: the first exchange, which also waited for the partner's release
        }
      }
    } else if (partner >= 0) {
      t.clear_marks();
      std::vector<int> marks;
      marks.push_back(t.mark());
      for (int i = 0; i < iters; ++i) {
        exchange();
        marks.push_back(t.mark());
      }
      t.sync();
      sample(marks, 1);
    }
    boot.barrier();
    return summarize(samples);
  };

  if (n == 1) {
    Summary s = run_round(0);
    LatencyResult r;
    r.a = r.b = 0;
    r.bytes = bytes;
    r.one_way_us = s;
    r.method = gated ? "preposted" : "host";
    out.push_back(r);
    return out;
  }
  for (const auto& round : round_robin_rounds(n)) {
    int partner = -1;
    for (auto& pr : round) {
      if (pr.first == me) partner = pr.second;
      if (pr.second == me) partner = pr.first;
    }
    Summary s = run_round(partner);
    auto all = boot.allgather_value(s);
    for (auto& pr : round) {
      LatencyResult r;
      r.a = pr.first;
      r.b = pr.second;
      r.bytes = bytes;
      r.one_way_us = all[static_cast<size_t>(pr.first)];
      r.method = gated ? "preposted" : "host";
      out.push_back(r);
    }
  }
  std::sort(out.begin(), out.end(), [](const LatencyResult& x, const LatencyResult& y) {
    return x.a != y.a ? x.a < y.a : x.b < y.b;
  });
  return out;
}

std::vector<LatencyResult> run_device_latency(Transport& t, Bootstrap& boot, size_t bytes, int iters, int warmup) {
  P2P_CHECK(t.supports_device_pingpong(),
            "device ping-pong needs a one-sided transport (--transport ipc); " + t.name() + " has none");
  P2P_CHECK(iters >= 1 && warmup >= 0, "bad device latency iterations");
  const int n = boot.size(), me = boot.rank();
  t.pingpong_setup();
  auto one = [&](int partner) -> Summary {
    std::vector<double> us;
    boot.barrier();  // both kernels start together (each spin has a deadline)
    if (partner >= 0) {
      us = t.device_pingpong(partner, bytes, warmup + iters);
      if (!us.empty()) us.erase(us.begin(), us.begin() + std::min<size_t>(us.size(), static_cast<size_t>(warmup)));
    }
    return summarize(us);
  };
  std::vector<LatencyResult> out;
  auto add = [&](int a, int b, const Summary& s) {
    LatencyResult r;
    r.a = a;
    r.b = b;
    r.bytes = std::max<size_t>(16, (bytes + 15) / 16 * 16);
    r.one_way_us = s;
    r.method = "device";
    out.push_back(r);
  };
  if (n == 1) {
    add(0, 0, one(0));
    return out;
  }
  for (const auto& round : round_robin_rounds(n)) {
    int partner = -1;
    for (auto& pr : round) {
      if (pr.first == me) partner = pr.second;
      if (pr.second == me) partner = pr.first;
    }
    Summary s = one(partner);
    auto all = boot.allgather_value(s);
    for (auto& pr : round) add(pr.first, pr.second, all[static_cast<size_t>(pr.first)]);
  }
  std::sort(out.begin(), out.end(), [](const LatencyResult& x, const LatencyResult& y) {
    return x.a != y.a ? x.a < y.a : x.b < y.b;
  });
  return out;
}

// ------------------------------------------------------ ring token chain ----

namespace {
RingLatencyResult ring_result(Bootstrap& boot, size_t bytes, int laps, const std::vector<double>& lap_us,
                              const char* method) {
  // Rank 0's samples, for every rank.
  const Summary lap = summarize(lap_us);
  std::vector<double> hop;
  for (double v : lap_us) hop.push_back(v / boot.size());
  const Summary h = summarize(hop);
  RingLatencyResult r;
  r.nranks = boot.size();
  r.bytes = bytes;
  r.laps = laps;
  r.lap_us = boot.allgather_value(lap)[0];
  r.hop_us = boot.allgather_value(h)[0];
  r.method = method;
  return r;
}
}  // namespace

RingLatencyResult run_ring_latency(Transport& t, Bootstrap& boot, size_t bytes, int laps, int warmup, Buffers& bufs) {
  const int n = boot.size(), me = boot.rank();
  P2P_CHECK(bytes <= bufs.capacity() && laps >= 1 && warmup >= 0, "ring latency: bad arguments");
  const int succ = (me + 1) % n, pred = (me + n - 1) % n;
  auto lap = [&]() {
    if (n == 1) {
      t.group_begin();
      t.send(bufs.send_buf(), bytes, me);
      t.recv(bufs.recv_buf(0), bytes, me);
      t.group_end();
      return;
    }
    auto send = [&] { t.group_begin(); t.send_to_slot(bufs.send_buf(), bytes, succ, 0); t.group_end(); };
    auto recv = [&] { t.group_begin(); t.recv(bufs.recv_buf(0), bytes, pred); t.group_end(); };
    if (me == 0) {
      send();
      recv();
    } else {
      recv();
      send();
    }
  };
  for (int i = 0; i < warmup; ++i) lap();
  t.sync();
  boot.barrier();
  t.clear_marks();
  std::vector<int> marks{t.mark()};
  for (int i = 0; i < laps; ++i) {
    lap();
    marks.push_back(t.mark());
  }
  t.sync();
  std::vector<double> us;
  if (me == 0)
    for (size_t i = 1; i < marks.size(); ++i) us.push_back(t.elapsed_ms(marks[i - 1], marks[i]) * 1e3);
  boot.barrier();
  return ring_result(boot, bytes, laps, us, "host");
}

RingLatencyResult run_device_ring_latency(Transport& t, Bootstrap& boot, size_t bytes, int laps, int warmup) {
  P2P_CHECK(t.supports_device_pingpong(),
            "device ring latency needs a one-sided transport (--transport ipc); " + t.name() + " has none");
  P2P_CHECK(laps >= 1 && warmup >= 0, "device ring latency: bad arguments");
  const int n = boot.size(), me = boot.rank();
  t.pingpong_setup();
  std::vector<double> us;
  if (n == 1) {
    // One rank: the token's hop is a self round trip through its own inbox.
    boot.barrier();
    us = t.device_pingpong(me, bytes, warmup + laps);
    us.erase(us.begin(), us.begin() + std::min<size_t>(us.size(), static_cast<size_t>(warmup)));
    for (double& v : us) v *= 2.0;  // device_pingpong returns half round trips
  } else {
    const int succ = (me + 1) % n, pred = (me + n - 1) % n;
    if (warmup > 0) {
      boot.barrier();  // every rank's kernel starts together (each spin has a deadline)
      t.device_ring_token(pred, succ, me == 0, bytes, warmup);
    }
    boot.barrier();
    us = t.device_ring_token(pred, succ, me == 0, bytes, laps);
  }
  boot.barrier();
  return ring_result(boot, std::max<size_t>(16, (bytes + 15) / 16 * 16), laps, us, "device");
}

// ----------------------------------------------------------------- fuzz ----

uint64_t fuzz_transport(Transport& t, Bootstrap& boot, int rounds, uint64_t seed, size_t max_bytes) {
  const int n = boot.size(), me = boot.rank();
  P2P_CHECK(max_bytes >= 16, "fuzz: max_bytes >= 16");
  constexpr int kMaxMsgs = 12;
  // One buffer set for the whole run, like a schedule's: every message a rank
  // sends in a round is a prefix of its send buffer (filled with the round's
  // stream), and the i-th message it receives lands in slot i.  This is what
  // the one-sided transports (IPC pull / push / relay) can move.
  Buffers bufs(t, max_bytes, kMaxMsgs);
  uint64_t rng = seed;
  auto next = [&]() {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return static_cast<uint64_t>(rng >> 33);
  };
  uint64_t mism = 0;
  struct Msg {
    int src, dst;
    size_t bytes;
    int slot;  // receive slot on dst
  };
  for (int r = 0; r < rounds; ++r) {
    std::vector<Msg> plan;
    std::vector<int> slots(static_cast<size_t>(n), 0);
    const int count = 1 + static_cast<int>(next() % kMaxMsgs);
    for (int k = 0; k < count; ++k) {
      Msg m{static_cast<int>(next() % static_cast<uint64_t>(n)), static_cast<int>(next() % static_cast<uint64_t>(n)), 0, 0};
      const uint64_t kind = next() % 4;  // tiny, one page, odd, large
      m.bytes = kind == 0 ? 1 + next() % 16 : kind == 1 ? 4096 : kind == 2 ? 1 + next() % (max_bytes / 4) : max_bytes / 2 + next() % (max_bytes / 2);
      m.bytes = std::min(std::max<size_t>(m.bytes, 1), max_bytes);
      m.slot = slots[static_cast<size_t>(m.dst)]++;
      plan.push_back(m);
    }
    auto seed_of = [&](int src) { return payload_seed(src, max_bytes, static_cast<uint64_t>(r) * 1000 + 7); };
    bool sends = false;
    for (const Msg& m : plan) sends = sends || m.src == me;
    if (sends) t.fill(bufs.send_buf(), max_bytes, seed_of(me));
    for (const Msg& m : plan)
      if (m.dst == me) t.zero(bufs.recv_buf(m.slot), m.bytes);
    t.sync();
    boot.barrier();  // every payload written and every slot poisoned before anyone moves data
    t.group_begin();
    if (t.wants_group_flows())
      for (const Msg& m : plan) t.group_flows(bufs.send_buf(), {Transport::GroupFlow{m.src, m.dst, m.slot}}, m.bytes);
    for (const Msg& m : plan)
      if (m.src == me) t.send_to_slot(bufs.send_buf(), m.bytes, m.dst, m.slot);
    for (const Msg& m : plan)
      if (m.dst == me) t.recv(bufs.recv_buf(m.slot), m.bytes, m.src);
    t.group_end();
    t.sync();
    for (const Msg& m : plan)
      if (m.dst == me) mism += t.verify(bufs.recv_buf(m.slot), m.bytes, seed_of(m.src)).mismatches;
    boot.barrier();  // nobody refills its send buffer while a peer may still read it
  }
  return mism;
}

}  // namespace p2p
