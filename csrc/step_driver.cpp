// StepDriver (runner.hpp): the engine behind bench.py's timed steps.  One
// phase of the schedule per step, posted with no host sync between steps;
// payload layout and verification as described in runner.hpp.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "bootstrap.hpp"
#include "common.hpp"
#include "prng.hpp"
#include "runner.hpp"
#include "runner_detail.hpp"

namespace p2p {

using detail::fault_applies;
using detail::flow_slots;
using detail::posts_phase;
using detail::slot_stride;

namespace {

// [rank][phase] -> first slot of the phase within a generation; the last
// entry of each row is the generation size.
std::vector<std::vector<int>> step_layout(const Schedule& s, int msgs) {
  P2P_CHECK(msgs >= 1, "msgs per step must be >= 1");
  std::vector<std::vector<int>> base(static_cast<size_t>(s.nranks));
  for (int r = 0; r < s.nranks; ++r) {
    int at = 0;
    for (const Phase& p : s.phases) {
      base[static_cast<size_t>(r)].push_back(at);
      at += p.recv_slots(r) * msgs;
    }
    base[static_cast<size_t>(r)].push_back(at);
  }
  return base;
}

std::vector<int> generation_sizes(const std::vector<std::vector<int>>& base) {
  std::vector<int> out;
  for (const auto& row : base) out.push_back(row.back());
  return out;
}

// Receive generations: as many as asked and the budget allows, the same on
// every rank (every rank computes every peer's slot numbers).
int agreed_depth(Transport& t, Bootstrap& boot, const StepOptions& o, size_t per_gen_bytes) {
  long d = std::max(1, o.depth);
  size_t budget = o.recv_budget;
  if (budget == 0) budget = shared_free_budget(t, boot, size_t{256} << 20, SIZE_MAX);
  if (per_gen_bytes > 0) d = std::min<long>(d, std::max<long>(1, static_cast<long>(budget / per_gen_bytes)));
  return static_cast<int>(-boot.allreduce_max(-static_cast<double>(d)));
}

}  // namespace

StepDriver::StepDriver(Transport& t, Bootstrap& boot, Schedule sched, size_t bytes, int msgs, bool verify, uint64_t salt,
                       StepOptions opt)
    : t_(t), boot_(boot), sched_(std::move(sched)), bytes_(bytes), msgs_(msgs), verify_(verify), salt_(salt), opt_(opt),
      phase_base_(step_layout(sched_, msgs)), gen_slots_(generation_sizes(phase_base_)),
      depth_(agreed_depth(t, boot, opt, slot_stride(bytes) * static_cast<size_t>(gen_slots_.at(static_cast<size_t>(t.rank()))))),
      bufs_(t, bytes, std::max(1, depth_ * gen_slots_[static_cast<size_t>(t.rank())]),
            slot_stride(bytes) * static_cast<size_t>(msgs)) {
  if (opt_.graph && !t_.supports_graphs()) opt_.graph = false;
  if (const char* g = std::getenv("P2P_STEP_GROUP_MSGS"); g && opt_.group_msgs == 0) opt_.group_msgs = std::atoi(g);
  if (const char* g = std::getenv("P2P_STEP_FIRST_GROUP_MSGS"); g && opt_.first_group_msgs == 0)
    opt_.first_group_msgs = std::atoi(g);
  std::string bad = validate(sched_);
  P2P_CHECK(bad.empty(), "invalid schedule: " + bad);
  P2P_CHECK(!sched_.phases.empty(), "empty schedule");
  P2P_CHECK(sched_.nranks == t_.nranks(), "schedule and transport disagree on the number of ranks");
  // Message m is sent from region m; regions start at 4 KiB boundaries like
  // the receive slots, so every kernel sees 16-byte aligned payloads.
  for (int m = 0; m < msgs_; ++m) t_.fill(bufs_.send_at(region_offset(m)), bytes_, msg_seed(t_.rank(), m));
  if (verify_) t_.zero(bufs_.recv_base(), recv_bytes());
  t_.sync();
}

StepDriver::~StepDriver() {
  if (skip_armed_ || skip_some_armed_) t_.set_discard(false);
}

int StepDriver::slot_index(int rank, int gen, int phase, int msg, int i) const {
  const Phase& p = sched_.phases[static_cast<size_t>(phase)];
  const int r = p.recv_slots(rank);
  P2P_CHECK(i >= 0 && i < r && msg >= 0 && msg < msgs_ && gen >= 0 && gen < depth_, "bad step slot");
  return gen * gen_slots_[static_cast<size_t>(rank)] + phase_base_[static_cast<size_t>(rank)][static_cast<size_t>(phase)] +
         msg * r + i;
}

size_t StepDriver::region_offset(int msg) const { return slot_stride(bytes_) * static_cast<size_t>(msg); }

uint64_t StepDriver::msg_seed(int src, int msg) const {
  return payload_seed(src, bytes_, salt_ * 1000003ull + static_cast<uint64_t>(msg) + 1);
}

void StepDriver::connect() {
  warm_connections(t_, boot_, sched_, bufs_, std::min<size_t>(bytes_, 4096));
  // One full step of every phase: small messages may take another path than
  // the step's (RCCL with several communicators keeps them on the first), so
  // every connection the timed steps use is made here, not in a timed step.
  for (size_t pi = 0; pi < sched_.phases.size(); ++pi)
    if (posts_phase(t_, sched_.phases[pi], t_.rank())) post_step_ops(sched_.phases[pi], static_cast<int>(pi), 0);
  t_.sync();
  boot_.barrier();
  if (verify_) t_.zero(bufs_.recv_base(), recv_bytes());
  t_.sync();
  // Every connection exists now: the transport re-derives its per-peer op
  // limits from what it connected (RCCL's connection lines), before any graph
  // records op sizes and before any timed step.
  if (t_.refine_op_limits(boot_)) ++limit_changes_;
  // Graph capture only records launches (no peer interaction), so it must
  // follow the warm-up that established every lazy connection.
  if (opt_.graph && graphs_.empty()) capture_graphs();
}

void StepDriver::capture_graphs() {
  // A recapture (rechunk fallback) replaces the graphs: the transport frees
  // the old ones instead of keeping them until it is destroyed.
  for (int h : graphs_)
    if (h >= 0) t_.graph_release(h);
  graphs_.clear();
  for (int g = 0; g < depth_; ++g)
    for (size_t pi = 0; pi < sched_.phases.size(); ++pi) {
      const Phase& p = sched_.phases[pi];
      if (!p.participates(t_.rank())) {
        graphs_.push_back(-1);
        continue;
      }
      t_.capture_begin();
      post_step_ops(p, static_cast<int>(pi), g);
      graphs_.push_back(t_.capture_end());
    }
  boot_.barrier();
}

void StepDriver::recapture() {
  // A graph replays the ops it recorded, op sizes included: after the
  // transport's chunking changed, the steps must be recorded again.
  if (!opt_.graph) return;
  sync();
  capture_graphs();
  ++recaptures_;
}

void StepDriver::post_step_ops(const Phase& p, int pi, int gen) {
  const int me = t_.rank();
  const RankOps& ops = p.ranks[static_cast<size_t>(me)];
  const std::vector<int> rs = remote_slots(p, me);
  const bool all_flows = t_.wants_group_flows();
  std::vector<int> fslot;
  if (all_flows) fslot = flow_slots(p);
  auto one_message = [&](int m) {
    const size_t off = region_offset(m);
    if (all_flows) {
      std::vector<Transport::GroupFlow> flows(p.flows.size());
      for (size_t i = 0; i < p.flows.size(); ++i) {
        flows[i].src = p.flows[i].src;
        flows[i].dst = p.flows[i].dst;
        flows[i].slot = slot_index(p.flows[i].dst, gen, pi, m, fslot[i]);
        flows[i].src_offset = off;
      }
      t_.group_flows(bufs_.send_buf(), flows, bytes_);
    }
    for (size_t j = 0; j < ops.send_to.size(); ++j)
      t_.send_to_slot(bufs_.send_at(off), bytes_, ops.send_to[j], slot_index(ops.send_to[j], gen, pi, m, rs[j]));
    for (size_t i = 0; i < ops.recv_from.size(); ++i)
      t_.recv_from(bufs_.recv_buf(slot_index(me, gen, pi, m, static_cast<int>(i))), bytes_, ops.recv_from[i], off);
  };
  if (opt_.batch) {
    // One group: every message of the step, fused into one launch by RCCL
    // (or groups of per_group_ whole messages, post_step_groups).
    const int per = per_group_ > 0 && per_group_ < msgs_ ? per_group_ : msgs_;
    for (int m0 = 0; m0 < msgs_; m0 += per) {
      t_.group_begin();
      for (int m = m0; m < std::min(msgs_, m0 + per); ++m) one_message(m);
      t_.group_end();
    }
  } else {
    for (int m = 0; m < msgs_; ++m) {
      t_.group_begin();
      one_message(m);
      t_.group_end();
    }
  }
}

// A step posted in groups of `per_group` whole messages (0: one group).  A
// transport launches nothing of a group before its end (RCCL prepares all of
// a group's work first), so smaller groups let the GPU start on a step while
// the host is still posting it; with 8 communicators and messages routed
// round-robin over them, 16 messages per group give every communicator its
// usual two-message kernel (profiles/r3b_post/).
void StepDriver::post_step_groups(const Phase& p, int pi, int gen, int per_group) {
  per_group_ = per_group;
  post_step_ops(p, pi, gen);
  per_group_ = 0;
}

void StepDriver::step(long k) { step_impl(k, false); }

void StepDriver::run_steps(long first, long count) {
  for (long k = first; k < first + count; ++k) step_impl(k, k > first);
}

void StepDriver::step_impl(long k, bool chain) {
  const auto posted_from = std::chrono::steady_clock::now();
  const int pi = static_cast<int>(k % phases());
  const int g = gen_of(k);
  const Phase& p = sched_.phases[static_cast<size_t>(pi)];
  if (!chain) chain_mark_ = -1;
  // skip-some: every other step moves no payload (a graph replay would not
  // honour the discard, so such steps are posted eagerly).
  if (skip_some_armed_) t_.set_discard(k % 2 == 0);
  const bool replay = opt_.graph && !skip_armed_ && !skip_some_armed_;
  const int per_group = !chain && opt_.first_group_msgs > 0 ? opt_.first_group_msgs : opt_.group_msgs;
  if (!p.participates(t_.rank())) {
    if (posts_phase(t_, p, t_.rank())) post_step_groups(p, pi, g, per_group);  // relay only: no flow of its own
    marks_.emplace_back(-1, -1);
    chain_mark_ = -1;
  } else {
    // Nothing is posted between two steps of one run_steps call, so the
    // previous step's end mark is this step's start: one event per step
    // (the IPC self step's inter-step gap drops from 8.2 to ~4 us,
    // profiles/r2_mark_fence/).
    const int a = chain_mark_ >= 0 ? chain_mark_ : t_.mark();
    const size_t gi = static_cast<size_t>(g) * sched_.phases.size() + static_cast<size_t>(pi);
    if (replay && gi < graphs_.size() && graphs_[gi] >= 0)
      t_.graph_launch(graphs_[gi]);
    else
      post_step_groups(p, pi, g, per_group);
    const int b = t_.mark();
    marks_.emplace_back(a, b);
    chain_mark_ = b;
  }
  last_step_ = k;
  post_ms_.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - posted_from).count());
}

void StepDriver::sync() {
  t_.sync();
  std::string err = t_.async_error();
  if (!err.empty()) P2P_FATAL("transport reported an asynchronous error: " + err);
}

std::vector<double> StepDriver::step_ms() {
  std::vector<double> out;
  out.reserve(marks_.size());
  for (auto& m : marks_) out.push_back(m.first < 0 ? 0.0 : t_.elapsed_ms(m.first, m.second));
  return out;
}

void StepDriver::reset() {
  marks_.clear();
  post_ms_.clear();
  t_.clear_marks();
}

void StepDriver::clear() {
  // Every rank drains first: with a push transport a peer writes into this
  // rank's slots, and its writes are complete once this rank's receives are.
  sync();
  boot_.barrier();
  if (verify_) {
    t_.zero(bufs_.recv_base(), recv_bytes());
    t_.sync();
  }
  boot_.barrier();
}

void StepDriver::poison() {
  clear();
  const int me = t_.rank();
  if (!skip_armed_ && fault_applies("skip", me, -1)) {
    std::fprintf(stderr, "[p2p] injected fault: rank %d moves no payload in the steps after poison()\n", me);
    skip_armed_ = true;
    t_.set_discard(true);
  }
  if (!skip_some_armed_ && fault_applies("skip-some", me, -1)) {
    std::fprintf(stderr, "[p2p] injected fault: rank %d moves no payload in every other step after poison()\n", me);
    skip_some_armed_ = true;
  }
}

StepVerifyReport StepDriver::verify_steps(long first, long count) {
  if (skip_armed_ || skip_some_armed_) {
    t_.set_discard(false);
    skip_armed_ = skip_some_armed_ = false;
  }
  const int me = t_.rank();
  uint64_t timed = 0, bad = 0;
  std::map<int, std::pair<int, int>> last;  // slot -> (sender, message) of its last write in the range
  for (long k = first; k < first + count; ++k) {
    const int pi = static_cast<int>(k % phases());
    const Phase& p = sched_.phases[static_cast<size_t>(pi)];
    const RankOps& ops = p.ranks[static_cast<size_t>(me)];
    timed += static_cast<uint64_t>(msgs_) * ops.recv_from.size();
    for (int m = 0; m < msgs_; ++m)
      for (size_t i = 0; i < ops.recv_from.size(); ++i)
        last[slot_index(me, gen_of(k), pi, m, static_cast<int>(i))] = {ops.recv_from[i], m};
  }
  if (verify_) {
    // Every slot in one batched check (Transport::verify_many: one readback).
    std::vector<Transport::VerifyJob> jobs;
    jobs.reserve(last.size());
    for (const auto& kv : last) jobs.push_back({bufs_.recv_buf(kv.first), bytes_, msg_seed(kv.second.first, kv.second.second)});
    for (const auto& r : t_.verify_many(jobs)) bad += r.mismatches;
  }
  const uint64_t mine[4] = {bad, verify_ ? static_cast<uint64_t>(last.size()) : 0, timed, verify_ ? last.size() : 0};
  std::vector<uint64_t> all(4 * static_cast<size_t>(boot_.size()));
  boot_.allgather(mine, all.data(), sizeof(mine));
  StepVerifyReport r;
  for (int q = 0; q < boot_.size(); ++q) {
    r.mismatches += all[4 * static_cast<size_t>(q)];
    r.verified_msgs += all[4 * static_cast<size_t>(q) + 1];
    r.timed_msgs += all[4 * static_cast<size_t>(q) + 2];
    r.slots += all[4 * static_cast<size_t>(q) + 3];
  }
  return r;
}

uint64_t StepDriver::verify_last() {
  if (last_step_ < 0) return boot_.allreduce_sum_u64(0);
  return verify_steps(last_step_, 1).mismatches;
}

double StepDriver::bytes_sent_per_step(long k) const {
  const Phase& p = sched_.phases[static_cast<size_t>(k % static_cast<long>(sched_.phases.size()))];
  return static_cast<double>(p.ranks[static_cast<size_t>(t_.rank())].send_to.size()) * static_cast<double>(bytes_) * msgs_;
}

double StepDriver::job_bytes_per_step(long k) const {
  return static_cast<double>(flows_per_step(k)) * static_cast<double>(bytes_) * msgs_;
}

int StepDriver::flows_per_step(long k) const {
  return static_cast<int>(sched_.phases[static_cast<size_t>(k % static_cast<long>(sched_.phases.size()))].flows.size());
}

}  // namespace p2p
