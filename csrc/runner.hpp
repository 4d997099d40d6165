// Measurement engine: executes schedules on a Transport and times them.
//
// Reference: the cell loops at /root/reference/p2p_matrix.cc:141-186 (uni) and
// :196-267 (bi).  Two timing methodologies:
//   * Timing::Wallclock — reference semantics: barrier, steady clock, one
//     group + host stream-sync per message, barrier, clock; no warmup unless
//     asked, so first-use connection setup lands inside the cell, exactly like
//     the reference (which also used the non-monotonic system_clock; we use
//     steady_clock).
//   * Timing::Events (default) — barrier, `warmup` untimed iterations (which
//     also establish the lazy RCCL p2p connections), barrier, then all `iters`
//     groups are posted back to back on the stream with a hipEvent between
//     iterations, one sync at the end; per-rank durations are all-gathered and
//     each flow is charged the max of its two endpoints.  The per-iteration
//     event deltas give the per-message time distribution (p50/p99).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "schedule.hpp"
#include "stats.hpp"
#include "transport.hpp"

namespace p2p {

class Bootstrap;

enum class Timing { Events, Wallclock };
const char* timing_name(Timing t);
Timing parse_timing(const std::string& s);

struct RunConfig {
  size_t bytes = 32u << 20;  // reference: msg_size = 32 MiB (p2p_matrix.cc:124)
  int iters = 128;           // reference: count = 128 (p2p_matrix.cc:132)
  int warmup = 8;            // reference: none (p2p_matrix.cc:153-172)
  Timing timing = Timing::Events;
  // Random-filled sends, every received buffer checked on the device after
  // the timed loop (never inside it).  On by default: the
  // reference's zeroed buffers are never read back (p2p_matrix.cc:129-130),
  // so a transfer that silently drops bytes would print as a fast cell.
  // p2p_matrix --no-verify opts out.
  bool verify = true;
  bool samples = true;       // record an event per iteration for the distribution
  uint64_t salt = 0;
  // With verify: receive generations.  Iteration i (warmup and timed alike)
  // sends from send region i mod G, filled with that generation's PRNG stream,
  // into receive slots g * P + 0..P-1 (P = the phase's most receive slots on
  // any rank), so up to G timed deliveries per slot are checked, not only the
  // last one (run_phase caps G by the buffers; verify_generations() sizes it).
  int gens = 1;
  // With verify: a warmup that does not verify makes every rank post smaller
  // ops (rechunk_until_warmup_verifies) -- the second line of defence against
  // RCCL's half-delivery.  P2P_RECHUNK=0 turns it off, so the timed check
  // reports the loss instead.
  bool rechunk = true;
};

struct FlowResult {
  Flow flow;
  double seconds = 0;     // per message
  double gbps = 0;        // reference unit: bytes*8/s/1e9
  double gbs = 0;         // GB/s (1e9 B/s)
  Summary iter_us;        // per-iteration time seen by the receiver, microseconds
  bool verified = false;
  uint64_t mismatches = 0;
  uint64_t checksum = 0;
};

struct PhaseResult {
  size_t index = 0;
  std::string label;
  int row = -1, col = -1;
  bool idle = false;
  size_t bytes = 0;
  int iters = 0;
  double seconds_per_iter = 0;  // phase time per iteration (max over participants)
  double wall_seconds = 0;      // host barrier-to-barrier time of the timed region
  double bytes_per_iter = 0;    // all flows of the phase
  double agg_gbs = 0;           // bytes_per_iter / seconds_per_iter
  std::vector<double> rank_seconds;  // each rank's own timed duration (0 = not participating)
  std::vector<double> host_begin;    // each rank's steady-clock time at the start / end of the
  std::vector<double> host_end;      // timed region (seconds; one clock per host) -> --trace
  std::vector<FlowResult> flows;
  uint64_t total_mismatches = 0;
  // Verification coverage (all ranks): timed deliveries, and those checked
  // (one per receive slot and generation; G >= iters checks every one).
  int generations = 1;
  uint64_t timed_msgs = 0;
  uint64_t verified_msgs = 0;
  // Op size the phase's messages were posted as (largest over this rank's
  // peers; 0 = one op per message) and what the warmup check saw: wrong words
  // in the first warmup and the op sizes it had to fall back to.
  size_t op_bytes = 0;
  uint64_t warmup_mismatches = 0;
  std::vector<size_t> rechunked_to;
  // Wrong words the warmup still had after the last re-chunking (0: the
  // smaller ops fixed it).  Non-zero: the loss does not follow the op size.
  uint64_t warmup_residual = 0;
};

// Send buffer + receive slots for one rank.  The slots are carved from one
// receive arena (one allocation, one IPC export), `stride()` bytes apart, so
// a step driver can hold thousands of them -- one per message of every timed
// step -- within the 288 GB of HBM3E.
class Buffers {
 public:
  // `slot_bytes` per receive slot; the send buffer holds `send_bytes`
  // (default: one message).
  Buffers(Transport& t, size_t slot_bytes, int recv_slots, size_t send_bytes = 0);
  ~Buffers();
  Buffers(const Buffers&) = delete;
  Buffers& operator=(const Buffers&) = delete;
  void* send_buf() const { return send_; }
  void* send_at(size_t offset) const { return static_cast<char*>(send_) + offset; }
  void* recv_buf(int slot) const;
  void* recv_base() const { return recv_; }
  size_t capacity() const { return cap_; }          // bytes per receive slot
  size_t send_capacity() const { return send_cap_; }
  size_t stride() const { return stride_; }
  int slots() const { return nslots_; }

 private:
  Transport& t_;
  size_t cap_;
  size_t send_cap_;
  size_t stride_;
  int nslots_;
  void* send_ = nullptr;
  void* recv_ = nullptr;
};

// Receive slot on `peer` that holds messages from `me` in `phase` (position
// of `me` in the peer's recv list).
int remote_slot(const Phase& phase, int me, int peer);
// For each entry of `me`'s send list, the receive index on that peer: the
// k-th send to a peer meets the k-th receive from `me` there (a phase may
// hold several flows between the same two ranks, e.g. ring-bi with 2 ranks).
std::vector<int> remote_slots(const Phase& phase, int me);

// Posts one iteration (one group) of `phase` for this rank, generation `gen`:
// the payload comes from send region gen (slot_stride(bytes) apart) and lands
// in receive slots gen * phase.max_recv_slots() + i.
void post_phase_iteration(Transport& t, const Phase& phase, size_t bytes, Buffers& bufs, int gen = 0);

// Receive generations for verified runs of messages up to `max_bytes` with
// `slots` receive slots per iteration and up to `iters` iterations: as many as
// P2P_VERIFY_BUDGET bytes of send regions + receive slots allow (default a
// quarter of free device memory, at most 32 GiB; 256 MiB where the transport
// cannot tell), agreed by every rank (collective).
int verify_generations(Transport& t, Bootstrap& boot, size_t max_bytes, int slots, int iters);
// Collective: a quarter of this rank's GPU's free memory (at most `cap`;
// `fallback` where the transport cannot tell), divided between the ranks that
// share the GPU (Transport::device_key).  Every rank drains its stream and
// meets a barrier before any reads the free memory, and another before any
// allocates (ranks sharing a GPU read it while peers still freed).
size_t shared_free_budget(Transport& t, Bootstrap& boot, size_t fallback, size_t cap);

// Receive-slot / send-region stride for messages of `bytes` (4 KiB aligned).
size_t slot_stride_bytes(size_t bytes);

// PRNG stream of generation `gen` of a run's payload from `src`.
uint64_t generation_seed(int src, size_t bytes, uint64_t salt, int gen);

// Runs one phase on every rank (collective over `boot`).
PhaseResult run_phase(Transport& t, Bootstrap& boot, const Phase& phase, size_t phase_index, const RunConfig& cfg,
                      Buffers& bufs);

using PhaseCallback = std::function<void(const PhaseResult&)>;

// Runs every phase of a schedule (collective).  `on_phase` fires on every rank
// after each phase, so reports can stream like the reference's fflush'd rows.
std::vector<PhaseResult> run_schedule(Transport& t, Bootstrap& boot, const Schedule& s, const RunConfig& cfg,
                                      Buffers& bufs, const PhaseCallback& on_phase = nullptr);

// Establish every lazy connection a schedule will use (one tiny untimed
// iteration per phase), so no timed cell pays connection setup.
void warm_connections(Transport& t, Bootstrap& boot, const Schedule& s, Buffers& bufs, size_t bytes = 4096);

// ---- latency: ping-pong between disjoint pairs, concurrently per round ----
struct LatencyResult {
  int a = -1, b = -1;   // a < b; a == b for the self path
  size_t bytes = 0;
  Summary one_way_us;   // half round trip, microseconds
  // host: posted ping-pong through the transport; preposted: the same, posted
  // in batches behind a stream gate (GPU timeline only); device: ping-pong kernel
  std::string method = "host";
};

// Ping-pong over round-robin rounds (every unordered pair once; each round's
// pairs run concurrently on disjoint xGMI links).  n == 1 measures the self
// path (one grouped self send/recv per sample).
//
// preposted == 0: every exchange is posted as the previous one runs, so a
// sample is max(operation time on the GPU, host posting time).  preposted =
// B > 0 (transports with Transport::gate_arm): exchanges are posted B at a
// time behind a stream gate on every rank and released together, so they run
// back to back on the GPU and a sample is the operation's own GPU-timeline
// time (the first exchange of each batch, which also absorbs the ranks'
// release skew, is not sampled).  Transports without a gate fall back to 0.
std::vector<LatencyResult> run_latency(Transport& t, Bootstrap& boot, size_t bytes, int iters, int warmup,
                                       Buffers& bufs, int preposted = 0);

// Device-initiated ping-pong (Transport::device_pingpong; the IPC transport):
// one wave per GPU bounces a message through the peer's memory with no host
// in the loop, timed on the device clock.  Same round structure as
// run_latency; payloads are rounded up to 16 bytes (at most 64 KiB).
std::vector<LatencyResult> run_device_latency(Transport& t, Bootstrap& boot, size_t bytes, int iters, int warmup);

// ---- ring token chain: pipeline-parallel hop latency ----
// Rank 0 sends a small message to rank 1; every rank forwards it to its
// successor only after it has arrived from its predecessor (0 -> 1 -> ... ->
// N-1 -> 0), `laps` times.  Unlike the concurrent ring phase (every rank
// sends every iteration, which measures pipelined issue rate), each hop here
// depends on the previous one, as a pipeline stage waits for its input.
// Rank 0 times each lap (hipEvents / steady clock); hop = lap / N.
struct RingLatencyResult {
  int nranks = 0;
  size_t bytes = 0;
  int laps = 0;
  Summary hop_us;  // lap time / nranks
  Summary lap_us;
  std::string method = "host";  // host: grouped send/recv through the transport; device: ring token kernel
};

// Host-posted chain: every lap is two groups per rank (rank 0: send, then
// receive; the others: receive, then send), posted without host syncs, so on
// a GPU transport the stream order makes each send wait for the preceding
// receive.  Collective; n == 1 is the self send/recv.  Not meaningful on the
// IPC pull engines (a pull does not wait for the sender).
RingLatencyResult run_ring_latency(Transport& t, Bootstrap& boot, size_t bytes, int laps, int warmup, Buffers& bufs);
// Device chain (Transport::device_ring_token, IPC): one wave per GPU spins
// on its inbox and writes into its successor's; no host or runtime in the loop.
RingLatencyResult run_device_ring_latency(Transport& t, Bootstrap& boot, size_t bytes, int laps, int warmup);

// ---- transport fuzz (tests) ----
// `rounds` groups of random messages (src, dst, size <= max_bytes; self
// messages and repeated pairs included) drawn from `seed`, identical on every
// rank; each rank posts its sends and receives in plan order inside one group,
// then checks every received message against the sender's PRNG stream.
// Collective; returns this rank's mismatching words.  Transports that only
// move registered buffer sets (IPC) are not supported.
uint64_t fuzz_transport(Transport& t, Bootstrap& boot, int rounds, uint64_t seed, size_t max_bytes);

// ---- step driver (used by bench.py): one phase per step, no host syncs ----
// Step k posts `msgs` messages per flow of phase (k mod phases) with a
// timestamp around them; nothing blocks until sync().  Per-step durations are
// read after sync().
//
// Payload layout, so that verification covers the timed work:
//   * the send buffer holds `msgs` regions; message m of every step is sent
//     from region m, filled with its own PRNG stream (msg_seed(src, m));
//   * every message of every step lands in its own receive slot: generation
//     g = (k / phases) mod depth, then phase, message and receive index.
//     With depth >= the laps of the timed steps, no timed delivery is
//     overwritten, and verify_steps() checks each one against the stream of
//     the region it was sent from;
//   * poison() zeroes every slot after the warmup, so a slot passes only if
//     a timed step wrote it.
struct StepOptions {
  bool batch = false;  // all msgs of a step in ONE group (one launch) instead of one group per message
  bool graph = false;  // capture each (phase, generation) step into a hipGraph (transports that support it)
  int depth = 1;       // receive generations requested (capped by recv_budget)
  size_t recv_budget = 0;  // bytes of receive slots this rank may hold (0: a quarter of free memory)
  // batch: messages per group (0: the whole step).  group_msgs applies to every
  // step, first_group_msgs to the first step of a run_steps call only (the one
  // the GPU waits for while the host posts it).  Every group holds whole
  // messages, and every rank splits alike.  Env P2P_STEP_GROUP_MSGS /
  // P2P_STEP_FIRST_GROUP_MSGS set them where the caller did not.
  int group_msgs = 0;
  int first_group_msgs = 0;
};

struct StepVerifyReport {
  uint64_t mismatches = 0;     // 32-bit words that differ, all ranks
  uint64_t verified_msgs = 0;  // timed deliveries checked (the last one into each slot), all ranks
  uint64_t timed_msgs = 0;     // timed deliveries in the range, all ranks
  uint64_t slots = 0;          // receive slots checked, all ranks
};

class StepDriver {
 public:
  StepDriver(Transport& t, Bootstrap& boot, Schedule sched, size_t bytes, int msgs, bool verify, uint64_t salt = 0,
             StepOptions opt = StepOptions());
  ~StepDriver();
  void connect();               // warm every phase once (collective, blocking)
  void step(long k);            // enqueue step k
  // Enqueue steps [first, first + count): consecutive steps share their
  // boundary mark (step k's end is step k + 1's start), so a step costs one
  // timestamp event instead of two (each is a barrier packet on the queue).
  void run_steps(long first, long count);
  void sync();                  // wait for everything posted
  std::vector<double> step_ms();       // this rank's per-step durations since the last reset
  // Host time each of those steps took to post (ms, steady clock): a step the
  // GPU waits for is one whose posting is slower than the step before it ran.
  const std::vector<double>& post_ms() const { return post_ms_; }
  void reset();                 // forget recorded steps
  // Collective, blocking, untimed: zero every receive slot of every rank once
  // every rank has drained.
  void clear();
  // clear(), then arm P2P_INJECT_FAULT=skip (no payload) or skip-some (no
  // payload in every other step) for the steps that follow.
  void poison();
  // Collective: record the step graphs again (opt.graph), after the
  // transport's op sizes changed (Transport::set_chunk_cap); a graph replays
  // the ops it recorded.
  void recapture();
  int recaptures() const { return recaptures_; }
  // connect() calls that changed the transport's per-peer op limits.
  int limit_changes() const { return limit_changes_; }
  bool graphs() const { return opt_.graph; }
  // Collective: checks every receive slot written by steps [first, first +
  // count) against the payload of the message that wrote it last.
  StepVerifyReport verify_steps(long first, long count);
  uint64_t verify_last();       // mismatches in the receive slots of the last step (collective)
  double bytes_sent_per_step(long k) const;  // by THIS rank
  double job_bytes_per_step(long k) const;   // by all ranks
  int flows_per_step(long k) const;          // directed flows of step k's phase
  const Schedule& schedule() const { return sched_; }
  int phases() const { return static_cast<int>(sched_.phases.size()); }
  int depth() const { return depth_; }
  int msgs() const { return msgs_; }
  size_t recv_bytes() const { return bufs_.stride() * static_cast<size_t>(bufs_.slots()); }

  // Receive slot on `rank` of message `msg` from its `i`-th sender in
  // `phase`, generation `gen` (every rank computes every rank's layout).
  int slot_index(int rank, int gen, int phase, int msg, int i) const;
  uint64_t msg_seed(int src, int msg) const;
  size_t region_offset(int msg) const;  // where message `msg` starts in the send buffer

 private:
  Transport& t_;
  Bootstrap& boot_;
  Schedule sched_;
  size_t bytes_;
  int msgs_;
  bool verify_;
  uint64_t salt_;
  StepOptions opt_;
  std::vector<std::vector<int>> phase_base_;  // [rank][phase]: first slot of the phase in generation 0
  std::vector<int> gen_slots_;                // [rank]: slots per generation
  int depth_;                                 // receive generations (the same on every rank)
  Buffers bufs_;
  std::vector<std::pair<int, int>> marks_;
  std::vector<double> post_ms_;  // host posting time per recorded step
  std::vector<int> graphs_;  // per (generation, phase), when opt_.graph
  long last_step_ = -1;
  bool skip_armed_ = false;
  bool skip_some_armed_ = false;
  int recaptures_ = 0;
  int limit_changes_ = 0;
  int chain_mark_ = -1;  // run_steps: the previous step's end mark, the next one's start
  int per_group_ = 0;    // post_step_ops: messages per group of the step being posted (0: all)

  void step_impl(long k, bool chain);
  void post_step_groups(const Phase& p, int pi, int gen, int per_group);
  void capture_graphs();

  void post_step_ops(const Phase& p, int pi, int gen);
  int gen_of(long k) const { return static_cast<int>((k / phases()) % depth_); }
};

}  // namespace p2p
