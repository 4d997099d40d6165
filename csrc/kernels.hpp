// Host-side launch API for the gfx950 buffer kernels (kernels.hip).
//
// The reference has no device code at all: its buffers are zeroed with
// cudaMemset (p2p_matrix.cc:129-130) and never read back.
// These kernels replace that with verifiable random payloads:
//   fill    — counter-based PRNG, one 16-byte global_store_dwordx4 per lane
//   verify  — regenerates the stream and compares; two stagings, the A/B
//             SURVEY.md §7.5 item 6 asks for:
//               * LDS (Lds8, the default): non-temporal global_load_lds_dwordx4
//                           (LDS-DMA, 1 KiB per wave instruction) into a
//                           per-wave LDS slot of 8 KiB, then ds_read_b128 —
//                           the LDS-staged form the north star asks for;
//                           6.44 / 6.64 TB/s at 1 / 4 GiB, within 1-2% of
//                           register staging
//               * stride:   register staging, 4 x global_load_dwordx4 in flight
//                           per lane, grid capped at 16 workgroups per CU so the
//                           reduction epilogue is amortised over 64 KiB+
//             (round 5 removed the variants that lost: profiles/r1_tuned/,
//             r4_verify_span/)
//   reduce  — fused epilogue of verify: wave64 __shfl_xor tree -> LDS across
//             the 4 waves -> one atomic per block into one of kVerifyShards
//             64-byte counters (no single hot address), then a one-wave
//             finalize kernel folds the shards
//   copy    — multi-source copy for the IPC transport (remote loads over xGMI)
//
// Measured on MI355X (profiles/, scripts/fill_probe.hip): streaming at one
// 16 B access per lane with one block per 4 KiB (a "full grid", up to 2^20
// blocks, then grid-stride) reaches 6.9-7.0 TB/s for stores and 6.7-6.8 TB/s
// for loads, against 5.1-5.6 / 6.3 TB/s for grid-stride loops over a grid
// capped at 4-32 blocks per CU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>

#include "prng.hpp"

namespace p2p {
namespace dev {

// One 64-byte shard of the device-side accumulator; `first_bad` starts at ~0
// (launch_verify_reset).  Allocate verify_accum_bytes() for the whole array;
// after launch_verify the totals are in shard 0.
struct alignas(64) VerifyAccum {
  unsigned long long mismatches;
  unsigned long long checksum;
  unsigned long long first_bad;
};
constexpr int kVerifyShards = 64;
constexpr size_t verify_accum_bytes() { return sizeof(VerifyAccum) * kVerifyShards; }

// Verify staging (app.hpp parse_verify_impl maps the CLI / Python names).
enum class VerifyImpl : int { Auto = 0, Lds8 = 1, Stride = 2 };
// One fill kernel, the full grid; the enum stays so callers name it.
enum class FillImpl : int { Auto = 0, Grid = 1 };

// Geometry chosen for a launch (exposed for tests / profiling scripts).
struct LaunchGeom {
  unsigned grid = 0;
  unsigned block = 256;
  size_t lds_bytes = 0;
};

LaunchGeom fill_geometry(size_t bytes, FillImpl impl = FillImpl::Auto);
// max_grid > 0 caps the workgroup count (the kernels grid-stride beyond it);
// 0 = the tuned default of the variant.
LaunchGeom verify_geometry(size_t bytes, VerifyImpl impl, unsigned max_grid = 0);

void launch_fill(void* p, size_t bytes, uint64_t seed, hipStream_t stream, FillImpl impl = FillImpl::Auto);
void launch_verify_reset(VerifyAccum* acc, hipStream_t stream);
// check_prng=false only sums the words (checksum of an arbitrary buffer).
// Leaves the totals in acc[0] (stream-ordered).
void launch_verify(const void* p, size_t bytes, uint64_t seed, VerifyAccum* acc, VerifyImpl impl, bool check_prng,
                   hipStream_t stream, unsigned max_grid = 0);

// ---- batched verify (the post-timing check of many receive slots) ----
// Job i's totals land in out[i] (device memory, njobs entries; nothing needs
// resetting).  Batches of kMaxVerifyJobs, three launches each (reset, the
// LDS-DMA verify over all the batch's buffers, finalize); `scratch` holds
// multi_verify_scratch_bytes() and is reused by every batch (stream order).
struct VerifyJob {
  const void* p;
  size_t bytes;
  uint64_t seed;
};
constexpr int kMaxVerifyJobs = 32;
constexpr size_t multi_verify_scratch_bytes() { return verify_accum_bytes() * kMaxVerifyJobs; }
void launch_multi_verify(const VerifyJob* jobs, int njobs, VerifyAccum* scratch, VerifyAccum* out, hipStream_t stream);

// The device scratch, device results and pinned host results of
// launch_multi_verify for one stream's user (a transport), grown on demand.
// reserve() makes room for njobs results: should the arrays grow, it calls
// `drain` first -- the stream may still read the old ones -- which is the
// caller's own wait for its stream (the transports' is bounded and
// abort-aware).  enqueue() then puts the batched verify and ONE
// readback of every job's totals on `stream`; results() is valid once the
// caller has synchronised the stream.
class BatchVerifier {
 public:
  BatchVerifier() = default;
  BatchVerifier(const BatchVerifier&) = delete;
  BatchVerifier& operator=(const BatchVerifier&) = delete;
  ~BatchVerifier();
  void reserve(int njobs, const std::function<void()>& drain);
  void enqueue(const VerifyJob* jobs, int njobs, hipStream_t stream);  // after reserve(njobs)
  const VerifyAccum* results() const { return host_; }

 private:
  VerifyAccum* scratch_ = nullptr;
  VerifyAccum* out_ = nullptr;
  VerifyAccum* host_ = nullptr;
  int cap_ = 0;
};

// Device attributes cached per device (CU count drives grid sizing).
int cu_count();

// ---- multi-source copy (IPC transport data plane) ----
// One launch moves every receive of a group: op i copies ops[i].bytes from
// src (typically a peer GPU's buffer mapped through hipIpcOpenMemHandle, so
// the loads travel over xGMI) to dst.  Full grid: one 16 B load + store per
// lane, one 4 KiB block per workgroup, workgroups split across ops by size.
// coherent = the op crosses GPUs (a hipIpc-mapped peer buffer on either side):
// its loads and stores carry system-scope cache bits (sc0 sc1), so a reader
// never sees a line its L2 kept from an earlier run of the peer's buffer and
// the payload is written through to the owner's HBM before the kernel ends.
// Local ops (the self path) keep plain accesses.
struct CopyOp {
  const void* src;
  void* dst;
  size_t bytes;
  bool coherent = false;
};
constexpr int kMaxCopyOps = 32;  // ops per launch (one bit each in CopyArgs::coherent)
void launch_multi_copy(const CopyOp* ops, int nops, hipStream_t stream, int max_blocks = 0);

// ---- device-initiated ping-pong (pingpong.hip) ----
// One wave per role.  The leader writes message i (payload words = base+i+1,
// then the flag) into the peer's inbox and spins on its own inbox for the
// reply; the follower mirrors it.  stamps[0..iters] (leader only) are
// s_memrealtime ticks; status[0] bit 0 = a spin hit the deadline, status[1] =
// payloads that arrived without their sequence number.
struct PingRole {
  unsigned long long* out_flag;        // peer's inbox flag
  unsigned char* out_payload;          // peer's inbox payload
  const unsigned long long* in_flag;   // own inbox flag (written by the peer)
  const unsigned char* in_payload;     // own inbox payload
  unsigned long long bytes;            // payload bytes, multiple of 16, >= 16
  unsigned long long base;             // sequence base of what this wave writes (iteration i: base + i + 1)
  unsigned long long in_base;          // sequence base of what it waits for (== base for a ping-pong pair;
                                       // a ring token chain reads its predecessor's count, writes its own)
  int iters;
  int leader;
  unsigned long long* stamps;          // leader: iters + 1 entries
  unsigned int* status;                // 2 words, zeroed by the caller
  unsigned long long timeout_ticks;    // per kernel, in s_memrealtime ticks
};
// b == nullptr: one wave (cross-process partner).  Otherwise both roles run
// as two waves of one workgroup (self ping-pong on one GPU).
void launch_pingpong(const PingRole& a, const PingRole* b, hipStream_t stream);

// ---- stream-ordered flag signalling (pingpong.hip; IPC push engine) ----
// One wave: optionally a system-scope release fence (so the writes of earlier
// kernels in the stream, e.g. a copy into a peer's memory, reach their
// memory first), then every post stores its value to its flag (system scope),
// then the wave spins until every wait flag is >= its value (system-scope
// acquire), each spin bounded by timeout_ticks; a deadline sets bit 0 of
// *status (host-visible memory) and ends the kernel.
constexpr int kMaxSignals = 16;
struct SignalArgs {
  unsigned long long* post_flag[kMaxSignals];
  unsigned long long post_value[kMaxSignals];
  const unsigned long long* wait_flag[kMaxSignals];
  unsigned long long wait_value[kMaxSignals];
  int nposts;
  int nwaits;
  int release_first;
  unsigned int* status;
  unsigned long long timeout_ticks;
};
void launch_signal(const SignalArgs& args, hipStream_t stream);

}  // namespace dev
}  // namespace p2p
