// Host-side launch API for the gfx950 buffer kernels (kernels.hip).
//
// The reference has no device code at all: its buffers are zeroed with
// cudaMemset (p2p_matrix.cc:129-130) and never read back.
// These kernels replace that with verifiable random payloads:
//   fill    — counter-based PRNG, one 16-byte global_store_dwordx4 per lane
//   verify  — regenerates the stream and compares; two staging variants:
//               * register: global_load_dwordx4, UNROLL loads in flight/lane
//               * LDS:      global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave
//                           instruction) into a double-buffered per-wave LDS
//                           ring, then ds_read_b128 — the LDS-staged form the
//                           north star asks for, A/B-tested against register
//                           staging
//   reduce  — fused epilogue of verify: wave64 __shfl_xor tree -> LDS across
//             the 4 waves -> one atomic per block (mismatches, checksum,
//             first bad offset)
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "prng.hpp"

namespace p2p {
namespace dev {

// Device-side accumulator; `first_bad` must start at ~0 (verify_reset does it).
struct VerifyAccum {
  unsigned long long mismatches;
  unsigned long long checksum;
  unsigned long long first_bad;
};

enum class VerifyImpl : int { Auto = 0, Register = 1, Lds = 2, Register8 = 3 };
enum class FillImpl : int { Auto = 0, Plain = 1, Nontemporal = 2 };

// Geometry chosen for a launch (exposed for tests / profiling scripts).
struct LaunchGeom {
  unsigned grid = 0;
  unsigned block = 256;
  size_t lds_bytes = 0;
};

LaunchGeom fill_geometry(size_t bytes);
LaunchGeom verify_geometry(size_t bytes, VerifyImpl impl);

void launch_fill(void* p, size_t bytes, uint64_t seed, hipStream_t stream, FillImpl impl = FillImpl::Auto);
void launch_verify_reset(VerifyAccum* acc, hipStream_t stream);
// check_prng=false only sums the words (checksum of an arbitrary buffer).
void launch_verify(const void* p, size_t bytes, uint64_t seed, VerifyAccum* acc, VerifyImpl impl, bool check_prng,
                   hipStream_t stream);

// Device attributes cached per device (CU count drives grid sizing).
int cu_count();

// ---- multi-source copy (IPC transport data plane) ----
// One launch moves every receive of a group: op i copies ops[i].bytes from
// src (typically a peer GPU's buffer mapped through hipIpcOpenMemHandle, so
// the loads travel over xGMI) to dst.  Workgroups are split across ops in
// proportion to their size; each lane keeps UNROLL x 16 B loads in flight to
// cover the remote-read latency.
struct CopyOp {
  const void* src;
  void* dst;
  size_t bytes;
};
constexpr int kMaxCopyOps = 16;
void launch_multi_copy(const CopyOp* ops, int nops, hipStream_t stream, int max_blocks = 0);

}  // namespace dev
}  // namespace p2p
