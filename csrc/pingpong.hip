// Device-initiated ping-pong, ring token chain and stream-ordered flag
// signalling over hipIpc-mapped memory (IPC transport).
//
// The reference has no latency measurement at all; the host-
// posted ping-pong in runner.cpp (run_latency) measures what an application
// sees through RCCL: launch, proxy and protocol overhead included.  This
// kernel measures the fabric itself: one wave on each GPU bounces a message
// through the peer's memory with no host or runtime in the loop:
//
//   leader:   write payload (seq) into the peer's inbox -> release flag=seq
//             -> spin on its own inbox flag until >= seq -> timestamp
//   follower: spin until its inbox flag >= seq -> check payload -> reply
//
// The same kernel runs the ring token chain (pipeline-parallel hop latency,
// runner.cpp run_ring_latency): every rank's `out` is its successor's inbox,
// its `in` is the slot its predecessor writes; rank 0 leads (writes, then
// waits for the token to come round), every other rank follows (waits, then
// forwards), so one leader iteration is one lap of N dependent hops.
//
// Stores to the peer travel over xGMI (remote writes, the direction xGMI and
// RCCL's LL protocols favour); the spin is on local memory.  Flags are
// monotonic sequence numbers, so consecutive calls need no reset.  Every spin
// is bounded by a wall-clock deadline (s_memrealtime, constant 100 MHz on
// CDNA), so a missing partner ends the kernel with status bit 0 set instead
// of hanging the GPU.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace p2p {
namespace dev {
namespace {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64 now_ticks() { return static_cast<u64>(wall_clock64()); }

__device__ __forceinline__ void ping_send(const PingRole& r, u64 seq, int lane) {
  const u64x2 v = {seq, seq};
  for (u64 off = static_cast<u64>(lane) * 16; off < r.bytes; off += 64 * 16)
    *reinterpret_cast<u64x2*>(r.out_payload + off) = v;
  // All of this wave's payload stores are complete (vmcnt is per wave) and
  // written back before the flag becomes visible to the peer.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) __hip_atomic_store(r.out_flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wave-uniform: every lane loads the same flag and reads the same scalar clock.
__device__ __forceinline__ bool ping_wait(const PingRole& r, u64 seq, u64 deadline) {
  while (__hip_atomic_load(r.in_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq)
    if (now_ticks() > deadline) return false;
  return true;
}

// After the acquire: first and last 16 B of the payload must carry seq (the
// writer's sequence number for this message).
__device__ __forceinline__ void ping_check(const PingRole& r, u64 seq, int lane) {
  if (lane < 2) {
    const u64 off = lane == 0 ? 0 : r.bytes - 16;
    const u64x2 v = *reinterpret_cast<const u64x2*>(r.in_payload + off);
    if (v.x != seq || v.y != seq) atomicAdd(r.status + 1, 1u);
  }
}

__global__ __launch_bounds__(128) void pingpong_kernel(PingRole a, PingRole b) {
  const int lane = threadIdx.x & 63;
  const PingRole& r = (threadIdx.x >> 6) == 0 ? a : b;
  const u64 deadline = now_ticks() + r.timeout_ticks;
  if (r.leader) {
    if (lane == 0) r.stamps[0] = now_ticks();
    for (int i = 0; i < r.iters; ++i) {
      const u64 seq = r.base + static_cast<u64>(i) + 1;
      const u64 want = r.in_base + static_cast<u64>(i) + 1;
      ping_send(r, seq, lane);
      if (!ping_wait(r, want, deadline)) {
        if (lane == 0) atomicOr(r.status, 1u);
        return;
      }
      ping_check(r, want, lane);
      if (lane == 0) r.stamps[i + 1] = now_ticks();
    }
  } else {
    for (int i = 0; i < r.iters; ++i) {
      const u64 seq = r.base + static_cast<u64>(i) + 1;
      const u64 want = r.in_base + static_cast<u64>(i) + 1;
      if (!ping_wait(r, want, deadline)) {
        if (lane == 0) atomicOr(r.status, 1u);
        return;
      }
      ping_check(r, want, lane);
      ping_send(r, seq, lane);
    }
  }
}

__global__ __launch_bounds__(64) void signal_kernel(SignalArgs a) {
  const int lane = threadIdx.x;
  if (a.release_first) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane < a.nposts) __hip_atomic_store(a.post_flag[lane], a.post_value[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const u64 deadline = now_ticks() + a.timeout_ticks;
  // Lane i watches wait i; the wave leaves when every lane's flag arrived.
  bool ok = true;
  if (lane < a.nwaits) {
    while (__hip_atomic_load(a.wait_flag[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.wait_value[lane]) {
      if (now_ticks() > deadline) {
        ok = false;
        break;
      }
    }
  }
  if (!ok) __hip_atomic_fetch_or(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

void launch_signal(const SignalArgs& args, hipStream_t stream) {
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, stream, args);
}

void launch_pingpong(const PingRole& a, const PingRole* b, hipStream_t stream) {
  PingRole second = b ? *b : a;
  hipLaunchKernelGGL(pingpong_kernel, dim3(1), dim3(b ? 128 : 64), 0, stream, a, second);
}

}  // namespace dev
}  // namespace p2p
