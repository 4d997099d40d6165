#include "stream_gate.hpp"

#include "common.hpp"
#include "hip_check.hpp"
#include "kernels.hpp"

namespace p2p {

StreamGate::~StreamGate() {
  if (flag_) (void)hipHostFree(flag_);
  if (status_) (void)hipFree(status_);
}

void StreamGate::arm(hipStream_t stream, double timeout_s) {
  if (!flag_) {
    // Fine-grained (coherent) host memory: the gate's system-scope loads see the
    // host's store without any cache maintenance.
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&flag_), 64, hipHostMallocCoherent));
    __atomic_store_n(flag_, 0ull, __ATOMIC_RELEASE);
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&status_), sizeof(unsigned int)));
    HIPCHECK(hipMemsetAsync(status_, 0, sizeof(unsigned int), stream));
  }
  dev::SignalArgs a{};
  a.nposts = 0;
  a.nwaits = 1;
  a.wait_flag[0] = flag_;
  a.wait_value[0] = ++seq_;
  a.release_first = 0;
  a.status = status_;
  a.timeout_ticks = static_cast<unsigned long long>(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  dev::launch_signal(a, stream);
}

void StreamGate::release() {
  if (flag_) __atomic_store_n(flag_, seq_, __ATOMIC_RELEASE);
}

bool StreamGate::timed_out() {
  if (!status_) return false;
  unsigned int st = 0;
  HIPCHECK(hipMemcpy(&st, status_, sizeof(st), hipMemcpyDeviceToHost));
  if (st & 1u) HIPCHECK(hipMemset(status_, 0, sizeof(st)));  // report each expiry once
  return (st & 1u) != 0;
}

}  // namespace p2p
