// StreamGate: holds a HIP stream until the host releases it (Transport::
// gate_arm / gate_release, the pre-posted latency of runner.cpp).  The gate is
// the one-wave signal kernel of pingpong.hip waiting on a monotonic sequence
// number in host-pinned memory (system-scope acquire loads), bounded by a
// wall-clock deadline so a host that never releases cannot hang the GPU.
#pragma once

#include <hip/hip_runtime.h>

namespace p2p {

class StreamGate {
 public:
  StreamGate() = default;
  StreamGate(const StreamGate&) = delete;
  StreamGate& operator=(const StreamGate&) = delete;
  ~StreamGate();
  void arm(hipStream_t stream, double timeout_s);  // enqueue the gate kernel
  void release();                                  // let every armed gate pass
  bool timed_out();  // blocking: did a gate expire since the last call?

 private:
  unsigned long long* flag_ = nullptr;  // host-pinned, written by the host only
  unsigned int* status_ = nullptr;      // device: bit 0 = a gate expired
  unsigned long long seq_ = 0;
};

}  // namespace p2p
