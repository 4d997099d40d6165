// HIP error check for the GPU translation units (host builds never include
// it): a failing call goes through p2p::fatal, so abort hooks run (reference
// equivalent: CUDACHECK, p2p_matrix.cc:25-32, which exit()s one rank).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "common.hpp"

#define HIPCHECK(cmd)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (cmd);                                                                       \
    if (e_ != hipSuccess) P2P_FATAL(::p2p::strfmt("HIP error in %s: %s", #cmd, hipGetErrorString(e_))); \
  } while (0)

namespace p2p {

// Flags of the events that only timestamp the stream (Transport::mark).  A
// default event's record ends in a system-scope release: the L2 writes back
// every dirty line before the event reads "recorded", which after a bulk copy
// is ~10 us of idle GPU per mark (two marks per bench step: 10.5 us gaps
// between steps in the IPC trace, profiles/r2_mark_fence/).  Timing needs no
// fence -- the host never reads payload through these events, and stream
// order, not the event, orders the work -- so marks skip it
// (hipEventDisableSystemFence).  P2P_MARK_FENCE=system restores the default.
inline unsigned timing_event_flags() {
  static const unsigned flags = [] {
    const char* e = std::getenv("P2P_MARK_FENCE");
    return (e && std::strcmp(e, "system") == 0) ? unsigned{hipEventDefault} : unsigned{hipEventDisableSystemFence};
  }();
  return flags;
}

}  // namespace p2p
