// Transport::verify_many for the GPU transports: every buffer of the list
// in batched dev::launch_multi_verify launches with one readback and one
// stream sync, instead of reset + verify + finalize +
// copy + sync per buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.hpp"
#include "transport.hpp"

namespace p2p {

// P2P_VERIFY_BATCH=0: the one-buffer-at-a-time check (the A/B of round 3's
// post-timing verification against the batched one).
inline bool batch_verify_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("P2P_VERIFY_BATCH");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// Transport::verify_many through dev::BatchVerifier on `stream`; `sync` waits
// for the stream the transport's way (bounded, abort-aware).
template <class SyncFn>
inline std::vector<VerifyResult> batch_verify(dev::BatchVerifier& bv, const std::vector<Transport::VerifyJob>& jobs,
                                              hipStream_t stream, SyncFn&& sync) {
  std::vector<dev::VerifyJob> dj;
  dj.reserve(jobs.size());
  for (const auto& j : jobs) dj.push_back({j.p, j.bytes, j.seed});
  bv.reserve(static_cast<int>(dj.size()), sync);
  bv.enqueue(dj.data(), static_cast<int>(dj.size()), stream);
  sync();
  std::vector<VerifyResult> out(jobs.size());
  for (size_t i = 0; i < jobs.size(); ++i) {
    out[i].mismatches = bv.results()[i].mismatches;
    out[i].checksum = bv.results()[i].checksum;
    out[i].first_bad = bv.results()[i].first_bad;
  }
  return out;
}

}  // namespace p2p
