// Multi-path routing over a fully connected xGMI mesh (pure host code).
//
// MI355X GPUs of one node are connected point-to-point: every GPU has a
// direct xGMI link to each of the other 7.  A message between two GPUs that
// travels only on their direct link uses 1/7 of either endpoint's links.  The
// reference measures exactly that case: its matrix runs one ordered pair at a
// time while every other GPU idles (p2p_matrix.cc:141-186), and NCCL/RCCL
// send/recv moves a message on the direct path only.
//
// plan_routes() splits each message of a group into stripes: one on the
// direct link and one per two-hop path s -> k -> d through a rank k that is
// not an endpoint.  The IPC transport's relay engine then moves each two-hop
// stripe with one kernel on k that loads from s's send buffer and stores into
// d's receive slot (both hipIpc-mapped), so the bytes cross s->k and k->d and
// never touch k's HBM.
//
// Split rule (identical on every rank; inputs are the group's global flows):
//   * a two-hop path is used only if neither of its links carries a direct
//     flow of the group (relaying over a busy link only adds traffic, e.g.
//     in all-pairs mode every link is busy and nothing is relayed);
//   * C(a,b) = number of two-hop segments that would cross directed link a->b;
//     a path's share is 1 for the direct link and relay_weight / max(C(s,k),
//     C(k,d)) for a relay, and bytes are split in proportion to the shares,
//     in `align`-byte units, the direct stripe taking the remainder (at the
//     end of the message, so that every stripe starts aligned).
// A single pair on N GPUs thus gets N-1 equal stripes (up to (N-1)x one
// link); the N/2 disjoint pairs of a tournament round get a direct share of 1
// and N-2 relay shares of 1/2 (up to N/2x one link); all-pairs stays direct.
#pragma once

#include <cstddef>
#include <utility>
#include <vector>

namespace p2p {

struct Stripe {
  int via = -1;        // relay rank; -1 = the direct link
  size_t offset = 0;   // byte offset in the message
  size_t bytes = 0;
};

struct RouteOptions {
  size_t min_bytes = size_t{1} << 20;  // messages below this stay on the direct link
  size_t align = 4096;                 // stripe granularity
  double relay_weight = 1.0;           // relative share of a relay path (0 = no relays)
  int max_relays = -1;                 // cap on relays per flow (-1 = all candidates)
};

// Options from the environment: P2P_RELAY_MIN (size), P2P_RELAY_WEIGHT,
// P2P_RELAY_MAX.
RouteOptions route_options_from_env();

// One entry per flow of `flows` (same order; duplicates allowed and planned
// identically): the stripes that cover [0, bytes), direct stripe first in the
// vector.  In the message the relay stripes come first (each a whole number
// of `align` units, so every stripe offset is aligned) and the direct stripe
// takes the rest, including any unaligned tail.
// Self flows (src == dst) are one direct stripe.
std::vector<std::vector<Stripe>> plan_routes(int nranks, const std::vector<std::pair<int, int>>& flows, size_t bytes,
                                             const RouteOptions& opt = RouteOptions());

}  // namespace p2p
