// Communication schedules: which rank sends to / receives from whom, and in
// which order the concurrent "phases" run.  Pure host code (no HIP, no RCCL),
// unit-tested on CPU.
//
// Reference parity:
//   * Mode::Pair + Direction::Uni  == the uni-directional matrix loop,
//     /root/reference/p2p_matrix.cc:141-186: ordered pairs (src,dst) one at a
//     time, row-major, a barrier per cell including the diagonal, which prints
//     0.00 and moves no data.
//   * Mode::Pair + Direction::Bi   == the bi-directional loop,
//     /root/reference/p2p_matrix.cc:196-267: both endpoints send and receive
//     inside one group.
// Extensions (BASELINE.json north star / SURVEY.md §2.5):
//   * Ring        — rank r sends to r+1 and receives from r-1 concurrently:
//                   the pipeline-parallel / ring-attention hop pattern.
//   * AllPairs    — every rank exchanges with every peer in ONE group: the
//                   expert-parallel all-to-all shape; bisection-bandwidth stress.
//   * Tournament  — round-robin 1-factorisation of the complete graph: N-1
//                   rounds (N even), each a perfect matching of disjoint pairs.
//                   MI355X's xGMI is fully connected point-to-point, so the
//                   N/2 pairs of a round never share a link and the whole N x N
//                   matrix is measured in N-1 concurrent rounds instead of
//                   N(N-1) serial cells.
//   * Self        — every rank sends to itself (the 1-GPU path).
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace p2p {

enum class Mode { Pair, Ring, AllPairs, Tournament, Self };
enum class Direction { Uni, Bi };

const char* mode_name(Mode m);
const char* direction_name(Direction d);
Mode parse_mode(const std::string& s);
Direction parse_direction(const std::string& s);

struct Flow {
  int src = -1;
  int dst = -1;
  bool operator==(const Flow& o) const { return src == o.src && dst == o.dst; }
};

// What one rank posts per iteration, all inside one ncclGroupStart/End.
// recv_from[i] lands in receive slot i.
struct RankOps {
  std::vector<int> send_to;
  std::vector<int> recv_from;
  bool active() const { return !send_to.empty() || !recv_from.empty(); }
};

struct Phase {
  std::string label;
  int row = -1;       // pair-mode cell (src, dst); -1 for concurrent modes
  int col = -1;
  bool idle = false;  // pair-mode diagonal: barrier only, reported as 0.00
  std::vector<RankOps> ranks;  // one entry per rank
  std::vector<Flow> flows;     // every directed transfer of one iteration

  bool participates(int r) const { return r >= 0 && r < static_cast<int>(ranks.size()) && ranks[r].active(); }
  int recv_slots(int r) const { return participates(r) ? static_cast<int>(ranks[r].recv_from.size()) : 0; }
  int max_recv_slots() const;
};

struct Schedule {
  Mode mode = Mode::Pair;
  Direction dir = Direction::Uni;
  int nranks = 0;
  std::vector<Phase> phases;
  std::string name() const;
  int max_recv_slots() const;
};

Schedule make_pair_schedule(int n, Direction dir);
Schedule make_ring_schedule(int n, Direction dir);
Schedule make_allpairs_schedule(int n, Direction dir);
Schedule make_tournament_schedule(int n, Direction dir);
Schedule make_self_schedule(int n);
Schedule make_schedule(Mode mode, Direction dir, int n);

// Pair mode: measure only the listed (src, dst) cells.  With drop_others the
// other phases are removed (a sweep over a few cells pays no barriers for the
// rest); otherwise they become idle phases, so printed matrices keep their
// shape (--cells).  Other modes are returned unchanged.
void restrict_cells(Schedule* s, const std::vector<std::pair<int, int>>& cells, bool drop_others);

// Round-robin (circle-method) pairing.  Returns rounds of disjoint unordered
// pairs (a < b); for odd n one rank sits out each round.  Every unordered
// pair appears exactly once.
std::vector<std::vector<std::pair<int, int>>> round_robin_rounds(int n);

// Self-consistency: every send has a matching recv on the peer within the
// phase (as a multiset) and flows agree with the per-rank op lists.  Returns
// an empty string when valid, else a description of the first problem.
std::string validate(const Schedule& s);

}  // namespace p2p
