#include "schedule.hpp"

#include <algorithm>
#include <map>

#include "common.hpp"

namespace p2p {

const char* mode_name(Mode m) {
  switch (m) {
    case Mode::Pair: return "pair";
    case Mode::Ring: return "ring";
    case Mode::AllPairs: return "allpairs";
    case Mode::Tournament: return "tournament";
    case Mode::Self: return "self";
  }
  return "?";
}

const char* direction_name(Direction d) { return d == Direction::Uni ? "uni" : "bi"; }

Mode parse_mode(const std::string& s) {
  if (s == "pair" || s == "pairs" || s == "serial") return Mode::Pair;
  if (s == "ring") return Mode::Ring;
  if (s == "allpairs" || s == "all-pairs" || s == "alltoall" || s == "a2a") return Mode::AllPairs;
  if (s == "tournament" || s == "rounds" || s == "matching") return Mode::Tournament;
  if (s == "self") return Mode::Self;
  P2P_FATAL("unknown mode '" + s + "' (pair|ring|allpairs|tournament|self)");
}

Direction parse_direction(const std::string& s) {
  if (s == "uni") return Direction::Uni;
  if (s == "bi") return Direction::Bi;
  P2P_FATAL("unknown direction '" + s + "' (uni|bi)");
}

int Phase::max_recv_slots() const {
  int m = 0;
  for (const auto& r : ranks) m = std::max(m, static_cast<int>(r.recv_from.size()));
  return m;
}

std::string Schedule::name() const { return std::string(mode_name(mode)) + "-" + direction_name(dir); }

int Schedule::max_recv_slots() const {
  int m = 0;
  for (const auto& p : phases) m = std::max(m, p.max_recv_slots());
  return m;
}

namespace {

Phase empty_phase(int n, std::string label) {
  Phase p;
  p.label = std::move(label);
  p.ranks.resize(static_cast<size_t>(n));
  return p;
}

void add_flow(Phase& p, int src, int dst) {
  p.ranks[static_cast<size_t>(src)].send_to.push_back(dst);
  p.ranks[static_cast<size_t>(dst)].recv_from.push_back(src);
  p.flows.push_back({src, dst});
}

}  // namespace

Schedule make_pair_schedule(int n, Direction dir) {
  P2P_CHECK(n >= 1, "need at least one rank");
  Schedule s;
  s.mode = Mode::Pair;
  s.dir = dir;
  s.nranks = n;
  // Row-major over (src, dst) exactly like p2p_matrix.cc:141-145 / 196-200.
  for (int src = 0; src < n; ++src) {
    for (int dst = 0; dst < n; ++dst) {
      Phase p = empty_phase(n, strfmt("%d->%d", src, dst));
      p.row = src;
      p.col = dst;
      if (src == dst) {
        p.idle = true;  // p2p_matrix.cc:147-151: barrier, print 0.00, no transfer
      } else {
        add_flow(p, src, dst);
        if (dir == Direction::Bi) add_flow(p, dst, src);  // p2p_matrix.cc:211-249
      }
      s.phases.push_back(std::move(p));
    }
  }
  return s;
}

Schedule make_self_schedule(int n) {
  Schedule s;
  s.mode = Mode::Self;
  s.dir = Direction::Uni;
  s.nranks = n;
  Phase p = empty_phase(n, "self");
  for (int r = 0; r < n; ++r) add_flow(p, r, r);
  s.phases.push_back(std::move(p));
  return s;
}

Schedule make_ring_schedule(int n, Direction dir) {
  if (n == 1) {
    Schedule s = make_self_schedule(1);
    s.mode = Mode::Ring;
    s.dir = dir;
    return s;
  }
  Schedule s;
  s.mode = Mode::Ring;
  s.dir = dir;
  s.nranks = n;
  Phase p = empty_phase(n, dir == Direction::Uni ? "ring+1" : "ring+-1");
  for (int r = 0; r < n; ++r) add_flow(p, r, (r + 1) % n);
  // Bi ring adds the reverse hop; with n == 2 next == prev, so skip duplicates.
  if (dir == Direction::Bi && n > 2)
    for (int r = 0; r < n; ++r) add_flow(p, r, (r + n - 1) % n);
  s.phases.push_back(std::move(p));
  return s;
}

Schedule make_allpairs_schedule(int n, Direction dir) {
  if (n == 1) {
    Schedule s = make_self_schedule(1);
    s.mode = Mode::AllPairs;
    s.dir = dir;
    return s;
  }
  Schedule s;
  s.mode = Mode::AllPairs;
  s.dir = dir;
  s.nranks = n;
  Phase p = empty_phase(n, "all-pairs");
  // Staggered order (r+k) so that no single peer is everyone's first op.
  for (int k = 1; k < n; ++k)
    for (int r = 0; r < n; ++r) add_flow(p, r, (r + k) % n);
  s.phases.push_back(std::move(p));
  return s;
}

std::vector<std::vector<std::pair<int, int>>> round_robin_rounds(int n) {
  std::vector<std::vector<std::pair<int, int>>> rounds;
  if (n < 2) return rounds;
  int m = (n % 2 == 0) ? n : n + 1;  // pad with a dummy player for odd n
  int fixed = m - 1;
  for (int r = 0; r < m - 1; ++r) {
    std::vector<std::pair<int, int>> pairs;
    auto push = [&](int a, int b) {
      if (a >= n || b >= n) return;  // dummy: that rank sits out
      pairs.emplace_back(std::min(a, b), std::max(a, b));
    };
    push(fixed, r);
    for (int k = 1; k < m / 2; ++k) push((r + k) % (m - 1), (r - k + (m - 1)) % (m - 1));
    std::sort(pairs.begin(), pairs.end());
    rounds.push_back(std::move(pairs));
  }
  return rounds;
}

Schedule make_tournament_schedule(int n, Direction dir) {
  if (n == 1) {
    Schedule s = make_self_schedule(1);
    s.mode = Mode::Tournament;
    s.dir = dir;
    return s;
  }
  Schedule s;
  s.mode = Mode::Tournament;
  s.dir = dir;
  s.nranks = n;
  auto rounds = round_robin_rounds(n);
  for (size_t r = 0; r < rounds.size(); ++r) {
    if (dir == Direction::Bi) {
      Phase p = empty_phase(n, strfmt("round %zu", r));
      for (auto& pr : rounds[r]) {
        add_flow(p, pr.first, pr.second);
        add_flow(p, pr.second, pr.first);
      }
      s.phases.push_back(std::move(p));
    } else {
      // Uni: each round becomes two phases, low->high then high->low, so all
      // N(N-1) ordered cells are covered.
      Phase up = empty_phase(n, strfmt("round %zu a", r));
      Phase down = empty_phase(n, strfmt("round %zu b", r));
      for (auto& pr : rounds[r]) {
        add_flow(up, pr.first, pr.second);
        add_flow(down, pr.second, pr.first);
      }
      s.phases.push_back(std::move(up));
      s.phases.push_back(std::move(down));
    }
  }
  return s;
}

Schedule make_schedule(Mode mode, Direction dir, int n) {
  switch (mode) {
    case Mode::Pair: return make_pair_schedule(n, dir);
    case Mode::Ring: return make_ring_schedule(n, dir);
    case Mode::AllPairs: return make_allpairs_schedule(n, dir);
    case Mode::Tournament: return make_tournament_schedule(n, dir);
    case Mode::Self: return make_self_schedule(n);
  }
  P2P_FATAL("bad mode");
}

std::string validate(const Schedule& s) {
  for (size_t pi = 0; pi < s.phases.size(); ++pi) {
    const Phase& p = s.phases[pi];
    if (static_cast<int>(p.ranks.size()) != s.nranks) return strfmt("phase %zu: rank list size", pi);
    std::map<std::pair<int, int>, int> sends, recvs, flows;
    for (int r = 0; r < s.nranks; ++r) {
      for (int d : p.ranks[r].send_to) {
        if (d < 0 || d >= s.nranks) return strfmt("phase %zu: rank %d sends to bad peer %d", pi, r, d);
        sends[{r, d}]++;
      }
      for (int src : p.ranks[r].recv_from) {
        if (src < 0 || src >= s.nranks) return strfmt("phase %zu: rank %d receives from bad peer %d", pi, r, src);
        recvs[{src, r}]++;
      }
    }
    for (const auto& f : p.flows) flows[{f.src, f.dst}]++;
    if (sends != recvs) return strfmt("phase %zu (%s): send/recv multisets differ", pi, p.label.c_str());
    if (sends != flows) return strfmt("phase %zu (%s): flows disagree with ops", pi, p.label.c_str());
    if (p.idle && !p.flows.empty()) return strfmt("phase %zu: idle phase has flows", pi);
  }
  return "";
}

void restrict_cells(Schedule* s, const std::vector<std::pair<int, int>>& cells, bool drop_others) {
  if (s->mode != Mode::Pair || cells.empty()) return;
  std::vector<Phase> kept;
  for (auto& p : s->phases) {
    bool keep = std::find(cells.begin(), cells.end(), std::make_pair(p.row, p.col)) != cells.end();
    if (keep) {
      kept.push_back(p);
    } else if (!drop_others) {
      if (!p.idle) {
        p.idle = true;
        p.flows.clear();
        for (auto& r : p.ranks) r = RankOps{};
      }
      kept.push_back(p);
    }
  }
  s->phases = std::move(kept);
}

}  // namespace p2p
