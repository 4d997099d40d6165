#include "routing.hpp"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <set>

#include "common.hpp"
#include "units.hpp"

namespace p2p {

RouteOptions route_options_from_env() {
  RouteOptions o;
  if (const char* v = std::getenv("P2P_RELAY_MIN")) o.min_bytes = parse_size(v);
  if (const char* v = std::getenv("P2P_RELAY_WEIGHT")) o.relay_weight = std::atof(v);
  if (const char* v = std::getenv("P2P_RELAY_MAX")) o.max_relays = std::atoi(v);
  P2P_CHECK(o.relay_weight >= 0.0, "P2P_RELAY_WEIGHT must be >= 0");
  return o;
}

std::vector<std::vector<Stripe>> plan_routes(int nranks, const std::vector<std::pair<int, int>>& flows, size_t bytes,
                                             const RouteOptions& opt) {
  const size_t n = static_cast<size_t>(std::max(nranks, 0));
  const size_t align = std::max<size_t>(opt.align, 1);
  auto at = [n](int a, int b) { return static_cast<size_t>(a) * n + static_cast<size_t>(b); };
  // Distinct directed flows of the group: duplicates (several messages of one
  // flow in a group) neither make a link busier nor change the split.
  std::set<std::pair<int, int>> uniq;
  for (const auto& f : flows) {
    P2P_CHECK(f.first >= 0 && f.first < nranks && f.second >= 0 && f.second < nranks, "plan_routes: rank out of range");
    if (f.first != f.second) uniq.insert(f);
  }
  std::vector<char> busy(n * n, 0);
  for (const auto& f : uniq) busy[at(f.first, f.second)] = 1;

  const bool relaying = bytes >= opt.min_bytes && opt.relay_weight > 0.0 && opt.max_relays != 0 && nranks > 2;
  // Relay candidates per flow, in a rotated order starting after the
  // destination, so that capped plans (P2P_RELAY_MAX) spread over ranks.
  std::map<std::pair<int, int>, std::vector<int>> cand;
  std::vector<int> load(n * n, 0);  // C(a,b): two-hop segments over a->b
  if (relaying) {
    for (const auto& f : uniq) {
      std::vector<int>& c = cand[f];
      for (int step = 1; step < nranks; ++step) {
        const int k = (f.second + step) % nranks;
        if (k == f.first || k == f.second) continue;
        if (busy[at(f.first, k)] || busy[at(k, f.second)]) continue;
        c.push_back(k);
        if (opt.max_relays > 0 && static_cast<int>(c.size()) == opt.max_relays) break;
      }
      for (int k : c) {
        ++load[at(f.first, k)];
        ++load[at(k, f.second)];
      }
    }
  }

  std::map<std::pair<int, int>, std::vector<Stripe>> plans;
  for (const auto& f : uniq) {
    std::vector<Stripe> relays;
    size_t relayed = 0;
    const auto it = cand.find(f);
    const size_t units = bytes / align;
    if (it != cand.end() && !it->second.empty() && units > 1) {
      std::vector<double> share;
      double total = 1.0;  // the direct link
      for (int k : it->second) {
        const int c = std::max(load[at(f.first, k)], load[at(k, f.second)]);
        share.push_back(opt.relay_weight / std::max(c, 1));
        total += share.back();
      }
      for (size_t i = 0; i < share.size(); ++i) {
        const size_t u = static_cast<size_t>(static_cast<double>(units) * share[i] / total);
        if (u == 0) continue;
        Stripe s;
        s.via = it->second[i];
        s.bytes = u * align;
        relays.push_back(s);
        relayed += s.bytes;
      }
    }
    // Byte layout: the relay stripes first (whole `align` units, so every
    // stripe starts aligned for the 16-byte copy kernel), the direct stripe
    // last with the remainder and the message's unaligned tail.
    std::vector<Stripe> out;
    Stripe direct;
    direct.offset = relayed;
    direct.bytes = bytes - relayed;
    out.push_back(direct);
    size_t off = 0;
    for (Stripe& s : relays) {
      s.offset = off;
      off += s.bytes;
      out.push_back(s);
    }
    plans[f] = std::move(out);
  }

  std::vector<std::vector<Stripe>> result;
  result.reserve(flows.size());
  for (const auto& f : flows) {
    if (f.first == f.second) {
      Stripe s;
      s.bytes = bytes;
      result.push_back({s});
    } else {
      result.push_back(plans.at(f));
    }
  }
  return result;
}

}  // namespace p2p
