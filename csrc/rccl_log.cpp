#include "rccl_log.hpp"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <map>
#include <set>
#include <sstream>

namespace p2p {
namespace {

// Integer right after `key` (spaces skipped) in `line`; -1 if absent.
int int_after(const std::string& line, const std::string& key) {
  size_t at = line.find(key);
  if (at == std::string::npos) return -1;
  at += key.size();
  while (at < line.size() && line[at] == ' ') ++at;
  if (at >= line.size() || !std::isdigit(static_cast<unsigned char>(line[at]))) return -1;
  return std::atoi(line.c_str() + at);
}

// Integer ending right before position `end` (spaces skipped); -1 if none.
int int_before(const std::string& line, size_t end) {
  size_t e = end;
  while (e > 0 && line[e - 1] == ' ') --e;
  size_t b = e;
  while (b > 0 && std::isdigit(static_cast<unsigned char>(line[b - 1]))) --b;
  if (b == e) return -1;
  return std::atoi(line.substr(b, e - b).c_str());
}

// "<int>[<int>]" at `at`; returns the rank, advances `at`.
bool rank_dev(const std::string& s, size_t* at, int* rank) {
  size_t i = *at;
  while (i < s.size() && s[i] == ' ') ++i;
  size_t b = i;
  while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
  if (i == b || i >= s.size() || s[i] != '[') return false;
  *rank = std::atoi(s.substr(b, i - b).c_str());
  size_t close = s.find(']', i);
  if (close == std::string::npos) return false;
  *at = close + 1;
  return true;
}

std::string transport_class(const std::string& via) {
  if (via.rfind("P2P", 0) == 0) return "P2P";
  if (via.rfind("SHM", 0) == 0) return "SHM";
  if (via.rfind("NET", 0) == 0 || via.rfind("COLLNET", 0) == 0) return "NET";
  return via.substr(0, via.find('/'));
}

}  // namespace

RcclInitInfo parse_rccl_init(const std::string& text) {
  RcclInitInfo info;
  std::istringstream in(text);
  for (std::string line; std::getline(in, line);) {
    if (line.find(" nNodes ") != std::string::npos && line.find(" nRanks ") != std::string::npos) {
      info.nranks = int_after(line, " nRanks ");
      info.nnodes = int_after(line, " nNodes ");
    }
    const size_t uf = line.find("Unroll Factor");
    if (uf != std::string::npos) {
      const size_t colon = line.find(':', uf);
      if (colon != std::string::npos) info.unroll = std::atoi(line.c_str() + colon + 1);
    }
    const size_t pp = line.find(" p2p channels per peer");
    if (pp != std::string::npos) {
      info.p2p_per_peer = int_before(line, pp);
      const size_t pc = line.rfind(" p2p channels,", pp);
      info.p2p_channels = pc == std::string::npos ? -1 : int_before(line, pc);
    }
  }
  return info;
}

std::vector<RcclConnection> parse_rccl_connections(const std::string& text) {
  std::vector<RcclConnection> out;
  std::istringstream in(text);
  for (std::string line; std::getline(in, line);) {
    const size_t ch = line.find("Channel ");
    const size_t via = line.find(" via ");
    if (ch == std::string::npos || via == std::string::npos || via < ch) continue;
    RcclConnection c;
    size_t at = ch + 8;
    c.channel = std::atoi(line.c_str() + at);
    const size_t colon = line.find(" : ", at);
    const size_t slash = line.find('/', at);
    if (slash != std::string::npos && slash < colon) c.conn_index = std::atoi(line.c_str() + slash + 1);
    if (colon == std::string::npos || colon > via) continue;
    at = colon + 3;
    if (!rank_dev(line, &at, &c.src)) continue;
    const size_t arrow = line.find("->", at);
    if (arrow == std::string::npos || arrow > via) continue;
    at = arrow + 2;
    if (!rank_dev(line, &at, &c.dst)) continue;
    size_t t = via + 5;
    while (t < line.size() && line[t] == ' ') ++t;
    size_t e = t;
    while (e < line.size() && line[e] != ' ' && line[e] != '\r') ++e;
    c.via = line.substr(t, e - t);
    if (c.via.empty()) continue;
    const size_t cm = line.find(" comm ", e);
    if (cm != std::string::npos) {
      size_t b = cm + 6, x = b;
      while (x < line.size() && line[x] != ' ' && line[x] != '\r') ++x;
      c.comm = line.substr(b, x - b);
    }
    out.push_back(c);
  }
  return out;
}

std::vector<RcclConnection> connections_of(const std::vector<RcclConnection>& conns, const std::vector<std::string>& comms) {
  std::vector<RcclConnection> out;
  for (const auto& c : conns)
    if (c.comm.empty() || std::find(comms.begin(), comms.end(), c.comm) != comms.end()) out.push_back(c);
  return out;
}

std::vector<RcclPeerLink> rccl_peer_links(const std::vector<RcclConnection>& conns, int me, int nranks) {
  std::vector<RcclPeerLink> out(static_cast<size_t>(std::max(nranks, 0)));
  // (peer, communicator) -> channels of its send / receive-side lines
  std::map<std::pair<int, std::string>, std::set<int>> send_ch, recv_ch;
  std::set<int> p2p_peers;  // peers with p2p (conn_index > 0) lines: only those count
  for (const auto& c : conns)
    if (c.conn_index > 0) p2p_peers.insert(c.src == me ? c.dst : c.src);
  for (int p = 0; p < nranks; ++p) {
    out[static_cast<size_t>(p)].peer = p;
    if (p == me) out[static_cast<size_t>(p)].transport = "self";
  }
  for (const auto& c : conns) {
    int peer = -1;
    bool send = false;
    if (c.src == me && c.dst != me) {
      peer = c.dst;
      send = true;
    } else if (c.dst == me && c.src != me) {
      peer = c.src;
    }
    if (peer < 0 || peer >= nranks) continue;
    if (c.conn_index > 0 || !p2p_peers.count(peer)) (send ? send_ch : recv_ch)[{peer, c.comm}].insert(c.channel);
    auto& l = out[static_cast<size_t>(peer)];
    if (l.via.empty()) {
      l.via = c.via;
      l.transport = transport_class(c.via);
    }
  }
  // Per communicator: its send lines, or its receive-side lines where it
  // logged no send line; the peer's count is the fewest of any communicator.
  std::map<std::pair<int, std::string>, int> per_comm;
  for (const auto& kv : recv_ch) per_comm[kv.first] = static_cast<int>(kv.second.size());
  for (const auto& kv : send_ch) per_comm[kv.first] = static_cast<int>(kv.second.size());
  for (const auto& kv : per_comm) {
    auto& l = out[static_cast<size_t>(kv.first.first)];
    l.channels_connected = l.channels_connected == 0 ? kv.second : std::min(l.channels_connected, kv.second);
  }
  return out;
}

int rccl_op_channels(const RcclInitInfo& info, bool net_peer, int net_per_peer) {
  if (!info.found()) return 0;
  int c = std::min(info.p2p_channels, info.p2p_per_peer);
  if (net_peer && net_per_peer > 0) c = std::min(c, net_per_peer);
  return std::max(c, 1);
}

std::vector<int> proposed_op_channels(const std::vector<int>& init_channels, const std::vector<RcclPeerLink>& links,
                                      int me) {
  std::vector<int> out(init_channels.size(), 0);
  for (size_t p = 0; p < out.size() && p < links.size(); ++p) {
    if (static_cast<int>(p) == me || init_channels[p] <= 0 || links[p].channels_connected <= 0) continue;
    out[p] = std::min(init_channels[p], links[p].channels_connected);
  }
  return out;
}

std::vector<int> agree_op_channels(const std::vector<int>& all, int n, int me, const std::vector<int>& current,
                                   std::vector<std::string>* sources) {
  std::vector<int> out(current);
  out.resize(static_cast<size_t>(n), 0);
  for (int p = 0; p < n; ++p) {
    const int a = all[static_cast<size_t>(me) * n + p], b = all[static_cast<size_t>(p) * n + me];
    if (a <= 0 && b <= 0) continue;
    out[static_cast<size_t>(p)] = a > 0 && b > 0 ? std::min(a, b) : std::max(a, b);
    if (sources && static_cast<size_t>(p) < sources->size()) (*sources)[static_cast<size_t>(p)] = "connection lines";
  }
  return out;
}

bool link_transport_mismatch(const std::string& link, const std::string& transport) {
  const bool direct_xgmi = link.rfind("XGMI/1", 0) == 0 && link.size() == 6;
  return direct_xgmi && !transport.empty() && transport != "?" && transport != "P2P" && transport != "self";
}

}  // namespace p2p
