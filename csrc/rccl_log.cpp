#include "rccl_log.hpp"

#include <strings.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>

#include "common.hpp"

namespace p2p {
namespace {

// RCCL's INFO log, which this process reads to learn the p2p channels and
// transports RCCL set up (rccl_log.hpp).  Unless the user asked for RCCL's
// log themselves (NCCL_DEBUG / NCCL_DEBUG_FILE) or P2P_RCCL_LOG=0, the
// first transport of the process points it at a private file before RCCL's
// first initialisation reads the variables; the file is removed at exit
// (P2P_RCCL_LOG=keep keeps it).  Empty path: no log to read.
//
// What this process sets in its environment for RCCL (the private log's
// NCCL_DEBUG* below and RCCL_UNROLL_FACTOR) is inherited by every child it
// starts: bench.py's comparison children, a test's p2p_matrix.  Each setting
// is made by set_owned(), which records the value it replaced
// (P2P_RCCL_PREV_<name>: "=<value>", or "" for unset) and this pid
// (P2P_RCCL_ENV_OWNER).  A process that finds another pid's settings puts the
// replaced values back before it decides anything, so a child never writes
// RCCL's log into its parent's file or mistakes the parent's unroll for the
// user's (profiles/r4_session: p2p_matrix --reference under pytest ran at the
// parent's unroll 4).
constexpr const char* kOwnedVars[] = {"NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE", "RCCL_UNROLL_FACTOR"};

void undo_inherited_rccl_env() {
  static const bool done = [] {
    const char* owner = std::getenv("P2P_RCCL_ENV_OWNER");
    if (!owner || std::atoi(owner) == static_cast<int>(getpid())) return true;
    for (const char* k : kOwnedVars) {
      const std::string saved = strfmt("P2P_RCCL_PREV_%s", k);
      const char* v = std::getenv(saved.c_str());
      if (!v) continue;
      if (*v == '=')
        setenv(k, v + 1, 1);
      else
        unsetenv(k);
      unsetenv(saved.c_str());
    }
    unsetenv("P2P_RCCL_ENV_OWNER");
    return true;
  }();
  (void)done;
}

void set_owned(const char* name, const char* value) {
  const std::string saved = strfmt("P2P_RCCL_PREV_%s", name);
  if (!std::getenv(saved.c_str())) {
    const char* prev = std::getenv(name);
    setenv(saved.c_str(), prev ? (std::string("=") + prev).c_str() : "", 1);
  }
  setenv(name, value, 1);
  setenv("P2P_RCCL_ENV_OWNER", std::to_string(static_cast<int>(getpid())).c_str(), 1);
}

}  // namespace

const RcclLogFile& rccl_log_file() {
  static RcclLogFile log = [] {
    undo_inherited_rccl_env();
    RcclLogFile l;
    const char* mode = std::getenv("P2P_RCCL_LOG");
    if (mode && std::strcmp(mode, "0") == 0) return l;
    if (const char* f = std::getenv("NCCL_DEBUG_FILE")) {
      // The user's file: readable only if it names no per-process pattern.
      if (!std::strchr(f, '%')) l.path = f;
      return l;
    }
    // NCCL_DEBUG=VERSION (set in the image's environment) asks only for the
    // version banner; any other level is the user asking for RCCL's log on
    // stderr, which is then left alone.
    if (const char* lvl = std::getenv("NCCL_DEBUG"); lvl && *lvl && strcasecmp(lvl, "VERSION") != 0) return l;
    const char* tmp = std::getenv("TMPDIR");
    l.path = strfmt("%s/p2p_rccl_info_%d.log", tmp && *tmp ? tmp : "/tmp", static_cast<int>(getpid()));
    l.ours = true;
    set_owned("NCCL_DEBUG", "INFO");
    if (!std::getenv("NCCL_DEBUG_SUBSYS")) set_owned("NCCL_DEBUG_SUBSYS", "INIT,ENV,P2P,NET,SHM");
    set_owned("NCCL_DEBUG_FILE", l.path.c_str());
    if (!(mode && std::strcmp(mode, "keep") == 0))
      std::atexit([] { std::remove(rccl_log_file().path.c_str()); });
    return l;
  }();
  return log;
}

// RCCL's copy-loop unroll factor for the kernels of every communicator of
// this process.  RCCL's kernel table holds unroll 1, 2 and 4 and picks 1 on
// MI355X; with 4, a single communicator's self send/recv step runs in 0.92 ms
// instead of 1.13 ms and the 4-communicator bench gains 7% (2428 vs 2272 GB/s
// over 4 interleaved runs, profiles/r3_unroll/), small-message latency
// unchanged.  Set before RCCL's first init (it reads the variable once), never
// over the user's own RCCL_UNROLL_FACTOR; P2P_RCCL_UNROLL=<n> picks another,
// 0 leaves RCCL's choice.  The value is in every provenance record (env) and
// RCCL's log confirms it per communicator (link_report comms[].unroll).
void rccl_unroll_setup() {
  static const bool done = [] {
    undo_inherited_rccl_env();
    if (std::getenv("RCCL_UNROLL_FACTOR")) return true;
    const char* want = std::getenv("P2P_RCCL_UNROLL");
    const std::string v = want ? want : "4";
    if (v != "0" && !v.empty()) set_owned("RCCL_UNROLL_FACTOR", v.c_str());
    return true;
  }();
  (void)done;
}

size_t rccl_log_size() {
  const std::string& p = rccl_log_file().path;
  if (p.empty()) return 0;
  std::ifstream in(p, std::ios::binary | std::ios::ate);
  return in ? static_cast<size_t>(in.tellg()) : 0;
}

std::string rccl_log_since(size_t offset) {
  const std::string& p = rccl_log_file().path;
  if (p.empty()) return "";
  std::ifstream in(p, std::ios::binary);
  if (!in) return "";
  in.seekg(static_cast<std::streamoff>(offset));
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

// The last few WARN lines of the log since `offset` (RCCL's own account of an
// error, which the private log would otherwise hide).
std::string rccl_log_warnings(size_t offset) {
  std::istringstream in(rccl_log_since(offset));
  std::vector<std::string> warn;
  for (std::string line; std::getline(in, line);)
    if (line.find("NCCL WARN") != std::string::npos) warn.push_back(line);
  std::string out;
  for (size_t i = warn.size() > 4 ? warn.size() - 4 : 0; i < warn.size(); ++i) out += "\n  rccl: " + warn[i];
  return out;
}

// The host RCCL places a rank on: NCCL_HOSTID when set, else the hostname.
std::string rccl_host_id() {
  if (const char* h = std::getenv("NCCL_HOSTID")) return h;
  char name[256] = {0};
  if (gethostname(name, sizeof(name) - 1) != 0) return "?";
  return name;
}


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

namespace {
// Does `line` name rank `r` as a connection endpoint or a peer?
bool names_rank(const std::string& line, int r) {
  const std::string d = std::to_string(r);
  for (size_t at = line.find(d); at != std::string::npos; at = line.find(d, at + 1)) {
    const bool digit_before = at > 0 && std::isdigit(static_cast<unsigned char>(line[at - 1]));
    const size_t end = at + d.size();
    const bool digit_after = end < line.size() && std::isdigit(static_cast<unsigned char>(line[end]));
    if (digit_before || digit_after) continue;
    size_t b = at;
    while (b > 0 && line[b - 1] == ' ') --b;
    size_t e = end;
    while (e < line.size() && line[e] == ' ') ++e;
    const std::string before = line.substr(b >= 5 ? b - 5 : 0, b >= 5 ? 5 : b);
    if ((end < line.size() && line[end] == '[') || line.compare(e, 2, "->") == 0 ||
        (b >= 2 && line.compare(b - 2, 2, "->") == 0) || (b >= 2 && line.compare(b - 2, 2, "=>") == 0) ||
        line.compare(e, 2, "=>") == 0 || before == " rank" || before == "rank" || before == " peer" ||
        before == "peer")
      return true;
  }
  return false;
}

bool connection_like(const std::string& line) {
  for (const char* k : {"Channel", "channel", " via ", "P2P", "Connect", "connect"})
    if (line.find(k) != std::string::npos) return true;
  return false;
}
}  // namespace

std::vector<RcclUnparsedPeer> rccl_unparsed_peers(const std::string& text, const std::vector<RcclPeerLink>& links,
                                                  const std::vector<char>& net_peer, const std::vector<char>& touched,
                                                  int me, size_t max_lines) {
  std::vector<RcclUnparsedPeer> out;
  for (size_t p = 0; p < links.size(); ++p) {
    const int peer = static_cast<int>(p);
    if (peer == me || links[p].channels_connected > 0) continue;
    if (p < net_peer.size() && net_peer[p]) continue;
    if (p >= touched.size() || !touched[p]) continue;
    RcclUnparsedPeer u;
    u.peer = peer;
    std::vector<std::string> other;
    std::istringstream in(text);
    for (std::string line; std::getline(in, line);) {
      if (!names_rank(line, peer)) continue;
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (connection_like(line)) {
        if (u.lines.size() < max_lines) u.lines.push_back(line);
      } else if (other.size() < max_lines) {
        other.push_back(line);
      }
    }
    for (size_t i = 0; i < other.size() && u.lines.size() < max_lines; ++i) u.lines.push_back(other[i]);
    out.push_back(std::move(u));
  }
  return out;
}

std::vector<std::string> rccl_log_sample(const std::string& text, size_t max_conn) {
  std::string version, channels;
  std::vector<std::string> p2p, other;  // connection lines of p2p ops ("Channel xx/1") first
  std::istringstream in(text);
  for (std::string line; std::getline(in, line);) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (version.empty() && line.find("RCCL version") != std::string::npos) version = line;
    if (line.find(" p2p channels per peer") != std::string::npos) channels = line;
    const size_t ch = line.find("Channel ");
    if (ch == std::string::npos || line.find(" via ", ch) == std::string::npos) continue;
    const size_t slash = line.find('/', ch), colon = line.find(" : ", ch);
    const bool is_p2p = slash != std::string::npos && slash < colon && std::atoi(line.c_str() + slash + 1) > 0;
    auto& v = is_p2p ? p2p : other;
    if (v.size() < max_conn) v.push_back(line);
  }
  std::vector<std::string> out;
  if (!version.empty()) out.push_back(version);
  if (!channels.empty()) out.push_back(channels);
  for (size_t i = 0; i < other.size() && p2p.size() < max_conn; ++i) p2p.push_back(other[i]);
  out.insert(out.end(), p2p.begin(), p2p.end());
  return out;
}

bool link_transport_mismatch(const std::string& link, const std::string& transport) {
  const bool direct_xgmi = link.rfind("XGMI/1", 0) == 0 && link.size() == 6;
  return direct_xgmi && !transport.empty() && transport != "?" && transport != "P2P" && transport != "self";
}

}  // namespace p2p
