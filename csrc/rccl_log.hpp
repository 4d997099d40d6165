// What RCCL set up, read from its own INFO log (pure host code, unit-tested).
//
// RCCL reports neither how many p2p channels a send/recv to a peer is split
// over nor which transport (P2P/IPC over xGMI, SHM, NET) carries it -- except
// in its INFO log.  Both matter here:
//   * RCCL 2.26 / 2.27 on MI355X deliver exactly the first half of an op whose
//     share of one p2p channel exceeds 16 MiB, silently
//     (scripts/rccl_half_repro.cpp, profiles/r3_rccl_half_repro/), so the
//     transport posts messages as ops of at most 16 MiB x channels;
//   * a pair that silently fell back from xGMI to SHM or NET would look like a
//     slow link.
// The transport points NCCL_DEBUG_FILE at a private file (when the user has not
// set NCCL_DEBUG), reads it after each communicator's init and after the lazy
// p2p connects, and records what it found (provenance.rccl_peers).
#pragma once

#include <string>
#include <vector>

namespace p2p {

// From a communicator's init block.
struct RcclInitInfo {
  int nranks = -1;           // "comm 0x.. rank r nRanks N nNodes H localRanks L ..."
  int nnodes = -1;
  int p2p_channels = -1;     // "... %d p2p channels, %d p2p channels per peer"
  int p2p_per_peer = -1;
  int from_rank = -1;        // set when another rank's log supplied the counts
  int unroll = -1;           // "RCCL Unroll Factor (pre-set|user-defined): U"
  bool found() const { return p2p_channels > 0 && p2p_per_peer > 0; }
};

// One connection line: "Channel 03/0 : 0[2] -> 1[5] [send] via NET/Socket/0".
struct RcclConnection {
  int channel = -1;
  int conn_index = 0;  // "Channel 03/1": 1 = the connections p2p ops use (0: collectives' rings / trees)
  int src = -1;  // ranks
  int dst = -1;
  std::string via;  // first token after "via": "P2P/IPC/read", "NET/Socket/0", "SHM/direct/direct", ...
  std::string comm;  // the "comm 0x..." token RCCL appends ("" when absent)
};

// The last init block in `text` (fields not seen stay -1).
RcclInitInfo parse_rccl_init(const std::string& text);
// Every connection line in `text`, in order.
std::vector<RcclConnection> parse_rccl_connections(const std::string& text);

// The lines of the communicators named in `comms` ("0x..." as RCCL prints a
// pointer) and lines without a comm token; another transport of the process
// may log into the same file.
std::vector<RcclConnection> connections_of(const std::vector<RcclConnection>& conns, const std::vector<std::string>& comms);

// Per peer of rank `me`: the channels connected towards it (send lines
// me -> peer; receive-side lines peer -> me where no send line exists; lines
// of p2p connections, conn_index > 0, where there are any; counted per
// communicator, and the fewest of any communicator with lines) and
// the transport class: "P2P" (xGMI / PCIe peer access through IPC), "SHM",
// "NET", "self" (peer == me: RCCL copies inside the kernel and logs no
// connection) or "" (not connected yet).
struct RcclPeerLink {
  int peer = -1;
  int channels_connected = 0;
  std::string transport;  // class, as above
  std::string via;        // the full token of the first line seen
};
std::vector<RcclPeerLink> rccl_peer_links(const std::vector<RcclConnection>& conns, int me, int nranks);

// Channels a send/recv to a peer is split over: min(p2p channels, per peer)
// of the communicator, and for a peer RCCL reaches through its network
// transport at most `net_per_peer` (NCCL_NCHANNELS_PER_NET_PEER, 2 by
// default).  0 when the init block was not found.
int rccl_op_channels(const RcclInitInfo& info, bool net_peer, int net_per_peer);

// Op channels once RCCL's connection lines are known.
// The init line gives the channels a communicator may split an op to a peer
// over; the connection lines give the channels it did connect to that peer.
// proposed_op_channels(): per peer, min(init_channels[p], channels connected)
// for a remote peer with connection lines; 0 (no opinion) for `me` and for a
// peer without lines (or without an init count).
std::vector<int> proposed_op_channels(const std::vector<int>& init_channels, const std::vector<RcclPeerLink>& links,
                                      int me);
// Both ends of a pair must split a message alike.  `all` holds every rank's
// proposals (all[r * n + p]: rank r's for peer p).  Rank me's op channels per
// peer: the smaller proposal where both ends have one, the one proposal where
// only one end has, else `current[p]`.  sources[p] (if given) is set to
// "connection lines" where a proposal was used, left alone otherwise.
std::vector<int> agree_op_channels(const std::vector<int>& all, int n, int me, const std::vector<int>& current,
                                   std::vector<std::string>* sources = nullptr);

// Link check (--min-gbs): a pair whose GPUs share a direct xGMI link
// (`link` "XGMI/1", provenance rank_links) must be carried by RCCL's P2P
// transport; a known transport of another class (SHM, NET) there is a silent
// fallback that would read as a slow link.
bool link_transport_mismatch(const std::string& link, const std::string& transport);

// Peers whose connections the parser did not see: a
// remote peer on this host (not `me`, net_peer[p] == 0) that this rank has
// exchanged messages with (touched[p] != 0) but for which rccl_peer_links
// found no channel -- RCCL connected it, so a line in a layout
// parse_rccl_connections does not know was missed, and the peer's op limit
// stayed at the unconnected default.  For each, up to `max_lines` lines of
// `text` that name the peer's rank as an endpoint ("<p>[", "-> <p>",
// "<p> ->", "rank <p>", "peer <p>"), preferring connection-like lines, so the
// record shows the format that was missed.
struct RcclUnparsedPeer {
  int peer = -1;
  std::vector<std::string> lines;
};
std::vector<RcclUnparsedPeer> rccl_unparsed_peers(const std::string& text, const std::vector<RcclPeerLink>& links,
                                                  const std::vector<char>& net_peer, const std::vector<char>& touched,
                                                  int me, size_t max_lines = 20);

// Raw lines of `text` for the record (link_report log_sample): RCCL's version
// line, the last line that states the p2p channel counts, and the first
// `max_conn` connection lines ("Channel .. via .."; those of p2p connections,
// "Channel xx/1", before the collectives' "xx/0"), so a node run keeps the
// real format its parser was checked against (the fixtures in tests/data are
// hand-written in RCCL 2.26's layout).
std::vector<std::string> rccl_log_sample(const std::string& text, size_t max_conn = 4);

// ---- this process's RCCL environment and INFO log file -----------------
// RCCL's INFO log, which this process reads to learn the p2p channels and
// transports RCCL set up.  Unless the user asked for RCCL's log themselves
// (NCCL_DEBUG / NCCL_DEBUG_FILE) or P2P_RCCL_LOG=0, the first call points it
// at a private file before RCCL's first initialisation reads the variables;
// the file is removed at exit (P2P_RCCL_LOG=keep keeps it).  Empty path: no
// log to read.  What this sets in the environment (NCCL_DEBUG*,
// RCCL_UNROLL_FACTOR) is recorded with the values it replaced, so a child
// process puts them back before deciding anything (rccl_log.cpp set_owned).
struct RcclLogFile {
  std::string path;
  bool ours = false;
};
const RcclLogFile& rccl_log_file();
// RCCL's copy-loop unroll factor for this process (4 unless the user set
// RCCL_UNROLL_FACTOR; P2P_RCCL_UNROLL=<n>, 0 = RCCL's choice).
void rccl_unroll_setup();
size_t rccl_log_size();                            // bytes in the log so far
std::string rccl_log_since(size_t offset);         // the log from `offset` on
std::string rccl_log_warnings(size_t offset);      // its last 4 WARN lines, one "\n  rccl: " each
std::string rccl_host_id();                        // NCCL_HOSTID, else the hostname

// RCCL's half-delivery threshold: bytes of one op per p2p channel.
constexpr size_t kRcclBytesPerChannel = size_t{16} << 20;

}  // namespace p2p
