// Top-level application: CLI -> bootstrap -> placement -> transport ->
// schedules -> reports.  Shared by the p2p_matrix executable (main.cpp) and
// the Python extension (pymodule.cpp).
//
// The reference has no CLI at all (argv only reaches MPI_Init_thread,
// p2p_matrix.cc:105; message size and iteration count are compile-time
// constants, :124 and :132).  Defaults here reproduce it: with no flags,
// `mpirun -n N ./p2p_matrix` runs the serial pair schedule, uni then bi, at
// 32 MiB x 128 and prints the same two matrices first.
#pragma once

#include <cstdio>
#include <string>
#include <vector>

#include "report.hpp"
#include "runner.hpp"
#include "schedule.hpp"

namespace p2p {

class Bootstrap;

struct AppConfig {
  std::vector<Mode> modes{Mode::Pair};
  std::vector<Direction> dirs{Direction::Uni, Direction::Bi};
  std::vector<size_t> sizes{32u << 20};
  RunConfig run;                 // iters / warmup / timing / verify
  bool iters_auto = false;       // scale iterations per size (target_bytes per cell)
  size_t target_bytes = 4ull << 30;
  bool latency = false;
  bool device_latency = false;   // ping-pong kernel matrix (one-sided transports)
  int latency_preposted = 0;     // > 0: ping-pong also posted in batches of this many behind a stream gate
  int fuzz_rounds = 0;           // --fuzz N: N groups of random verified messages (data-integrity stress)
  size_t latency_bytes = 8;
  int latency_iters = 1000;
  std::string transport = "rccl";  // rccl | ipc | host
  std::string ipc_engine = "kernel";
  std::string bootstrap = "auto";  // auto | mpi | env | local
  int device = -1;
  std::string json_path;
  std::string csv_path;
  std::string trace_path;
  bool resume = false;
  std::vector<std::pair<int, int>> cells;  // pair-mode cell filter (empty = all)
  bool compat = true;      // reference matrices for pair mode
  bool extended = true;    // GB/s / latency tables after the compat section
  double timeout_s = 300;
  bool reference_buffers = false;  // --reference: one send / receive region for every iteration
  int verify_impl = 0;
  bool dry_run = false;    // print the schedules and exit (no transport)
  bool topology_only = false;  // print the GPU link matrix and exit
  bool warm_connections = true;
  double min_gbs = 0;          // link check: any off-diagonal flow below this fails the run (exit 3)
  bool two_streams = false;  // RCCL receives on a second stream (reference layout)
  bool rccl_stock = false;   // --reference: RCCL's own kernel unroll (no P2P_RCCL_UNROLL)
  int comms = 1;             // RCCL communicators per rank (messages spread round-robin)
  int repeat = 1;            // --repeat R: every (mode, dir, size) run R times; repeat summary (median)
  int verbose = 0;
};

// Parses argv (after the program name).  Sets *exit_code and returns false
// when the program should exit immediately (--help, --version, bad flag).
bool parse_cli(int argc, char** argv, AppConfig* cfg, int* exit_code, FILE* out = stdout);
std::string usage_text();
// --verify-impl / ops.verify(impl=) names -> dev::VerifyImpl values
// (kernels.hpp): auto 0, lds8 (alias lds) 1, stride (aliases reg, register)
// 2.  Returns -2 for a variant removed in round 5 and -1 for an unknown
// name, with the reason in *note.
int parse_verify_impl(const std::string& name, std::string* note);

// Iterations for a message size under --iters auto.
int auto_iters(size_t bytes, size_t target_bytes);

struct AppResult {
  std::vector<RunRecord> runs;
  std::vector<LatencyResult> latency;
  std::vector<LatencyResult> device_latency;
  std::vector<LatencyResult> preposted_latency;
  std::vector<RingLatencyResult> ring_latency;  // --mode ring with --latency / --device-latency
  uint64_t mismatches = 0;
  int slow_flows = 0;  // flows under --min-gbs, or carried by the wrong transport (see count_slow_flows)
  // After the runs (collective): per pair (row-major n x n) the transport
  // class the data plane reached the peer through (Transport::peer_transports,
  // "" unknown) and the GPU link type (provenance rank_links); each rank's
  // Transport::link_report().
  std::vector<std::string> transport_matrix;
  std::vector<std::string> link_matrix;
  std::vector<std::string> link_reports;
};

// Runs everything collectively; rank 0 prints to `out`.  Returns 0 on success,
// 2 if verification found corrupted data, 3 if a link ran below --min-gbs.
int run_app(const AppConfig& cfg, Bootstrap& boot, FILE* out, AppResult* result = nullptr);

}  // namespace p2p
