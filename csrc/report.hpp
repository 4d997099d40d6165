// Reporting: the reference-compatible text matrices, extended tables, JSON.
//
// Compat format (byte-exact with /root/reference/p2p_matrix.cc):
//   title   "Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n"   :134
//           "\nEvaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)\n"  :189
//   corner  "   D\\D"                                                     :135/:190
//   col id  "%6d "                                                        :137/:192
//   row id  "%6d "                                                        :143/:198
//   cell    "%6.02f " (diagonal 0.00), fflush after each cell             :149,179/:204,260
//   row end "\n"                                                          :184/:265
// Values >= 1000 Gbps overflow the 6-char field exactly as the reference's
// printf would; aligned GB/s tables follow after.
#pragma once

#include <cstdio>
#include <string>
#include <vector>

#include "runner.hpp"
#include "schedule.hpp"

namespace p2p {

class CompatPrinter {
 public:
  CompatPrinter(FILE* out, int nranks) : out_(out), n_(nranks) {}
  void begin(Direction dir, bool leading_blank_line);
  void on_phase(const PhaseResult& r);  // pair-mode phases, in row-major order
 private:
  FILE* out_;
  int n_;
};

// Gbps value the reference would print for a pair-mode cell: uni = the one
// flow; bi = sum of both directions (p2p_matrix.cc:258 "* 2").
double compat_cell_gbps(const PhaseResult& r);

struct RunRecord {
  Mode mode;
  Direction dir;
  size_t bytes;
  RunConfig cfg;
  std::vector<PhaseResult> phases;
  int repeat = 0;  // --repeat: which run of this (mode, dir, size), 0-based
};

// N x N (row = src, col = dst) matrices built from all flows of a run.
std::vector<double> flow_matrix_gbs(const RunRecord& rec, int n);
std::vector<double> flow_matrix_p50_us(const RunRecord& rec, int n);

// Fabric checks of one node's matrices (GB/s per direction, row = sender;
// the multi-GPU tier's test_fabric_is_uniform and bench.py fabric_findings
// carry the same rules): on a fully connected xGMI node every link is alike,
// so an off-diagonal cell of `uni` below min_ratio x the median cell, or a
// pair whose bi-directional total (bi[a][b] + bi[b][a], p2p_matrix.cc:258)
// is below its uni cell (:177), is reported.  Cells never measured (0) are
// not judged; `bi` may be null.  One line per finding, [] when all pass.
std::vector<std::string> fabric_findings(const std::vector<double>& uni, const std::vector<double>* bi, int n,
                                         double min_ratio = 0.5);

// Human-readable tables appended after the compat section.
void print_extended(FILE* out, const RunRecord& rec, int n);
// The fabric lines of every pair-mode size with both a uni and a bi run
// (fabric_findings), after the extended tables.
void print_fabric_check(FILE* out, const std::vector<RunRecord>& runs, int n);

// --repeat: per (mode, dir, size), every run's mean cell and their median /
// min / max.  A run's value is its mean compat cell in GB/s for pair mode
// (the reference's printed cell / 8: bi = both directions summed,
// p2p_matrix.cc:258) and its mean off-diagonal flow (per direction) for the
// other modes.  One wall-clock run of the reference's method varied by +-9%
// between records on one GPU, so the median is the number to
// compare.
struct RepeatSummary {
  Mode mode;
  Direction dir;
  size_t bytes;
  std::vector<double> runs;
  double median = 0, min = 0, max = 0;
};
std::vector<RepeatSummary> repeat_summaries(const std::vector<RunRecord>& runs, int n);
void print_repeat_summary(FILE* out, const std::vector<RepeatSummary>& sums);
std::string repeat_summary_json(const RepeatSummary& s);
void print_latency(FILE* out, const std::vector<LatencyResult>& lat, int n);
void print_matrix(FILE* out, const std::string& title, const std::vector<double>& m, int n, const char* fmt,
                  bool blank_diag);

// Machine-readable JSON (one object per run / latency set).
std::string run_to_json(const RunRecord& rec, int n);
std::string latency_to_json(const std::vector<LatencyResult>& lat, int n);
// {"type":"ring_latency","method":...,"nranks":N,"bytes":B,"laps":L,"hop_us":{...},"lap_us":{...}}
std::string ring_latency_to_json(const RingLatencyResult& r);
void print_ring_latency(FILE* out, const RingLatencyResult& r);

// CSV rows: mode,dir,bytes,iters,timing,phase,src,dst,seconds,gbps,gbs,p50_us,p99_us,mismatches
std::string csv_header();
std::string run_to_csv(const RunRecord& rec);

// Chrome / Perfetto trace ("traceEvents" JSON): one complete event per rank
// per timed phase (host steady clock), pid = run, tid = rank.
std::string chrome_trace(const std::vector<RunRecord>& runs, int n);

// Resume support: the (mode, dir, bytes) key of a run and of a JSON line.
std::string run_key(Mode m, Direction d, size_t bytes);
std::string run_key_from_json(const std::string& line);  // "" if not a run line

// Minimal JSON string escaping.
std::string json_escape(const std::string& s);

}  // namespace p2p
