#include "report.hpp"

#include <algorithm>
#include <cmath>
#include <sstream>

#include "common.hpp"
#include "stats.hpp"
#include "units.hpp"

namespace p2p {

// -------------------------------------------------------------- compat ----

void CompatPrinter::begin(Direction dir, bool leading_blank_line) {
  if (dir == Direction::Uni) {
    std::fprintf(out_, "%sEvaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n", leading_blank_line ? "\n" : "");
  } else {
    // The reference's bi title always starts with "\n" (p2p_matrix.cc:189).
    std::fprintf(out_, "\nEvaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)\n");
  }
  std::fprintf(out_, "   D\\D");
  for (int i = 0; i < n_; ++i) std::fprintf(out_, "%6d ", i);
  std::fprintf(out_, "\n");
  std::fflush(out_);
}

double compat_cell_gbps(const PhaseResult& r) {
  if (r.idle) return 0.0;
  return gbps(r.bytes_per_iter, r.seconds_per_iter);
}

void CompatPrinter::on_phase(const PhaseResult& r) {
  if (r.row < 0) return;
  if (r.col == 0) std::fprintf(out_, "%6d ", r.row);
  std::fprintf(out_, "%6.02f ", compat_cell_gbps(r));
  std::fflush(out_);  // p2p_matrix.cc:180: partial results survive a kill
  if (r.col == n_ - 1) std::fprintf(out_, "\n");
}

// -------------------------------------------------------------- matrices --

std::vector<double> flow_matrix_gbs(const RunRecord& rec, int n) {
  std::vector<double> m(static_cast<size_t>(n) * n, 0.0);
  for (const auto& ph : rec.phases)
    for (const auto& f : ph.flows) m[static_cast<size_t>(f.flow.src) * n + f.flow.dst] = f.gbs;
  return m;
}

std::vector<double> flow_matrix_p50_us(const RunRecord& rec, int n) {
  std::vector<double> m(static_cast<size_t>(n) * n, 0.0);
  for (const auto& ph : rec.phases)
    for (const auto& f : ph.flows) m[static_cast<size_t>(f.flow.src) * n + f.flow.dst] = f.iter_us.p50;
  return m;
}

void print_matrix(FILE* out, const std::string& title, const std::vector<double>& m, int n, const char* fmt,
                  bool blank_diag) {
  std::fprintf(out, "%s\n", title.c_str());
  std::fprintf(out, "  src\\dst");
  for (int j = 0; j < n; ++j) std::fprintf(out, " %9d", j);
  std::fprintf(out, "\n");
  for (int i = 0; i < n; ++i) {
    std::fprintf(out, "  %7d", i);
    for (int j = 0; j < n; ++j) {
      double v = m[static_cast<size_t>(i) * n + j];
      if ((blank_diag && i == j && n > 1) || v == 0.0) {
        std::fprintf(out, " %9s", "-");
      } else {
        std::fprintf(out, " ");
        std::fprintf(out, fmt, v);
      }
    }
    std::fprintf(out, "\n");
  }
}

std::vector<std::string> fabric_findings(const std::vector<double>& uni, const std::vector<double>* bi, int n,
                                         double min_ratio) {
  std::vector<std::string> out;
  std::vector<double> cells;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (i != j && uni[static_cast<size_t>(i) * n + j] > 0) cells.push_back(uni[static_cast<size_t>(i) * n + j]);
  if (cells.size() >= 2) {
    std::sort(cells.begin(), cells.end());
    const size_t h = cells.size() / 2;
    const double med = cells.size() % 2 ? cells[h] : 0.5 * (cells[h - 1] + cells[h]);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        const double v = uni[static_cast<size_t>(i) * n + j];
        if (i != j && v > 0 && v < min_ratio * med)
          out.push_back(strfmt("cell %d->%d %.2f GB/s < %.2f x median %.2f", i, j, v, min_ratio, med));
      }
  }
  if (bi)
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) {
        const double total = (*bi)[static_cast<size_t>(i) * n + j] + (*bi)[static_cast<size_t>(j) * n + i];
        for (const auto& [a, b] : {std::pair<int, int>{i, j}, std::pair<int, int>{j, i}}) {
          const double u = uni[static_cast<size_t>(a) * n + b];
          if (total > 0 && u > 0 && total < u)
            out.push_back(strfmt("pair %d<->%d both directions %.2f GB/s < its uni cell %d->%d %.2f", i, j, total, a,
                                 b, u));
        }
      }
  return out;
}

void print_fabric_check(FILE* out, const std::vector<RunRecord>& runs, int n) {
  if (n < 2) return;
  for (const auto& u : runs) {
    if (u.mode != Mode::Pair || u.dir != Direction::Uni) continue;
    const RunRecord* b = nullptr;
    for (const auto& r : runs)
      if (r.mode == Mode::Pair && r.dir == Direction::Bi && r.bytes == u.bytes) b = &r;
    const auto ug = flow_matrix_gbs(u, n);
    std::vector<double> bg;
    if (b) bg = flow_matrix_gbs(*b, n);
    const auto f = fabric_findings(ug, b ? &bg : nullptr, n);
    std::fprintf(out, "\n== fabric check, pair %s: %s ==\n", format_size(u.bytes).c_str(),
                 f.empty() ? "every link alike (no cell below half the median, bi >= uni)" : "FINDINGS");
    for (const auto& line : f) std::fprintf(out, "  %s\n", line.c_str());
  }
  std::fflush(out);
}

std::vector<RepeatSummary> repeat_summaries(const std::vector<RunRecord>& runs, int n) {
  std::vector<RepeatSummary> out;
  for (const auto& r : runs) {
    double v = 0;
    if (r.mode == Mode::Pair) {
      double sum = 0;
      size_t cells = 0;
      for (const auto& ph : r.phases)
        if (!ph.idle) {
          sum += compat_cell_gbps(ph) / 8.0;
          ++cells;
        }
      v = cells ? sum / static_cast<double>(cells) : 0.0;
    } else {
      v = summarize_offdiag(flow_matrix_gbs(r, n), n).mean;
    }
    auto it = std::find_if(out.begin(), out.end(), [&](const RepeatSummary& s) {
      return s.mode == r.mode && s.dir == r.dir && s.bytes == r.bytes;
    });
    if (it == out.end()) {
      out.push_back(RepeatSummary{r.mode, r.dir, r.bytes, {}, 0, 0, 0});
      it = out.end() - 1;
    }
    it->runs.push_back(v);
  }
  for (auto& s : out) {
    std::vector<double> v = s.runs;
    std::sort(v.begin(), v.end());
    const size_t k = v.size();
    s.median = k % 2 ? v[k / 2] : 0.5 * (v[k / 2 - 1] + v[k / 2]);
    s.min = v.front();
    s.max = v.back();
  }
  return out;
}

void print_repeat_summary(FILE* out, const std::vector<RepeatSummary>& sums) {
  if (sums.empty()) return;
  std::fprintf(out, "\n== repeats: mean cell GB/s of every run (pair: the compat cell / 8, bi both directions) ==\n");
  std::fprintf(out, "  %-10s %-4s %8s  %5s %10s %10s %10s %7s  runs\n", "mode", "dir", "size", "n", "median", "min", "max",
               "spread");
  for (const auto& s : sums) {
    std::string runs;
    for (double v : s.runs) runs += strfmt(" %.2f", v);
    std::fprintf(out, "  %-10s %-4s %8s  %5zu %10.2f %10.2f %10.2f %6.1f%% %s\n", mode_name(s.mode),
                 direction_name(s.dir), format_size(s.bytes).c_str(), s.runs.size(), s.median, s.min, s.max,
                 s.median > 0 ? 100.0 * (s.max - s.min) / s.median : 0.0, runs.c_str());
  }
  std::fflush(out);
}

void print_extended(FILE* out, const RunRecord& rec, int n) {
  std::string head = strfmt("[%s %s | %s x %d | timing=%s warmup=%d%s]", mode_name(rec.mode), direction_name(rec.dir),
                            format_size(rec.bytes).c_str(), rec.cfg.iters, timing_name(rec.cfg.timing), rec.cfg.warmup,
                            rec.cfg.verify ? " verify" : "");
  std::fprintf(out, "\n== %s ==\n", head.c_str());
  bool blank_diag = rec.mode != Mode::Self && n > 1;
  auto gbs = flow_matrix_gbs(rec, n);
  print_matrix(out, "GB/s per direction (1 GB = 1e9 B; row = sender, col = receiver)", gbs, n, "%9.2f", blank_diag);
  MatrixSummary ms = summarize_offdiag(gbs, n);
  std::fprintf(out, "  flow GB/s: min %.2f  mean %.2f  max %.2f  (%zu cells)\n", ms.min, ms.mean, ms.max, ms.cells);
  auto p50 = flow_matrix_p50_us(rec, n);
  print_matrix(out, "p50 per-message time (us, receiver GPU timeline)", p50, n, "%9.1f", blank_diag);

  // Concurrent modes: per-phase aggregate (bisection / ring throughput).
  if (rec.mode != Mode::Pair) {
    for (const auto& ph : rec.phases) {
      std::fprintf(out, "  phase '%s': %zu flows, %.2f GB/s aggregate, %.1f us per iteration\n", ph.label.c_str(),
                   ph.flows.size(), ph.agg_gbs, ph.seconds_per_iter * 1e6);
    }
    if (rec.mode == Mode::AllPairs || rec.mode == Mode::Ring) {
      std::vector<double> egress(static_cast<size_t>(n), 0.0), ingress(static_cast<size_t>(n), 0.0);
      for (const auto& ph : rec.phases)
        for (const auto& f : ph.flows) {
          egress[static_cast<size_t>(f.flow.src)] += static_cast<double>(rec.bytes) / ph.seconds_per_iter / 1e9;
          ingress[static_cast<size_t>(f.flow.dst)] += static_cast<double>(rec.bytes) / ph.seconds_per_iter / 1e9;
        }
      std::fprintf(out, "  per-rank egress/ingress GB/s:");
      for (int r = 0; r < n; ++r) std::fprintf(out, " [%d] %.1f/%.1f", r, egress[static_cast<size_t>(r)], ingress[static_cast<size_t>(r)]);
      std::fprintf(out, "\n");
    }
  }
  uint64_t bad = 0, timed = 0, checked = 0;
  bool verified = false;
  for (const auto& ph : rec.phases) {
    bad += ph.total_mismatches;
    timed += ph.timed_msgs;
    checked += ph.verified_msgs;
    for (const auto& f : ph.flows) verified |= f.verified;
  }
  if (verified)
    std::fprintf(out, "  verification: %s (%llu mismatching words; %llu of %llu timed deliveries checked)\n",
                 bad ? "FAILED" : "OK", static_cast<unsigned long long>(bad), static_cast<unsigned long long>(checked),
                 static_cast<unsigned long long>(timed));
  // Phases whose warmup did not verify and were re-posted with smaller ops.
  for (const auto& ph : rec.phases)
    if (!ph.rechunked_to.empty())
      std::fprintf(out, "  %s: warmup had %llu wrong words; timed as ops of <= %s\n", ph.label.c_str(),
                   static_cast<unsigned long long>(ph.warmup_mismatches), format_size(ph.rechunked_to.back()).c_str());
  std::fflush(out);
}

void print_latency(FILE* out, const std::vector<LatencyResult>& lat, int n) {
  if (lat.empty()) return;
  std::vector<double> m(static_cast<size_t>(n) * n, 0.0);
  std::vector<double> p50s;
  for (const auto& l : lat) {
    m[static_cast<size_t>(l.a) * n + l.b] = l.one_way_us.p50;
    m[static_cast<size_t>(l.b) * n + l.a] = l.one_way_us.p50;
    p50s.push_back(l.one_way_us.p50);
  }
  std::fprintf(out, "\n== latency: %s messages, %s ==\n", format_size(lat[0].bytes).c_str(),
               lat[0].method == "device"      ? "device-initiated ping-pong (one wave per GPU, no host in the loop)"
               : lat[0].method == "preposted" ? "ping-pong pre-posted behind a stream gate (GPU timeline)"
                                              : "ping-pong");
  print_matrix(out, "p50 one-way latency (us)", m, n, "%9.2f", n > 1);
  Summary s = summarize(p50s);
  std::fprintf(out, "  p50 over pairs: min %.2f  median %.2f  max %.2f us\n", s.min, s.p50, s.max);
  std::fflush(out);
}

// ---------------------------------------------------------------- json ----

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20)
          o += strfmt("\\u%04x", c);
        else
          o += c;
    }
  }
  return o;
}

namespace {
std::string num(double v) {
  if (!std::isfinite(v)) return "null";
  return strfmt("%.6g", v);
}
std::string summary_json(const Summary& s) {
  return strfmt("{\"n\":%zu,\"min\":%s,\"p50\":%s,\"p90\":%s,\"p99\":%s,\"max\":%s,\"mean\":%s}", s.n, num(s.min).c_str(),
                num(s.p50).c_str(), num(s.p90).c_str(), num(s.p99).c_str(), num(s.max).c_str(), num(s.mean).c_str());
}
std::string matrix_json(const std::vector<double>& m, int n) {
  std::string o = "[";
  for (int i = 0; i < n; ++i) {
    o += i ? ",[" : "[";
    for (int j = 0; j < n; ++j) o += (j ? "," : "") + num(m[static_cast<size_t>(i) * n + j]);
    o += "]";
  }
  return o + "]";
}
}  // namespace

std::string repeat_summary_json(const RepeatSummary& s) {
  std::string runs = "[";
  for (size_t i = 0; i < s.runs.size(); ++i) runs += (i ? "," : "") + num(s.runs[i]);
  return strfmt("{\"type\":\"repeats\",\"mode\":\"%s\",\"dir\":\"%s\",\"bytes\":%zu,\"runs\":%s],"
                "\"median\":%s,\"min\":%s,\"max\":%s}",
                mode_name(s.mode), direction_name(s.dir), s.bytes, runs.c_str(), num(s.median).c_str(),
                num(s.min).c_str(), num(s.max).c_str());
}

std::string run_to_json(const RunRecord& rec, int n) {
  auto gbs = flow_matrix_gbs(rec, n);
  MatrixSummary ms = summarize_offdiag(gbs, n);
  std::ostringstream o;
  uint64_t timed = 0, checked = 0;
  bool rechunked = false;
  for (const auto& ph : rec.phases) {
    timed += ph.timed_msgs;
    checked += ph.verified_msgs;
    rechunked = rechunked || !ph.rechunked_to.empty();
  }
  o << "{\"type\":\"run\",\"mode\":\"" << mode_name(rec.mode) << "\",\"dir\":\"" << direction_name(rec.dir)
    << "\",\"bytes\":" << rec.bytes << ",\"repeat\":" << rec.repeat << ",\"iters\":" << rec.cfg.iters << ",\"warmup\":" << rec.cfg.warmup
    << ",\"timing\":\"" << timing_name(rec.cfg.timing) << "\",\"nranks\":" << n << ",\"verify\":"
    << (rec.cfg.verify ? "true" : "false") << ",\"timed_msgs\":" << timed << ",\"verified_msgs\":" << checked
    << ",\"verify_coverage\":" << (rec.cfg.verify && timed ? num(static_cast<double>(checked) / static_cast<double>(timed)) : "null")
    << ",\"rechunked\":" << (rechunked ? "true" : "false")
    << ",\"gbs_matrix\":" << matrix_json(gbs, n) << ",\"p50_us_matrix\":" << matrix_json(flow_matrix_p50_us(rec, n), n)
    << ",\"gbs_min\":" << num(ms.min) << ",\"gbs_mean\":" << num(ms.mean) << ",\"gbs_max\":" << num(ms.max)
    << ",\"phases\":[";
  bool first = true;
  for (const auto& ph : rec.phases) {
    if (ph.idle) continue;
    o << (first ? "" : ",") << "{\"label\":\"" << json_escape(ph.label) << "\",\"row\":" << ph.row << ",\"col\":" << ph.col
      << ",\"seconds_per_iter\":" << num(ph.seconds_per_iter) << ",\"agg_gbs\":" << num(ph.agg_gbs)
      << ",\"compat_gbps\":" << num(compat_cell_gbps(ph)) << ",\"wall_seconds\":" << num(ph.wall_seconds)
      << ",\"mismatches\":" << ph.total_mismatches << ",\"generations\":" << ph.generations
      << ",\"timed_msgs\":" << ph.timed_msgs << ",\"verified_msgs\":" << ph.verified_msgs << ",\"op_bytes\":" << ph.op_bytes
      << ",\"warmup_mismatches\":" << ph.warmup_mismatches << ",\"warmup_residual\":" << ph.warmup_residual
      << ",\"rechunked_to\":[";
    for (size_t i = 0; i < ph.rechunked_to.size(); ++i) o << (i ? "," : "") << ph.rechunked_to[i];
    o << "],\"flows\":[";
    for (size_t i = 0; i < ph.flows.size(); ++i) {
      const auto& f = ph.flows[i];
      o << (i ? "," : "") << "{\"src\":" << f.flow.src << ",\"dst\":" << f.flow.dst << ",\"seconds\":" << num(f.seconds)
        << ",\"gbps\":" << num(f.gbps) << ",\"gbs\":" << num(f.gbs) << ",\"iter_us\":" << summary_json(f.iter_us);
      if (f.verified) o << ",\"mismatches\":" << f.mismatches << ",\"checksum\":" << f.checksum;
      o << "}";
    }
    o << "]}";
    first = false;
  }
  o << "]}";
  return o.str();
}

std::string latency_to_json(const std::vector<LatencyResult>& lat, int n) {
  std::ostringstream o;
  o << "{\"type\":\"latency\",\"method\":\"" << (lat.empty() ? "host" : lat[0].method) << "\",\"nranks\":" << n
    << ",\"bytes\":" << (lat.empty() ? 0 : lat[0].bytes) << ",\"pairs\":[";
  for (size_t i = 0; i < lat.size(); ++i)
    o << (i ? "," : "") << "{\"a\":" << lat[i].a << ",\"b\":" << lat[i].b << ",\"one_way_us\":" << summary_json(lat[i].one_way_us) << "}";
  o << "]}";
  return o.str();
}

std::string ring_latency_to_json(const RingLatencyResult& r) {
  return strfmt("{\"type\":\"ring_latency\",\"method\":\"%s\",\"nranks\":%d,\"bytes\":%zu,\"laps\":%d,\"hop_us\":%s,"
                "\"lap_us\":%s}",
                r.method.c_str(), r.nranks, r.bytes, r.laps, summary_json(r.hop_us).c_str(), summary_json(r.lap_us).c_str());
}

void print_ring_latency(FILE* out, const RingLatencyResult& r) {
  std::fprintf(out, "\n== ring token latency: %d rank(s), %s, %s dependent chain 0 -> 1 -> ... -> 0, %d laps ==\n",
               r.nranks, format_size(r.bytes).c_str(),
               r.method == "device" ? "device-initiated (one wave per GPU)" : "host-posted", r.laps);
  std::fprintf(out, "  per hop (lap / %d): p50 %.2f  p99 %.2f us   per lap: p50 %.2f  p99 %.2f us\n", r.nranks,
               r.hop_us.p50, r.hop_us.p99, r.lap_us.p50, r.lap_us.p99);
  std::fflush(out);
}

std::string chrome_trace(const std::vector<RunRecord>& runs, int n) {
  double t0 = 0;
  bool have = false;
  for (const auto& rec : runs)
    for (const auto& ph : rec.phases)
      for (double b : ph.host_begin)
        if (!have || b < t0) {
          t0 = b;
          have = true;
        }
  std::ostringstream o;
  o << "{\"displayTimeUnit\":\"ms\",\"traceEvents\":[";
  bool first = true;
  for (size_t ri = 0; ri < runs.size(); ++ri) {
    const RunRecord& rec = runs[ri];
    std::string run_name = strfmt("%s-%s %s", mode_name(rec.mode), direction_name(rec.dir), format_size(rec.bytes).c_str());
    o << (first ? "" : ",") << "{\"name\":\"process_name\",\"ph\":\"M\",\"pid\":" << ri
      << ",\"args\":{\"name\":\"" << json_escape(run_name) << "\"}}";
    first = false;
    for (const auto& ph : rec.phases) {
      for (int r = 0; r < n && r < static_cast<int>(ph.host_begin.size()); ++r) {
        double b = (ph.host_begin[static_cast<size_t>(r)] - t0) * 1e6;
        double d = (ph.host_end[static_cast<size_t>(r)] - ph.host_begin[static_cast<size_t>(r)]) * 1e6;
        o << ",{\"name\":\"" << json_escape(ph.label) << "\",\"ph\":\"X\",\"pid\":" << ri << ",\"tid\":" << r
          << ",\"ts\":" << num(b) << ",\"dur\":" << num(d) << ",\"args\":{\"gpu_ms\":"
          << num(ph.rank_seconds.size() > static_cast<size_t>(r) ? ph.rank_seconds[static_cast<size_t>(r)] * 1e3 : 0)
          << ",\"agg_gbs\":" << num(ph.agg_gbs) << "}}";
      }
    }
  }
  o << "]}";
  return o.str();
}

std::string run_key(Mode m, Direction d, size_t bytes) {
  return strfmt("%s/%s/%zu", mode_name(m), direction_name(d), bytes);
}

std::string run_key_from_json(const std::string& line) {
  auto field = [&](const char* key) -> std::string {
    std::string k = std::string("\"") + key + "\":";
    auto p = line.find(k);
    if (p == std::string::npos) return "";
    p += k.size();
    if (line[p] == '"') {
      auto e = line.find('"', p + 1);
      return line.substr(p + 1, e - p - 1);
    }
    auto e = line.find_first_of(",}", p);
    return line.substr(p, e - p);
  };
  if (field("type") != "run") return "";
  return field("mode") + "/" + field("dir") + "/" + field("bytes");
}

std::string csv_header() { return "mode,dir,bytes,iters,timing,phase,src,dst,seconds,gbps,gbs,p50_us,p99_us,mismatches\n"; }

std::string run_to_csv(const RunRecord& rec) {
  std::ostringstream o;
  for (const auto& ph : rec.phases)
    for (const auto& f : ph.flows)
      o << mode_name(rec.mode) << ',' << direction_name(rec.dir) << ',' << rec.bytes << ',' << rec.cfg.iters << ','
        << timing_name(rec.cfg.timing) << ",\"" << ph.label << "\"," << f.flow.src << ',' << f.flow.dst << ','
        << num(f.seconds) << ',' << num(f.gbps) << ',' << num(f.gbs) << ',' << num(f.iter_us.p50) << ','
        << num(f.iter_us.p99) << ',' << f.mismatches << '\n';
  return o.str();
}

}  // namespace p2p
