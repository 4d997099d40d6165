#include "stats.hpp"

#include <algorithm>
#include <cmath>
#include <limits>

namespace p2p {

double percentile(std::vector<double> s, double q) {
  if (s.empty()) return 0.0;
  std::sort(s.begin(), s.end());
  if (q <= 0) return s.front();
  if (q >= 100) return s.back();
  double pos = q / 100.0 * static_cast<double>(s.size() - 1);
  size_t lo = static_cast<size_t>(std::floor(pos));
  size_t hi = std::min(lo + 1, s.size() - 1);
  double frac = pos - static_cast<double>(lo);
  return s[lo] + (s[hi] - s[lo]) * frac;
}

Summary summarize(const std::vector<double>& samples) {
  Summary r;
  r.n = samples.size();
  if (samples.empty()) return r;
  std::vector<double> s(samples);
  std::sort(s.begin(), s.end());
  r.min = s.front();
  r.max = s.back();
  double sum = 0;
  for (double v : s) sum += v;
  r.mean = sum / static_cast<double>(s.size());
  double var = 0;
  for (double v : s) var += (v - r.mean) * (v - r.mean);
  r.stdev = s.size() > 1 ? std::sqrt(var / static_cast<double>(s.size() - 1)) : 0.0;
  r.p50 = percentile(s, 50);
  r.p90 = percentile(s, 90);
  r.p99 = percentile(s, 99);
  return r;
}

MatrixSummary summarize_offdiag(const std::vector<double>& m, int n, bool skip_zero) {
  MatrixSummary r;
  double mn = std::numeric_limits<double>::infinity(), mx = -mn, sum = 0;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n; ++j) {
      if (n > 1 && i == j) continue;
      double v = m[static_cast<size_t>(i) * n + j];
      if (skip_zero && v == 0.0) continue;
      mn = std::min(mn, v);
      mx = std::max(mx, v);
      sum += v;
      ++r.cells;
    }
  }
  if (r.cells) {
    r.min = mn;
    r.max = mx;
    r.mean = sum / static_cast<double>(r.cells);
  }
  return r;
}

}  // namespace p2p
