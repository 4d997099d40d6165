// Sample statistics for latency / bandwidth distributions.
//
// The reference only reports a single mean per cell (one wall-clock interval
// divided by 128, p2p_matrix.cc:174-177).  The north star asks for p50
// latency, so every timed cell keeps its per-iteration samples and is
// summarised here.
#pragma once

#include <cstddef>
#include <vector>

namespace p2p {

struct Summary {
  size_t n = 0;
  double min = 0, max = 0, mean = 0, stdev = 0;
  double p50 = 0, p90 = 0, p99 = 0;
};

// Percentile with linear interpolation between closest ranks (numpy's default).
double percentile(std::vector<double> samples, double q);
Summary summarize(const std::vector<double>& samples);

// Off-diagonal min / mean of an N x N row-major matrix (diagonal excluded when
// n > 1; for n == 1 the single cell is used).  Zero cells that were never
// measured are skipped when `skip_zero` is set.
struct MatrixSummary {
  double min = 0, mean = 0, max = 0;
  size_t cells = 0;
};
MatrixSummary summarize_offdiag(const std::vector<double>& m, int n, bool skip_zero = true);

}  // namespace p2p
