// Sizes and bandwidth units.
//
// The reference hard-codes `const int msg_size = 32*1024*1024` (p2p_matrix.cc:124),
// which caps messages below 2 GiB.  Everything here is size_t so sweeps can go
// to multi-GiB buffers sized for 288 GB of HBM3E per MI355X.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace p2p {

// "4096", "4K", "4KiB", "32M", "1G", "1.5G", "256MB" (binary multiples: K=2^10).
size_t parse_size(const std::string& text);

// "32M" -> {32M};  "4K:4G" -> powers of two 4K..4G;  "4K:64K:4" -> factor 4;
// "4K,1M,3M" -> explicit list.  Combinations are comma separated.
std::vector<size_t> parse_size_list(const std::string& text);

// 33554432 -> "32M", 4096 -> "4K", 1000 -> "1000".
std::string format_size(size_t bytes);

// Reference units: Gbps = bytes*8/seconds/1e9 (p2p_matrix.cc:177).  GB/s is
// decimal (1e9 bytes/s) so GB/s == Gbps/8.
inline double gbps(double bytes, double seconds) { return seconds > 0 ? bytes * 8.0 / seconds / 1e9 : 0.0; }
inline double gbytes_per_s(double bytes, double seconds) { return seconds > 0 ? bytes / seconds / 1e9 : 0.0; }

}  // namespace p2p
