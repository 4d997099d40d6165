#include "units.hpp"

#include <cctype>
#include <cmath>
#include <sstream>

#include "common.hpp"

namespace p2p {

size_t parse_size(const std::string& raw) {
  std::string t;
  for (char c : raw)
    if (!std::isspace(static_cast<unsigned char>(c))) t.push_back(c);
  P2P_CHECK(!t.empty(), "empty size");
  size_t pos = 0;
  while (pos < t.size() && (std::isdigit(static_cast<unsigned char>(t[pos])) || t[pos] == '.')) ++pos;
  P2P_CHECK(pos > 0, "size must start with a number: '" + raw + "'");
  double value = std::stod(t.substr(0, pos));
  std::string suffix = t.substr(pos);
  for (auto& c : suffix) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  double mult = 1;
  if (suffix.empty() || suffix == "B") {
    mult = 1;
  } else {
    char unit = suffix[0];
    std::string rest = suffix.substr(1);
    P2P_CHECK(rest.empty() || rest == "B" || rest == "IB", "bad size suffix in '" + raw + "'");
    switch (unit) {
      case 'K': mult = 1024.0; break;
      case 'M': mult = 1024.0 * 1024; break;
      case 'G': mult = 1024.0 * 1024 * 1024; break;
      case 'T': mult = 1024.0 * 1024 * 1024 * 1024; break;
      default: P2P_FATAL("bad size unit in '" + raw + "'");
    }
  }
  double bytes = value * mult;
  P2P_CHECK(bytes >= 1 && std::floor(bytes) == bytes, "size must be a positive whole number of bytes: '" + raw + "'");
  return static_cast<size_t>(bytes);
}

std::vector<size_t> parse_size_list(const std::string& text) {
  std::vector<size_t> out;
  std::stringstream ss(text);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    auto c1 = item.find(':');
    if (c1 == std::string::npos) {
      out.push_back(parse_size(item));
      continue;
    }
    auto c2 = item.find(':', c1 + 1);
    size_t lo = parse_size(item.substr(0, c1));
    size_t hi = parse_size(item.substr(c1 + 1, c2 == std::string::npos ? std::string::npos : c2 - c1 - 1));
    size_t factor = 2;
    if (c2 != std::string::npos) factor = static_cast<size_t>(std::stoull(item.substr(c2 + 1)));
    P2P_CHECK(factor >= 2, "sweep factor must be >= 2");
    P2P_CHECK(lo <= hi, "sweep range lo > hi in '" + item + "'");
    for (size_t s = lo; s <= hi; s *= factor) {
      out.push_back(s);
      if (s > hi / factor) break;  // overflow guard
    }
  }
  P2P_CHECK(!out.empty(), "no sizes in '" + text + "'");
  return out;
}

std::string format_size(size_t b) {
  const char* units[] = {"", "K", "M", "G", "T"};
  int u = 0;
  size_t v = b;
  while (u < 4 && v >= 1024 && v % 1024 == 0) {
    v /= 1024;
    ++u;
  }
  return std::to_string(v) + units[u];
}

}  // namespace p2p
