// GPU link topology probe (HIP).  See topology.cpp.
#pragma once

#include <string>
#include <vector>

namespace p2p {

struct LinkInfo {
  std::string type = "?";  // XGMI, PCIE, ... ("self" on the diagonal)
  int hops = 0;
  bool peer_access = false;
};

// Row-major ndev x ndev matrix over the GPUs visible to this process.
std::vector<LinkInfo> probe_topology(int* ndev);
std::string topology_report();

// Path of the shared object that defines `sym` (dladdr; "" if unknown).
std::string library_of(const void* sym);

}  // namespace p2p
