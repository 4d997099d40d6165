// Host-only builds (CPU test binaries) link this instead of
// transport_rccl.cpp + transport_ipc.cpp + kernels.hip: the GPU transports
// are unavailable there.
#include "common.hpp"
#include "transport.hpp"

namespace p2p {

std::unique_ptr<Transport> make_rccl_transport(Bootstrap&, const TransportOptions&) {
  P2P_FATAL("this binary was built without HIP/RCCL; use --transport host");
}

std::unique_ptr<Transport> make_ipc_transport(Bootstrap&, const TransportOptions&) {
  P2P_FATAL("this binary was built without HIP; use --transport host");
}

bool rccl_transport_available() { return false; }

}  // namespace p2p

// Topology probe stubs for host-only builds.
#include "topology.hpp"

namespace p2p {
std::vector<LinkInfo> probe_topology(int* ndev) {
  *ndev = 0;
  return {};
}
std::string topology_report() { return "GPU link topology: not available in this host-only build\n"; }
}  // namespace p2p

// Provenance stubs for host-only builds: no GPU runtime in the process.
#include "provenance.hpp"

namespace p2p {
std::string hip_runtime_json() { return "null"; }
std::string rccl_runtime_json() { return "null"; }
std::string device_pci_id(int) { return ""; }
}  // namespace p2p
