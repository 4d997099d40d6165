// Node topology probe: link type and hop count between every pair of visible
// GPUs (hipExtGetLinkTypeAndHopCount; HSA link types, XGMI = 4) plus peer
// access.  On an MI355X node every pair should read XGMI with one hop: the
// fully connected point-to-point fabric the tournament / all-pairs schedules
// are designed around (docs/DESIGN.md §1).  SURVEY.md §7.2 (bootstrap: xGMI
// topology probe).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "common.hpp"
#include "provenance.hpp"
#include "report.hpp"
#include "topology.hpp"

namespace p2p {

namespace {
const char* link_name(uint32_t t) {
  switch (t) {
    case 0: return "HT";
    case 1: return "QPI";
    case 2: return "PCIE";
    case 3: return "IB";
    case 4: return "XGMI";
    default: return "?";
  }
}
}  // namespace

std::vector<LinkInfo> probe_topology(int* ndev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *ndev = n;
  std::vector<LinkInfo> m(static_cast<size_t>(n) * static_cast<size_t>(n));
  for (int a = 0; a < n; ++a) {
    for (int b = 0; b < n; ++b) {
      LinkInfo& li = m[static_cast<size_t>(a) * n + b];
      if (a == b) {
        li.type = "self";
        continue;
      }
      uint32_t type = 0, hops = 0;
      if (hipExtGetLinkTypeAndHopCount(a, b, &type, &hops) == hipSuccess) {
        li.type = link_name(type);
        li.hops = static_cast<int>(hops);
      } else {
        li.type = "n/a";
      }
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess) li.peer_access = can != 0;
    }
  }
  return m;
}

std::string topology_report() {
  int n = 0;
  auto m = probe_topology(&n);
  std::string out = strfmt("GPU link topology (%d visible; type/hops, * = peer access)\n       ", n);
  for (int b = 0; b < n; ++b) out += strfmt(" %9d", b);
  out += "\n";
  int xgmi = 0, pairs = 0;
  for (int a = 0; a < n; ++a) {
    out += strfmt("  %4d ", a);
    for (int b = 0; b < n; ++b) {
      const LinkInfo& li = m[static_cast<size_t>(a) * n + b];
      if (a == b) {
        out += strfmt(" %9s", "-");
        continue;
      }
      ++pairs;
      xgmi += li.type == "XGMI" && li.hops == 1;
      out += strfmt(" %9s", strfmt("%s/%d%s", li.type.c_str(), li.hops, li.peer_access ? "*" : "").c_str());
    }
    out += "\n";
  }
  if (pairs) out += strfmt("  %d of %d ordered pairs are direct (1-hop) xGMI links\n", xgmi, pairs);
  return out;
}

// Path of the shared object that defines `sym` ("" if unknown).
std::string library_of(const void* sym) {
  Dl_info info{};
  if (dladdr(sym, &info) && info.dli_fname) {
    char real[4096];
    if (realpath(info.dli_fname, real)) return real;
    return info.dli_fname;
  }
  return "";
}

std::string hip_runtime_json() {
  int rt = 0, drv = 0;
  if (hipRuntimeGetVersion(&rt) != hipSuccess) rt = -1;
  if (hipDriverGetVersion(&drv) != hipSuccess) drv = -1;
  return strfmt("{\"runtime_version\":%d,\"driver_version\":%d,\"library\":\"%s\"}", rt, drv,
                json_escape(library_of(reinterpret_cast<const void*>(&hipRuntimeGetVersion))).c_str());
}

std::string device_pci_id(int device) {
  char pci[64] = {0};
  if (hipDeviceGetPCIBusId(pci, sizeof(pci), device) != hipSuccess) return "";
  return pci;
}

std::string gpu_memory_key(int device) {
  char host[256] = {0};
  if (gethostname(host, sizeof(host) - 1) != 0) host[0] = 0;
  const std::string pci = device_pci_id(device);
  return pci.empty() ? strfmt("%s:hip%d", host, device) : std::string(host) + ":" + pci;
}

}  // namespace p2p
