#include "provenance.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "bootstrap.hpp"
#include "common.hpp"
#include "report.hpp"
#include "topology.hpp"

extern char** environ;

namespace p2p {

namespace {

bool is_knob(const std::string& name) {
  static const char* kPrefixes[] = {"NCCL_", "RCCL_", "HSA_", "HIP_", "ROCR_", "GPU_", "AMD_", "P2P_", "ROCM_", "MSCCL"};
  for (const char* p : kPrefixes)
    if (name.rfind(p, 0) == 0) return true;
  return name == "CUDA_VISIBLE_DEVICES" || name == "OMP_NUM_THREADS";
}

std::string quoted(const std::string& s) { return "\"" + json_escape(s) + "\""; }

}  // namespace

std::string env_knobs_json() {
  std::vector<std::pair<std::string, std::string>> kv;
  for (char** e = environ; e && *e; ++e) {
    const char* eq = std::strchr(*e, '=');
    if (!eq) continue;
    std::string name(*e, static_cast<size_t>(eq - *e));
    if (is_knob(name)) kv.emplace_back(name, eq + 1);
  }
  std::sort(kv.begin(), kv.end());
  std::string o = "{";
  bool hwq = false;
  for (size_t i = 0; i < kv.size(); ++i) {
    o += (i ? "," : "") + quoted(kv[i].first) + ":" + quoted(kv[i].second);
    hwq = hwq || kv[i].first == "GPU_MAX_HW_QUEUES";
  }
  // HIP's hardware queues per process bound how many communicators' kernels
  // run side by side (docs/DESIGN.md §3); unset means the runtime default, 4.
  if (!hwq) o += std::string(kv.empty() ? "" : ",") + "\"GPU_MAX_HW_QUEUES\":null";
  return o + "}";
}

std::string runtime_json() {
  int n = 0;
  auto links = probe_topology(&n);
  std::string o = "{\"hip\":" + hip_runtime_json() + ",\"rccl\":" + rccl_runtime_json() +
                  strfmt(",\"visible_devices\":%d,\"device_links\":[", n);
  for (int a = 0; a < n; ++a) {
    o += a ? ",[" : "[";
    for (int b = 0; b < n; ++b) {
      const LinkInfo& li = links[static_cast<size_t>(a) * n + b];
      o += (b ? "," : "") + quoted(a == b ? "self" : strfmt("%s/%d", li.type.c_str(), li.hops));
    }
    o += "]";
  }
  return o + "]}";
}

namespace {
struct RankDev {
  int32_t device;
  char pci[60];
  uint64_t host;
};
RankDev my_rank_dev(int device) {
  RankDev mine{};
  mine.device = device;
  std::snprintf(mine.pci, sizeof(mine.pci), "%s", device >= 0 ? device_pci_id(device).c_str() : "");
  mine.host = host_hash(real_hostname());
  return mine;
}
// Link between the GPUs of every two ranks, from this host's probe (ranks on
// other hosts, or ranks without a GPU, read "n/a").  GPUs are matched by PCI
// bus id, not by device index: a launcher that shows every rank only its own
// GPU (HIP_VISIBLE_DEVICES per process) leaves every rank on its device 0, and
// a GPU this process cannot see reads "n/a" rather than "same-gpu".
std::vector<std::string> link_matrix(const std::vector<RankDev>& all, const RankDev& mine) {
  const int n = static_cast<int>(all.size());
  int ndev = 0;
  auto links = probe_topology(&ndev);
  std::vector<std::string> visible_pci(static_cast<size_t>(ndev));
  for (int d = 0; d < ndev; ++d) visible_pci[static_cast<size_t>(d)] = device_pci_id(d);
  // This process's index of rank r's GPU, -1 if it is not visible here.
  auto local_index = [&](const RankDev& r) {
    if (r.device < 0) return -1;
    if (r.pci[0] == '\0') return r.device < ndev ? r.device : -1;
    for (int d = 0; d < ndev; ++d)
      if (visible_pci[static_cast<size_t>(d)] == r.pci) return d;
    return -1;
  };
  std::vector<std::string> out(static_cast<size_t>(n) * static_cast<size_t>(n), "n/a");
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      const RankDev& ra = all[static_cast<size_t>(a)];
      const RankDev& rb = all[static_cast<size_t>(b)];
      if (ra.host != mine.host || rb.host != mine.host || ra.device < 0 || rb.device < 0) continue;
      std::string& cell = out[static_cast<size_t>(a) * n + b];
      if (ra.pci[0] != '\0' && std::strcmp(ra.pci, rb.pci) == 0) {
        cell = "same-gpu";
        continue;
      }
      const int da = local_index(ra), db = local_index(rb);
      if (da < 0 || db < 0) continue;
      if (da == db) {
        cell = "same-gpu";
        continue;
      }
      const LinkInfo& li = links[static_cast<size_t>(da) * ndev + db];
      cell = strfmt("%s/%d", li.type.c_str(), li.hops);
    }
  return out;
}
}  // namespace

std::vector<std::string> rank_link_matrix(Bootstrap& boot, int device) {
  const RankDev mine = my_rank_dev(device);
  return link_matrix(boot.allgather_value(mine), mine);
}

std::string provenance_json(Bootstrap& boot, int device) {
  const RankDev mine = my_rank_dev(device);
  auto all = boot.allgather_value(mine);
  const int n = boot.size();
  std::string o = "{\"type\":\"provenance\",\"runtime\":" + runtime_json() + ",\"env\":" + env_knobs_json() +
                  ",\"rank_devices\":[";
  for (int r = 0; r < n; ++r)
    o += strfmt("%s{\"rank\":%d,\"device\":%d,\"pci\":%s}", r ? "," : "", r, all[static_cast<size_t>(r)].device,
                quoted(all[static_cast<size_t>(r)].pci).c_str());
  const auto lm = link_matrix(all, mine);
  o += "],\"rank_links\":[";
  for (int a = 0; a < n; ++a) {
    o += a ? ",[" : "[";
    for (int b = 0; b < n; ++b) o += (b ? "," : "") + quoted(lm[static_cast<size_t>(a) * n + b]);
    o += "]";
  }
  return o + "]}";
}

}  // namespace p2p
