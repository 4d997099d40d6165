// Provenance: what produced a number.
//
// The reference sets no RCCL/NCCL knob and inherits whatever NCCL_* the shell
// has, invisibly ("sweep and record them; never hard-code
// them silently").  Every result this framework writes -- the bench JSON line
// and the `p2p_matrix --json` file -- therefore carries:
//   * the environment knobs (NCCL_* / RCCL_* / HSA_* / HIP_* / GPU_* ...),
//     including GPU_MAX_HW_QUEUES (null = HIP's default of 4);
//   * the HIP runtime and RCCL library actually loaded: version and path
//     (dladdr on an entry point), so a number can be tied to one library;
//   * each rank's GPU (index, PCI bus id) and the link type / hop count
//     between every pair of ranks (hipExtGetLinkTypeAndHopCount).
#pragma once

#include <string>
#include <vector>

namespace p2p {

class Bootstrap;

// JSON object of every environment variable that can change P2P behaviour.
std::string env_knobs_json();

// JSON object describing the GPU runtime of this process: HIP runtime /
// driver versions and library, RCCL version and library, visible devices and
// their link matrix.  Host-only builds report {"gpu": false}.
std::string runtime_json();

// Collective: runtime_json() + env_knobs_json() + every rank's device and the
// rank-to-rank link types (device = this rank's GPU index, -1 for none).
std::string provenance_json(Bootstrap& boot, int device);

// Collective: the link type between every two ranks' GPUs (row-major n x n,
// "XGMI/1", "PCIE/2", "same-gpu", "n/a"), as in provenance_json's rank_links.
std::vector<std::string> rank_link_matrix(Bootstrap& boot, int device);

// ---- pieces implemented per build (GPU: topology.cpp / transport_rccl.cpp;
// host-only: transport_rccl_stub.cpp) ----
std::string hip_runtime_json();
std::string rccl_runtime_json();
std::string device_pci_id(int device);  // "" when unknown
// "<hostname>:<PCI bus id>" of a local GPU (Transport::device_key).
std::string gpu_memory_key(int device);

}  // namespace p2p
