// Control plane: rank identity, barriers, small all-gathers and broadcasts.
//
// The reference's control plane is MPI only (MPI_Init_thread, MPI_Allgather,
// MPI_Bcast of the ncclUniqueId, MPI_Barrier — /root/reference/p2p_matrix.cc:
// 70-76, 105-118, 146, 173, 271).  Here it is an interface with three
// implementations so the same engine runs under
//   * `mpirun -n N ./p2p_matrix`        (MpiBootstrap, reference-compatible),
//   * `torchrun` / any RANK+WORLD_SIZE+MASTER_ADDR launcher, including the
//     Python bench (TcpBootstrap: a native star over TCP, no MPI needed),
//   * a single process                  (LocalBootstrap).
// The data plane (RCCL over xGMI) never goes through this interface; it only
// carries the 128-byte unique id, timing results and barriers.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace p2p {

class Bootstrap {
 public:
  virtual ~Bootstrap() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // `all` receives size() * bytes, rank-major.
  virtual void allgather(const void* mine, void* all, size_t bytes) = 0;
  virtual void bcast(void* buf, size_t bytes, int root) = 0;
  virtual void barrier() = 0;
  // Tear the job down from this rank (called from the fatal() hook).
  virtual void abort(int code) = 0;
  virtual std::string name() const = 0;
  // Seconds any one receive may wait (TCP); shrunk as a deadline approaches.
  virtual void set_timeout(double /*seconds*/) {}

  template <class T>
  std::vector<T> allgather_value(const T& v) {
    std::vector<T> out(static_cast<size_t>(size()));
    allgather(&v, out.data(), sizeof(T));
    return out;
  }
  // Strings of any length, one per rank.
  std::vector<std::string> allgather_string(const std::string& mine) {
    const auto lens = allgather_value(static_cast<uint64_t>(mine.size()));
    uint64_t most = 0;
    for (uint64_t l : lens) most = l > most ? l : most;
    std::string padded = mine;
    padded.resize(static_cast<size_t>(most) + 1, '\0');
    std::string all(padded.size() * lens.size(), '\0');
    allgather(padded.data(), &all[0], padded.size());
    std::vector<std::string> out;
    for (size_t r = 0; r < lens.size(); ++r) out.push_back(all.substr(r * padded.size(), static_cast<size_t>(lens[r])));
    return out;
  }
  template <class T>
  std::vector<T> allgather_vector(const std::vector<T>& v) {  // equal lengths on all ranks
    std::vector<T> out(v.size() * static_cast<size_t>(size()));
    allgather(v.data(), out.data(), v.size() * sizeof(T));
    return out;
  }
  double allreduce_max(double v);
  double allreduce_sum(double v);
  uint64_t allreduce_sum_u64(uint64_t v);
};

std::unique_ptr<Bootstrap> make_local_bootstrap();

// A listening socket, created before the peers know the port (port 0 picks an
// ephemeral one; the Python bench shares it through torch.distributed).
class TcpListener {
 public:
  explicit TcpListener(int port = 0, const std::string& bind_addr = "0.0.0.0");
  ~TcpListener();
  TcpListener(const TcpListener&) = delete;
  TcpListener& operator=(const TcpListener&) = delete;
  int port() const { return port_; }
  int fd() const { return fd_; }
  int release();  // hand the fd over to the bootstrap

 private:
  int fd_ = -1;
  int port_ = 0;
};

// Star topology rooted at rank 0.  Rank 0 accepts size-1 connections on
// `port` (or on `listener` if given); others connect to host:port, retrying
// until `timeout_s`.  Every receive is bounded by `timeout_s` so a dead peer
// turns into an error instead of a hang.
std::unique_ptr<Bootstrap> make_tcp_bootstrap(int rank, int size, const std::string& host, int port,
                                              double timeout_s = 600.0, TcpListener* listener = nullptr);

// MPI support is linked in only by the executable: bootstrap_mpi.cpp
// registers its factory at static-initialisation time.
using MpiFactory = std::unique_ptr<Bootstrap> (*)(int* argc, char*** argv);
void register_mpi_factory(MpiFactory f);
bool mpi_available();
bool mpi_launch_detected();  // PMI_RANK / OMPI_COMM_WORLD_RANK / PMIX_RANK in the env

// Picks MPI when launched by mpirun, TCP when RANK/WORLD_SIZE are set (the
// TCP port is P2P_BOOTSTRAP_PORT or MASTER_PORT+1, because torchrun's own
// store already owns MASTER_PORT), else local.  `kind` forces one of
// "auto", "mpi", "env", "local".
std::unique_ptr<Bootstrap> make_bootstrap(const std::string& kind, int* argc, char*** argv);

// ---- host topology (reference: p2p_matrix.cc:44-100) ----------------------

// DJB2a-style string hash, bit-compatible with getHostHash (p2p_matrix.cc:44-51).
uint64_t host_hash(const std::string& s);
// gethostname() truncated at the first '.' (p2p_matrix.cc:53-61).
std::string short_hostname();
// Full gethostname() result, ignoring the P2P_HOSTNAME override (used for
// socket addressing).
std::string real_hostname();

struct Placement {
  bool ok = false;
  std::string error;
  int num_hosts = 0;
  int ranks_per_host = 0;
  int host_index = 0;
  int local_rank = 0;  // == GPU index on this host
};

// Pure logic of check_process_placement_policy (p2p_matrix.cc:63-100): ranks
// must come in contiguous equal-sized blocks per host; local rank = rank %
// ranks_per_host.
Placement compute_placement(const std::vector<uint64_t>& hashes, int rank);
Placement check_placement(Bootstrap& boot);

}  // namespace p2p
