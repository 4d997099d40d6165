// MPI control plane, for `mpirun -n N ./p2p_matrix` (README.md:5 of the
// reference).  Same calls as the reference: MPI_Init_thread requesting
// MPI_THREAD_MULTIPLE (p2p_matrix.cc:105), MPI_Allgather (:70-76), MPI_Bcast
// (:118), MPI_Barrier (:146 etc).  Differences: a lower thread level is a
// warning, not an assert (the program is single-threaded); errors call
// MPI_Abort so the job dies together; MPI_Finalize runs at exit (the
// reference comments it out, :272).
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <thread>

#include "bootstrap.hpp"
#include "common.hpp"

namespace p2p {
namespace {

#define P2P_MPICHECK(cmd)                                                  \
  do {                                                                     \
    int e_ = (cmd);                                                        \
    if (e_ != MPI_SUCCESS) {                                               \
      char s_[MPI_MAX_ERROR_STRING];                                       \
      int l_ = 0;                                                          \
      MPI_Error_string(e_, s_, &l_);                                       \
      P2P_FATAL(strfmt("MPI error in %s: %s", #cmd, s_));                  \
    }                                                                      \
  } while (0)

class MpiBootstrap final : public Bootstrap {
 public:
  MpiBootstrap(int* argc, char*** argv) {
    int inited = 0;
    MPI_Initialized(&inited);
    if (!inited) {
      int provided = 0;
      P2P_MPICHECK(MPI_Init_thread(argc, argv, MPI_THREAD_MULTIPLE, &provided));
      owns_ = true;
      if (provided < MPI_THREAD_MULTIPLE)
        P2P_INFO("MPI provides thread level %d < MPI_THREAD_MULTIPLE; fine for this single-threaded tool", provided);
    }
    P2P_MPICHECK(MPI_Comm_rank(MPI_COMM_WORLD, &rank_));
    P2P_MPICHECK(MPI_Comm_size(MPI_COMM_WORLD, &size_));
  }
  ~MpiBootstrap() override {
    int fin = 0;
    MPI_Finalized(&fin);
    if (owns_ && !fin) MPI_Finalize();
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return "mpi"; }
  void allgather(const void* mine, void* all, size_t bytes) override {
    P2P_CHECK(bytes < (1u << 31), "allgather too large");
    P2P_MPICHECK(MPI_Allgather(mine, static_cast<int>(bytes), MPI_BYTE, all, static_cast<int>(bytes), MPI_BYTE,
                               MPI_COMM_WORLD));
  }
  void bcast(void* buf, size_t bytes, int root) override {
    P2P_MPICHECK(MPI_Bcast(buf, static_cast<int>(bytes), MPI_BYTE, root, MPI_COMM_WORLD));
  }
  void barrier() override { P2P_MPICHECK(MPI_Barrier(MPI_COMM_WORLD)); }
  void abort(int code) override {
    // Give mpirun's I/O forwarding a moment to drain the error this rank just
    // printed: MPI_Abort tears the job down at once, and under load the last
    // stderr lines of the ranks could otherwise be lost.
    std::fflush(nullptr);
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
    MPI_Abort(MPI_COMM_WORLD, code);
  }

 private:
  int rank_ = 0, size_ = 1;
  bool owns_ = false;
};

std::unique_ptr<Bootstrap> make_mpi_bootstrap(int* argc, char*** argv) {
  return std::make_unique<MpiBootstrap>(argc, argv);
}

struct Registrar {
  Registrar() { register_mpi_factory(&make_mpi_bootstrap); }
} g_registrar;

}  // namespace

}  // namespace p2p
