// Framework-free two-rank reproducer for RCCL point-to-point data loss.
//
// Nothing from csrc/: raw HIP + RCCL + MPI.  Two MPI ranks, one ncclSend on
// rank 0 and one ncclRecv on rank 1 per message, each inside its own group
// (the reference's call pattern, /root/reference/p2p_matrix.cc:156-169).  The
// payload is a host-generated word pattern copied in with hipMemcpy, the
// receive buffer is zeroed with hipMemset, and rank 1 copies the result back
// and compares it on the host.  Whatever it reports is RCCL's behaviour, not
// the benchmark engine's.
//
// Round 4 (profiles/r4_node_rehearsal/): with NCCL_NCHANNELS_PER_PEER=8 and
// ranks on RCCL's socket transport (4 p2p channels), p2p_matrix lost exactly
// half of every message at any op size.  This program asks the same of RCCL
// alone.
//
//   mpirun -n 2 rccl_net_repro [--sizes 1M,32M] [--iters I] [--distinct-hosts] [--device D]
//
// --distinct-hosts: each rank sets NCCL_HOSTID to a value of its own before
//   RCCL starts, so two ranks on one GPU are accepted and connected through
//   RCCL's network transport (sockets; NCCL_SOCKET_IFNAME=lo on one box).
// --device D: the GPU of every rank (default: the rank, for a 2-GPU node).
// Rank 1 prints one line of JSON per message size: wrong bytes, the first
// wrong byte range, and how the wrong bytes split between the two halves.
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <rccl/rccl.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIP_OK(x)                                                                                    \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                  \
    }                                                                                                \
  } while (0)
#define NCCL_OK(x)                                                                                   \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) {                                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));        \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                  \
    }                                                                                                \
  } while (0)

namespace {

size_t parse_size(const std::string& s) {
  char* end = nullptr;
  errno = 0;
  const unsigned long long v = std::strtoull(s.c_str(), &end, 10);
  if (errno || end == s.c_str()) {
    std::fprintf(stderr, "bad size '%s'\n", s.c_str());
    std::exit(2);
  }
  const char u = *end;
  return static_cast<size_t>(v) << (u == 'K' ? 10 : u == 'M' ? 20 : u == 'G' ? 30 : 0);
}

// Word w of message `iter`: distinct per word and per iteration, never zero.
uint32_t pattern(size_t w, int iter) { return static_cast<uint32_t>(w * 2654435761u) ^ (0x9E3779B9u + iter) ^ 1u; }

}  // namespace

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, world = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &world);
  std::vector<size_t> sizes;
  int iters = 2, device = -1;
  bool distinct = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "%s needs a value\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--sizes") {
      const std::string list = next();
      for (size_t p = 0; p <= list.size();) {
        size_t q = list.find(',', p);
        if (q == std::string::npos) q = list.size();
        if (q > p) sizes.push_back(parse_size(list.substr(p, q - p)));
        p = q + 1;
      }
    } else if (a == "--iters") {
      iters = std::atoi(next().c_str());
    } else if (a == "--device") {
      device = std::atoi(next().c_str());
    } else if (a == "--distinct-hosts") {
      distinct = true;
    } else {
      if (rank == 0) std::fprintf(stderr, "usage: mpirun -n 2 %s [--sizes a,b] [--iters I] [--distinct-hosts] [--device D]\n", argv[0]);
      MPI_Finalize();
      return 2;
    }
  }
  if (world != 2) {
    if (rank == 0) std::fprintf(stderr, "needs exactly 2 ranks (mpirun -n 2)\n");
    MPI_Finalize();
    return 2;
  }
  if (sizes.empty()) sizes = {1u << 20, 32u << 20};
  if (distinct) setenv("NCCL_HOSTID", ("rccl-net-repro-host-" + std::to_string(rank)).c_str(), 1);
  HIP_OK(hipSetDevice(device >= 0 ? device : rank));

  ncclUniqueId id;
  if (rank == 0) NCCL_OK(ncclGetUniqueId(&id));
  MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, MPI_COMM_WORLD);
  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, 2, id, rank));
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  int ver = 0;
  NCCL_OK(ncclGetVersion(&ver));
  if (rank == 1) {
    const char* pp = std::getenv("NCCL_NCHANNELS_PER_PEER");
    std::printf("{\"rccl_version\":%d,\"distinct_hosts\":%s,\"NCCL_NCHANNELS_PER_PEER\":\"%s\",\"iters\":%d}\n", ver,
                distinct ? "true" : "false", pp ? pp : "", iters);
    std::fflush(stdout);
  }

  int failed = 0;
  for (const size_t bytes : sizes) {
    const size_t words = bytes / 4;
    void* buf = nullptr;
    HIP_OK(hipMalloc(&buf, bytes));
    std::vector<uint32_t> host(words);
    unsigned long long wrong = 0, wrong_first_half = 0, first_bad = ~0ull, last_bad = 0;
    for (int it = 0; it < iters; ++it) {
      if (rank == 0) {
        for (size_t w = 0; w < words; ++w) host[w] = pattern(w, it);
        HIP_OK(hipMemcpy(buf, host.data(), bytes, hipMemcpyHostToDevice));
      } else {
        HIP_OK(hipMemset(buf, 0, bytes));
      }
      HIP_OK(hipDeviceSynchronize());
      MPI_Barrier(MPI_COMM_WORLD);
      NCCL_OK(ncclGroupStart());
      if (rank == 0)
        NCCL_OK(ncclSend(buf, bytes, ncclInt8, 1, comm, stream));
      else
        NCCL_OK(ncclRecv(buf, bytes, ncclInt8, 0, comm, stream));
      NCCL_OK(ncclGroupEnd());
      HIP_OK(hipStreamSynchronize(stream));
      if (rank == 1) {
        HIP_OK(hipMemcpy(host.data(), buf, bytes, hipMemcpyDeviceToHost));
        for (size_t w = 0; w < words; ++w)
          if (host[w] != pattern(w, it)) {
            wrong += 4;
            wrong_first_half += w < words / 2 ? 4 : 0;
            if (w * 4 < first_bad) first_bad = w * 4;
            last_bad = w * 4 + 4;
          }
      }
      MPI_Barrier(MPI_COMM_WORLD);
    }
    if (rank == 1) {
      std::printf("{\"bytes\":%zu,\"iters\":%d,\"wrong_bytes\":%llu,\"wrong_fraction\":%.4f,\"wrong_in_first_half\":%llu,"
                  "\"first_bad\":%lld,\"last_bad_end\":%llu}\n",
                  bytes, iters, wrong, static_cast<double>(wrong) / (static_cast<double>(bytes) * iters),
                  wrong_first_half, wrong ? static_cast<long long>(first_bad) : -1LL, last_bad);
      std::fflush(stdout);
      failed |= wrong != 0;
    }
    HIP_OK(hipFree(buf));
  }
  MPI_Allreduce(MPI_IN_PLACE, &failed, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
  NCCL_OK(ncclCommDestroy(comm));
  HIP_OK(hipStreamDestroy(stream));
  MPI_Finalize();
  return failed ? 3 : 0;
}
