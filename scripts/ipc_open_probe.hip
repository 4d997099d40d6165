// Does hipIpcOpenMemHandle of a large block return, and how fast?  One
// process exports a hipMalloc block of SIZE bytes and waits; another opens
// it (same GPU), touches both ends with a memset, and reports the time.
//   build/ipc_open_probe export <bytes> <handle-file>   (waits until the file is removed)
//   build/ipc_open_probe open <handle-file>
//   build/ipc_open_probe mesh <n> <rank> <bytes> <dir>   (n processes export one block each,
//                                                         then every one opens all the others)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unistd.h>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 3) return 1;
  if (hipSetDevice(0) != hipSuccess) return 2;
  if (!std::strcmp(argv[1], "mesh")) {
    const int n = std::atoi(argv[2]), rank = std::atoi(argv[3]);
    const size_t size = std::strtoull(argv[4], nullptr, 10);
    const std::string dir = argv[5];
    void* p = nullptr;
    if (hipMalloc(&p, size) != hipSuccess) return 3;
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) != hipSuccess) return 4;
    auto path = [&](const char* what, int r) { return dir + "/" + what + std::to_string(r); };
    std::string tmp = path("h", rank) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    std::fwrite(&h, sizeof(h), 1, f);
    std::fclose(f);
    std::rename(tmp.c_str(), path("h", rank).c_str());
    // P2P_PROBE_SERIAL=1: one process opens at a time (token files t<rank>).
    const bool serial = std::getenv("P2P_PROBE_SERIAL") != nullptr;
    if (serial && rank > 0)
      while (access(path("t", rank).c_str(), F_OK) != 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    for (int k = 1; k < n; ++k) {
      const int r = (rank + k) % n;
      while (access(path("h", r).c_str(), F_OK) != 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
      hipIpcMemHandle_t hr;
      FILE* g = std::fopen(path("h", r).c_str(), "rb");
      if (std::fread(&hr, sizeof(hr), 1, g) != 1) return 5;
      std::fclose(g);
      double t0 = now();
      void* q = nullptr;
      hipError_t e = hipIpcOpenMemHandle(&q, hr, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) return 6;
      // Touch the first and the last page of the peer's block through the mapping.
      hipError_t m1 = hipMemset(q, 1, 4096);
      hipError_t m2 = hipMemset(static_cast<char*>(q) + size - 4096, 1, 4096);
      hipError_t m3 = hipDeviceSynchronize();
      std::printf("rank %d: open rank %d's %zu B: %s in %.3f s, touch %s/%s/%s\n", rank, r, size, hipGetErrorString(e),
                  now() - t0, hipGetErrorString(m1), hipGetErrorString(m2), hipGetErrorString(m3));
      std::fflush(stdout);
    }
    if (serial) std::fclose(std::fopen(path("t", rank + 1).c_str(), "wb"));
    FILE* d = std::fopen(path("d", rank).c_str(), "wb");
    std::fclose(d);
    for (int r = 0; r < n; ++r)
      while (access(path("d", r).c_str(), F_OK) != 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    std::printf("rank %d: all opened\n", rank);
    return 0;
  }
  if (!std::strcmp(argv[1], "export")) {
    const size_t size = std::strtoull(argv[2], nullptr, 10);
    void* p = nullptr;
    if (hipMalloc(&p, size) != hipSuccess) return 3;
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) != hipSuccess) return 4;
    std::string tmp = std::string(argv[3]) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    std::fwrite(&h, sizeof(h), 1, f);
    std::fwrite(&size, sizeof(size), 1, f);
    std::fclose(f);
    std::rename(tmp.c_str(), argv[3]);
    while (access(argv[3], F_OK) == 0) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    (void)hipFree(p);
    return 0;
  }
  hipIpcMemHandle_t h;
  size_t size = 0;
  while (access(argv[2], F_OK) != 0) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  FILE* f = std::fopen(argv[2], "rb");
  if (std::fread(&h, sizeof(h), 1, f) != 1 || std::fread(&size, sizeof(size), 1, f) != 1) return 5;
  std::fclose(f);
  double t0 = now();
  void* q = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess);
  double t1 = now();
  if (e != hipSuccess) {
    std::printf("open %zu B failed: %s\n", size, hipGetErrorString(e));
    std::remove(argv[2]);
    return 6;
  }
  (void)hipMemset(q, 1, 4096);
  (void)hipMemset(static_cast<char*>(q) + size - 4096, 1, 4096);
  (void)hipDeviceSynchronize();
  double t2 = now();
  (void)hipIpcCloseMemHandle(q);
  std::printf("open %zu B (%.2f GiB): %.3f s, touch %.3f s\n", size, size / 1073741824.0, t1 - t0, t2 - t1);
  std::remove(argv[2]);
  return 0;
}
