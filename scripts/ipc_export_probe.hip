// How often does hipIpcGetMemHandle refuse a fresh hipMalloc block?  Each
// process allocates, exports and frees `iters` blocks of 2 MiB .. 256 MiB
// (optionally keeping `keep` of them alive) and prints how many exports
// failed, with the first error string.  Run several copies at once to
// reproduce the multi-process case:
//   hipcc --offload-arch=gfx950 -O2 scripts/ipc_export_probe.hip -o build/ipc_export_probe
//   for i in $(seq 8); do ./build/ipc_export_probe 500 16 & done; wait
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <deque>
#include <unistd.h>

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 500;
  const size_t keep = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 16;
  if (hipSetDevice(0) != hipSuccess) return 2;
  std::deque<void*> live;
  int fails = 0, first_fail = -1;
  const char* first_err = "";
  unsigned seed = static_cast<unsigned>(getpid());
  for (int i = 0; i < iters; ++i) {
    seed = seed * 1664525u + 1013904223u;
    const size_t size = (size_t{2} << 20) << (seed >> 29);  // 2 MiB .. 256 MiB
    void* p = nullptr;
    if (hipMalloc(&p, size) != hipSuccess) {
      std::printf("pid %d: hipMalloc(%zu) failed at %d\n", getpid(), size, i);
      return 1;
    }
    hipIpcMemHandle_t h;
    hipError_t e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) {
      if (!fails++) {
        first_fail = i;
        first_err = hipGetErrorString(e);
      }
      (void)hipGetLastError();
    }
    live.push_back(p);
    while (live.size() > keep) {
      (void)hipFree(live.front());
      live.pop_front();
    }
  }
  for (void* p : live) (void)hipFree(p);
  std::printf("pid %d: %d / %d exports refused (first at %d: %s)\n", getpid(), fails, iters, first_fail, first_err);
  return 0;
}
