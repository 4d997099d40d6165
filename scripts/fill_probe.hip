// Probe: what limits the PRNG fill kernel on gfx950?  Times store-only
// variants of the same grid shape at 1 GiB (hipEvents, 20 reps each):
//   const       16 B/lane stores of a constant          (store roof)
//   fmix        the production generator (4 x fmix32 per 16 B)
//   mul1        one multiply per word: (lo * golden) ^ key
//   fmix-u8     production generator, 8 stores in flight per lane
//   fmix-g16    production generator, 16 blocks per CU
// Build: hipcc --offload-arch=gfx950 -O3 scripts/fill_probe.hip -o build/fill_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

template <int MODE, int UNROLL>
__global__ __launch_bounds__(256) void probe(uint4* __restrict__ p, uint64_t nvec, uint32_t key) {
  const uint64_t tile = 256ull * UNROLL;
  for (uint64_t base = blockIdx.x * tile; base < nvec; base += static_cast<uint64_t>(gridDim.x) * tile) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + u * 256ull + threadIdx.x;
      if (i >= nvec) continue;
      const uint32_t lo = static_cast<uint32_t>(i * 4);
      uint4 v;
      if (MODE == 0) {
        v = make_uint4(key, key, key, key);
      } else if (MODE == 1) {
        v = make_uint4(fmix32((lo * 0x9E3779B1u) ^ key), fmix32(((lo + 1) * 0x9E3779B1u) ^ key),
                       fmix32(((lo + 2) * 0x9E3779B1u) ^ key), fmix32(((lo + 3) * 0x9E3779B1u) ^ key));
      } else {
        v = make_uint4((lo * 0x9E3779B1u) ^ key, ((lo + 1) * 0x9E3779B1u) ^ key, ((lo + 2) * 0x9E3779B1u) ^ key,
                       ((lo + 3) * 0x9E3779B1u) ^ key);
      }
      p[i] = v;
    }
  }
}

// One contiguous chunk of UNROLL x 4 KiB per block, no grid-stride loop.
template <int MODE, int UNROLL>
__global__ __launch_bounds__(256) void probe_chunk(uint4* __restrict__ p, uint64_t nvec, uint32_t key) {
  const uint64_t base = blockIdx.x * 256ull * UNROLL;
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const uint64_t i = base + u * 256ull + threadIdx.x;
    if (i >= nvec) continue;
    const uint32_t lo = static_cast<uint32_t>(i * 4);
    uint4 v = MODE == 0 ? make_uint4(key, key, key, key)
                        : make_uint4(fmix32((lo * 0x9E3779B1u) ^ key), fmix32(((lo + 1) * 0x9E3779B1u) ^ key),
                                     fmix32(((lo + 2) * 0x9E3779B1u) ^ key), fmix32(((lo + 3) * 0x9E3779B1u) ^ key));
    p[i] = v;
  }
}

// Read probe: sum of words, grid-stride (capped grid) vs one chunk per block.
template <bool CHUNK, int UNROLL>
__global__ __launch_bounds__(256) void read_probe(const uint4* __restrict__ p, uint64_t nvec, unsigned long long* out) {
  unsigned long long s = 0;
  const uint64_t tile = 256ull * UNROLL;
  const uint64_t start = blockIdx.x * tile;
  const uint64_t stride = CHUNK ? nvec : static_cast<uint64_t>(gridDim.x) * tile;
  for (uint64_t base = start; base < nvec; base += stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + u * 256ull + threadIdx.x;
      v[u] = i < nvec ? p[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) s += static_cast<unsigned long long>(v[u].x) + v[u].y + v[u].z + v[u].w;
  }
  if (s == 0x1234567) atomicAdd(out, s);  // keep the loads alive
}

template <bool CHUNK, int UNROLL>
double run_read(const uint4* p, uint64_t nvec, int grid, unsigned long long* out) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  read_probe<CHUNK, UNROLL><<<grid, 256>>>(p, nvec, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 20; ++r) read_probe<CHUNK, UNROLL><<<grid, 256>>>(p, nvec, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return static_cast<double>(nvec) * 16 * 20 / (ms * 1e-3) / 1e12;
}

template <int MODE, int UNROLL>
double run_chunk(uint4* p, uint64_t nvec) {
  const int grid = static_cast<int>((nvec + 256ull * UNROLL - 1) / (256ull * UNROLL));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  probe_chunk<MODE, UNROLL><<<grid, 256>>>(p, nvec, 7);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 20; ++r) probe_chunk<MODE, UNROLL><<<grid, 256>>>(p, nvec, 7 + r);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return static_cast<double>(nvec) * 16 * 20 / (ms * 1e-3) / 1e12;
}

template <int MODE, int UNROLL>
double run(uint4* p, uint64_t nvec, int grid) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  probe<MODE, UNROLL><<<grid, 256>>>(p, nvec, 7);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 20; ++r) probe<MODE, UNROLL><<<grid, 256>>>(p, nvec, 7 + r);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return static_cast<double>(nvec) * 16 * 20 / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? std::atoll(argv[1]) : 1) << 30;
  uint4* p = nullptr;
  CHECK(hipMalloc(&p, bytes));
  const uint64_t nvec = bytes / 16;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("const     g8  u4: %.2f TB/s\n", run<0, 4>(p, nvec, cus * 8));
  std::printf("fmix      g8  u4: %.2f TB/s\n", run<1, 4>(p, nvec, cus * 8));
  std::printf("mul1      g8  u4: %.2f TB/s\n", run<2, 4>(p, nvec, cus * 8));
  std::printf("fmix      g8  u8: %.2f TB/s\n", run<1, 8>(p, nvec, cus * 8));
  std::printf("fmix      g16 u4: %.2f TB/s\n", run<1, 4>(p, nvec, cus * 16));
  std::printf("fmix      g4  u4: %.2f TB/s\n", run<1, 4>(p, nvec, cus * 4));
  std::printf("const     g16 u4: %.2f TB/s\n", run<0, 4>(p, nvec, cus * 16));
  std::printf("const     g32 u1: %.2f TB/s\n", run<0, 1>(p, nvec, cus * 32));
  std::printf("fmix      g32 u1: %.2f TB/s\n", run<1, 1>(p, nvec, cus * 32));
  std::printf("fmix  full-grid u1: %.2f TB/s\n", run<1, 1>(p, nvec, static_cast<int>(nvec / 256)));
  std::printf("const full-grid u1: %.2f TB/s\n", run<0, 1>(p, nvec, static_cast<int>(nvec / 256)));
  std::printf("fmix  chunk u2: %.2f TB/s\n", run_chunk<1, 2>(p, nvec));
  std::printf("fmix  chunk u4: %.2f TB/s\n", run_chunk<1, 4>(p, nvec));
  std::printf("fmix  chunk u8: %.2f TB/s\n", run_chunk<1, 8>(p, nvec));
  std::printf("const chunk u4: %.2f TB/s\n", run_chunk<0, 4>(p, nvec));
  unsigned long long* out = nullptr;
  CHECK(hipMalloc(&out, 8));
  std::printf("read  stride g8 u4: %.2f TB/s\n", run_read<false, 4>(p, nvec, cus * 8, out));
  std::printf("read  stride g16 u4: %.2f TB/s\n", run_read<false, 4>(p, nvec, cus * 16, out));
  std::printf("read  chunk u1: %.2f TB/s\n", run_read<true, 1>(p, nvec, static_cast<int>(nvec / 256), out));
  std::printf("read  chunk u4: %.2f TB/s\n", run_read<true, 4>(p, nvec, static_cast<int>(nvec / 1024), out));
  std::printf("read  chunk u8: %.2f TB/s\n", run_read<true, 8>(p, nvec, static_cast<int>(nvec / 2048), out));
  CHECK(hipFree(out));
  CHECK(hipFree(p));
  return 0;
}
