// Probe: can a device-local copy on gfx950 beat the production copy kernel
// (one 16 B load + store per lane, one 4 KiB chunk per workgroup, full grid,
// 3.14 TB/s of payload)?  Times variants of the same copy at 1 and 4 GiB
// (hipEvents, 20 reps each, payload bytes counted once):
//   plain        d[i] = s[i]                                 (production form)
//   nt-ld        nontemporal load, plain store
//   nt-st        plain load, nontemporal store
//   nt-both      nontemporal load and store
//   u2 / u4      2 / 4 x 16 B per lane (8 / 16 KiB per workgroup), nt both
//   u2-plain     2 x 16 B per lane, plain
//   stride16     grid-stride over 16 workgroups per CU, 4 in flight per lane
// Build: hipcc --offload-arch=gfx950 -O3 scripts/copy_probe.hip -o build/copy_probe
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_chunk(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t nvec) {
  const uint64_t base = blockIdx.x * 256ull * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + u * 256ull;
    if (i < nvec) v[u] = NTL ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + u * 256ull;
    if (i < nvec) {
      if (NTS)
        __builtin_nontemporal_store(v[u], d + i);
      else
        d[i] = v[u];
    }
  }
}

__global__ __launch_bounds__(256) void copy_stride(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t nvec) {
  const uint64_t tile = 256ull * 4;
  for (uint64_t b = blockIdx.x * tile + threadIdx.x; b < nvec; b += static_cast<uint64_t>(gridDim.x) * tile) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * 256ull < nvec) v[u] = __builtin_nontemporal_load(s + b + u * 256ull);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * 256ull < nvec) __builtin_nontemporal_store(v[u], d + b + u * 256ull);
  }
}

using Kern = void (*)(const u32x4*, u32x4*, uint64_t);

int main(int argc, char** argv) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t sizes[] = {1ull << 30, 4ull << 30};
  struct V {
    const char* name;
    Kern k;
    int u;
    bool stride;
  } vs[] = {{"plain", copy_chunk<false, false, 1>, 1, false}, {"nt-ld", copy_chunk<true, false, 1>, 1, false},
            {"nt-st", copy_chunk<false, true, 1>, 1, false},  {"nt-both", copy_chunk<true, true, 1>, 1, false},
            {"u2", copy_chunk<true, true, 2>, 2, false},      {"u4", copy_chunk<true, true, 4>, 4, false},
            {"u2-plain", copy_chunk<false, false, 2>, 2, false}, {"stride16", copy_stride, 4, true}};
  for (size_t bytes : sizes) {
    u32x4 *s = nullptr, *d = nullptr;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(s, 1, bytes));
    CHECK(hipMemset(d, 0, bytes));
    const uint64_t nvec = bytes / 16;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int pass = 0; pass < 2; ++pass) {  // two interleaved passes: noise check
      for (const V& v : vs) {
        const uint64_t grid = v.stride ? static_cast<uint64_t>(cus) * 16 : (nvec + 256ull * v.u - 1) / (256ull * v.u);
        v.k<<<grid, 256>>>(s, d, nvec);  // warm
        CHECK(hipDeviceSynchronize());
        const int reps = 20;
        CHECK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) v.k<<<grid, 256>>>(s, d, nvec);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        std::printf("%5.1f GiB pass %d %-9s grid %8llu  %.3f TB/s payload\n", bytes / double(1ull << 30), pass, v.name,
                    static_cast<unsigned long long>(grid), bytes * double(reps) / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
      }
    }
    CHECK(hipFree(s));
    CHECK(hipFree(d));
  }
  return 0;
}
