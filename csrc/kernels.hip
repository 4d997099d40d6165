// gfx950 (MI355X, CDNA4) buffer kernels: fill / verify / reduce.
// See kernels.hpp for the contract.  Design notes (numbers from
// /opt/skills/guides/MI355X_MICROARCH.md):
//   * Pure streaming, so the target is the HBM3E roofline (~6.3 TB/s
//     measured).  Every access is 16 B/lane so one wave instruction moves a
//     contiguous 1 KiB (Guideline 13).
//   * Grids are sized to the chip (CU count x resident blocks) and grid-stride
//     the rest (Guideline 11); 256-thread blocks = 4 wave64s.
//   * ~50 KB must be in flight per CU to cover HBM latency under load: the
//     register variant keeps UNROLL=4 x 16 B per lane outstanding at up to 8
//     blocks/CU; the LDS variant keeps two STAGES-deep batches of 1 KiB
//     LDS-DMA pieces per wave in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace p2p {
namespace dev {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kFillUnroll = 4;
constexpr int kVerifyUnroll = 4;   // register variant, default
constexpr int kVerifyUnroll8 = 8;  // register variant with twice the loads in flight
constexpr int kLdsStages = 4;  // 1 KiB pieces per wave per batch
// Defaults picked from scripts/kernel_bench.py A/B runs (profiles/).
constexpr FillImpl kDefaultFill = FillImpl::Plain;
constexpr VerifyImpl kDefaultVerify = VerifyImpl::Register;

#define HIP_OK(cmd)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (cmd);                                                                   \
    if (e_ != hipSuccess) P2P_FATAL(strfmt("HIP error %s: %s", #cmd, hipGetErrorString(e_))); \
  } while (0)

// The key depends only on (seed, word_index >> 32).  Every tile below is a
// multiple of 4096 words and starts on such a multiple, so it never straddles
// a 2^32-word boundary: the key is computed once per tile from tile-uniform
// values (scalar ALU) and only the 4 per-word mixes run on the vector ALU.
__device__ __forceinline__ uint4 prng_vec_k(uint32_t key, uint64_t vec_index) {
  const uint32_t lo = static_cast<uint32_t>(vec_index * 4);
  return make_uint4(prng_word_k(key, lo), prng_word_k(key, lo + 1), prng_word_k(key, lo + 2), prng_word_k(key, lo + 3));
}

// ------------------------------------------------------------------ fill ----

template <bool NT>
__global__ __launch_bounds__(kBlock) void fill_kernel(uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                      uint8_t* __restrict__ tail, uint32_t tail_bytes,
                                                      uint64_t tail_offset) {
  const uint64_t tile = static_cast<uint64_t>(kBlock) * kFillUnroll;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * tile; base < nvec; base += static_cast<uint64_t>(gridDim.x) * tile) {
    const uint32_t key = prng_key(seed, base * 4);
#pragma unroll
    for (int u = 0; u < kFillUnroll; ++u) {
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < nvec) {
        const uint4 v = prng_vec_k(key, i);
        if (NT) {
          u32x4 w = {v.x, v.y, v.z, v.w};
          __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p) + i);
        } else {
          p[i] = v;
        }
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < tail_bytes) tail[threadIdx.x] = prng_byte(seed, tail_offset + threadIdx.x);
}

// ---------------------------------------------------------------- verify ----

struct Partial {
  unsigned long long mism;
  unsigned long long sum;
  unsigned long long first;
};

template <bool CHECK>
__device__ __forceinline__ void check_vec(const uint4 v, uint32_t key, uint64_t vec_index, Partial& acc) {
  acc.sum += static_cast<unsigned long long>(v.x) + v.y + static_cast<unsigned long long>(v.z) + v.w;
  if (CHECK) {
    const uint4 e = prng_vec_k(key, vec_index);
    const unsigned bad = (v.x != e.x) + (v.y != e.y) + (v.z != e.z) + (v.w != e.w);
    if (bad) {
      acc.mism += bad;
      const unsigned first_word = v.x != e.x ? 0 : v.y != e.y ? 1 : v.z != e.z ? 2 : 3;
      acc.first = min(acc.first, static_cast<unsigned long long>(vec_index * 16 + first_word * 4));
    }
  }
}

// Sub-16-byte tail: whole words, then a masked partial word (host_verify
// applies the same rule).
template <bool CHECK>
__device__ void check_tail(const uint8_t* tail, uint32_t tail_bytes, uint64_t tail_offset, uint64_t seed, Partial& acc) {
  for (uint32_t off = 0; off < tail_bytes; off += 4) {
    const uint32_t n = min(4u, tail_bytes - off);
    uint32_t got = 0;
    for (uint32_t b = 0; b < n; ++b) got |= static_cast<uint32_t>(tail[off + b]) << (8 * b);
    acc.sum += got;
    if (CHECK) {
      const uint64_t word = (tail_offset + off) / 4;
      const uint32_t mask = n == 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
      if ((got & mask) != (prng_word(seed, word) & mask)) {
        acc.mism += 1;
        acc.first = min(acc.first, static_cast<unsigned long long>(tail_offset + off));
      }
    }
  }
}

// Reduction epilogue: wave64 butterfly, then the 4 wave partials through LDS,
// then one atomic per block and per field (skipped when zero).
__device__ __forceinline__ void block_commit(Partial acc, VerifyAccum* out) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc.mism += __shfl_xor(acc.mism, off, 64);
    acc.sum += __shfl_xor(acc.sum, off, 64);
    acc.first = min(acc.first, __shfl_xor(acc.first, off, 64));
  }
  __shared__ Partial red[kWaves];
  const int wave = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial t = red[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) {
      t.mism += red[w].mism;
      t.sum += red[w].sum;
      t.first = min(t.first, red[w].first);
    }
    if (t.sum) atomicAdd(&out->checksum, t.sum);
    if (t.mism) {
      atomicAdd(&out->mismatches, t.mism);
      atomicMin(&out->first_bad, t.first);
    }
  }
}

template <bool CHECK, int UNROLL>
__global__ __launch_bounds__(kBlock) void verify_reg_kernel(const uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                            const uint8_t* __restrict__ tail, uint32_t tail_bytes,
                                                            uint64_t tail_offset, VerifyAccum* __restrict__ out) {
  Partial acc{0, 0, ~0ull};
  const uint64_t tile = static_cast<uint64_t>(kBlock) * UNROLL;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * tile; base < nvec; base += static_cast<uint64_t>(gridDim.x) * tile) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {  // all loads issued before any compare
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < nvec) {
        const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i);
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = make_uint4(0, 0, 0, 0);
      }
    }
    const uint32_t key = prng_key(seed, base * 4);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < nvec) check_vec<CHECK>(v[u], key, i, acc);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) check_tail<CHECK>(tail, tail_bytes, tail_offset, seed, acc);
  block_commit(acc, out);
}

// LDS-staged verify.  Each wave owns a private double-buffered ring of
// 2 x kLdsStages x 1 KiB in LDS.  A "super-chunk" is kLdsStages consecutive
// KiB; wave g of G handles super-chunks g, g+G, ...  While the compare loop
// reads batch b from LDS (ds_read_b128, each lane its own 16 B: conflict
// free), the LDS-DMA of batch b+1 is already in flight; the counted
// s_waitcnt vmcnt(kLdsStages) waits only for the older batch.  No
// workgroup barrier is needed: a wave only reads bytes its own DMAs wrote.
template <bool CHECK>
__global__ __launch_bounds__(kBlock) void verify_lds_kernel(const uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                            const uint8_t* __restrict__ tail, uint32_t tail_bytes,
                                                            uint64_t tail_offset, VerifyAccum* __restrict__ out) {
  __shared__ uint4 ring[kWaves][2][kLdsStages][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x / 64;
  const uint64_t waves_total = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
  const uint64_t sc_vecs = static_cast<uint64_t>(kLdsStages) * 64;
  const uint64_t n_sc = (nvec + sc_vecs - 1) / sc_vecs;

  auto issue = [&](uint64_t sc, int buf) {
#pragma unroll
    for (int s = 0; s < kLdsStages; ++s) {
      const uint64_t i = sc * sc_vecs + static_cast<uint64_t>(s) * 64 + lane;
      if (i < nvec)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(p + i),
                                         (__attribute__((address_space(3))) void*)(&ring[wave][buf][s][0]),
                                         16, 0, 0);
    }
  };

  Partial acc{0, 0, ~0ull};
  uint64_t sc = g;
  int buf = 0;
  if (sc < n_sc) issue(sc, 0);
  for (; sc < n_sc; sc += waves_total) {
    const uint64_t next = sc + waves_total;
    const bool next_full = (next + 1) * sc_vecs <= nvec;  // wave-uniform
    if (next < n_sc) issue(next, buf ^ 1);
    if (next_full) {
      // Older batch done; the kLdsStages youngest (next batch) may still fly.
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLdsStages) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // The four ds_read_b128 live in one asm statement: hipcc cannot tell which
    // LDS-DMA a ds_read aliases and would put a full vmcnt(0) in front of
    // each one, serialising the ring; here the only VMEM wait is the counted
    // one above and the asm drains its own reads (lgkmcnt(0)).
    static_assert(kLdsStages == 4, "asm block reads exactly four stages");
    const uint32_t lds_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) void*)(&ring[wave][buf][0][lane])));
    u32x4 r0, r1, r2, r3;
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %4 offset:1024\n\t"
        "ds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(lds_addr)
        : "memory");
    const u32x4 rv[kLdsStages] = {r0, r1, r2, r3};
    const uint32_t key = prng_key(seed, sc * sc_vecs * 4);
#pragma unroll
    for (int s = 0; s < kLdsStages; ++s) {
      const uint64_t i = sc * sc_vecs + static_cast<uint64_t>(s) * 64 + lane;
      if (i < nvec) check_vec<CHECK>(make_uint4(rv[s].x, rv[s].y, rv[s].z, rv[s].w), key, i, acc);
    }
    buf ^= 1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) check_tail<CHECK>(tail, tail_bytes, tail_offset, seed, acc);
  block_commit(acc, out);
}

__global__ void verify_reset_kernel(VerifyAccum* acc) {
  acc->mismatches = 0;
  acc->checksum = 0;
  acc->first_bad = ~0ull;
}

struct DevCache {
  std::mutex mu;
  std::vector<int> cus;
};

DevCache& dev_cache() {
  static DevCache c;
  return c;
}

}  // namespace

int cu_count() {
  int d = 0;
  HIP_OK(hipGetDevice(&d));
  auto& c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  if (static_cast<int>(c.cus.size()) <= d) c.cus.resize(static_cast<size_t>(d) + 1, 0);
  if (!c.cus[static_cast<size_t>(d)]) {
    int v = 0;
    HIP_OK(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d));
    c.cus[static_cast<size_t>(d)] = v > 0 ? v : 256;
  }
  return c.cus[static_cast<size_t>(d)];
}

LaunchGeom fill_geometry(size_t bytes) {
  LaunchGeom g;
  const uint64_t nvec = bytes / 16;
  const uint64_t tiles = (nvec + kBlock * kFillUnroll - 1) / (kBlock * kFillUnroll);
  const uint64_t cap = static_cast<uint64_t>(cu_count()) * 8;  // 8 resident 256-thread blocks per CU
  g.grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min(tiles, cap)));
  return g;
}

LaunchGeom verify_geometry(size_t bytes, VerifyImpl impl) {
  LaunchGeom g;
  const uint64_t nvec = bytes / 16;
  if (impl == VerifyImpl::Lds) {
    const uint64_t sc_vecs = static_cast<uint64_t>(kLdsStages) * 64;
    const uint64_t waves = (nvec + sc_vecs - 1) / sc_vecs;
    const uint64_t blocks = (waves + kWaves - 1) / kWaves;
    g.lds_bytes = sizeof(uint4) * kWaves * 2 * kLdsStages * 64;
    // 160 KiB LDS per CU / 32 KiB per block -> 5 resident blocks per CU.
    const uint64_t per_cu = std::max<uint64_t>(1, (160u * 1024u) / (g.lds_bytes + 256));
    const uint64_t cap = static_cast<uint64_t>(cu_count()) * std::min<uint64_t>(per_cu, 8);
    g.grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min(blocks, cap)));
  } else {
    const int unroll = impl == VerifyImpl::Register8 ? kVerifyUnroll8 : kVerifyUnroll;
    const uint64_t tiles = (nvec + static_cast<uint64_t>(kBlock) * unroll - 1) / (static_cast<uint64_t>(kBlock) * unroll);
    const uint64_t cap = static_cast<uint64_t>(cu_count()) * 8;
    g.grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min(tiles, cap)));
  }
  return g;
}

void launch_fill(void* p, size_t bytes, uint64_t seed, hipStream_t stream, FillImpl impl) {
  if (!bytes) return;
  P2P_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "fill: buffer must be 16-byte aligned");
  if (impl == FillImpl::Auto) impl = kDefaultFill;
  const uint64_t nvec = bytes / 16;
  const uint32_t tail = static_cast<uint32_t>(bytes - nvec * 16);
  LaunchGeom g = fill_geometry(bytes);
  auto* base = static_cast<uint8_t*>(p);
  if (impl == FillImpl::Nontemporal)
    fill_kernel<true><<<g.grid, kBlock, 0, stream>>>(reinterpret_cast<uint4*>(p), nvec, seed, base + nvec * 16, tail, nvec * 16);
  else
    fill_kernel<false><<<g.grid, kBlock, 0, stream>>>(reinterpret_cast<uint4*>(p), nvec, seed, base + nvec * 16, tail, nvec * 16);
  HIP_OK(hipGetLastError());
}

void launch_verify_reset(VerifyAccum* acc, hipStream_t stream) {
  verify_reset_kernel<<<1, 1, 0, stream>>>(acc);
  HIP_OK(hipGetLastError());
}

namespace {
template <bool CHECK>
void launch_verify_t(const uint4* vp, uint64_t nvec, uint64_t seed, const uint8_t* tp, uint32_t tail, VerifyAccum* acc,
                     VerifyImpl impl, const LaunchGeom& g, hipStream_t stream) {
  switch (impl) {
    case VerifyImpl::Lds:
      verify_lds_kernel<CHECK><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
      break;
    case VerifyImpl::Register8:
      verify_reg_kernel<CHECK, kVerifyUnroll8><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
      break;
    default:
      verify_reg_kernel<CHECK, kVerifyUnroll><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
  }
}
}  // namespace

void launch_verify(const void* p, size_t bytes, uint64_t seed, VerifyAccum* acc, VerifyImpl impl, bool check_prng,
                   hipStream_t stream) {
  if (!bytes) return;
  P2P_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "verify: buffer must be 16-byte aligned");
  if (impl == VerifyImpl::Auto) impl = kDefaultVerify;
  const uint64_t nvec = bytes / 16;
  const uint32_t tail = static_cast<uint32_t>(bytes - nvec * 16);
  const auto* vp = static_cast<const uint4*>(p);
  const auto* tp = static_cast<const uint8_t*>(p) + nvec * 16;
  LaunchGeom g = verify_geometry(bytes, impl);
  if (check_prng)
    launch_verify_t<true>(vp, nvec, seed, tp, tail, acc, impl, g, stream);
  else
    launch_verify_t<false>(vp, nvec, seed, tp, tail, acc, impl, g, stream);
  HIP_OK(hipGetLastError());
}

// ------------------------------------------------------------ multi copy ----

namespace {

constexpr int kCopyUnroll = 4;

// Passed by value in the kernarg segment: no device-side descriptor upload,
// so a launch is a single stream operation (and graph-capturable).
struct CopyArgs {
  const uint4* src[kMaxCopyOps];
  uint4* dst[kMaxCopyOps];
  uint64_t nvec[kMaxCopyOps];
  uint32_t tail[kMaxCopyOps];
  uint32_t block_begin[kMaxCopyOps + 1];
  int nops;
};

__global__ __launch_bounds__(kBlock) void multi_copy_kernel(const CopyArgs a) {
  // Workgroup -> op: block ranges are contiguous per op; the scan is over at
  // most kMaxCopyOps wave-uniform values.
  int op = 0;
  while (op + 1 < a.nops && blockIdx.x >= a.block_begin[op + 1]) ++op;
  const uint32_t b = blockIdx.x - a.block_begin[op];
  const uint32_t nb = a.block_begin[op + 1] - a.block_begin[op];
  const uint4* __restrict__ s = a.src[op];
  uint4* __restrict__ d = a.dst[op];
  const uint64_t n = a.nvec[op];
  const uint64_t tile = static_cast<uint64_t>(kBlock) * kCopyUnroll;
  for (uint64_t base = static_cast<uint64_t>(b) * tile; base < n; base += static_cast<uint64_t>(nb) * tile) {
    uint4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {  // all (remote) loads in flight before the stores
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < n) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < n) d[i] = v[u];
    }
  }
  if (b == 0 && threadIdx.x < a.tail[op]) {
    const uint8_t* st = reinterpret_cast<const uint8_t*>(s + n);
    uint8_t* dt = reinterpret_cast<uint8_t*>(d + n);
    dt[threadIdx.x] = st[threadIdx.x];
  }
}

}  // namespace

void launch_multi_copy(const CopyOp* ops, int nops, hipStream_t stream, int max_blocks) {
  for (int first = 0; first < nops; first += kMaxCopyOps) {
    const int cnt = std::min(kMaxCopyOps, nops - first);
    CopyArgs a{};
    a.nops = cnt;
    uint64_t need[kMaxCopyOps] = {0};
    uint64_t total_need = 0;
    const uint64_t tile = static_cast<uint64_t>(kBlock) * kCopyUnroll;
    for (int i = 0; i < cnt; ++i) {
      const CopyOp& o = ops[first + i];
      P2P_CHECK(reinterpret_cast<uintptr_t>(o.src) % 16 == 0 && reinterpret_cast<uintptr_t>(o.dst) % 16 == 0,
                "multi_copy: 16-byte aligned buffers required");
      a.src[i] = static_cast<const uint4*>(o.src);
      a.dst[i] = static_cast<uint4*>(o.dst);
      a.nvec[i] = o.bytes / 16;
      a.tail[i] = static_cast<uint32_t>(o.bytes - a.nvec[i] * 16);
      need[i] = std::max<uint64_t>(1, (a.nvec[i] + tile - 1) / tile);
      total_need += need[i];
    }
    const uint64_t cap = max_blocks > 0 ? static_cast<uint64_t>(max_blocks) : static_cast<uint64_t>(cu_count()) * 8;
    uint32_t acc = 0;
    for (int i = 0; i < cnt; ++i) {
      a.block_begin[i] = acc;
      uint64_t share = total_need <= cap ? need[i] : std::max<uint64_t>(1, need[i] * cap / total_need);
      acc += static_cast<uint32_t>(std::min(share, need[i]));
    }
    a.block_begin[cnt] = acc;
    multi_copy_kernel<<<acc, kBlock, 0, stream>>>(a);
    HIP_OK(hipGetLastError());
  }
}

}  // namespace dev
}  // namespace p2p
