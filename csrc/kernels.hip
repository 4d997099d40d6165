// gfx950 (MI355X, CDNA4) buffer kernels: fill / verify / reduce / copy.
// See kernels.hpp for the contract.  Design notes:
//   * Pure streaming: the target is the HBM3E roofline.  Every access is
//     16 B per lane, so one wave instruction moves a contiguous 1 KiB
//     (cdna_hip_programming.md Guideline 13).
//   * Grid shape (measured, scripts/fill_probe.hip): one 16 B access per lane
//     and one 4 KiB block per 256-thread workgroup, up to kMaxGrid = 2^20
//     workgroups and grid-striding only beyond 4 GiB.  On MI355X this "full
//     grid" streams stores at 6.9-7.0 TB/s (torch zero_: 6.87) and loads at
//     6.7-6.8 TB/s, while the textbook grid-stride loop over a grid capped at
//     4-32 blocks per CU tops out at 5.1-5.6 (stores) / 6.3 (loads) TB/s.
//   * The PRNG key depends only on word_index >> 32; a block iteration covers
//     1024 words starting at a multiple of 1024, so the key is computed once per
//     iteration from block-uniform values on the scalar unit and the vector ALU
//     only runs the 4 per-word mixes.
//   * The verify epilogue never funnels into one hot address: each block
//     commits with one atomic per field into shard (blockIdx % 64) of a
//     64-line accumulator, and a one-wave finalize kernel folds the shards.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
constexpr uint64_t kBlockVecs = kBlock;     // 16 B vectors per block iteration (4 KiB)
constexpr uint64_t kMaxGrid = 1ull << 20;   // 4 GiB per grid pass
constexpr int kStrideUnroll = 4;            // register verify: loads in flight per lane
constexpr int kLdsStages = 8;               // 1 KiB LDS-DMA pieces per wave (8 KiB per wave)
// Below this size the single-buffer LDS verify stages 4 KiB per wave (16 KiB
// of LDS per workgroup: 8 workgroups, 32 waves per CU, the register kernel's
// occupancy) instead of 8 KiB (20 waves).  Interleaved A/B (scripts/verify_ab.py
// with 4 KiB per wave as a temporary impl 3, profiles/r6_verify_ab/r6_vab11-12):
// 4 KiB per wave read 2.4% faster at 512 MiB, 1.7-2.4% at 1 GiB (= register
// staging), equal at 2 GiB and 4.6% slower at 4 GiB.
constexpr uint64_t kLds4Below = 2ull << 30;
constexpr int lds_stages_for(uint64_t bytes) { return bytes < kLds4Below ? 4 : kLdsStages; }
// Verify grid caps (workgroups per CU).  Register stride: 16 (2 generations
// of its 8 resident per CU), from scripts/verify_grid_sweep.py.  LDS-DMA: 8,
// from round 6's interleaved A/B (scripts/verify_ab.py, profiles/r6_verify_ab/,
// 5 boxes): at 1 GiB 0.3-4% faster than 16, at 256 MiB and 4 GiB within
// +-1%.  The batched kernel keeps 16 (its 32 MiB-slot layout was measured
// there).  Variants that lost their A/Bs: 4 KiB/wave, default-cache LDS-DMA,
// two 4 KiB halves per wave, per-block spans, 32 slices each walked by its
// own workgroups, the full-grid register loop (profiles/r1_tuned/,
// r4_verify_span/, r6_verify_ab/).
constexpr int kVerifyStridePerCu = 16;
constexpr int kVerifyLdsPerCu = 8;
constexpr int kMultiVerifyPerCu = 16;
// LDS-staged verify is the default (the north star's LDS staging).  Against
// register staging in interleaved A/Bs (profiles/r6_verify_ab/): 3-8% faster
// at 256 MiB, 0.97-1.0x at 1 GiB (4 KiB per wave), 0.98-1.0x at 2-4 GiB (8 KiB
// per wave); tests/test_zz_perf_floors_gpu.py test_verify_staging_ab puts the
// box's lds_over_stride on the PERF line (0.991: 1 GiB 0.973, 4 GiB 0.996).
constexpr VerifyImpl kDefaultVerify = VerifyImpl::Lds8;

#define HIP_OK(cmd)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (cmd);                                                                   \
    if (e_ != hipSuccess) P2P_FATAL(strfmt("HIP error %s: %s", #cmd, hipGetErrorString(e_))); \
  } while (0)

__device__ __forceinline__ uint4 prng_vec_k(uint32_t key, uint64_t vec_index) {
  const uint32_t lo = static_cast<uint32_t>(vec_index * 4);
  return make_uint4(prng_word_k(key, lo), prng_word_k(key, lo + 1), prng_word_k(key, lo + 2), prng_word_k(key, lo + 3));
}

__device__ __forceinline__ void store_tail(uint8_t* tail, uint32_t tail_bytes, uint64_t tail_offset, uint64_t seed) {
  if (blockIdx.x == 0 && threadIdx.x < tail_bytes) tail[threadIdx.x] = prng_byte(seed, tail_offset + threadIdx.x);
}

// ------------------------------------------------------------------ fill ----

// Vectors [begin, nvec) of the buffer at p (launch_fill issues one full grid
// per 4 GiB chunk); the tail bytes go with the last chunk (tail_bytes > 0).
// The one fill: one 16 B store per lane, one 4 KiB block per workgroup
// (7.0 TB/s by WRITE_SIZE, profiles/r4_pmc/).  Its A/B losers -- non-temporal
// stores, an XCD-ordered block map, a grid-stride loop over a capped grid, 2
// or 4 stores per lane (6.0-6.9 TB/s, profiles/r3b_nt_ab/, r4_gpu_tier/) --
// were removed in round 5.
__global__ __launch_bounds__(kBlock) void fill_grid_kernel(uint4* __restrict__ p, uint64_t begin, uint64_t nvec,
                                                           uint64_t seed, uint8_t* __restrict__ tail,
                                                           uint32_t tail_bytes, uint64_t tail_offset) {
  for (uint64_t base = begin + static_cast<uint64_t>(blockIdx.x) * kBlockVecs; base < nvec;
       base += static_cast<uint64_t>(gridDim.x) * kBlockVecs) {
    const uint32_t key = prng_key(seed, base * 4);  // block-uniform: scalar ALU
    const uint64_t i = base + threadIdx.x;
    if (i < nvec) p[i] = prng_vec_k(key, i);
  }
  store_tail(tail, tail_bytes, tail_offset, seed);
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

// Reduction epilogue: wave64 butterfly, the 4 wave partials through LDS, then
// one atomic per non-zero field into this block's shard.  Wave w's partial
// goes to red + w * red_stride bytes: the stride kernel passes a small array
// of its own, the LDS-staged kernels the first bytes of each wave's own
// staging slots (free once that wave's loop is done), so those kernels use
// exactly 32 KiB of LDS and 5 workgroups fit a CU's 160 KiB (a separate
// 96-byte array made it 32,864 B: 4 per CU).
__device__ __forceinline__ void block_commit(Partial acc, VerifyAccum* out, uint32_t shard_key, char* red,
                                             uint32_t red_stride) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc.mism += __shfl_xor(acc.mism, off, 64);
    acc.sum += __shfl_xor(acc.sum, off, 64);
    acc.first = min(acc.first, __shfl_xor(acc.first, off, 64));
  }
  const int wave = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) *reinterpret_cast<Partial*>(red + wave * red_stride) = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial t = *reinterpret_cast<const Partial*>(red);
#pragma unroll
    for (int w = 1; w < kWaves; ++w) {
      const Partial& r = *reinterpret_cast<const Partial*>(red + w * red_stride);
      t.mism += r.mism;
      t.sum += r.sum;
      t.first = min(t.first, r.first);
    }
    VerifyAccum* s = out + (shard_key % kVerifyShards);
    if (t.sum) atomicAdd(&s->checksum, t.sum);
    if (t.mism) {
      atomicAdd(&s->mismatches, t.mism);
      atomicMin(&s->first_bad, t.first);
    }
  }
}

__device__ __forceinline__ uint4 load_nt(const uint4* p, uint64_t i) {
  const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i);
  return make_uint4(t.x, t.y, t.z, t.w);
}

template <bool CHECK>
__global__ __launch_bounds__(kBlock) void verify_stride_kernel(const uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                               const uint8_t* __restrict__ tail, uint32_t tail_bytes,
                                                               uint64_t tail_offset, VerifyAccum* __restrict__ out) {
  Partial acc{0, 0, ~0ull};
  const uint64_t tile = static_cast<uint64_t>(kBlock) * kStrideUnroll;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * tile; base < nvec; base += static_cast<uint64_t>(gridDim.x) * tile) {
    uint4 v[kStrideUnroll];
#pragma unroll
    for (int u = 0; u < kStrideUnroll; ++u) {  // all loads issued before any compare
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      v[u] = i < nvec ? load_nt(p, i) : make_uint4(0, 0, 0, 0);
    }
    const uint32_t key = prng_key(seed, base * 4);
#pragma unroll
    for (int u = 0; u < kStrideUnroll; ++u) {
      const uint64_t i = base + static_cast<uint64_t>(u) * kBlock + threadIdx.x;
      if (i < nvec) check_vec<CHECK>(v[u], key, i, acc);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) check_tail<CHECK>(tail, tail_bytes, tail_offset, seed, acc);
  __shared__ Partial red[kWaves];
  block_commit(acc, out, blockIdx.x, reinterpret_cast<char*>(red), sizeof(Partial));
}

// LDS-staged verify.  Wave g owns super-chunk g (STAGES consecutive KiB: 4 or
// 8, lds_stages_for) of each grid pass: it issues STAGES LDS-DMA pieces
// (global_load_lds_dwordx4: the wave's 64 lanes x 16 B land contiguously at
// the LDS address in M0), waits for its own DMAs (vmcnt(0)), reads each lane's
// 16 B back with ds_read_b128 (contiguous per lane: bank-conflict free) and
// compares.  No workgroup barrier: a wave only reads bytes its own DMAs
// wrote.  The ds_read_b128s live in one asm statement: hipcc cannot tell
// which LDS-DMA a ds_read aliases and would put a vmcnt(0) in front of each
// one.  lds_read_stages reads this lane's 16 B of each of the STAGES
// consecutive 1 KiB LDS pieces and drains them (lgkmcnt(0)) before returning.
template <int STAGES>
__device__ __forceinline__ void lds_read_stages(uint32_t addr, u32x4 (&r)[STAGES]) {
  static_assert(STAGES == 8 || STAGES == 4, "one ds_read_b128 per stage below (lds_stages_for)");
  if constexpr (STAGES == 8) {
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:1024\n\t"
        "ds_read_b128 %2, %8 offset:2048\n\t"
        "ds_read_b128 %3, %8 offset:3072\n\t"
        "ds_read_b128 %4, %8 offset:4096\n\t"
        "ds_read_b128 %5, %8 offset:5120\n\t"
        "ds_read_b128 %6, %8 offset:6144\n\t"
        "ds_read_b128 %7, %8 offset:7168\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7])
        : "v"(addr)
        : "memory");
  } else {
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %4 offset:1024\n\t"
        "ds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3])
        : "v"(addr)
        : "memory");
  }
}

// The LDS-staged kernels' only LDS: STAGES KiB of staging slots per wave
// (8: 32 KiB per workgroup), whose first bytes also carry the block_commit
// partials.
template <int STAGES>
struct LdsSlots {
  uint4 s[kWaves][STAGES][64];
};
static_assert(sizeof(LdsSlots<kLdsStages>) == 32768, "5 workgroups per CU need <= 32 KiB each");

template <int STAGES>
__device__ __forceinline__ LdsSlots<STAGES>& lds_slots() {
  __shared__ LdsSlots<STAGES> slots;
  return slots;
}

template <int STAGES>
__device__ __forceinline__ void lds_block_commit(Partial acc, VerifyAccum* out, uint32_t shard_key) {
  block_commit(acc, out, shard_key, reinterpret_cast<char*>(&lds_slots<STAGES>().s[0][0][0]),
               sizeof(lds_slots<STAGES>().s[0]));
}

// Blocks `block` of `nblocks` of one buffer: the LDS-staged loop below, with
// the workgroup's own LDS slots (the single and the batched verify share it).
// aux = 2 on the LDS-DMA: non-temporal (6.3-6.6 TB/s against 5.7-5.9 with the
// default cache policy; MI355X_MICROARCH.md ldsdma-fill row agrees).
//
// Pipelined: as soon as a chunk's ds_reads have drained into VGPRs its
// slots are free, so the wave issues the NEXT chunk's DMAs into them before
// it checks this one, and its loads stay in flight through the PRNG compare.
// The check's VALU work cost the unpipelined loop 4% (6.55 -> 6.30 TB/s,
// checksum-only vs check, profiles/r5_prof/pmc_summary.txt) against 0.75%
// for register staging at 32 waves per CU (LDS staging runs 20); pipelined
// +0.6% at 1 GiB, +1.2% at 4 GiB in one interleaved A/B (profiles/r6_verify_ab/).
template <bool CHECK, int STAGES = kLdsStages>
__device__ __forceinline__ Partial lds_verify_blocks(const uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                     uint64_t block, uint64_t nblocks) {
  auto& slot = lds_slots<STAGES>().s;
  const int lane = threadIdx.x & 63;
  // Wave-uniform by construction; readfirstlane tells the compiler, so the
  // chunk walk below stays on the scalar unit.
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x / 64));
  const uint64_t sc_vecs = static_cast<uint64_t>(STAGES) * 64;
  const uint64_t n_sc = (nvec + sc_vecs - 1) / sc_vecs;
  const uint64_t step = nblocks * kWaves;
  const uint32_t lds_addr = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)(&slot[wave][0][lane])));
  auto issue = [&](uint64_t sc) {
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
      const uint64_t i = sc * sc_vecs + static_cast<uint64_t>(s) * 64 + lane;
      if (i < nvec)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(p + i),
                                         (__attribute__((address_space(3))) void*)(&slot[wave][s][0]), 16, 0, 2);
    }
  };
  Partial acc{0, 0, ~0ull};
  uint64_t sc = block * kWaves + wave;
  if (sc < n_sc) issue(sc);
  for (; sc < n_sc; sc += step) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's DMAs (the only ones in flight)
    u32x4 rv[STAGES];
    lds_read_stages<STAGES>(lds_addr, rv);  // drained (lgkmcnt(0)): the slots are free again
    if (sc + step < n_sc) issue(sc + step);
    const uint32_t key = prng_key(seed, sc * sc_vecs * 4);  // wave-uniform
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
      const uint64_t i = sc * sc_vecs + static_cast<uint64_t>(s) * 64 + lane;
      if (i < nvec) check_vec<CHECK>(make_uint4(rv[s].x, rv[s].y, rv[s].z, rv[s].w), key, i, acc);
    }
  }
  return acc;
}

template <bool CHECK, int STAGES>
__global__ __launch_bounds__(kBlock) void verify_lds_kernel(const uint4* __restrict__ p, uint64_t nvec, uint64_t seed,
                                                            const uint8_t* __restrict__ tail, uint32_t tail_bytes,
                                                            uint64_t tail_offset, VerifyAccum* __restrict__ out) {
  Partial acc = lds_verify_blocks<CHECK, STAGES>(p, nvec, seed, blockIdx.x, gridDim.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) check_tail<CHECK>(tail, tail_bytes, tail_offset, seed, acc);
  lds_block_commit<STAGES>(acc, out, blockIdx.x);
}

// Batched verify: up to kMaxVerifyJobs buffers, each with
// its own seed, in one launch.  Workgroups are split across the jobs in
// contiguous ranges (block_begin, as multi_copy_kernel); job j commits into
// its own kVerifyShards shards of the scratch.  The post-timing check of a
// bench run was one reset + verify + finalize + D2H copy + host sync per
// 32 MiB slot (3336 of each per run, profiles/r3b_close/bench_kernel_stats.csv).
struct MultiVerifyArgs {
  const uint4* p[kMaxVerifyJobs];
  uint64_t nvec[kMaxVerifyJobs];
  uint64_t seed[kMaxVerifyJobs];
  uint32_t tail[kMaxVerifyJobs];
  uint32_t block_begin[kMaxVerifyJobs + 1];
  int njobs;
};

__global__ __launch_bounds__(kBlock) void multi_verify_lds_kernel(const MultiVerifyArgs a,
                                                                  VerifyAccum* __restrict__ scratch) {
  int lo = 0, hi = a.njobs - 1;  // largest job with block_begin[job] <= blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (blockIdx.x >= a.block_begin[mid]) lo = mid; else hi = mid - 1;
  }
  const int job = lo;
  const uint32_t b = blockIdx.x - a.block_begin[job];
  const uint32_t nb = a.block_begin[job + 1] - a.block_begin[job];
  const uint64_t nvec = a.nvec[job];
  Partial acc = lds_verify_blocks<true>(a.p[job], nvec, a.seed[job], b, nb);
  if (b == 0 && threadIdx.x == 0)
    check_tail<true>(reinterpret_cast<const uint8_t*>(a.p[job] + nvec), a.tail[job], nvec * 16, a.seed[job], acc);
  lds_block_commit<kLdsStages>(acc, scratch + static_cast<size_t>(job) * kVerifyShards, b);
}

// One workgroup (one wave) per job: reset its shards.
__global__ __launch_bounds__(64) void multi_verify_reset_kernel(VerifyAccum* scratch) {
  VerifyAccum* a = scratch + static_cast<size_t>(blockIdx.x) * kVerifyShards + threadIdx.x;
  a->mismatches = 0;
  a->checksum = 0;
  a->first_bad = ~0ull;
}

// One wave per job folds its shards into out[job].
__global__ __launch_bounds__(64) void multi_verify_finalize_kernel(const VerifyAccum* __restrict__ scratch,
                                                                   VerifyAccum* __restrict__ out) {
  const VerifyAccum& s = scratch[static_cast<size_t>(blockIdx.x) * kVerifyShards + threadIdx.x];
  unsigned long long m = s.mismatches, c = s.checksum, f = s.first_bad;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m += __shfl_xor(m, off, 64);
    c += __shfl_xor(c, off, 64);
    f = min(f, __shfl_xor(f, off, 64));
  }
  if (threadIdx.x == 0) {
    out[blockIdx.x].mismatches = m;
    out[blockIdx.x].checksum = c;
    out[blockIdx.x].first_bad = f;
  }
}

__global__ void verify_reset_kernel(VerifyAccum* acc) {
  if (threadIdx.x < kVerifyShards) {
    acc[threadIdx.x].mismatches = 0;
    acc[threadIdx.x].checksum = 0;
    acc[threadIdx.x].first_bad = ~0ull;
  }
}

// One wave folds the 64 shards into shard 0.
__global__ __launch_bounds__(64) void verify_finalize_kernel(VerifyAccum* acc) {
  const int l = threadIdx.x;
  unsigned long long m = acc[l].mismatches, s = acc[l].checksum, f = acc[l].first_bad;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m += __shfl_xor(m, off, 64);
    s += __shfl_xor(s, off, 64);
    f = min(f, __shfl_xor(f, off, 64));
  }
  __syncthreads();  // every lane has read its shard before shard 0 is overwritten
  if (l == 0) {
    acc[0].mismatches = m;
    acc[0].checksum = s;
    acc[0].first_bad = f;
  }
}

struct DevCache {
  std::mutex mu;
  std::vector<int> cus;
};

DevCache& dev_cache() {
  static DevCache c;
  return c;
}

unsigned grid_for(uint64_t units) { return static_cast<unsigned>(std::max<uint64_t>(1, std::min(units, kMaxGrid))); }

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

LaunchGeom fill_geometry(size_t bytes, FillImpl) {
  LaunchGeom g;
  g.grid = grid_for((bytes / 16 + kBlockVecs - 1) / kBlockVecs);
  return g;
}

LaunchGeom verify_geometry(size_t bytes, VerifyImpl impl, unsigned max_grid) {
  LaunchGeom g;
  const uint64_t nvec = bytes / 16;
  if (impl == VerifyImpl::Auto) impl = kDefaultVerify;
  // Unlike fill/copy, verify ends every workgroup with a reduction and an
  // atomic commit, so a full grid (one 4 KiB block per workgroup) pays that
  // epilogue 256K times per GiB; the caps below let each workgroup stream
  // tens of KiB per epilogue (kernel_bench A/B).
  const uint64_t cap = max_grid ? max_grid
                                : static_cast<uint64_t>(cu_count()) *
                                      (impl == VerifyImpl::Stride ? kVerifyStridePerCu : kVerifyLdsPerCu);
  if (impl == VerifyImpl::Stride) {
    const uint64_t tiles = (nvec + kBlock * kStrideUnroll - 1) / (kBlock * kStrideUnroll);
    g.grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min(tiles, cap)));
  } else {
    // Waves of 4 or 8 KiB chunks (lds_stages_for), and the LDS each wave owns.
    const int stages = lds_stages_for(bytes);
    const uint64_t sc_vecs = static_cast<uint64_t>(stages) * 64;
    const uint64_t waves = (nvec + sc_vecs - 1) / sc_vecs;
    g.grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min((waves + kWaves - 1) / kWaves, cap)));
    g.lds_bytes = sizeof(uint4) * kWaves * stages * 64;
  }
  return g;
}

void launch_fill(void* p, size_t bytes, uint64_t seed, hipStream_t stream, FillImpl) {
  if (!bytes) return;
  P2P_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "fill: buffer must be 16-byte aligned");
  const uint64_t nvec = bytes / 16;
  const uint32_t tail = static_cast<uint32_t>(bytes - nvec * 16);
  auto* vp = reinterpret_cast<uint4*>(p);
  auto* tp = static_cast<uint8_t*>(p) + nvec * 16;
  // Full grids: one launch per 4 GiB chunk (a capped grid striding over a
  // larger buffer streams 16% slower: 5.9 vs 7.0 TB/s at 16 GiB).
  const uint64_t chunk = kMaxGrid * kBlockVecs;
  for (uint64_t begin = 0;; begin += chunk) {
    const uint64_t end = std::min(nvec, begin + chunk);
    const bool last = end == nvec;
    const unsigned grid = grid_for((end - begin + kBlockVecs - 1) / kBlockVecs);
    fill_grid_kernel<<<grid, kBlock, 0, stream>>>(vp, begin, end, seed, tp, last ? tail : 0, nvec * 16);
    HIP_OK(hipGetLastError());
    if (last) break;
  }
}

void launch_verify_reset(VerifyAccum* acc, hipStream_t stream) {
  verify_reset_kernel<<<1, 64, 0, stream>>>(acc);
  HIP_OK(hipGetLastError());
}

namespace {
template <bool CHECK>
void launch_verify_t(const uint4* vp, uint64_t nvec, uint64_t seed, const uint8_t* tp, uint32_t tail, VerifyAccum* acc,
                     VerifyImpl impl, const LaunchGeom& g, hipStream_t stream) {
  if (impl == VerifyImpl::Stride)
    verify_stride_kernel<CHECK><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
  else if (lds_stages_for(nvec * 16) == 4)
    verify_lds_kernel<CHECK, 4><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
  else
    verify_lds_kernel<CHECK, kLdsStages><<<g.grid, kBlock, 0, stream>>>(vp, nvec, seed, tp, tail, nvec * 16, acc);
}
}  // namespace

void launch_verify(const void* p, size_t bytes, uint64_t seed, VerifyAccum* acc, VerifyImpl impl, bool check_prng,
                   hipStream_t stream, unsigned max_grid) {
  if (bytes) {
    P2P_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "verify: buffer must be 16-byte aligned");
    if (impl == VerifyImpl::Auto) impl = kDefaultVerify;
    const uint64_t nvec = bytes / 16;
    const uint32_t tail = static_cast<uint32_t>(bytes - nvec * 16);
    const auto* vp = static_cast<const uint4*>(p);
    const auto* tp = static_cast<const uint8_t*>(p) + nvec * 16;
    LaunchGeom g = verify_geometry(bytes, impl, max_grid);
    if (check_prng)
      launch_verify_t<true>(vp, nvec, seed, tp, tail, acc, impl, g, stream);
    else
      launch_verify_t<false>(vp, nvec, seed, tp, tail, acc, impl, g, stream);
    HIP_OK(hipGetLastError());
  }
  verify_finalize_kernel<<<1, 64, 0, stream>>>(acc);
  HIP_OK(hipGetLastError());
}

void launch_multi_verify(const VerifyJob* jobs, int njobs, VerifyAccum* scratch, VerifyAccum* out,
                         hipStream_t stream) {
  // Workgroups: kMultiVerifyPerCu (16) per CU shared by the jobs of a
  // batch in proportion to their size, at least one each.
  const uint64_t cap = static_cast<uint64_t>(cu_count()) * kMultiVerifyPerCu;
  constexpr uint64_t kChunkVecs = kLdsStages * 64 * kWaves;  // 32 KiB per workgroup pass
  for (int first = 0; first < njobs; first += kMaxVerifyJobs) {
    const int cnt = std::min(kMaxVerifyJobs, njobs - first);
    MultiVerifyArgs a{};
    a.njobs = cnt;
    uint64_t need[kMaxVerifyJobs] = {0}, total = 0;
    for (int i = 0; i < cnt; ++i) {
      const VerifyJob& j = jobs[first + i];
      P2P_CHECK(reinterpret_cast<uintptr_t>(j.p) % 16 == 0, "verify: buffer must be 16-byte aligned");
      a.p[i] = static_cast<const uint4*>(j.p);
      a.nvec[i] = j.bytes / 16;
      a.tail[i] = static_cast<uint32_t>(j.bytes - a.nvec[i] * 16);
      a.seed[i] = j.seed;
      need[i] = std::max<uint64_t>(1, (a.nvec[i] + kChunkVecs - 1) / kChunkVecs);
      total += need[i];
    }
    uint32_t acc = 0;
    for (int i = 0; i < cnt; ++i) {
      a.block_begin[i] = acc;
      const uint64_t share = total <= cap ? need[i] : std::max<uint64_t>(1, need[i] * cap / total);
      acc += static_cast<uint32_t>(std::min(share, need[i]));
    }
    a.block_begin[cnt] = acc;
    multi_verify_reset_kernel<<<cnt, 64, 0, stream>>>(scratch);
    HIP_OK(hipGetLastError());
    multi_verify_lds_kernel<<<acc, kBlock, 0, stream>>>(a, scratch);
    HIP_OK(hipGetLastError());
    multi_verify_finalize_kernel<<<cnt, 64, 0, stream>>>(scratch, out + first);
    HIP_OK(hipGetLastError());
  }
}

BatchVerifier::~BatchVerifier() {
  if (scratch_) (void)hipFree(scratch_);
  if (out_) (void)hipFree(out_);
  if (host_) (void)hipHostFree(host_);
}

void BatchVerifier::reserve(int njobs, const std::function<void()>& drain) {
  if (!scratch_) HIP_OK(hipMalloc(&scratch_, multi_verify_scratch_bytes()));
  if (njobs <= cap_) return;
  // The stream may still read the old arrays: the caller drains it first.
  if (out_ || host_) drain();
  if (out_) HIP_OK(hipFree(out_));
  if (host_) HIP_OK(hipHostFree(host_));
  out_ = host_ = nullptr;
  cap_ = std::max(njobs, 2 * cap_);
  HIP_OK(hipMalloc(&out_, sizeof(VerifyAccum) * static_cast<size_t>(cap_)));
  HIP_OK(hipHostMalloc(&host_, sizeof(VerifyAccum) * static_cast<size_t>(cap_), hipHostMallocDefault));
}

void BatchVerifier::enqueue(const VerifyJob* jobs, int njobs, hipStream_t stream) {
  if (njobs <= 0) return;
  P2P_CHECK(scratch_ && njobs <= cap_, "BatchVerifier::enqueue: reserve(njobs) first");
  launch_multi_verify(jobs, njobs, scratch_, out_, stream);
  HIP_OK(hipMemcpyAsync(host_, out_, sizeof(VerifyAccum) * static_cast<size_t>(njobs), hipMemcpyDeviceToHost, stream));
}

// ------------------------------------------------------------ multi copy ----

namespace {

// Passed by value in the kernarg segment: no device-side descriptor upload,
// so a launch is a single stream operation (and graph-capturable).
struct CopyArgs {
  const uint4* src[kMaxCopyOps];
  uint4* dst[kMaxCopyOps];
  uint64_t nvec[kMaxCopyOps];
  uint32_t tail[kMaxCopyOps];
  uint32_t block_begin[kMaxCopyOps + 1];
  uint32_t coherent;  // bit i: op i moves between GPUs (system-coherent accesses)
  int nops;
  // Workgroup -> op lookup: > 0 every op has this many blocks (one division);
  // 0 binary search of block_begin.
  int32_t uniform;
};

// gfx940+ cache-policy bits of a buffer access: sc0 | sc1 = system scope.
// A load with them never returns a line the reader's L2 kept from an earlier
// run (the peer may have refilled that buffer since); a store with them is
// written through to the owner's memory, so the flag kernel that follows only
// has to order, not flush (kernels.hpp CopyOp::coherent).
constexpr int kSystemCoherent = 1 | 16;
constexpr int kRsrcFlags = 0x00020000;  // raw buffer descriptor word 3 for gfx950

__global__ __launch_bounds__(kBlock) void multi_copy_kernel(const CopyArgs a) {
  // Workgroup -> op: block ranges are contiguous per op.  Every workgroup
  // moves a single 4 KiB chunk, so this lookup is on its critical path: a
  // linear scan of up to 16 dependent scalar loads cost 6% at 16 ops x 32 MiB
  // (2.95 vs 3.14 TB/s, profiles/r2_copy_lookup/); equal-sized ops (every
  // bench step) take one division, others a 4-step binary search.
  int op = 0;
  if (a.uniform > 0) {
    op = min(static_cast<int>(blockIdx.x / static_cast<uint32_t>(a.uniform)), a.nops - 1);
  } else {
    int lo = 0, hi = a.nops - 1;  // largest op with block_begin[op] <= blockIdx.x
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (blockIdx.x >= a.block_begin[mid]) lo = mid; else hi = mid - 1;
    }
    op = lo;
  }
  const uint32_t b = blockIdx.x - a.block_begin[op];
  const uint32_t nb = a.block_begin[op + 1] - a.block_begin[op];
  const uint4* __restrict__ s = a.src[op];
  uint4* __restrict__ d = a.dst[op];
  const uint64_t n = a.nvec[op];
  if ((a.coherent >> op) & 1u) {
    // One descriptor pair per 4 KiB chunk (block-uniform base, lane offset in
    // voffset); the range check drops the lanes past the end of the op.
    for (uint64_t base = static_cast<uint64_t>(b) * kBlockVecs; base < n; base += static_cast<uint64_t>(nb) * kBlockVecs) {
      const int bytes = static_cast<int>(min<uint64_t>(kBlockVecs, n - base) * 16);
      auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(s + base), 0, bytes, kRsrcFlags);
      auto rd = __builtin_amdgcn_make_buffer_rsrc(d + base, 0, bytes, kRsrcFlags);
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(threadIdx.x) * 16, 0, kSystemCoherent);
      __builtin_amdgcn_raw_buffer_store_b128(v, rd, static_cast<int>(threadIdx.x) * 16, 0, kSystemCoherent);
    }
    if (b == 0 && threadIdx.x < a.tail[op]) {
      auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(s + n), 0, static_cast<int>(a.tail[op]), kRsrcFlags);
      auto rd = __builtin_amdgcn_make_buffer_rsrc(d + n, 0, static_cast<int>(a.tail[op]), kRsrcFlags);
      const auto v = __builtin_amdgcn_raw_buffer_load_b8(rs, static_cast<int>(threadIdx.x), 0, kSystemCoherent);
      __builtin_amdgcn_raw_buffer_store_b8(v, rd, static_cast<int>(threadIdx.x), 0, kSystemCoherent);
    }
    return;
  }
  // Device-local op: non-temporal load and store (3.25-3.28 TB/s of payload
  // at 1 / 4 GiB vs 3.09-3.14 for plain accesses, scripts/copy_probe.hip,
  // profiles/r2_copy_nt/).
  const u32x4* __restrict__ sv = reinterpret_cast<const u32x4*>(s);
  u32x4* __restrict__ dv = reinterpret_cast<u32x4*>(d);
  for (uint64_t i = static_cast<uint64_t>(b) * kBlockVecs + threadIdx.x; i < n; i += static_cast<uint64_t>(nb) * kBlockVecs)
    __builtin_nontemporal_store(__builtin_nontemporal_load(sv + i), dv + i);
  if (b == 0 && threadIdx.x < a.tail[op]) {
    const uint8_t* st = reinterpret_cast<const uint8_t*>(s + n);
    uint8_t* dt = reinterpret_cast<uint8_t*>(d + n);
    dt[threadIdx.x] = st[threadIdx.x];
  }
}

}  // namespace

namespace {

// One launch over at most kMaxCopyOps ops; with max_blocks == 0 the caller
// keeps the total at or under kMaxGrid blocks, so every op gets a full grid.
void launch_copy_group(const CopyOp* ops, int cnt, hipStream_t stream, int max_blocks) {
  CopyArgs a{};
  a.nops = cnt;
  a.coherent = 0;
  uint64_t need[kMaxCopyOps] = {0};
  uint64_t total_need = 0;
  for (int i = 0; i < cnt; ++i) {
    const CopyOp& o = ops[i];
    P2P_CHECK(reinterpret_cast<uintptr_t>(o.src) % 16 == 0 && reinterpret_cast<uintptr_t>(o.dst) % 16 == 0,
              "multi_copy: 16-byte aligned buffers required");
    a.src[i] = static_cast<const uint4*>(o.src);
    a.dst[i] = static_cast<uint4*>(o.dst);
    a.nvec[i] = o.bytes / 16;
    a.tail[i] = static_cast<uint32_t>(o.bytes - a.nvec[i] * 16);
    if (o.coherent) a.coherent |= 1u << i;
    need[i] = std::max<uint64_t>(1, (a.nvec[i] + kBlockVecs - 1) / kBlockVecs);
    total_need += need[i];
  }
  const uint64_t cap = max_blocks > 0 ? static_cast<uint64_t>(max_blocks) : kMaxGrid;
  uint32_t acc = 0;
  for (int i = 0; i < cnt; ++i) {
    a.block_begin[i] = acc;
    uint64_t share = total_need <= cap ? need[i] : std::max<uint64_t>(1, need[i] * cap / total_need);
    acc += static_cast<uint32_t>(std::min(share, need[i]));
  }
  a.block_begin[cnt] = acc;
  a.uniform = static_cast<int32_t>(a.block_begin[1] - a.block_begin[0]);
  for (int i = 1; i < cnt; ++i)
    if (a.block_begin[i + 1] - a.block_begin[i] != static_cast<uint32_t>(a.uniform)) a.uniform = 0;
  multi_copy_kernel<<<acc, kBlock, 0, stream>>>(a);
  HIP_OK(hipGetLastError());
}

uint64_t copy_blocks(size_t bytes) { return std::max<uint64_t>(1, (bytes / 16 + kBlockVecs - 1) / kBlockVecs); }


}  // namespace

void launch_multi_copy(const CopyOp* ops, int nops, hipStream_t stream, int max_blocks) {
  constexpr int max_ops = kMaxCopyOps;
  if (max_blocks > 0) {  // explicit grid cap (grid-shape experiments): the ops share it
    for (int first = 0; first < nops; first += max_ops)
      launch_copy_group(ops + first, std::min(max_ops, nops - first), stream, max_blocks);
    return;
  }
  // Full grids only: ops above 4 GiB are split into 4 GiB pieces and pieces
  // are packed so that no launch needs more than kMaxGrid blocks.  A second
  // grid-stride pass over a capped grid streams ~5% slower (IPC self path:
  // 2.98 TB/s at 16-64 GiB vs 3.12 at 4 GiB, profiles/r1_sweeps).
  const size_t piece = static_cast<size_t>(kMaxGrid * kBlockVecs * 16);
  std::vector<CopyOp> pieces;
  for (int i = 0; i < nops; ++i) {
    const CopyOp& o = ops[i];
    size_t off = 0;
    do {
      const size_t n = std::min(piece, o.bytes - off);
      pieces.push_back({static_cast<const char*>(o.src) + off, static_cast<char*>(o.dst) + off, n, o.coherent});
      off += n;
    } while (off < o.bytes);
  }
  size_t i = 0;
  while (i < pieces.size()) {
    size_t j = i;
    uint64_t blocks = 0;
    while (j < pieces.size() && j - i < static_cast<size_t>(max_ops) &&
           (j == i || blocks + copy_blocks(pieces[j].bytes) <= kMaxGrid))
      blocks += copy_blocks(pieces[j++].bytes);
    launch_copy_group(pieces.data() + i, static_cast<int>(j - i), stream, 0);
    i = j;
  }
}

}  // namespace dev
}  // namespace p2p
