// Counter-based PRNG shared by the device fill/verify kernels and the host
// (CPU transport, tests).  Word i of the stream for `seed` is a pure function
// of (seed, i), so a receiver can regenerate what the sender wrote without any
// extra traffic, and any byte range can be checked independently.
//
// The reference fills buffers with zeros (cudaMemset, p2p_matrix.cc:129-130)
// and never reads them back; the north star asks for random-filled buffers
// with device-side verification.
//
// Cost on CDNA4: 1 key derivation per 16-byte lane chunk + 4 x fmix32 (two
// 32-bit multiplies each) ~= 35 VALU ops per 16 B, ~20% of the VALU budget at
// the HBM roofline, so fill/verify stay memory-bound.
#pragma once

#include <cstddef>
#include <cstdint>

#if defined(__HIP__)  // HIP language mode (.hip sources): usable on both sides
#define P2P_HD __host__ __device__ __attribute__((always_inline)) inline
#else
#define P2P_HD inline
#endif

namespace p2p {

P2P_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Per-2^32-word-region key; constant across a 16-byte chunk (4 words never
// straddle a 2^32 boundary because chunks start at multiples of 4 words).
P2P_HD uint32_t prng_key(uint64_t seed, uint64_t word_index) {
  uint32_t hi = static_cast<uint32_t>(word_index >> 32);
  return fmix32(static_cast<uint32_t>(seed) ^ fmix32(static_cast<uint32_t>(seed >> 32) + hi * 0x27D4EB2Fu + 0x165667B1u));
}

P2P_HD uint32_t prng_word_k(uint32_t key, uint32_t lo) { return fmix32((lo * 0x9E3779B1u) ^ key); }

P2P_HD uint32_t prng_word(uint64_t seed, uint64_t word_index) {
  return prng_word_k(prng_key(seed, word_index), static_cast<uint32_t>(word_index));
}

// Byte b of the stream (little-endian words).
P2P_HD uint8_t prng_byte(uint64_t seed, uint64_t b) {
  return static_cast<uint8_t>(prng_word(seed, b >> 2) >> (8 * (b & 3)));
}

// Seed for the payload rank `src` sends in a phase.  Distinct per sender and
// message size, so a message delivered from the wrong peer or a stale buffer
// from the previous size fails verification.
P2P_HD uint64_t payload_seed(int src, uint64_t bytes, uint64_t salt) {
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (static_cast<uint64_t>(static_cast<uint32_t>(src)) << 40) ^ bytes ^ (salt * 0xD6E8FEB86659FD93ull);
  return s ^ (s >> 29);
}

// Checksum convention (device verify and host reference agree): the sum,
// modulo 2^64, of every *received* 32-bit word (tail bytes zero-extended into
// a final partial word).
struct VerifyResult {
  uint64_t mismatches = 0;       // number of 32-bit words (or tail bytes) that differ
  uint64_t checksum = 0;         // sum of received words mod 2^64
  uint64_t first_bad = ~0ull;    // lowest mismatching byte offset, ~0 if none
};

}  // namespace p2p
