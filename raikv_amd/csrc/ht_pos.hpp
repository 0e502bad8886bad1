// ht_pos.hpp -- device side of SURVEY.md §8 row f1: one fixed-up key hash
// (h1, h2) -> the hash-table positions raikv's KeyCtx probes.
//
//   home slot   FileHdr::ht_mod (include/raikv/shm_ht.h:181-184):
//               ((k & mask) * fraction) >> shift, u64 arithmetic
//   alternates  CuckooAltHash::calc_hash (src/ht_cuckoo.cpp:38-79):
//               alt0 = h1, alt1 = h2 unless its slot clashes with alt0's;
//               further alternates step a xoroshiro128+ pair
//               (ht_cuckoo.cpp:20-27) seeded 0x9e3779b97f4a7c13 ^ h2 until
//               clear of every earlier slot
//   clash       equal low 13 bits (the 8K PositionBits index,
//               ht_cuckoo.cpp:15-16) or ring distance either way
//               (KeyCtx::calc_offset, key_ctx.h:473-477) < cuckoo_buckets
//   linear      cuckoo_buckets <= 1 or arity <= 1: home slot only
//               (KeyCtx::acquire, src/key_ctx.cpp:130)
//
// Integer-only and data-parallel: every lane owns one key, every array is
// indexed by compile-time constants (arity A is a template parameter) so
// the positions stay in VGPRs.  The rejection loop is reached by ~1 key in
// 2000 (13-bit index clashes dominate), so divergence is negligible.
#pragma once
#include <stdint.h>

namespace kvh {

struct HtGeom {
  uint64_t size, mask, frac;
  uint32_t shift, buckets;
};

__device__ __forceinline__ uint64_t ht_mod(const HtGeom& g, uint64_t k) {
  return ((k & g.mask) * g.frac) >> g.shift;
}

__device__ __forceinline__ uint64_t ring_dist(uint64_t a, uint64_t b, uint64_t size) {
  return b >= a ? b - a : b + size - a;
}

__device__ __forceinline__ bool slot_clash(const HtGeom& g, uint64_t a, uint64_t b) {
  return ((uint32_t)(a ^ b) & 8191u) == 0 || ring_dist(a, b, g.size) < g.buckets ||
         ring_dist(b, a, g.size) < g.buckets;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// Bound on rejection steps per alternate.  The reference loops without a
// bound; a geometry where no clash-free slot exists (table smaller than
// arity * (2 * buckets - 1)) is refused on the host, so the bound is never
// reached by a valid geometry (expected steps < 1.1).  A lane that reaches
// it stores the KVH_POS_NONE sentinel.
constexpr uint32_t kMaxCuckooSteps = 1u << 20;

template <int A>
__device__ __forceinline__ void cuckoo_positions(const HtGeom& g, uint64_t h1, uint64_t h2, uint64_t (&q)[A]) {
  q[0] = ht_mod(g, h1);
  if constexpr (A > 1) {
    uint64_t st = 0x9e3779b97f4a7c13ull ^ h2;
    uint64_t alt = h2;
    q[1] = ht_mod(g, h2);
    const bool redo1 = slot_clash(g, q[0], q[1]);
    if (redo1) alt = h1;
#pragma unroll
    for (int i = 1; i < A; i++) {
      if (i == 1 && !redo1) continue;
      uint32_t steps = 0;
      bool bad;
      do {
        const uint64_t x = alt, y = st ^ x;
        alt = rotl64(x, 55) ^ y ^ (y << 14);
        st = rotl64(y, 36);
        q[i] = ht_mod(g, alt);
        bad = false;
#pragma unroll
        for (int j = 0; j < i; j++) bad |= slot_clash(g, q[i], q[j]);
      } while (bad && ++steps < kMaxCuckooSteps);
      if (bad) q[i] = ~0ull;
    }
  }
}

}  // namespace kvh
