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

// Geometry in kernel-argument form.  frac < 2^31 always (shift <= 30 and
// entries <= mask + 1, ht_init.cpp:139-150), so ht_mod is a 64x32 multiply.
// "Narrow" tables (mask and ht_size below 2^32, i.e. < 4G entries = maps
// under 256 GiB of 64 B entries) run every position computation in 32-bit
// arithmetic; the result is the same u64 value, since the product
// (k & mask) * frac < 2^64 does not wrap and every slot is < ht_size.
struct HtGeom {
  uint64_t size, mask;
  uint32_t frac, shift, buckets;
};

template <typename W> struct Slot;

template <> struct Slot<uint32_t> {  // narrow tables
  __device__ static __forceinline__ uint32_t mod(const HtGeom& g, uint64_t k) {
    const uint64_t p = (uint64_t)((uint32_t)k & (uint32_t)g.mask) * g.frac;
    return (uint32_t)(p >> g.shift);
  }
};

template <> struct Slot<uint64_t> {  // >= 4G-entry tables: u64 product, wraps like the reference
  __device__ static __forceinline__ uint64_t mod(const HtGeom& g, uint64_t k) {
    const uint64_t x = k & g.mask;
    const uint64_t p = (uint64_t)(uint32_t)x * g.frac + (((uint64_t)((uint32_t)(x >> 32) * g.frac)) << 32);
    return p >> g.shift;
  }
};

__device__ __forceinline__ uint64_t ht_mod(const HtGeom& g, uint64_t k) { return Slot<uint64_t>::mod(g, k); }

// KeyCtx::calc_offset(a, b) < B || calc_offset(b, a) < B for slots a, b <
// size: with d = calc_offset(a, b), calc_offset(b, a) is size - d (d > 0)
// or 0, so the pair clashes iff d < B or d > size - B.
template <typename W>
__device__ __forceinline__ bool slot_clash(W a, W b, W size, W buckets) {
  const W d = b >= a ? b - a : b + (size - a);
  return ((uint32_t)(a ^ b) & 8191u) == 0 || d < buckets || d > size - buckets;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// Bound on rejection steps per alternate.  The reference loops without a
// bound; a geometry where no clash-free slot exists (table smaller than
// arity * (2 * buckets - 1)) is refused on the host, so the bound is never
// reached by a valid geometry (expected steps < 1.1).  A lane that reaches
// it stores the ~0 sentinel.
constexpr uint32_t kMaxCuckooSteps = 1u << 20;

// The reference's loop (ht_cuckoo.cpp:50-78), kept for the rare lanes
// whose first candidates clash.
template <int A, typename W>
__device__ __forceinline__ void cuckoo_positions_loop(const HtGeom& g, uint64_t h1, uint64_t h2, W (&q)[A]) {
  q[0] = Slot<W>::mod(g, h1);
  if constexpr (A > 1) {
    const W size = (W)g.size, bk = (W)g.buckets;
    uint64_t st = 0x9e3779b97f4a7c13ull ^ h2;
    uint64_t alt = h2;
    q[1] = Slot<W>::mod(g, h2);
    const bool redo1 = slot_clash<W>(q[0], q[1], size, bk);
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
        q[i] = Slot<W>::mod(g, alt);
        bad = false;
#pragma unroll
        for (int j = 0; j < i; j++) bad |= slot_clash<W>(q[i], q[j], size, bk);
      } while (bad && ++steps < kMaxCuckooSteps);
      if (bad) q[i] = (W)~(W)0;
    }
  }
}

// Straight-line common case: alt1 = h2 and every alternate's first
// xoroshiro candidate clear of the earlier slots (all but ~1 key in 1400
// for A = 4).  Lanes where any candidate clashes redo the key through the
// loop form; both forms produce the reference's slots.
template <int A, typename W>
__device__ __forceinline__ void cuckoo_positions(const HtGeom& g, uint64_t h1, uint64_t h2, W (&q)[A]) {
  q[0] = Slot<W>::mod(g, h1);
  if constexpr (A > 1) {
    const W size = (W)g.size, bk = (W)g.buckets;
    uint64_t st = 0x9e3779b97f4a7c13ull ^ h2;
    uint64_t alt = h2;
    q[1] = Slot<W>::mod(g, h2);
    bool bad = slot_clash<W>(q[0], q[1], size, bk);
#pragma unroll
    for (int i = 2; i < A; i++) {
      const uint64_t x = alt, y = st ^ x;
      alt = rotl64(x, 55) ^ y ^ (y << 14);
      st = rotl64(y, 36);
      q[i] = Slot<W>::mod(g, alt);
#pragma unroll
      for (int j = 0; j < i; j++) bad |= slot_clash<W>(q[i], q[j], size, bk);
    }
    if (__builtin_expect(bad, 0)) cuckoo_positions_loop<A, W>(g, h1, h2, q);
  }
}

}  // namespace kvh
