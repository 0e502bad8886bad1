// meow_exp.hpp -- device helpers used only by the research kernels of
// tools/exp/kvh_exp.hip (experiments build, `make experiments`): the LDS
// key-byte source of k_var5, the prefetching variable-length Meow of
// k_var/k_var3/k_var6x/k_var7, its precursor of meow_a (meow_u) and the
// two-lanes-per-key Meow of k_var9x (meow_pair).  Not part of libkvh.so.
#pragma once
#include "../../raikv_amd/csrc/meow_dev.hpp"

namespace kvh {

// Key-byte source: an LDS staging buffer (dword reads only: misaligned LDS
// b128 reads replay at 64 cycles).
struct LdsLd {
  static __device__ __forceinline__ Blk full(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(p - (a & 3));  // pointer arithmetic keeps the global address space
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[5];
#pragma unroll
    for (int j = 0; j < 5; j++) d[j] = q[j];
    Blk r;
#pragma unroll
    for (int c = 0; c < 4; c++) r.w[c] = __builtin_amdgcn_alignbyte(d[c + 1], d[c], sh);
    return r;
  }
  static __device__ __forceinline__ Blk part(const uint8_t* p, uint32_t n) {
    Blk r = full(p);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int keep = (int)n - 4 * c;
      r.w[c] &= keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
    }
    return r;
  }
};


// Variable-length Meow with every load issued before the rounds that need
// it: the trail chunks and block 0 are requested up front, block b+1 while
// block b is absorbed.  Same dataflow and folding as meow_rt.
template <class Tab, class KGet, class LenT = uint32_t>
__device__ __forceinline__ Blk meow_var(const uint8_t* p, LenT L, const KGet& K, const Tab& T) {
  const LenT nb = L >> 6;
  const uint32_t C = (uint32_t)L & 48, t = (uint32_t)L & 15;
  const uint8_t* q = p + 64 * (uint64_t)nb;
  const Blk z = bzero();
  // trail chunks (key_hash.c:1200-1210) and the first full block, all in flight together
  const Blk r3 = t ? load_bytes(q + C, t) : z;
  const Blk r2 = C >= 48 ? load16_full(q + 32) : z;
  const Blk r1 = C >= 32 ? load16_full(q + 16) : z;
  const Blk r0 = C >= 16 ? load16_full(q) : z;
  Blk S0, S1, S2, S3;
  if (nb > 0) {
    Blk k0 = load16_full(p), k1 = load16_full(p + 16), k2 = load16_full(p + 32), k3 = load16_full(p + 48);
    Blk n0 = z, n1 = z, n2 = z, n3 = z;
    if (nb > 1) { n0 = load16_full(p + 64); n1 = load16_full(p + 80); n2 = load16_full(p + 96); n3 = load16_full(p + 112); }
    S0 = aesdec(bxor(K.F(0), k0), k0, T); S1 = aesdec(bxor(K.F(1), k1), k1, T);
    S2 = aesdec(bxor(K.F(2), k2), k2, T); S3 = aesdec(bxor(K.F(3), k3), k3, T);
    for (LenT b = 1; b < nb; b++) {
      k0 = n0; k1 = n1; k2 = n2; k3 = n3;
      if (b + 1 < nb) {
        const uint8_t* r = p + 64 * (uint64_t)(b + 1);
        n0 = load16_full(r); n1 = load16_full(r + 16); n2 = load16_full(r + 32); n3 = load16_full(r + 48);
      }
      S0 = aesdec(aesdec(S0, k0, T), k0, T); S1 = aesdec(aesdec(S1, k1, T), k1, T);
      S2 = aesdec(aesdec(S2, k2, T), k2, T); S3 = aesdec(aesdec(S3, k3, T), k3, T);
    }
  }
  const bool first = nb == 0;
  if (t) S3 = first ? aesdec(bxor(K.F(3), r3), r3, T) : aesdec(aesdec(S3, r3, T), r3, T);
  if (C >= 48) S2 = first ? aesdec(bxor(K.F(2), r2), r2, T) : aesdec(aesdec(S2, r2, T), r2, T);
  if (C >= 32) S1 = first ? aesdec(bxor(K.F(1), r1), r1, T) : aesdec(aesdec(S1, r1, T), r1, T);
  if (C >= 16) S0 = first ? aesdec(bxor(K.F(0), r0), r0, T) : aesdec(aesdec(S0, r0, T), r0, T);
  const bool T0 = !first || C >= 16, T1 = !first || C >= 32, T2 = !first || C >= 48, T3 = !first || t != 0;
  const Blk M = K.M();
  S3 = T3 ? aesdec(S3, M, T) : K.G(3);
  S2 = T2 ? aesdec(S2, M, T) : K.G(2);
  S1 = T1 ? aesdec(S1, M, T) : K.G(1);
  S0 = T0 ? aesdec(S0, M, T) : K.G(0);
  Blk S2b;
  if (T2) S2b = aesdec(aesdec(S2, S3, T), M, T);
  else if (T3) S2b = aesdec(bxor(K.TG2(), S3), M, T);
  else S2b = K.CS2b();
  Blk S0b;
  if (T0) S0b = aesdec(aesdec(S0, S1, T), S2b, T);
  else S0b = bxor(K.TCS0a(), S2b);
  return aesdec(S0b, M, T);
}

// First four 16-byte pieces a key consumes: block 0 for L >= 64, else the
// trail (full chunks at p, p+16, p+32 as present, partial tail at p+C).
// Issued one key ahead by k_var so the gather latency overlaps the rounds of
// the previous key.
__device__ __forceinline__ void prefetch_first(const uint8_t* p, uint32_t L, Blk (&pre)[4]) {
  const uint32_t nb = L >> 6, C = L & 48, t = L & 15;
  const Blk z = bzero();
  pre[0] = (nb || C >= 16) ? load16_full(p) : z;
  pre[1] = (nb || C >= 32) ? load16_full(p + 16) : z;
  pre[2] = (nb || C >= 48) ? load16_full(p + 32) : z;
  pre[3] = nb ? load16_full(p + 48) : (t ? load_bytes(p + C, t) : z);
}

// meow_var with the first four pieces supplied by prefetch_first; later
// blocks are fetched one block ahead and the trail of a long key together
// with its block 1.
template <class Tab, class KGet>
__device__ __forceinline__ Blk meow_var_pre(const uint8_t* p, uint32_t L, const Blk (&pre)[4], const KGet& K,
                                            const Tab& T) {
  const uint32_t nb = L >> 6, C = L & 48, t = L & 15;
  const bool first = nb == 0;
  Blk S0, S1, S2, S3, r0, r1, r2, r3;
  if (first) {
    r0 = pre[0]; r1 = pre[1]; r2 = pre[2]; r3 = pre[3];
  } else {
    const uint8_t* q = p + 64 * (uint64_t)nb;
    const Blk z = bzero();
    Blk n0 = z, n1 = z, n2 = z, n3 = z;
    if (nb > 1) { n0 = load16_full(p + 64); n1 = load16_full(p + 80); n2 = load16_full(p + 96); n3 = load16_full(p + 112); }
    r3 = t ? load_bytes(q + C, t) : z;
    r2 = C >= 48 ? load16_full(q + 32) : z;
    r1 = C >= 32 ? load16_full(q + 16) : z;
    r0 = C >= 16 ? load16_full(q) : z;
    S0 = aesdec(bxor(K.F(0), pre[0]), pre[0], T); S1 = aesdec(bxor(K.F(1), pre[1]), pre[1], T);
    S2 = aesdec(bxor(K.F(2), pre[2]), pre[2], T); S3 = aesdec(bxor(K.F(3), pre[3]), pre[3], T);
    for (uint32_t b = 1; b < nb; b++) {
      const Blk k0 = n0, k1 = n1, k2 = n2, k3 = n3;
      if (b + 1 < nb) {
        const uint8_t* r = p + 64 * (uint64_t)(b + 1);
        n0 = load16_full(r); n1 = load16_full(r + 16); n2 = load16_full(r + 32); n3 = load16_full(r + 48);
      }
      S0 = aesdec(aesdec(S0, k0, T), k0, T); S1 = aesdec(aesdec(S1, k1, T), k1, T);
      S2 = aesdec(aesdec(S2, k2, T), k2, T); S3 = aesdec(aesdec(S3, k3, T), k3, T);
    }
  }
  if (t) S3 = first ? aesdec(bxor(K.F(3), r3), r3, T) : aesdec(aesdec(S3, r3, T), r3, T);
  if (C >= 48) S2 = first ? aesdec(bxor(K.F(2), r2), r2, T) : aesdec(aesdec(S2, r2, T), r2, T);
  if (C >= 32) S1 = first ? aesdec(bxor(K.F(1), r1), r1, T) : aesdec(aesdec(S1, r1, T), r1, T);
  if (C >= 16) S0 = first ? aesdec(bxor(K.F(0), r0), r0, T) : aesdec(aesdec(S0, r0, T), r0, T);
  const bool T0 = !first || C >= 16, T1 = !first || C >= 32, T2 = !first || C >= 48, T3 = !first || t != 0;
  const Blk M = K.M();
  S3 = T3 ? aesdec(S3, M, T) : K.G(3);
  S2 = T2 ? aesdec(S2, M, T) : K.G(2);
  S1 = T1 ? aesdec(S1, M, T) : K.G(1);
  S0 = T0 ? aesdec(S0, M, T) : K.G(0);
  Blk S2b;
  if (T2) S2b = aesdec(aesdec(S2, S3, T), M, T);
  else if (T3) S2b = aesdec(bxor(K.TG2(), S3), M, T);
  else S2b = K.CS2b();
  Blk S0b;
  if (T0) S0b = aesdec(aesdec(S0, S1, T), S2b, T);
  else S0b = bxor(K.TCS0a(), S2b);
  return aesdec(S0b, M, T);
}

// Variable-length Meow written for a WAVE of keys whose shapes are bounded by
// two wave-uniform facts: AL = some lane's key has a full 64-byte block, CM =
// the largest trail-chunk count (L & 48) of any lane.  meow_rt's per-lane
// branches (one per trail chunk, one per Mix state, two in Compress) make the
// wave run every taken branch anyway, one after the other: each branch's
// load and each of its rounds is a separately exposed latency.  Here every
// trail load is issued before the first round, and the work any lane of the
// wave needs is done by all lanes in one basic block, so the (up to) four
// state chains of the trail and the Mix, and the two halves of Compress,
// interleave.  The LDS work is the same as the divergent code's (a round
// runs for the whole wave as soon as one lane needs it); lanes that do not
// need a state keep it at its init value ramp_i ^ M, for which the unfolded
// rounds give exactly the folded constants (AESDEC(init_i, M) = G_i,
// AESDEC(G2, S3) = TG2 ^ S3, T(AESDEC(G0, G1)) = TCS0a), so no lane needs a
// select after the trail.  Same dataflow as key_hash.c:1155-1226.
template <bool AL, int CM, class Tab, class KGet, class LenT = uint32_t>
__device__ __forceinline__ Blk meow_u(const uint8_t* p, LenT L, const KGet& K, const Tab& T) {
  constexpr bool P0 = AL || CM >= 16, P1 = AL || CM >= 32, P2 = AL || CM >= 48;  // state touched by some lane
  const LenT nb = L >> 6;
  const uint32_t C = (uint32_t)L & 48, t = (uint32_t)L & 15;
  const bool first = nb == 0;
  const uint8_t* q = p + (LenT)64 * nb;
  const Blk z = bzero();
  // short keys: every load before the first round; long keys: the trail's
  // loads together after the blocks (live across the block loop they spill)
#define KVH_TRAIL_LOADS                                                      \
  const Blk r3 = t ? load_bytes(q + C, t) : z;                               \
  const Blk r2 = (CM >= 48 && C >= 48) ? load16_full(q + 32) : z;            \
  const Blk r1 = (CM >= 32 && C >= 32) ? load16_full(q + 16) : z;            \
  const Blk r0 = (CM >= 16 && C >= 16) ? load16_full(q) : z;
  const Blk M = K.M();
  Blk S0 = bxor(ramp(0), M), S1 = bxor(ramp(1), M), S2 = bxor(ramp(2), M), S3 = bxor(ramp(3), M);
  if constexpr (AL) {
    if (!first) {
      const Blk k0 = load16_full(p), k1 = load16_full(p + 16), k2 = load16_full(p + 32), k3 = load16_full(p + 48);
      S0 = aesdec(bxor(K.F(0), k0), k0, T); S1 = aesdec(bxor(K.F(1), k1), k1, T);
      S2 = aesdec(bxor(K.F(2), k2), k2, T); S3 = aesdec(bxor(K.F(3), k3), k3, T);
      for (LenT b = 1; b < nb; b++) {
        const uint8_t* r = p + (LenT)64 * b;
        const Blk k0 = load16_full(r), k1 = load16_full(r + 16), k2 = load16_full(r + 32), k3 = load16_full(r + 48);
        S0 = aesdec(aesdec(S0, k0, T), k0, T); S1 = aesdec(aesdec(S1, k1, T), k1, T);
        S2 = aesdec(aesdec(S2, k2, T), k2, T); S3 = aesdec(aesdec(S3, k3, T), k3, T);
      }
    }
    KVH_TRAIL_LOADS
    // trail: a block-absorbed state takes two rounds, an init state the folded one
    {
      const Blk Y = aesdec(first ? bxor(K.F(3), r3) : aesdec(S3, r3, T), r3, T);
      if (t) S3 = Y;
    }
    if constexpr (CM >= 48) {
      const Blk Y = aesdec(first ? bxor(K.F(2), r2) : aesdec(S2, r2, T), r2, T);
      if (C >= 48) S2 = Y;
    }
    if constexpr (CM >= 32) {
      const Blk Y = aesdec(first ? bxor(K.F(1), r1) : aesdec(S1, r1, T), r1, T);
      if (C >= 32) S1 = Y;
    }
    if constexpr (CM >= 16) {
      const Blk Y = aesdec(first ? bxor(K.F(0), r0) : aesdec(S0, r0, T), r0, T);
      if (C >= 16) S0 = Y;
    }
  } else {
    KVH_TRAIL_LOADS
    {
      const Blk Y = aesdec(bxor(K.F(3), r3), r3, T);
      if (t) S3 = Y;
    }
    if constexpr (CM >= 48) { const Blk Y = aesdec(bxor(K.F(2), r2), r2, T); if (C >= 48) S2 = Y; }
    if constexpr (CM >= 32) { const Blk Y = aesdec(bxor(K.F(1), r1), r1, T); if (C >= 32) S1 = Y; }
    if constexpr (CM >= 16) { const Blk Y = aesdec(bxor(K.F(0), r0), r0, T); if (C >= 16) S0 = Y; }
  }
#undef KVH_TRAIL_LOADS
  // Mix_Meow: states no lane touched are the folded constants
  S3 = aesdec(S3, M, T);
  if constexpr (P2) S2 = aesdec(S2, M, T); else S2 = K.G(2);
  if constexpr (P1) S1 = aesdec(S1, M, T); else S1 = K.G(1);
  if constexpr (P0) S0 = aesdec(S0, M, T); else S0 = K.G(0);
  // Compress_Meow2 / Compress_Meow: the S2 chain and T(AESDEC(S0, S1)) are independent
  Blk S2b;
  if constexpr (P2) S2b = aesdec(aesdec(S2, S3, T), M, T);
  else S2b = aesdec(bxor(K.TG2(), S3), M, T);
  Blk S0b;
  if constexpr (P0) S0b = bxor(aesT(aesdec(S0, S1, T), T), S2b);
  else S0b = bxor(K.TCS0a(), S2b);
  return aesdec(S0b, M, T);
}


// Long keys, two lanes per key.  Until Compress a Meow state only ever meets
// its own 16-byte column of each block and its own trail chunk
// (key_hash.c:1155-1226), so lane half h (lane >> 5) carries states 2h and
// 2h+1 of the key both lanes of a pair were given: each lane loads the three
// dwordx4 groups its two columns need per block and runs two chains.  Mix is
// per state; Compress splits evenly: both halves form W = AESDEC(X, Y) and
// Z = T(W), which is T(AESDEC(S0, S1)) in the low half and, XORed with M,
// Compress_Meow2's AESDEC(AESDEC(S2, S3), M) in the high half; one
// v_permlane32_swap hands the high half's value down, and the low half runs
// the last round.  Against one lane per key this halves the lanes a chunk of
// long keys waits on its longest key for: a 64-key chunk is two 32-key
// halves, each as long as its own longest key (simulated over the C2 lengths:
// 1.60x -> 1.38x the ideal rounds).  Every lane must be active (permlane);
// a lane without a key passes L = 0.  The hash is valid in the low half.
template <class Tab, class KGet>
__device__ __forceinline__ Blk meow_pair(const uint8_t* p, uint32_t L, uint32_t h, bool safe, const KGet& K,
                                         const Tab& T) {
  const uint32_t nb = L >> 6, C = L & 48, t = L & 15;
  const bool first = nb == 0;
  const bool hi = h != 0;
  const int ix = 2 * (int)h, iy = ix + 1;
  const AChunks A(p, L, safe);
  const Blk M = K.M();
  Blk X = bxor(ramp(ix), M), Y = bxor(ramp(iy), M);
  if (!first) {
    {
      const Blk G0 = A.chunk(ix), G1 = A.chunk(ix + 1), G2 = A.chunk(ix + 2);
      const Blk kx = A.piece(G0, G1), ky = A.piece(G1, G2);
      X = aesdec(bxor(K.F(ix), kx), kx, T);
      Y = aesdec(bxor(K.F(iy), ky), ky, T);
    }
    for (uint32_t b = 1; b < nb; b++) {
      const uint64_t g = 4 * (uint64_t)b + ix;
      const Blk G0 = A.chunk(g), G1 = A.chunk(g + 1), G2 = A.chunk(g + 2);
      const Blk kx = A.piece(G0, G1), ky = A.piece(G1, G2);
      X = aesdec(aesdec(X, kx, T), kx, T);
      Y = aesdec(aesdec(Y, ky, T), ky, T);
    }
  }
  // trail: X takes piece 2h (state 0: C >= 16; state 2: C >= 48), Y piece 1
  // (state 1: C >= 32) or the partial piece C/16 of t bytes (state 3)
  const uint64_t i0 = 4 * (uint64_t)nb;
  const Blk z = bzero();
  const Blk g0 = A.chunk(i0), g1 = A.chunk(i0 + 1), g2 = A.chunk(i0 + 2);
  const Blk g3 = hi ? A.chunk(i0 + 3) : z, g4 = hi ? A.chunk(i0 + 4) : z;
  const Blk kx = A.piece(bsel(hi, g2, g0), bsel(hi, g3, g1));
  const uint32_t j = C >> 4;
  const Blk ya = bsel(j == 0, g0, bsel(j == 1, g1, bsel(j == 2, g2, g3)));
  const Blk yb = bsel(j == 0, g1, bsel(j == 1, g2, bsel(j == 2, g3, g4)));
  Blk ky = A.piece(bsel(hi, ya, g1), bsel(hi, yb, g2));
  ky = bsel(hi, mask_bytes(ky, t), ky);
  const bool cx = hi ? C >= 48 : C >= 16, cy = hi ? t != 0 : C >= 32;
  {
    const Blk X2 = aesdec(bsel(first, bxor(K.F0(ix), kx), aesdec(X, kx, T)), kx, T);
    const Blk Y2 = aesdec(bsel(first, bxor(K.F0(iy), ky), aesdec(Y, ky, T)), ky, T);
    X = bsel(cx, X2, X);
    Y = bsel(cy, Y2, Y);
  }
  X = aesdec(X, M, T);  // Mix_Meow (an untouched state holds its init value: this gives G)
  Y = aesdec(Y, M, T);
  const Blk Z = aesT(aesdec(X, Y, T), T);
  const Blk V = bsel(hi, bxor(Z, M), Z);
  Blk S0b;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const auto r = __builtin_amdgcn_permlane32_swap(V.w[w], V.w[w], false, false);
    S0b.w[w] = Z.w[w] ^ r[1];  // low half: T(AESDEC(S0, S1)) ^ S2b
  }
  return aesdec(S0b, M, T);
}


}  // namespace kvh
