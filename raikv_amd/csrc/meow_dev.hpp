// meow_dev.hpp -- CDNA4 (gfx950) device building blocks for raikv's 128-bit
// Meow-derived key hash (reference: /root/reference/src/key_hash.c:1070-1429).
//
// Design:
//  * one lane per key; the AESDEC round is lowered to integer ALU + LDS
//    T-table lookups (no AES instruction on the GPU, no MFMA: this is not a
//    contraction);
//  * the inverse-cipher T-tables live in LDS replicated 32x so that lane l
//    always reads copy (l & 31): every ds_read_b32 lane group hits 32
//    distinct banks, i.e. random lookups are bank-conflict free;
//  * the LDS byte address of a lookup is built by ONE v_perm_b32 from the
//    state word and a per-lane "lane word":
//        addr = (t>>1)<<16 | x<<8 | (t&1)<<7 | (lane&31)<<2
//    (t = table 0..3, x = state byte);
//  * data-independent work is folded per (seed, length): the first AESDEC
//    of a state that still holds init^Mixer is T(init^Mixer) ^ K, states
//    that never see data are constants, and an AESDEC whose *state* input is
//    a constant is a single XOR.  16-byte keys need 5 table rounds instead
//    of 11.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "aes_tables.hpp"

namespace kvh {

__constant__ TdTable c_td0 = kTd0;

struct Blk { uint32_t w[4]; };

__device__ __forceinline__ Blk bxor(const Blk& a, const Blk& b) {
  Blk r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.w[i] = a.w[i] ^ b.w[i];
  return r;
}
__device__ __forceinline__ Blk bzero() { Blk r; r.w[0] = r.w[1] = r.w[2] = r.w[3] = 0; return r; }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) {
  return r == 0 ? x : ((x << r) | (x >> (32 - r)));
}
// gfx950 v_bitop3_b32 with truth table 0x96 = a ^ b ^ c in one VALU op
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ---------------------------------------------------------------- tables
// LDS-resident, bank-replicated tables.  NT = 4: Td0..Td3 (128 KiB);
// NT = 2: Td0, Td1 (64 KiB), Td2/Td3 lookups reuse them rotated by 16.
// NT = 5 (the round-4 A/B layout): Td0..Td3 with 16 copies each in the same
// 64 KiB -- the four-table round (6 VALU per column instead of 7) at a 2-way
// bank conflict per lookup (lanes l and l + 16 of a ds_read_b32 lane group
// share a copy).  Byte address  x<<8 | t<<6 | (lane&15)<<2.
template <int NT>
struct LdsTab {
  static constexpr int kTabs = NT == 5 ? 4 : NT;
  static constexpr int kCopies = NT == 5 ? 16 : 32;
  static constexpr int kWords = kTabs * 256 * kCopies;
  const uint32_t* lds;
  uint32_t lw[kTabs];

  __device__ __forceinline__ explicit LdsTab(const uint32_t* p) : lds(p) {
#pragma unroll
    for (int t = 0; t < kTabs; t++) {
      if constexpr (NT == 5)
        lw[t] = ((uint32_t)t << 6) | ((threadIdx.x & 15u) << 2);
      else
        lw[t] = ((uint32_t)(t >> 1) << 16) | ((uint32_t)(t & 1) << 7) | ((threadIdx.x & 31u) << 2);
    }
  }
  __device__ __forceinline__ uint32_t ld(uint32_t byteaddr) const {
    return *(const uint32_t*)((const char*)lds + byteaddr);
  }
  // perm selector: byte0 <- lane word byte0, byte1 <- state byte k,
  // byte2 <- lane word byte2, byte3 <- lane word byte3 (= 0)
  template <int K> static constexpr uint32_t sel() { return 0x03020000u | ((4u + K) << 8); }

  // Td0[a.b0] ^ Td1[b.b1] ^ Td2[c.b2] ^ Td3[d.b3] ^ k  (v_bitop3 0x96 = 3-way XOR)
  __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
    if constexpr (kTabs == 4) {
      const uint32_t t0 = ld(__builtin_amdgcn_perm(a, lw[0], sel<0>()));
      const uint32_t t1 = ld(__builtin_amdgcn_perm(b, lw[1], sel<1>()));
      const uint32_t t2 = ld(__builtin_amdgcn_perm(c, lw[2], sel<2>()));
      const uint32_t t3 = ld(__builtin_amdgcn_perm(d, lw[3], sel<3>()));
      return xor3(xor3(t0, t1, k), t2, t3);
    } else {
      const uint32_t t0 = ld(__builtin_amdgcn_perm(a, lw[0], sel<0>()));
      const uint32_t t1 = ld(__builtin_amdgcn_perm(b, lw[1], sel<1>()));
      const uint32_t t2 = ld(__builtin_amdgcn_perm(c, lw[0], sel<2>()));
      const uint32_t t3 = ld(__builtin_amdgcn_perm(d, lw[1], sel<3>()));
      return xor3(t0, t1, k) ^ rotl32(t2 ^ t3, 16);
    }
  }
  // A round key as colk() takes it: with two tables the Td2/Td3 half of a
  // column is rotl16(Td0[c] ^ Td1[d]); XORing rotl16(k) into it before the
  // rotation (one v_bitop3) saves the separate XOR of k, so a key used in
  // several rounds (an absorbed chunk twice, the Mixer up to six times) is
  // rotated once.  With four tables the key is used as it is.
  __device__ __forceinline__ static uint32_t prep(uint32_t k) { return kTabs == 4 ? k : rotl32(k, 16); }
  __device__ __forceinline__ uint32_t colk(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kp) const {
    if constexpr (kTabs == 4) {
      return col(a, b, c, d, kp);
    } else {
      const uint32_t t0 = ld(__builtin_amdgcn_perm(a, lw[0], sel<0>()));
      const uint32_t t1 = ld(__builtin_amdgcn_perm(b, lw[1], sel<1>()));
      const uint32_t t2 = ld(__builtin_amdgcn_perm(c, lw[0], sel<2>()));
      const uint32_t t3 = ld(__builtin_amdgcn_perm(d, lw[1], sel<3>()));
      return xor3(t0, t1, rotl32(xor3(t2, t3, kp), 16));
    }
  }
};

// fill the replicated tables; dword index i = addr >> 2 decodes to
// copy = i & 31, table = ((i>>14)&1)*2 + ((i>>5)&1), x = (i>>6) & 255
// (NT = 5: copy = i & 15, table = (i>>4) & 3, x = (i>>6) & 255)
// Eight table words per thread per batch, every load of a batch issued
// before its first write: a word-at-a-time loop waits one full memory round
// trip per word (32 in a row for a 1024-thread workgroup filling 128 KiB).
template <int NT>
__device__ __forceinline__ void fill_tables(uint32_t* lds) {
  constexpr uint32_t W = (uint32_t)LdsTab<NT>::kWords;
  constexpr int B = 8;
  const uint32_t bd = blockDim.x;
  auto batch = [&](uint32_t i0, auto guarded) {
    uint32_t v[B];
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint32_t i = i0 + (uint32_t)k * bd;
      v[k] = c_td0.v[(((guarded && i >= W) ? 0u : i) >> 6) & 255u];
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint32_t i = i0 + (uint32_t)k * bd;
      const uint32_t t = NT == 5 ? (i >> 4) & 3u : (((i >> 14) & 1u) << 1) | ((i >> 5) & 1u);
      if (!guarded || i < W) lds[i] = rotl32(v[k], 8 * (int)t);
    }
  };
  if (W % (B * bd) == 0) {  // workgroup-uniform: whole batches (1024 and 512 threads)
    for (uint32_t i0 = threadIdx.x; i0 < W; i0 += B * bd) batch(i0, std::false_type{});
  } else {
    for (uint32_t i0 = threadIdx.x; i0 < W; i0 += B * bd) batch(i0, std::true_type{});
  }
}

// Table access through the constant segment (tiny batches / drop-ins:
// no per-workgroup LDS fill).
struct ConstTab {
  __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
    return c_td0.v[a & 255] ^ rotl32(c_td0.v[(b >> 8) & 255], 8) ^
           rotl32(c_td0.v[(c >> 16) & 255], 16) ^ rotl32(c_td0.v[d >> 24], 24) ^ k;
  }
};

// Ablation table (experiments build only, k_var9 AB = 5): a "round" that is
// one XOR per column -- the kernel's work with the table rounds taken out.
struct XorTab {
  __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
    return xor3(a, b, c) ^ d ^ k;
  }
  __device__ __forceinline__ static uint32_t prep(uint32_t k) { return k; }
  __device__ __forceinline__ uint32_t colk(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
    return col(a, b, c, d, k);
  }
};

// Intel AESDEC(s, k) = InvMixColumns(InvSubBytes(InvShiftRows(s))) ^ k.
// Output column c takes row r from input column (c - r) & 3.
template <class Tab>
__device__ __forceinline__ Blk aesdec(const Blk& s, const Blk& k, const Tab& T) {
  Blk o;
#pragma unroll
  for (int c = 0; c < 4; c++)
    o.w[c] = T.col(s.w[c], s.w[(c + 3) & 3], s.w[(c + 2) & 3], s.w[(c + 1) & 3], k.w[c]);
  return o;
}
// a round key prepared for T.colk (see LdsTab::prep), and AESDEC with it
struct PKey {
  uint32_t w[4];
};
template <class Tab>
__device__ __forceinline__ PKey pkey(const Blk& k, const Tab&) {
  PKey p;
#pragma unroll
  for (int c = 0; c < 4; c++) p.w[c] = Tab::prep(k.w[c]);
  return p;
}
template <class Tab>
__device__ __forceinline__ Blk aesdec_p(const Blk& s, const PKey& k, const Tab& T) {
  Blk o;
#pragma unroll
  for (int c = 0; c < 4; c++)
    o.w[c] = T.colk(s.w[c], s.w[(c + 3) & 3], s.w[(c + 2) & 3], s.w[(c + 1) & 3], k.w[c]);
  return o;
}
// the keyless half: T(s) = AESDEC(s, 0)
template <class Tab>
__device__ __forceinline__ Blk aesT(const Blk& s, const Tab& T) {
  Blk o;
#pragma unroll
  for (int c = 0; c < 4; c++)
    o.w[c] = T.col(s.w[c], s.w[(c + 3) & 3], s.w[(c + 2) & 3], s.w[(c + 1) & 3], 0u);
  return o;
}

// ------------------------------------------------------- Meow constants
// Meow state init ramps (key_hash.c:1106-1113): state i = bytes 16i..16i+15
__device__ __forceinline__ Blk ramp(int i) {
  Blk r;
#pragma unroll
  for (int c = 0; c < 4; c++) r.w[c] = 0x03020100u + 0x04040404u * (uint32_t)c + 0x10101010u * (uint32_t)i;
  return r;
}
// Mixer = _mm_set_epi64x(seed2 + sz + 1, seed1 - sz)   (key_hash.c:1418)
__device__ __forceinline__ Blk mixer(uint64_t s1, uint64_t s2, uint64_t sz) {
  const uint64_t lo = s1 - sz, hi = s2 + sz + 1;
  Blk m;
  m.w[0] = (uint32_t)lo; m.w[1] = (uint32_t)(lo >> 32);
  m.w[2] = (uint32_t)hi; m.w[3] = (uint32_t)(hi >> 32);
  return m;
}

// Everything about a hash that depends only on (seed, length):
//   F[i]  = T(ramp_i ^ M)           first absorb into state i = F[i] ^ K, then 1 round
//   G[i]  = F[i] ^ M                state i after Mix_Meow when it never saw data
//   TG2   = T(G2)                   Compress2 S2 <- AESDEC(G2, S3) = TG2 ^ S3
//   CS2b  = AESDEC(AESDEC(G2,G3),M) Compress2 result for S2 when S2,S3 untouched
//   TCS0a = T(AESDEC(G0, G1))       Compress S0 <- AESDEC(const, S2) = TCS0a ^ S2
struct MeowConst {
  Blk M, F[4], G[4], TG2, CS2b, TCS0a;
};

template <class Tab>
__device__ __forceinline__ MeowConst make_const(uint64_t s1, uint64_t s2, uint64_t len, const Tab& T) {
  MeowConst K;
  K.M = mixer(s1, s2, len);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    K.F[i] = aesT(bxor(ramp(i), K.M), T);
    K.G[i] = bxor(K.F[i], K.M);
  }
  K.TG2 = aesT(K.G[2], T);
  K.CS2b = aesdec(bxor(K.TG2, K.G[3]), K.M, T);
  K.TCS0a = aesT(bxor(aesT(K.G[0], T), K.G[1]), T);
  return K;
}

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ Blk rfl(const Blk& b) {
  Blk r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.w[i] = rfl(b.w[i]);
  return r;
}
// move wave-uniform constants to SGPRs
__device__ __forceinline__ MeowConst uniform(const MeowConst& k) {
  MeowConst r;
  r.M = rfl(k.M);
#pragma unroll
  for (int i = 0; i < 4; i++) { r.F[i] = rfl(k.F[i]); r.G[i] = rfl(k.G[i]); }
  r.TG2 = rfl(k.TG2); r.CS2b = rfl(k.CS2b); r.TCS0a = rfl(k.TCS0a);
  return r;
}

// ------------------------------------------------- compile-time length
// Key of compile-time length L given as NC = ceil(L/16) chunks, chunk j =
// bytes [16j, 16j+16) zero padded past L.  Follows Meow_Loop/Meow_Loop_Trail
// (key_hash.c:1200-1226), Mix_Meow (:1155-1160), Compress_Meow2/_Meow
// (:1167-1176) as used by kv_hash_meow128 (:1413-1429).
template <int L>
struct Plan {
  static constexpr int NB = L / 64;           // full 64-byte blocks
  static constexpr int C = (L % 64) & 48;     // trail full-chunk bytes
  static constexpr int T = L & 15;            // partial tail bytes -> S3
  static constexpr int NC = (L + 15) / 16;
  static constexpr bool T0 = NB > 0 || C >= 16;
  static constexpr bool T1 = NB > 0 || C >= 32;
  static constexpr bool T2 = NB > 0 || C >= 48;
  static constexpr bool T3 = NB > 0 || T != 0;
};

template <int L, class Tab>
__device__ __forceinline__ Blk meow_ct(const Blk* D, const MeowConst& K, const Tab& T) {
  using P = Plan<L>;
  Blk S0, S1, S2, S3;
  // absorb full blocks; the first AESDEC on a state is folded
#pragma unroll
  for (int b = 0; b < P::NB; b++) {
    const Blk& k0 = D[4 * b + 0]; const Blk& k1 = D[4 * b + 1];
    const Blk& k2 = D[4 * b + 2]; const Blk& k3 = D[4 * b + 3];
    if (b == 0) {
      S0 = aesdec(bxor(K.F[0], k0), k0, T); S1 = aesdec(bxor(K.F[1], k1), k1, T);
      S2 = aesdec(bxor(K.F[2], k2), k2, T); S3 = aesdec(bxor(K.F[3], k3), k3, T);
    } else {
      S0 = aesdec(aesdec(S0, k0, T), k0, T); S1 = aesdec(aesdec(S1, k1, T), k1, T);
      S2 = aesdec(aesdec(S2, k2, T), k2, T); S3 = aesdec(aesdec(S3, k3, T), k3, T);
    }
  }
  constexpr bool first = P::NB == 0;
  constexpr int base = 4 * P::NB;
  if constexpr (P::T != 0) {
    const Blk& k = D[base + P::C / 16];
    S3 = first ? aesdec(bxor(K.F[3], k), k, T) : aesdec(aesdec(S3, k, T), k, T);
  }
  if constexpr (P::C >= 48) {
    const Blk& k = D[base + 2];
    S2 = first ? aesdec(bxor(K.F[2], k), k, T) : aesdec(aesdec(S2, k, T), k, T);
  }
  if constexpr (P::C >= 32) {
    const Blk& k = D[base + 1];
    S1 = first ? aesdec(bxor(K.F[1], k), k, T) : aesdec(aesdec(S1, k, T), k, T);
  }
  if constexpr (P::C >= 16) {
    const Blk& k = D[base + 0];
    S0 = first ? aesdec(bxor(K.F[0], k), k, T) : aesdec(aesdec(S0, k, T), k, T);
  }
  // Mix_Meow
  if constexpr (P::T3) S3 = aesdec(S3, K.M, T); else S3 = K.G[3];
  if constexpr (P::T2) S2 = aesdec(S2, K.M, T); else S2 = K.G[2];
  if constexpr (P::T1) S1 = aesdec(S1, K.M, T); else S1 = K.G[1];
  if constexpr (P::T0) S0 = aesdec(S0, K.M, T); else S0 = K.G[0];
  // Compress_Meow2: S2 = AESDEC(S2,S3); S0 = AESDEC(S0,S1); S2 = AESDEC(S2,M)
  Blk S2b;
  if constexpr (P::T2) S2b = aesdec(aesdec(S2, S3, T), K.M, T);
  else if constexpr (P::T3) S2b = aesdec(bxor(K.TG2, S3), K.M, T);
  else S2b = K.CS2b;
  // Compress_Meow: S0 = AESDEC(S0, S2); S0 = AESDEC(S0, M)
  Blk S0b;
  if constexpr (P::T0) S0b = aesdec(aesdec(S0, S1, T), S2b, T);
  else S0b = bxor(K.TCS0a, S2b);
  return aesdec(S0b, K.M, T);
}

// ---------------------------------------------------- runtime lengths
// bytes [p, p+n), 0 <= n <= 16, zero padded; reads only the dwords that
// intersect [p, p+n), so it never touches memory past the key's last byte's
// dword (no fault at the end of an allocation).
__device__ __forceinline__ Blk load_bytes(const uint8_t* p, uint32_t n) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(p - (a & 3));  // pointer arithmetic keeps the global address space
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t nd = (sh + n + 3) >> 2;
  uint32_t d[5];
#pragma unroll
  for (uint32_t j = 0; j < 5; j++) d[j] = j < nd ? q[j] : 0u;
  Blk r;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t v = __builtin_amdgcn_alignbyte(d[c + 1], d[c], sh);
    const int keep = (int)n - 4 * c;
    const uint32_t m = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
    r.w[c] = v & m;
  }
  return r;
}

// 16 bytes at any byte address p whose 16 bytes are all valid: one dwordx4
// from the enclosing dword-aligned address (every dword of it holds a byte of
// [p-3, p+16), so it never leaves the key's pages) plus one more dword when p
// is not dword aligned, funnel-shifted with v_alignbyte.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ Blk load16_full(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(p - (a & 3));  // pointer arithmetic keeps the global address space
  const uint32_t sh = (uint32_t)(a & 3);
  const u32x4_a4 v = *(const u32x4_a4*)q;
  const uint32_t e = sh ? q[4] : 0u;
  Blk r;
  r.w[0] = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
  r.w[1] = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
  r.w[2] = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
  r.w[3] = __builtin_amdgcn_alignbyte(e, v.w, sh);
  return r;
}

// Key-byte source for meow_rt: global memory (HBM/L2).
struct GlobalLd {
  static __device__ __forceinline__ Blk full(const uint8_t* p) { return load16_full(p); }
  static __device__ __forceinline__ Blk part(const uint8_t* p, uint32_t n) { return load_bytes(p, n); }
};
// Bytes at or past `end` read as zero: a key whose hashed length runs one
// byte past its stored bytes (a token hashed with the NUL that
// kv_set_key_frag_string appends, key_ctx.cpp:1764-1772) never reads the
// separator that follows it in the buffer.
struct MaskLd {
  const uint8_t* end;
  __device__ __forceinline__ Blk full(const uint8_t* p) const {
    if (p + 16 <= end) return load16_full(p);
    return p < end ? load_bytes(p, (uint32_t)(end - p)) : bzero();
  }
  __device__ __forceinline__ Blk part(const uint8_t* p, uint32_t n) const {
    const uint32_t m = p + n <= end ? n : (p < end ? (uint32_t)(end - p) : 0u);
    return m ? load_bytes(p, m) : bzero();
  }
};

// Source of per-length constants for the runtime path.
struct ConstRef {
  const MeowConst* k;
};

// Runtime-length Meow over key bytes at p (global memory).  Branches are
// wave-uniform when every lane has the same length (generic fixed-length
// kernel) and lane-divergent (masked) for variable-length batches.  LenT is
// uint32_t on the hot paths; uint64_t for keys (or window spans) of 4 GiB
// and more (kv_hash_meow128 takes a size_t length, key_hash.c:1413).
template <class Tab, class KGet, class Ld = GlobalLd, class LenT = uint32_t>
__device__ __forceinline__ Blk meow_rt(const uint8_t* p, LenT L, const KGet& K, const Tab& T,
                                       const Ld& ld = Ld{}) {
  const LenT nb = L >> 6;
  const uint32_t C = (uint32_t)L & 48, t = (uint32_t)L & 15;
  Blk S0, S1, S2, S3;
  if (nb > 0) {
    Blk k0 = ld.full(p), k1 = ld.full(p + 16), k2 = ld.full(p + 32),
        k3 = ld.full(p + 48);
    S0 = aesdec(bxor(K.F(0), k0), k0, T); S1 = aesdec(bxor(K.F(1), k1), k1, T);
    S2 = aesdec(bxor(K.F(2), k2), k2, T); S3 = aesdec(bxor(K.F(3), k3), k3, T);
    for (LenT b = 1; b < nb; b++) {
      const uint8_t* q = p + (LenT)64 * b;
      k0 = ld.full(q); k1 = ld.full(q + 16);
      k2 = ld.full(q + 32); k3 = ld.full(q + 48);
      S0 = aesdec(aesdec(S0, k0, T), k0, T); S1 = aesdec(aesdec(S1, k1, T), k1, T);
      S2 = aesdec(aesdec(S2, k2, T), k2, T); S3 = aesdec(aesdec(S3, k3, T), k3, T);
    }
  }
  const bool first = nb == 0;
  const uint8_t* q = p + (LenT)64 * nb;
  // trail (key_hash.c:1200-1210); a state's first absorb is folded
  if (t) {
    const Blk k = ld.part(q + C, t);
    S3 = first ? aesdec(bxor(K.F(3), k), k, T) : aesdec(aesdec(S3, k, T), k, T);
  }
  if (C >= 48) {
    const Blk k = ld.full(q + 32);
    S2 = first ? aesdec(bxor(K.F(2), k), k, T) : aesdec(aesdec(S2, k, T), k, T);
  }
  if (C >= 32) {
    const Blk k = ld.full(q + 16);
    S1 = first ? aesdec(bxor(K.F(1), k), k, T) : aesdec(aesdec(S1, k, T), k, T);
  }
  if (C >= 16) {
    const Blk k = ld.full(q);
    S0 = first ? aesdec(bxor(K.F(0), k), k, T) : aesdec(aesdec(S0, k, T), k, T);
  }
  const bool T0 = !first || C >= 16, T1 = !first || C >= 32, T2 = !first || C >= 48,
             T3 = !first || t != 0;
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

// A key's bytes read as dwordx4 GROUPS from the dword-aligned address at or
// below it: group i = dwords 4i..4i+3.  The L1 does not merge the misses of
// different load instructions, so every load instruction of a gather is one
// L2 request per lane (two when it straddles a line): meow_rt's pieces
// (dwordx4 + one more dword each) and dword-by-dword tails cost ~7 requests
// per C2 key, and the L1->L2 queue sets k_var6's time.  Here a key costs
// ceil((s + L) / 16) loads (s = p & 3), and piece k (bytes 16k..16k+15) is
// group k plus the first dword of group k+1, funnel-shifted by s: four
// v_alignbyte.  A group may run up to 12 bytes past the key's last dword
// (into the next key); `safe` says the caller's buffer holds those bytes,
// otherwise the group is read dword by dword, never past the key.
struct AChunks {
  const u32x4_a4* g;  // dword-aligned address at or below the key
  uint64_t lim;       // s + L: group i holds key bytes iff 16 i < lim
  uint32_t bs;        // s
  bool safe;
  __device__ __forceinline__ AChunks(const uint8_t* p, uint64_t L, bool sf) {
    const uint32_t s = (uint32_t)((uintptr_t)p & 3);
    g = (const u32x4_a4*)(p - s);  // pointer arithmetic keeps the global address space
    lim = s + L;
    bs = s;
    safe = sf;
  }
  __device__ __forceinline__ Blk chunk(uint64_t i) const {
    Blk r = bzero();
    if (16 * i < lim) {
      if (safe) {
        const u32x4_a4 v = g[i];
        r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
      } else {
        const uint32_t* d = (const uint32_t*)(g + i);
#pragma unroll
        for (int j = 0; j < 4; j++) r.w[j] = 16 * i + 4 * j < lim ? d[j] : 0u;
      }
    }
    return r;
  }
  // chunk(i) without the zero fill (round 4, knob 7 = 45): with `safe`, a
  // group past the key's last one is read as that last group instead of
  // being zeroed -- no per-load compare and exec split.  Bit-exact: the bytes
  // such a group feeds lie past the key, and meow_a only uses them in the
  // partial piece (masked to t bytes) or in pieces of states whose lane does
  // not take them (bsel on C); see meow_a.
  __device__ __forceinline__ Blk chunk_cl(uint64_t i) const {
    if (safe) {
      const uint32_t il = lim ? (uint32_t)((lim - 1) >> 4) : 0u;
      const uint32_t j = (uint32_t)i < il ? (uint32_t)i : il;
      const u32x4_a4 v = g[j];
      Blk r;
      r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
      return r;
    }
    return chunk(i);
  }
  __device__ __forceinline__ Blk piece(const Blk& A, const Blk& B) const {
    Blk r;
    r.w[0] = __builtin_amdgcn_alignbyte(A.w[1], A.w[0], bs);
    r.w[1] = __builtin_amdgcn_alignbyte(A.w[2], A.w[1], bs);
    r.w[2] = __builtin_amdgcn_alignbyte(A.w[3], A.w[2], bs);
    r.w[3] = __builtin_amdgcn_alignbyte(B.w[0], A.w[3], bs);
    return r;
  }
};
// per-word select (a ?: on the struct can become a select of addresses,
// i.e. a scratch copy)
__device__ __forceinline__ Blk bsel(bool c, const Blk& a, const Blk& b) {
  Blk r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.w[i] = c ? a.w[i] : b.w[i];
  return r;
}
// the first n bytes of b (n < 16), zero padded
__device__ __forceinline__ Blk mask_bytes(Blk b, uint32_t n) {
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int keep = (int)n - 4 * c;
    b.w[c] &= keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
  }
  return b;
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
// select after the trail.  Key bytes come as dwordx4 groups (AChunks): all
// chunks of a short key, and each block's four new chunks of a long key, are
// requested before the rounds that use them.  Same dataflow as
// key_hash.c:1155-1226.
// F[i] of a key known to be shorter than 64 bytes: K.Fs(i) where the
// accessor has one (one LDS record read, no select against the long-key
// fold table), else K.F(i)
template <class KGet>
__device__ __forceinline__ auto f_short(const KGet& K, int i, int) -> decltype(K.Fs(i)) { return K.Fs(i); }
template <class KGet>
__device__ __forceinline__ Blk f_short(const KGet& K, int i, long) { return K.F(i); }

// AB (experiments build only, counter ablations of C2's non-round work,
// DESIGN.md §3.3): 2 = groups read without the per-group bounds compare,
// 3 = the per-lane state selects (bsel) dropped, 4 = the partial piece not
// masked, 7 = no key loads (group data made from the address).  Outputs of
// AB != 0 are not hashes.
template <bool AL, int CM, bool PF, bool PKY = false, bool CL = false, int AB = 0, class Tab, class KGet,
          class LenT = uint32_t>
__device__ __forceinline__ Blk meow_a(const uint8_t* p, LenT L, bool safe, const KGet& K, const Tab& T) {
  constexpr bool P0 = AL || CM >= 16, P1 = AL || CM >= 32, P2 = AL || CM >= 48;  // state touched by some lane
  const LenT nb = L >> 6;
  const uint32_t C = (uint32_t)L & 48, t = (uint32_t)L & 15;
  const bool first = nb == 0;
  const AChunks A(p, L, safe);
  auto ch = [&](uint64_t i) {
    if constexpr (AB == 7) {  // no key loads: data made from the address
      Blk r;
      const uint32_t a = (uint32_t)(uintptr_t)A.g + 16u * (uint32_t)i;
      r.w[0] = a; r.w[1] = a ^ 0x9e3779b9u; r.w[2] = a + 7u; r.w[3] = a * 3u;
      return r;
    } else if constexpr (AB == 2) {
      if (A.safe) {
        const u32x4_a4 v = A.g[i];
        Blk r;
        r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
        return r;
      }
      return A.chunk(i);
    } else if constexpr (CL) {
      return A.chunk_cl(i);
    } else {
      return A.chunk(i);
    }
  };
  auto bsel = [](bool c, const Blk& a, const Blk& b) { if constexpr (AB == 3) return a; else return kvh::bsel(c, a, b); };
  auto mask_bytes = [](const Blk& b, uint32_t n) { if constexpr (AB == 4) return b; else return kvh::mask_bytes(b, n); };
  const Blk M = K.M();
  // PKY: keys used in more than one round go through LdsTab::prep once
  PKey MP{};
  if constexpr (PKY) MP = pkey(M, T);
  auto adM = [&](const Blk& x) { if constexpr (PKY) return aesdec_p(x, MP, T); else return aesdec(x, M, T); };
  auto ad2 = [&](const Blk& x, const Blk& k) {
    if constexpr (PKY) { const PKey kp = pkey(k, T); return aesdec_p(aesdec_p(x, kp, T), kp, T); }
    else return aesdec(aesdec(x, k, T), k, T);
  };
  // AESDEC(first ? f ^ k : AESDEC(s, k), k)
  auto adT = [&](bool first_, const Blk& f, const Blk& s_, const Blk& k) {
    // (AB 3 keeps the absorbed-state round: the ablation removes selects, not rounds)
    auto bselr = [](bool c, const Blk& a, const Blk& b) { if constexpr (AB == 3) return b; else return kvh::bsel(c, a, b); };
    if constexpr (PKY) { const PKey kp = pkey(k, T); return aesdec_p(bselr(first_, f, aesdec_p(s_, kp, T)), kp, T); }
    else return aesdec(bselr(first_, f, aesdec(s_, k, T)), k, T);
  };
  Blk S0 = bxor(ramp(0), M), S1 = bxor(ramp(1), M), S2 = bxor(ramp(2), M), S3 = bxor(ramp(3), M);
  // groups 4nb .. 4nb+4 (the trail's) once the blocks are absorbed
  Blk c0 = ch(0), c1, c2 = bzero(), c3 = bzero(), c4 = bzero();
  if constexpr (AL && PF) {
    // one block ahead: block b's rounds run while block b+1's groups (and,
    // in the last block, the trail's) are in flight
    c1 = ch(1); c2 = ch(2); c3 = ch(3); c4 = ch(4);
    if (!first) {
#define KVH_BLOCK(FIRST)                                                                                   \
  {                                                                                                        \
    const Blk n1 = ch(i + 5), n2 = ch(i + 6), n3 = ch(i + 7), n4 = ch(i + 8);         \
    const Blk k0 = A.piece(c0, c1), k1 = A.piece(c1, c2), k2 = A.piece(c2, c3), k3 = A.piece(c3, c4);     \
    if (FIRST) {                                                                                           \
      S0 = aesdec(bxor(K.F(0), k0), k0, T); S1 = aesdec(bxor(K.F(1), k1), k1, T);                           \
      S2 = aesdec(bxor(K.F(2), k2), k2, T); S3 = aesdec(bxor(K.F(3), k3), k3, T);                           \
    } else {                                                                                               \
      S0 = ad2(S0, k0); S1 = ad2(S1, k1);                                                                   \
      S2 = ad2(S2, k2); S3 = ad2(S3, k3);                                                                   \
    }                                                                                                      \
    c0 = c4; c1 = n1; c2 = n2; c3 = n3; c4 = n4;                                                           \
  }
      {
        const uint64_t i = 0;
        KVH_BLOCK(true)
      }
      for (LenT b = 1; b < nb; b++) {
        const uint64_t i = 4 * (uint64_t)b;
        KVH_BLOCK(false)
      }
#undef KVH_BLOCK
    }
  } else {
    if constexpr (AL) {
      if (!first) {
        {
          const Blk c1 = ch(1), c2 = ch(2), c3 = ch(3), c4 = ch(4);
          const Blk k0 = A.piece(c0, c1), k1 = A.piece(c1, c2), k2 = A.piece(c2, c3), k3 = A.piece(c3, c4);
          c0 = c4;
          S0 = aesdec(bxor(K.F(0), k0), k0, T); S1 = aesdec(bxor(K.F(1), k1), k1, T);
          S2 = aesdec(bxor(K.F(2), k2), k2, T); S3 = aesdec(bxor(K.F(3), k3), k3, T);
        }
        for (LenT b = 1; b < nb; b++) {
          const uint64_t i = 4 * (uint64_t)b;
          const Blk c1 = ch(i + 1), c2 = ch(i + 2), c3 = ch(i + 3), c4 = ch(i + 4);
          const Blk k0 = A.piece(c0, c1), k1 = A.piece(c1, c2), k2 = A.piece(c2, c3), k3 = A.piece(c3, c4);
          c0 = c4;
          S0 = ad2(S0, k0); S1 = ad2(S1, k1);
          S2 = ad2(S2, k2); S3 = ad2(S3, k3);
        }
      }
    }
    // trail pieces: groups 4nb .. 4nb + CM/16 + 1; piece j feeds state j,
    // the partial piece C/16 (t bytes) state 3
    const uint64_t i0 = 4 * (uint64_t)nb;
    c1 = ch(i0 + 1);
    if constexpr (CM >= 16) c2 = ch(i0 + 2);
    if constexpr (CM >= 32) c3 = ch(i0 + 3);
    if constexpr (CM >= 48) c4 = ch(i0 + 4);
  }
  const Blk q0 = A.piece(c0, c1);
  Blk q1 = bzero(), q2 = bzero(), q3 = bzero();
  if constexpr (CM >= 16) q1 = A.piece(c1, c2);
  if constexpr (CM >= 32) q2 = A.piece(c2, c3);
  if constexpr (CM >= 48) q3 = A.piece(c3, c4);
  Blk r3 = q0;
  if constexpr (CM >= 16) r3 = bsel(C >= 16, q1, r3);
  if constexpr (CM >= 32) r3 = bsel(C >= 32, q2, r3);
  if constexpr (CM >= 48) r3 = bsel(C >= 48, q3, r3);
  r3 = mask_bytes(r3, t);
  if constexpr (AL) {
    // a block-absorbed state takes two rounds, an init state the folded one
    {
      const Blk Y = adT(first, bxor(K.F0(3), r3), S3, r3);
      S3 = bsel(t != 0, Y, S3);
    }
    if constexpr (CM >= 48) {
      const Blk Y = adT(first, bxor(K.F0(2), q2), S2, q2);
      S2 = bsel(C >= 48, Y, S2);
    }
    if constexpr (CM >= 32) {
      const Blk Y = adT(first, bxor(K.F0(1), q1), S1, q1);
      S1 = bsel(C >= 32, Y, S1);
    }
    if constexpr (CM >= 16) {
      const Blk Y = adT(first, bxor(K.F0(0), q0), S0, q0);
      S0 = bsel(C >= 16, Y, S0);
    }
  } else {
    {
      const Blk Y = aesdec(bxor(f_short(K, 3, 0), r3), r3, T);
      S3 = bsel(t != 0, Y, S3);
    }
    if constexpr (CM >= 48) { const Blk Y = aesdec(bxor(f_short(K, 2, 0), q2), q2, T); S2 = bsel(C >= 48, Y, S2); }
    if constexpr (CM >= 32) { const Blk Y = aesdec(bxor(f_short(K, 1, 0), q1), q1, T); S1 = bsel(C >= 32, Y, S1); }
    if constexpr (CM >= 16) { const Blk Y = aesdec(bxor(f_short(K, 0, 0), q0), q0, T); S0 = bsel(C >= 16, Y, S0); }
  }
  S3 = adM(S3);
  if constexpr (P2) S2 = adM(S2); else S2 = K.G(2);
  if constexpr (P1) S1 = adM(S1); else S1 = K.G(1);
  if constexpr (P0) S0 = adM(S0); else S0 = K.G(0);
  Blk S2b;
  if constexpr (P2) S2b = adM(aesdec(S2, S3, T));
  else S2b = adM(bxor(K.TG2(), S3));
  Blk S0b;
  if constexpr (P0) S0b = bxor(aesT(aesdec(S0, S1, T), T), S2b);
  else S0b = bxor(K.TCS0a(), S2b);
  return adM(S0b);
}

// constants held in registers (uniform length)
struct RegK {
  const MeowConst& k;
  __device__ __forceinline__ Blk M() const { return k.M; }
  __device__ __forceinline__ Blk F(int i) const { return k.F[i]; }
  __device__ __forceinline__ Blk G(int i) const { return k.G[i]; }
  __device__ __forceinline__ Blk TG2() const { return k.TG2; }
  __device__ __forceinline__ Blk CS2b() const { return k.CS2b; }
  __device__ __forceinline__ Blk TCS0a() const { return k.TCS0a; }
};

// ------------------------------------------- literal restatement (small)
// Straight-line kv_hash_meow128 with no folding: used by the tiny-batch /
// drop-in kernel, and as an independent second device path in tests.
template <class Tab>
__device__ __forceinline__ Blk absorb2(const Blk& s, const Blk& k, const Tab& T) {
  return aesdec(aesdec(s, k, T), k, T);
}

struct MeowState { Blk S[4]; };

// key-byte source of the literal path: global memory (bytes at or past the
// key's last dword never read), or an LDS copy (LdsBytes)
struct GlobalBytes {
  __device__ __forceinline__ Blk part(const uint8_t* p, uint32_t n) const { return load_bytes(p, n); }
};
// bytes [p, p+n) of an LDS buffer, zero padded: the five dwords around them
// (the buffer must hold 20 readable bytes from the dword at or below p),
// funnel-shifted and masked
struct LdsBytes {
  __device__ __forceinline__ Blk part(const uint8_t* p, uint32_t n) const {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(p - (a & 3));
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[5];
#pragma unroll
    for (int j = 0; j < 5; j++) d[j] = q[j];
    Blk r;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t v = __builtin_amdgcn_alignbyte(d[c + 1], d[c], sh);
      const int keep = (int)n - 4 * c;
      r.w[c] = v & (keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u));
    }
    return r;
  }
};

template <class Tab, class Ld = GlobalBytes>
__device__ __forceinline__ void absorb_blocks(MeowState& st, const uint8_t* p, uint64_t nblk, const Tab& T,
                                              const Ld& ld = Ld{}) {
  for (uint64_t b = 0; b < nblk; b++, p += 64) {
#pragma unroll
    for (int i = 0; i < 4; i++) st.S[i] = absorb2(st.S[i], ld.part(p + 16 * i, 16), T);
  }
}

// Meow_Loop with `sz` selecting the trail (key_hash.c:1212-1226)
template <class Tab, class Ld = GlobalBytes>
__device__ __forceinline__ void absorb_loop(MeowState& st, const uint8_t* p, uint64_t sz, const Tab& T,
                                            const Ld& ld = Ld{}) {
  const uint64_t nblk = sz >> 6;
  absorb_blocks(st, p, nblk, T, ld);
  p += 64 * nblk;
  const uint32_t t = (uint32_t)sz & 15, C = (uint32_t)sz & 48;
  if (t) st.S[3] = absorb2(st.S[3], ld.part(p + C, t), T);
  if (C >= 48) st.S[2] = absorb2(st.S[2], ld.part(p + 32, 16), T);
  if (C >= 32) st.S[1] = absorb2(st.S[1], ld.part(p + 16, 16), T);
  if (C >= 16) st.S[0] = absorb2(st.S[0], ld.part(p, 16), T);
}

template <class Tab>
__device__ __forceinline__ Blk finish(MeowState& st, const Blk& M, const Tab& T) {
  st.S[3] = aesdec(st.S[3], M, T); st.S[2] = aesdec(st.S[2], M, T);
  st.S[1] = aesdec(st.S[1], M, T); st.S[0] = aesdec(st.S[0], M, T);
  st.S[2] = aesdec(st.S[2], st.S[3], T);
  st.S[0] = aesdec(st.S[0], st.S[1], T);
  st.S[2] = aesdec(st.S[2], M, T);
  st.S[0] = aesdec(st.S[0], st.S[2], T);
  return aesdec(st.S[0], M, T);
}

__device__ __forceinline__ void state_init(MeowState& st, const Blk& M) {
#pragma unroll
  for (int i = 0; i < 4; i++) st.S[i] = bxor(ramp(i), M);
}

template <class Tab, class Ld = GlobalBytes>
__device__ __forceinline__ Blk meow_literal(const uint8_t* p, uint64_t sz, uint64_t s1, uint64_t s2, const Tab& T,
                                            const Ld& ld = Ld{}) {
  MeowState st;
  const Blk M = mixer(s1, s2, sz);
  state_init(st, M);
  absorb_loop(st, p, sz, T, ld);
  return finish(st, M, T);
}

// KeyFragment::hash epilogue (include/raikv/hash_entry.h:84-85):
// clear the ZOMBIE bit 63 of h1; 0 and 1 are reserved -> 2
__device__ __forceinline__ Blk fixup(Blk h) {
  h.w[1] &= 0x7fffffffu;
  if (h.w[1] == 0 && h.w[0] <= 1u) h.w[0] = 2u;
  return h;
}

}  // namespace kvh
