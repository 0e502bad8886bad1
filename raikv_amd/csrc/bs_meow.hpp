// bs_meow.hpp -- bitsliced Meow128 for fixed 16/32/48-byte keys, 8 keys per
// lane (raikv kv_hash_meow128, /root/reference/src/key_hash.c:1413-1429, with
// the folding of DESIGN.md §3.2).  Every AESDEC is the generated bitsliced
// round of bs_aes.hpp: VALU only, no LDS table lookups, so these keys can be
// hashed beside the T-table keys without competing for the LDS.
//
// Layout.  Key j (0..7) of a lane arrives as words w[j][c] (column c of a
// 16-byte chunk: byte r of w[j][c] = state byte (row r, column c)).  The
// bitsliced state R[8r + i] holds in byte lane c, bit j, bit i of state byte
// (r, c) of key j.  to_bits/from_bits convert (4x4 byte transpose per key
// with v_perm, then an 8x8 bit transpose inside each byte lane).
//
// Round keys.  A round with key k adds kappa(k) (bs_aes.hpp) in u-form: for a
// data-dependent key (a key chunk, or another state) that is a register
// array; for a (seed, length) constant it is a per-register mask whose byte
// lane c is 0x00 or 0xFF (the same bit for all 8 keys).  Masks are built in
// the kernel prologue, one register per constant: lane t < 32 holds the mask
// of register t; `KeySrc` expands one to 32 wave-uniform values per use.
#pragma once

namespace kvh {
namespace bs {

// ------------------------------------------------------------ transposes
// 4x4 byte transpose: out[r] byte c = in[c] byte r (an involution)
KVH_BS_DEV void btr4(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3) {
  const uint32_t t0 = perm(a1, a0, 0x06020400u), t1 = perm(a1, a0, 0x07030501u);
  const uint32_t t2 = perm(a3, a2, 0x06020400u), t3 = perm(a3, a2, 0x07030501u);
  a0 = perm(t2, t0, 0x05040100u);
  a2 = perm(t2, t0, 0x07060302u);
  a1 = perm(t3, t1, 0x05040100u);
  a3 = perm(t3, t1, 0x07060302u);
}

// 8x8 bit transpose inside every byte lane across x[0..7]:
// out[i] bit j = in[j] bit i (an involution)
KVH_BS_DEV void bitr8(uint32_t (&x)[8]) {
  constexpr uint32_t M4 = 0x0F0F0F0Fu, M2 = 0x33333333u, M1 = 0x55555555u;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t t = ((x[j] >> 4) ^ x[j + 4]) & M4;
    x[j + 4] ^= t; x[j] ^= t << 4;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (j & 2) continue;
    const uint32_t t = ((x[j] >> 2) ^ x[j + 2]) & M2;
    x[j + 2] ^= t; x[j] ^= t << 2;
  }
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const uint32_t t = ((x[j] >> 1) ^ x[j + 1]) & M1;
    x[j + 1] ^= t; x[j] ^= t << 1;
  }
}

// w[j][0..3] (8 keys, one 16-byte chunk each) -> bitsliced R[32]
KVH_BS_DEV void to_bits(const uint32_t (&w)[8][4], uint32_t (&R)[32]) {
  uint32_t X[4][8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t a0 = w[j][0], a1 = w[j][1], a2 = w[j][2], a3 = w[j][3];
    btr4(a0, a1, a2, a3);
    X[0][j] = a0; X[1][j] = a1; X[2][j] = a2; X[3][j] = a3;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    bitr8(X[r]);
#pragma unroll
    for (int i = 0; i < 8; i++) R[8 * r + i] = X[r][i];
  }
}

KVH_BS_DEV void from_bits(const uint32_t (&R)[32], uint32_t (&w)[8][4]) {
  uint32_t X[4][8];
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 8; i++) X[r][i] = R[8 * r + i];
    bitr8(X[r]);
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t a0 = X[0][j], a1 = X[1][j], a2 = X[2][j], a3 = X[3][j];
    btr4(a0, a1, a2, a3);
    w[j][0] = a0; w[j][1] = a1; w[j][2] = a2; w[j][3] = a3;
  }
}

// ------------------------------------------------------------ masks
enum MaskKind { kStd = 0, kKap = 1, kKapX = 2 };
// mask of register t for the 16-byte constant z (words z[0..3]):
// kStd: the bits of z; kKap: of kappa(z); kKapX: of kappa(z) ^ kappa(0)
KVH_BS_DEV uint32_t mask_of(const uint32_t (&z)[4], uint32_t t, int kind) {
  const uint32_t r = (t >> 3) & 3u, i = t & 7u;
  uint32_t m = 0;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    uint32_t b = (z[c] >> (8 * r)) & 255u;
    if (kind != kStd) b = kKappa[b] ^ (kind == kKapX ? kKappa[0] : 0u);
    if ((b >> i) & 1u) m |= 0xFFu << (8 * c);
  }
  return m;
}

// ------------------------------------------------------------ rounds
KVH_BS_DEV uint32_t rotrow(uint32_t x, int row) {  // rotate left by 8*row bits
  return row == 0 ? x : alignbit(x, x, 32u - 8u * (uint32_t)row);
}

// u <- u-form of AESDEC(state, key) for the state held in u-form; key = kappa(key)
KVH_BS_DEV void round_u(uint32_t (&u)[32], const uint32_t (&k)[32]) {
  uint32_t v[32];
#pragma unroll
  for (int row = 0; row < 4; row++) {
    uint32_t t[8];
    inv8(&u[8 * row], t);
#pragma unroll
    for (int i = 0; i < 8; i++) v[8 * row + i] = rotrow(t[i], row);
  }
  lin(v, k, u);
}

// last round: out (standard basis) = AESDEC(state, key); key in standard bits
KVH_BS_DEV void round_out(const uint32_t (&u)[32], const uint32_t (&k)[32], uint32_t (&out)[32]) {
  uint32_t v[32];
#pragma unroll
  for (int row = 0; row < 4; row++) {
    uint32_t t[8];
    inv8(&u[8 * row], t);
#pragma unroll
    for (int i = 0; i < 8; i++) v[8 * row + i] = rotrow(t[i], row);
  }
  lin_out(v, k, out);
}

// kappa(K) = M1 K ^ kappa(0) per byte (K: bitsliced standard chunk)
template <class KS>
KVH_BS_DEV void kappa_bits(const uint32_t (&R)[32], const KS& ks, uint32_t (&Kc)[32]) {
  uint32_t k0[32];
  ks.get(KS::kZero, k0);
#pragma unroll
  for (int row = 0; row < 4; row++) m1(&R[8 * row], &k0[8 * row], &Kc[8 * row]);
}

// first absorb into state i: u-form of AESDEC(F_i ^ K, K) from Kc = kappa(K)
template <class KS>
KVH_BS_DEV void first_absorb(const uint32_t (&Kc)[32], const KS& ks, int which, uint32_t (&u)[32]) {
  uint32_t a[32];
  ks.get(which, a);
#pragma unroll
  for (int t = 0; t < 32; t++) u[t] = Kc[t] ^ a[t];
  round_u(u, Kc);
}

// Meow128 of 8 keys of length L (16, 32 or 48: full 16-byte chunks, no
// 64-byte block) per lane.  w[c][j][*] = chunk c of key j; h[j][*] = hash.
// KS supplies the constant masks (see KeySrc): indices below.
template <int L, class KS>
KVH_BS_DEV void meow_bs(const uint32_t (&w)[L / 16][8][4], const KS& ks, uint32_t (&h)[8][4]) {
  static_assert(L == 16 || L == 32 || L == 48, "bitsliced Meow: 16, 32 or 48-byte keys");
  uint32_t R[32], Kc[32], km[32];
  uint32_t S0[32], S1[32], S2[32];
  // S_c for each present chunk c, in u-form after Mix_Meow (key_hash.c:1155-1160)
  if constexpr (L >= 48) {
    to_bits(w[2], R);
    kappa_bits(R, ks, Kc);
    first_absorb(Kc, ks, KS::kA2, S2);
    ks.get(KS::kM, km); round_u(S2, km);
    // Compress_Meow2 with S3 untouched: S2 = AESDEC(AESDEC(S2, G3), M)
    ks.get(KS::kG3, km); round_u(S2, km);
    ks.get(KS::kM, km); round_u(S2, km);
  }
  if constexpr (L >= 32) {
    to_bits(w[1], R);
    kappa_bits(R, ks, Kc);
    first_absorb(Kc, ks, KS::kA1, S1);
    ks.get(KS::kM, km); round_u(S1, km);
  }
  to_bits(w[0], R);
  kappa_bits(R, ks, Kc);
  first_absorb(Kc, ks, KS::kA0, S0);
  ks.get(KS::kM, km); round_u(S0, km);
  // Compress_Meow: S0 = AESDEC(AESDEC(S0, S1), S2b), S2b = CS2b when S2,S3 untouched
  if constexpr (L >= 32) round_u(S0, S1); else { ks.get(KS::kG1, km); round_u(S0, km); }
  if constexpr (L >= 48) round_u(S0, S2); else { ks.get(KS::kCS2b, km); round_u(S0, km); }
  uint32_t O[32];
  ks.get(KS::kMstd, km);
  round_out(S0, km, O);
  from_bits(O, h);
}

// Constant masks held lane-distributed in VGPRs (lane t < 32 = register t),
// expanded to wave-uniform values with v_readlane per use.
struct KeySrc {
  enum { kZero = 0, kA0, kA1, kA2, kM, kG1, kG3, kCS2b, kMstd, kN };
  uint32_t lv[kN];
  KVH_BS_DEV void get(int which, uint32_t (&k)[32]) const {
#pragma unroll
    for (int t = 0; t < 32; t++) k[t] = lane_val(lv[which], (uint32_t)t);
  }
};

}  // namespace bs
}  // namespace kvh
