// aes_tables.hpp -- compile-time inverse-cipher T-table for the Meow128
// AESDEC round (Intel _mm_aesdec_si128 semantics, used by the reference at
// /root/reference/src/key_hash.c:1075-1081).
//
// Td0[x] packs the InvMixColumns column of InvSbox[x] for row 0 as a
// little-endian word: bytes (14s, 9s, 13s, 11s).  Rows 1..3 are the byte
// rotations rotl(Td0, 8r).  Everything is derived from GF(2^8) arithmetic by
// constexpr code; no table literal is copied from anywhere.
#pragma once
#include <stdint.h>

namespace kvh {

struct TdTable { uint32_t v[256]; };
struct SboxTable { uint8_t v[256]; };

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}

constexpr SboxTable make_inv_sbox() {
  SboxTable inv{};
  // multiplicative inverse via generator 3: walk the cyclic group once
  uint8_t log_t[256] = {};
  uint8_t exp_t[256] = {};
  uint8_t x = 1;
  for (int i = 0; i < 255; i++) {
    exp_t[i] = x;
    log_t[x] = (uint8_t)i;
    x = gf_mul(x, 3);
  }
  for (int a = 0; a < 256; a++) {
    uint8_t ia = 0;
    if (a) ia = exp_t[(255 - log_t[a]) % 255];
    uint8_t s = ia;
    for (int k = 1; k <= 4; k++) s ^= (uint8_t)((ia << k) | (ia >> (8 - k)));
    s ^= 0x63;
    inv.v[s] = (uint8_t)a;
  }
  return inv;
}

constexpr TdTable make_td0() {
  TdTable t{};
  SboxTable inv = make_inv_sbox();
  for (int x = 0; x < 256; x++) {
    uint8_t s = inv.v[x];
    t.v[x] = (uint32_t)gf_mul(s, 14) | ((uint32_t)gf_mul(s, 9) << 8) |
             ((uint32_t)gf_mul(s, 13) << 16) | ((uint32_t)gf_mul(s, 11) << 24);
  }
  return t;
}

constexpr TdTable kTd0 = make_td0();
constexpr SboxTable kInvSbox = make_inv_sbox();

// spot checks against the published FIPS-197 inverse S-box
static_assert(kInvSbox.v[0x00] == 0x52 && kInvSbox.v[0x01] == 0x09 &&
              kInvSbox.v[0x63] == 0x00 && kInvSbox.v[0xff] == 0x7d,
              "inverse S-box derivation");

}  // namespace kvh
