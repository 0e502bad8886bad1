// bs_host_test.cpp -- TEST ONLY: runs the bitsliced Meow chain of
// raikv_amd/csrc/bs_meow.hpp (and the generated round, bs_aes.hpp) on the
// host, with the gfx950 primitives (v_bitop3, v_alignbit, v_perm) emulated
// bit by bit, and checks it against the clean-room oracle
// (oracle/liboracle.so: orc_meow128 = kv_hash_meow128, key_hash.c:1413-1429).
// The folding constants come from the oracle's AESDEC (orc_aesdec).
// Prints "bs_host_test ok N" on success; exits 1 on the first mismatch.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define KVH_BS_DEV inline
namespace kvh {
namespace bs {
template <uint32_t TT>
static inline uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r = 0;
  for (int bit = 0; bit < 32; bit++) {
    const uint32_t idx = (((a >> bit) & 1u) << 2) | (((b >> bit) & 1u) << 1) | ((c >> bit) & 1u);
    r |= ((TT >> idx) & 1u) << bit;
  }
  return r;
}
static inline uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)(((((uint64_t)hi) << 32) | lo) >> (s & 31u));
}
static inline uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  const uint64_t v = (((uint64_t)hi) << 32) | lo;
  uint32_t r = 0;
  for (int k = 0; k < 4; k++) {
    const uint32_t s = (sel >> (8 * k)) & 255u;
    if (s >= 8) { fprintf(stderr, "perm selector %u not emulated\n", s); exit(2); }
    r |= (uint32_t)((v >> (8 * s)) & 255u) << (8 * k);
  }
  return r;
}
static inline uint32_t lane_val(uint32_t v, uint32_t) { return v; }
}  // namespace bs
}  // namespace kvh
#include "../../raikv_amd/csrc/bs_aes.hpp"
#include "../../raikv_amd/csrc/bs_meow.hpp"

extern "C" {
void orc_meow128(const void* p, size_t sz, uint64_t* x1, uint64_t* x2);
void orc_aesdec(const uint8_t* state, const uint8_t* key, uint8_t* out);
}

using namespace kvh::bs;

struct Blk16 { uint8_t b[16]; };
static Blk16 bx(const Blk16& a, const Blk16& c) { Blk16 r; for (int i = 0; i < 16; i++) r.b[i] = a.b[i] ^ c.b[i]; return r; }
static Blk16 aesd(const Blk16& s, const Blk16& k) { Blk16 r; orc_aesdec(s.b, k.b, r.b); return r; }
static Blk16 T(const Blk16& s) { Blk16 z; memset(z.b, 0, 16); return aesd(s, z); }
static void words(const Blk16& a, uint32_t (&w)[4]) { memcpy(w, a.b, 16); }

struct HostKS {
  enum { kZero = 0, kA0, kA1, kA2, kM, kG1, kG3, kCS2b, kMstd, kN };
  uint32_t m[kN][32];
  void get(int which, uint32_t (&k)[32]) const { memcpy(k, m[which], sizeof k); }
};

static HostKS make_ks(uint64_t s1, uint64_t s2, uint64_t L) {
  Blk16 M, F[4], G[4];
  const uint64_t lo = s1 - L, hi = s2 + L + 1;  // key_hash.c:1418
  memcpy(M.b, &lo, 8); memcpy(M.b + 8, &hi, 8);
  for (int i = 0; i < 4; i++) {
    Blk16 ramp;
    for (int q = 0; q < 16; q++) ramp.b[q] = (uint8_t)(16 * i + q);
    F[i] = T(bx(ramp, M));
    G[i] = bx(F[i], M);
  }
  const Blk16 CS2b = aesd(bx(T(G[2]), G[3]), M);
  HostKS ks;
  uint32_t z[4];
  const uint32_t zero[4] = {0, 0, 0, 0};
  for (uint32_t t = 0; t < 32; t++) {
    ks.m[HostKS::kZero][t] = mask_of(zero, t, kKap);
    words(F[0], z); ks.m[HostKS::kA0][t] = mask_of(z, t, kKapX);
    words(F[1], z); ks.m[HostKS::kA1][t] = mask_of(z, t, kKapX);
    words(F[2], z); ks.m[HostKS::kA2][t] = mask_of(z, t, kKapX);
    words(M, z); ks.m[HostKS::kM][t] = mask_of(z, t, kKap);
    ks.m[HostKS::kMstd][t] = mask_of(z, t, kStd);
    words(G[1], z); ks.m[HostKS::kG1][t] = mask_of(z, t, kKap);
    words(G[3], z); ks.m[HostKS::kG3][t] = mask_of(z, t, kKap);
    words(CS2b, z); ks.m[HostKS::kCS2b][t] = mask_of(z, t, kKap);
  }
  return ks;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {  // splitmix64
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int L>
static int run(int iters) {
  int checked = 0;
  for (int it = 0; it < iters; it++) {
    const uint64_t s1 = it == 0 ? 0 : rnd(), s2 = it == 0 ? 0 : (it == 1 ? ~0ull : rnd());
    const HostKS ks = make_ks(s1, s2, L);
    uint8_t key[8][L];
    for (int j = 0; j < 8; j++)
      for (int q = 0; q < L; q++) key[j][q] = (uint8_t)(it < 2 ? (j * 31 + q) : rnd());
    uint32_t w[L / 16][8][4];
    for (int c = 0; c < L / 16; c++)
      for (int j = 0; j < 8; j++) memcpy(w[c][j], key[j] + 16 * c, 16);
    uint32_t h[8][4];
    meow_bs<L>(w, ks, h);
    for (int j = 0; j < 8; j++) {
      uint64_t x1 = s1, x2 = s2;
      orc_meow128(key[j], L, &x1, &x2);
      const uint64_t g1 = h[j][0] | ((uint64_t)h[j][1] << 32), g2 = h[j][2] | ((uint64_t)h[j][3] << 32);
      if (g1 != x1 || g2 != x2) {
        fprintf(stderr, "MISMATCH L=%d it=%d key=%d: got %016llx:%016llx want %016llx:%016llx\n", L, it, j,
                (unsigned long long)g1, (unsigned long long)g2, (unsigned long long)x1, (unsigned long long)x2);
        return -1;
      }
      checked++;
    }
  }
  return checked;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  // transposes are involutions and invert each other
  uint32_t w[8][4], R[32], w2[8][4];
  for (int j = 0; j < 8; j++) for (int c = 0; c < 4; c++) w[j][c] = (uint32_t)rnd();
  to_bits(w, R);
  for (int r = 0; r < 4; r++)
    for (int i = 0; i < 8; i++)
      for (int c = 0; c < 4; c++)
        for (int j = 0; j < 8; j++) {
          const uint32_t want = (w[j][c] >> (8 * r + i)) & 1u, got = (R[8 * r + i] >> (8 * c + j)) & 1u;
          if (want != got) { fprintf(stderr, "to_bits layout wrong r%d i%d c%d j%d\n", r, i, c, j); return 1; }
        }
  from_bits(R, w2);
  if (memcmp(w, w2, sizeof w)) { fprintf(stderr, "from_bits(to_bits(w)) != w\n"); return 1; }
  int n = 0, k;
  if ((k = run<16>(iters)) < 0) return 1; n += k;
  if ((k = run<32>(iters)) < 0) return 1; n += k;
  if ((k = run<48>(iters)) < 0) return 1; n += k;
  printf("bs_host_test ok %d\n", n);
  return 0;
}
