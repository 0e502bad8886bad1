/*
 * oracle/meow_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * Clean-room CPU restatement, in portable scalar C, of raikv's 128-bit
 * Meow-derived key hash.  Nothing in the product (raikv_amd/, include/)
 * links, loads or calls this file; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * Pinning: every function here is checked bit-exactly against golden
 * vectors produced by the reference itself (oracle/_ref, built from
 * /root/reference/src/key_hash.c by oracle/Makefile; fixtures committed in
 * tests/golden/, generator tests/golden/make_golden.py) and against the
 * README known-answer vector (README.md:130-137).
 *
 * Algorithm anchors (all in /root/reference):
 *   AESDEC                 = Intel _mm_aesdec_si128 semantics
 *                            (key_hash.c:1075-1081 uses it twice per block)
 *   state init ramps       key_hash.c:1106-1113, Declare_Meow :1149-1153
 *   Mixer                  key_hash.c:1418  (lo = seed1 - sz, hi = seed2 + sz + 1)
 *   Xor_Meow               key_hash.c:1178-1183
 *   Meow_Loop / _Trail     key_hash.c:1200-1226 (tail bytes -> S3 at sz&48)
 *   Mix_Meow               key_hash.c:1155-1160
 *   Compress_Meow2/_Meow   key_hash.c:1167-1176
 *   kv_hash_meow128        key_hash.c:1413-1429
 *   kv_hash_meow128_vec    key_hash.c:1431-1483
 *   kv_hash_meow64         key_hash.c:1485-1491
 *   kv_meow128_init/update/final  key_hash.c:1509-1568
 *   KeyFragment::hash fixup  include/raikv/hash_entry.h:80-86
 *
 * The AES S-box is derived from GF(2^8) arithmetic at first use (no table
 * is copied from anywhere).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

typedef struct { uint8_t b[16]; } orc_blk;

static uint8_t inv_sbox[256];
static int     sbox_ready;

static uint8_t gf_mul(uint8_t a, uint8_t b)
{
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}

static void init_sbox(void)
{
  if (sbox_ready) return;
  for (int x = 0; x < 256; x++) {
    uint8_t inv = 0;
    if (x) { /* brute-force multiplicative inverse */
      for (int y = 1; y < 256; y++)
        if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    }
    uint8_t s = inv;
    for (int k = 1; k <= 4; k++)
      s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    s ^= 0x63;
    inv_sbox[s] = (uint8_t)x;
  }
  sbox_ready = 1;
}

/* Intel AESDEC: InvShiftRows, InvSubBytes, InvMixColumns, then XOR key.
 * Byte i of the 16-byte block is row (i & 3), column (i >> 2). */
static orc_blk aesdec(orc_blk s, orc_blk k)
{
  orc_blk t, o;
  for (int c = 0; c < 4; c++)
    for (int r = 0; r < 4; r++)
      t.b[4 * c + r] = inv_sbox[s.b[4 * (((c - r) & 3)) + r]];
  for (int c = 0; c < 4; c++) {
    uint8_t a0 = t.b[4 * c], a1 = t.b[4 * c + 1], a2 = t.b[4 * c + 2],
            a3 = t.b[4 * c + 3];
    o.b[4 * c + 0] = gf_mul(a0, 14) ^ gf_mul(a1, 11) ^ gf_mul(a2, 13) ^ gf_mul(a3, 9);
    o.b[4 * c + 1] = gf_mul(a0, 9) ^ gf_mul(a1, 14) ^ gf_mul(a2, 11) ^ gf_mul(a3, 13);
    o.b[4 * c + 2] = gf_mul(a0, 13) ^ gf_mul(a1, 9) ^ gf_mul(a2, 14) ^ gf_mul(a3, 11);
    o.b[4 * c + 3] = gf_mul(a0, 11) ^ gf_mul(a1, 13) ^ gf_mul(a2, 9) ^ gf_mul(a3, 14);
  }
  for (int i = 0; i < 16; i++) o.b[i] ^= k.b[i];
  return o;
}

static orc_blk load16(const uint8_t *p) { orc_blk r; memcpy(r.b, p, 16); return r; }
static orc_blk xorb(orc_blk a, orc_blk b)
{
  for (int i = 0; i < 16; i++) a.b[i] ^= b.b[i];
  return a;
}
/* the first n bytes of p, zero padded (Meow_AESDECx2_Partial :1118-1147
 * semantically: the masked over-read yields exactly these bytes) */
static orc_blk load_partial(const uint8_t *p, size_t n)
{
  orc_blk r; memset(r.b, 0, 16); memcpy(r.b, p, n); return r;
}
static orc_blk absorb2(orc_blk s, orc_blk k) { return aesdec(aesdec(s, k), k); }

static orc_blk make_mixer(uint64_t s1, uint64_t s2, uint64_t sz)
{
  orc_blk m;
  uint64_t lo = s1 - sz, hi = s2 + sz + 1;
  memcpy(m.b, &lo, 8);
  memcpy(m.b + 8, &hi, 8);
  return m;
}

typedef struct { orc_blk S[4]; } orc_state;

static void state_init(orc_state *st, orc_blk mixer)
{
  for (int i = 0; i < 4; i++) {
    for (int j = 0; j < 16; j++) st->S[i].b[j] = (uint8_t)(16 * i + j);
    st->S[i] = xorb(st->S[i], mixer);
  }
}

/* full 64-byte blocks only (Meow_Loop64) */
static void absorb_blocks(orc_state *st, const uint8_t *p, size_t nblk)
{
  for (size_t b = 0; b < nblk; b++, p += 64)
    for (int i = 0; i < 4; i++) st->S[i] = absorb2(st->S[i], load16(p + 16 * i));
}

/* Meow_Loop: full blocks then the trail, using `sz` for the trail split */
static void absorb_loop(orc_state *st, const uint8_t *p, size_t sz)
{
  size_t nblk = sz / 64;
  absorb_blocks(st, p, nblk);
  p += 64 * nblk;
  uint32_t len8 = (uint32_t)sz & 15, len128 = (uint32_t)sz & 48;
  if (len8) st->S[3] = absorb2(st->S[3], load_partial(p + len128, len8));
  if (len128 >= 48) st->S[2] = absorb2(st->S[2], load16(p + 32));
  if (len128 >= 32) st->S[1] = absorb2(st->S[1], load16(p + 16));
  if (len128 >= 16) st->S[0] = absorb2(st->S[0], load16(p));
}

static void finish(orc_state *st, orc_blk m, uint64_t *x1, uint64_t *x2)
{
  for (int i = 3; i >= 0; i--) st->S[i] = aesdec(st->S[i], m); /* Mix */
  st->S[2] = aesdec(st->S[2], st->S[3]);                         /* Compress2 */
  st->S[0] = aesdec(st->S[0], st->S[1]);
  st->S[2] = aesdec(st->S[2], m);
  st->S[0] = aesdec(st->S[0], st->S[2]);                         /* Compress */
  st->S[0] = aesdec(st->S[0], m);
  memcpy(x1, st->S[0].b, 8);
  memcpy(x2, st->S[0].b + 8, 8);
}

void orc_meow128(const void *p, size_t sz, uint64_t *x1, uint64_t *x2)
{
  init_sbox();
  orc_state st;
  orc_blk m = make_mixer(*x1, *x2, sz);
  state_init(&st, m);
  absorb_loop(&st, (const uint8_t *)p, sz);
  finish(&st, m, x1, x2);
}

uint64_t orc_meow64(const void *p, size_t sz, uint64_t seed)
{
  uint64_t h1 = seed, h2 = seed;
  orc_meow128(p, sz, &h1, &h2);
  return h1;
}

/* scatter/gather key == hash of the concatenation (key_hash.c:1431-1483) */
typedef struct { const void *p; size_t sz; } orc_vec_t;
void orc_meow128_vec(const orc_vec_t *vec, size_t vec_sz, uint64_t *x1, uint64_t *x2)
{
  size_t total = 0;
  for (size_t i = 0; i < vec_sz; i++) total += vec[i].sz;
  uint8_t tmp_small[512];
  uint8_t *buf = tmp_small;
  if (total > sizeof(tmp_small)) return; /* oracle is for small test keys */
  size_t off = 0;
  for (size_t i = 0; i < vec_sz; i++) {
    memcpy(buf + off, vec[i].p, vec[i].sz);
    off += vec[i].sz;
  }
  orc_meow128(buf, total, x1, x2);
}

/* KeyFragment::hash epilogue (hash_entry.h:84-85) */
static uint64_t fixup_h1(uint64_t h1)
{
  h1 &= ~((uint64_t)1 << 63);
  if (h1 <= 1) h1 = 2;
  return h1;
}

uint64_t orc_fixup(uint64_t h1) { return fixup_h1(h1); }

/* batch forms used by tests: out is [n][arity][2] (h1,h2) */
void orc_batch_fixed(const uint8_t *keys, size_t len, size_t n, uint64_t s1,
                     uint64_t s2, uint64_t *out, int fixup)
{
  for (size_t i = 0; i < n; i++) {
    uint64_t h1 = s1, h2 = s2;
    orc_meow128(keys + i * len, len, &h1, &h2);
    out[2 * i] = fixup ? fixup_h1(h1) : h1;
    out[2 * i + 1] = h2;
  }
}

void orc_batch_var(const uint8_t *keys, const uint64_t *offs, size_t n,
                   uint64_t s1, uint64_t s2, uint64_t *out, int fixup)
{
  for (size_t i = 0; i < n; i++) {
    uint64_t h1 = s1, h2 = s2;
    orc_meow128(keys + offs[i], (size_t)(offs[i + 1] - offs[i]), &h1, &h2);
    out[2 * i] = fixup ? fixup_h1(h1) : h1;
    out[2 * i + 1] = h2;
  }
}

void orc_batch_multiseed(const uint8_t *keys, size_t len, size_t n,
                         const uint64_t *seeds, size_t arity, uint64_t *out,
                         int fixup)
{
  for (size_t i = 0; i < n; i++)
    for (size_t a = 0; a < arity; a++) {
      uint64_t h1 = seeds[2 * a], h2 = seeds[2 * a + 1];
      orc_meow128(keys + i * len, len, &h1, &h2);
      out[2 * (i * arity + a)] = fixup ? fixup_h1(h1) : h1;
      out[2 * (i * arity + a) + 1] = h2;
    }
}

/* streaming (key_hash.c:1509-1568); the state layout is our own */
typedef struct {
  orc_state st;
  uint8_t   block[64];
  size_t    off, total;
} orc_stream_t;

void orc_stream_init(orc_stream_t *s, uint64_t k1, uint64_t k2, size_t total)
{
  init_sbox();
  state_init(&s->st, make_mixer(k1, k2, total));
  s->off = 0;
  s->total = total;
}

void orc_stream_update(orc_stream_t *s, const void *p, size_t sz)
{
  const uint8_t *src = (const uint8_t *)p;
  size_t len = sz;
  if (s->off > 0) {
    size_t fill = 64 - s->off;
    if (fill > len) fill = len;
    memcpy(s->block + s->off, src, fill);
    s->off += fill; len -= fill; src += fill;
    if (s->off == 64) { absorb_blocks(&s->st, s->block, 1); s->off = 0; }
  }
  if (len > 0) {
    s->off = len & 63;
    absorb_blocks(&s->st, src, (len - s->off) / 64);
    memcpy(s->block, src + (len - s->off), s->off);
  }
}

void orc_stream_final(orc_stream_t *s, uint64_t *k1, uint64_t *k2)
{
  if (s->off > 0) absorb_loop(&s->st, s->block, s->off);
  finish(&s->st, make_mixer(*k1, *k2, s->total), k1, k2);
}

size_t orc_stream_size(void) { return sizeof(orc_stream_t); }

/* one bare AESDEC round, exposed so tests can pin the round itself */
void orc_aesdec(const uint8_t *state, const uint8_t *key, uint8_t *out)
{
  init_sbox();
  orc_blk r = aesdec(load16(state), load16(key));
  memcpy(out, r.b, 16);
}
