/*
 * oracle/cuckoo_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker
 * for SURVEY.md §8 row f1, table positions).  Linked into liboracle.so next
 * to meow_oracle.c; nothing in the product links, loads or calls it.
 *
 * Clean-room scalar restatement of how raikv turns one fixed-up key hash
 * (h1, h2) into hash-table positions:
 *
 *   geometry    HashTab::HashTab  src/ht_init.cpp:117-156
 *               (entries = ratio * data_area / entry_size; mask = 2^ceil(log2)-1;
 *               fraction chosen from shift = 30 down so that the largest
 *               index exceeds half the table, decremented if it hits it)
 *   home slot   FileHdr::ht_mod   include/raikv/shm_ht.h:181-184
 *               ((k & mask) * fraction) >> shift  (u64 arithmetic)
 *   alternates  CuckooAltHash::calc_hash  src/ht_cuckoo.cpp:38-79
 *               alt0 = h1 at its home slot; alt1 = h2 at ht_mod(h2) unless
 *               it collides with alt0; further alternates step a xoroshiro128+
 *               state (src/ht_cuckoo.cpp:20-27) seeded 0x9e3779b97f4a7c13 ^ h2
 *               until the position is clear of every earlier one
 *   collision   equal low 13 bits (the 8K PositionBits index,
 *               ht_cuckoo.cpp:15-16) or forward/backward ring distance
 *               (KeyCtx::calc_offset, include/raikv/key_ctx.h:473-477) below
 *               the bucket count
 *   linear      cuckoo_buckets <= 1 (KeyCtx::acquire takes the linear probe,
 *               src/key_ctx.cpp:130) or arity <= 1: the home slot only
 *               (KeyCtx::set_hash, src/key_ctx.cpp:89-94)
 *
 * Pinning: tests/golden/cuckoo_*.npz were produced by the reference's own
 * ht_init.cpp + ht_cuckoo.cpp compiled where they lie (oracle/ref_cuckoo.cpp,
 * oracle/Makefile -> oracle/_ref/libkvref_ht.so, generator
 * tests/golden/make_golden.py), including the SURVEY.md §8c "hello\0"
 * known-answer positions 727478/838349/167394/26629.
 */
#include <stdint.h>
#include <stddef.h>

typedef struct {
  uint64_t ht_size, ht_mod_mask, ht_mod_fraction;
  uint32_t ht_mod_shift;
  uint16_t cuckoo_buckets;
  uint8_t  cuckoo_arity, pad;
} orc_geom_t;

/* shm_ht.h:59-69 header regions that precede the table in the map */
#define ORC_HT_HDR_SIZE   (192u * 1024u)
#define ORC_HT_CTX_SIZE   (128u * 1024u)
#define ORC_HT_STATS_SIZE (128u * 1024u)

int orc_ht_geom(uint64_t map_size, uint32_t entry_size, float ratio,
                uint16_t buckets, uint8_t arity, orc_geom_t *g)
{
  const uint64_t hdr = ORC_HT_HDR_SIZE + ORC_HT_CTX_SIZE + ORC_HT_STATS_SIZE;
  uint64_t area, entries, mask = 0, frac = 0, top = 0;
  uint32_t bits = 1, shift;
  if (map_size <= hdr || entry_size == 0) return -1;
  area    = map_size - hdr;
  entries = (uint64_t) ((double) ratio * (double) area) / (uint64_t) entry_size;
  if (entries == 0) return -1;
  while (((uint64_t) 1 << bits) < entries) bits++;
  for (shift = 30; shift > 1; shift--) {
    mask = ((uint64_t) 1 << bits) - 1;
    frac = (uint64_t) (((double) entries / (double) mask) *
                       (double) ((uint64_t) 1 << shift));
    top  = (mask * frac) >> shift;
    if (top > entries / 2) {
      if (top == entries) frac--;
      break;
    }
  }
  g->ht_size = entries;
  g->ht_mod_mask = mask;
  g->ht_mod_fraction = frac;
  g->ht_mod_shift = shift;
  g->cuckoo_buckets = buckets;
  g->cuckoo_arity = arity;
  g->pad = 0;
  return 0;
}

static uint64_t home(const orc_geom_t *g, uint64_t k)
{
  return ((k & g->ht_mod_mask) * g->ht_mod_fraction) >> g->ht_mod_shift;
}

uint64_t orc_ht_mod(const orc_geom_t *g, uint64_t k) { return home(g, k); }

/* ring distance from a forward to b */
static uint64_t ring(uint64_t a, uint64_t b, uint64_t size)
{
  return b >= a ? b - a : b + size - a;
}

static int clash(const orc_geom_t *g, uint64_t a, uint64_t b)
{
  return ((a & 8191) == (b & 8191)) ||
         ring(a, b, g->ht_size) < g->cuckoo_buckets ||
         ring(b, a, g->ht_size) < g->cuckoo_buckets;
}

static uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* pos[0 .. orc_positions_per_key(g)) for one hash pair */
void orc_cuckoo_one(const orc_geom_t *g, uint64_t h1, uint64_t h2, uint64_t *pos)
{
  uint64_t st = 0x9e3779b97f4a7c13ULL ^ h2, alt;
  unsigned a = g->cuckoo_arity, i, j;
  pos[0] = home(g, h1);
  if (a <= 1 || g->cuckoo_buckets <= 1) return;
  alt    = h2;
  pos[1] = home(g, h2);
  i = 2;
  if (clash(g, pos[0], pos[1])) { alt = h1; i = 1; }
  for (; i < a; i++) {
    int bad;
    do {
      /* xoroshiro128+ step on (alt, st) */
      uint64_t x = alt, y = st ^ x;
      alt = rotl64(x, 55) ^ y ^ (y << 14);
      st  = rotl64(y, 36);
      pos[i] = home(g, alt);
      bad = 0;
      for (j = 0; j < i; j++) bad |= clash(g, pos[i], pos[j]);
    } while (bad);
  }
}

unsigned orc_positions_per_key(const orc_geom_t *g)
{
  return (g->cuckoo_arity > 1 && g->cuckoo_buckets > 1) ? g->cuckoo_arity : 1;
}

/* hashes: n x (h1,h2); pos: n x orc_positions_per_key(g) */
void orc_cuckoo_positions(const orc_geom_t *g, const uint64_t *hashes, size_t n, uint64_t *pos)
{
  const unsigned a = orc_positions_per_key(g);
  for (size_t i = 0; i < n; i++)
    orc_cuckoo_one(g, hashes[2 * i], hashes[2 * i + 1], pos + i * a);
}
