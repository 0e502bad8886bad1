/*
 * oracle/crc_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker for
 * SURVEY.md §8 row f4, batched CRC32C).  Linked into liboracle.so; nothing
 * in the product links, loads or calls it.
 *
 * Clean-room restatement of raikv's kv_crc_c (src/key_hash.c:53-63): the
 * SSE4.2 crc32 instruction chain, started at `seed`, no pre/post inversion.
 * That instruction is the reflected CRC with the Castagnoli polynomial
 * 0x82F63B78 processed LSB-first; the 8/4/2/1-byte chunking of the
 * reference does not change the value, so this is the plain bit-serial
 * definition.  Also kv_hash_uint/_uint2 (:27-37: one 4-byte step),
 * kv_crc_c_array (:122-142) and kv_crc_c_key_array (:168-179, prefixes of
 * one buffer).
 *
 * Pinning: tests/golden/crc32c.npz holds outputs of the reference's own
 * functions (oracle/_ref/libkvref.so, key_hash.c compiled where it lies;
 * generator tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stddef.h>

uint32_t orc_crc_c(const void *p, size_t sz, uint32_t seed)
{
  const uint8_t *s = (const uint8_t *) p;
  uint32_t r = seed;
  for (size_t i = 0; i < sz; i++) {
    r ^= s[i];
    for (int b = 0; b < 8; b++) r = (r >> 1) ^ (0x82F63B78u & (0u - (r & 1u)));
  }
  return r;
}

uint32_t orc_hash_uint2(uint32_t r, uint32_t i) { return orc_crc_c(&i, 4, r); }

/* out[i] = crc of keys[offs[i] .. offs[i+1]) from seeds[i] (or seed) */
void orc_crc_batch_var(const uint8_t *keys, const uint64_t *offs, size_t n,
                       const uint32_t *seeds, uint32_t seed, uint32_t *out)
{
  for (size_t i = 0; i < n; i++)
    out[i] = orc_crc_c(keys + offs[i], (size_t) (offs[i + 1] - offs[i]), seeds ? seeds[i] : seed);
}

void orc_crc_batch_fixed(const uint8_t *keys, size_t len, size_t n,
                         const uint32_t *seeds, uint32_t seed, uint32_t *out)
{
  for (size_t i = 0; i < n; i++)
    out[i] = orc_crc_c(keys + i * len, len, seeds ? seeds[i] : seed);
}
