/*
 * kvh_kv.h -- the kv_* symbols that libkvh_kv.so exports, for a raikv
 * build that links it in place of src/key_hash.c's Meow and CRC32C families.
 * The prototypes and types are the ones raikv's include/raikv/key_hash.h:8-20
 * (CRC32C) and :59-130 (Meow) declare (same names, argument meaning, x[] layouts and struct layouts), so
 * raikv's call sites (key_ctx.cpp:103, cli.cpp:846/1031, ctest.c:82, ...)
 * compile and link unchanged; only the Meow and CRC32C functions are
 * provided (HMAC-Meow is a different function, out of scope; kv_djb is an
 * inline function of key_hash.h itself).  Each call is one GPU round trip
 * (include/kvh.h, the drop-ins' latency note): link compatibility, not a
 * per-key hot path.  A GPU error aborts the process (the reference functions
 * cannot fail and have no error return).
 */
#ifndef KVH_KV_H
#define KVH_KV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef KVH_KV_NO_TYPES
typedef struct {
  uint64_t ctx[8];
} meow_ctx_t __attribute__((__aligned__(64)));

typedef struct {
  uint8_t block[64];
  size_t  off, total_update_sz;
} meow_block_t __attribute__((__aligned__(64)));

typedef struct {
  const void *p;
  size_t sz;
} meow_vec_t;
#endif

/* CRC32C (key_hash.h:8-20; key_hash.c:27-179) */
uint32_t kv_hash_uint(uint32_t i);
uint32_t kv_hash_uint2(uint32_t r, uint32_t i);
uint32_t kv_crc_c(const void *p, size_t sz, uint32_t seed);
void kv_crc_c_2_diff(const void *p, size_t sz, uint32_t *seed, const void *p2, size_t sz2, uint32_t *seed2);
void kv_crc_c_4_diff(const void *p, size_t sz, uint32_t *seed, const void *p2, size_t sz2, uint32_t *seed2,
                     const void *p3, size_t sz3, uint32_t *seed3, const void *p4, size_t sz4, uint32_t *seed4);
void kv_crc_c_array(const void **p, size_t *psz, uint32_t *seed, size_t count);
void kv_crc_c_key_array(const void *p, size_t *psz, uint32_t *seed, size_t count);

/* Meow (key_hash.h:59-130) */
uint64_t kv_hash_meow64(const void *p, size_t sz, uint64_t seed);
void kv_hash_meow128(const void *p, size_t sz, uint64_t *h1, uint64_t *h2);
void kv_hash_meow128_vec(const meow_vec_t *vec, size_t vec_sz, uint64_t *h1, uint64_t *h2);
void kv_meow128_init(meow_ctx_t *m, meow_block_t *b, uint64_t k1, uint64_t k2, size_t total_update_sz);
void kv_meow128_update(meow_ctx_t *m, meow_block_t *b, const void *p, size_t sz);
void kv_meow128_final(meow_ctx_t *m, meow_block_t *b, uint64_t *k1, uint64_t *k2);
void kv_meow_test(const void *p, size_t sz, uint64_t *k1, uint64_t *k2);
void kv_hash_meow128_2_same_length(const void *p, const void *p2, size_t sz, uint64_t *x4);
void kv_hash_meow128_4_same_length_a(const void **p, size_t sz, uint64_t *x);
void kv_hash_meow128_8_same_length_a(const void **p, size_t sz, uint64_t *x);
void kv_hash_meow128_4_same_length(const void *p, const void *p2, const void *p3, const void *p4, size_t sz,
                                   uint64_t *x);
void kv_hash_meow128_4_same_length_4_seed(const void *p, const void *p2, const void *p3, const void *p4,
                                          size_t sz, uint64_t *x);
void kv_hash_meow128_8_same_length(const void *p, const void *p2, const void *p3, const void *p4,
                                   const void *p5, const void *p6, const void *p7, const void *p8, size_t sz,
                                   uint64_t *x);
void kv_hash_meow128_2_diff_length(const void *p, size_t sz, const void *p2, size_t sz2, uint64_t *x);
void kv_hash_meow128_4_diff_length(const void *p, size_t sz, const void *p2, size_t sz2, const void *p3,
                                   size_t s3, const void *p4, size_t s4, uint64_t *x);

#ifdef __cplusplus
}
#endif

#endif /* KVH_KV_H */
